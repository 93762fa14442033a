# r05l: (1) the counters this rocprofv3 offers; (2) the traffic calibration probe: its timings,
# then one --pmc pass per counter group; (3) exclusive kernel times: one encode lane
# (experiment build, MIB_ENC_LANES=1), c4 with and without the near scan, kernel traces
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05l; mkdir -p $OUT
L=$PWD/brotli-lib_amd
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1; echo "list rc=$?"
P=$PWD/scripts/probe/traffic_probe
timeout -k 10 120 $P > $OUT/probe.jsonl 2> $OUT/probe.err || { echo "probe failed"; tail $OUT/probe.err; exit 1; }
for c in FETCH_SIZE TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum; do
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o probe -- $P > $OUT/pmc_$c.log 2>&1; echo "pmc $c rc=$?"
done
MIB_ENC_LANES=1 BROTLI_AMD_LIB=$L/libbrotli_amd_exp.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof1 -o near -- python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/lane1_near.json 2> $OUT/lane1_near.err || { echo "lane1 near failed"; tail $OUT/lane1_near.err; exit 1; }
MIB_NEAR=0 MIB_ENC_LANES=1 BROTLI_AMD_LIB=$L/libbrotli_amd_exp.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof1 -o nonear -- python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/lane1_nonear.json 2> $OUT/lane1_nonear.err || { echo "lane1 nonear failed"; tail $OUT/lane1_nonear.err; exit 1; }
echo "exit=0"
