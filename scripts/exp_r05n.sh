# r05n: small-call latency work (cached device count, 2-4 KiB parse pieces for calls of few
# segments, the metablock header and the context-mode scan as one-wave LDS kernels): GPU tests,
# c4 (stream bytes unchanged: 0.36281), the reference-cadence streaming leg and its kernel trace,
# latency and c2 legs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05n; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
timeout -k 10 300 python3 bench.py --workload c4 > $OUT/c4.json 2> $OUT/c4.err || { echo "c4 failed"; tail $OUT/c4.err; exit 1; }
MIB_DP_PIECES=3 BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_exp.so timeout -k 10 300 python3 bench.py --workload c4 --no-cpu-baseline > $OUT/c4_ps3.json 2> $OUT/c4_ps3.err || { echo "c4 ps3 failed"; exit 1; }
timeout -k 10 300 python3 bench.py --workload c5 --stream-chunk 0 --size 268435456 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/c5_cadence.json 2> $OUT/c5_cadence.err || { echo "cadence failed"; tail $OUT/c5_cadence.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o cad -- python3 bench.py --workload c5 --stream-chunk 0 --size 67108864 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/prof_cad.json 2> $OUT/prof_cad.err || { echo "prof failed"; tail $OUT/prof_cad.err; exit 1; }
for w in latency c2; do
  timeout -k 10 300 python3 bench.py --workload $w > $OUT/$w.json 2> $OUT/$w.err || { echo "$w failed"; tail $OUT/$w.err; exit 1; }
done
echo "exit=0"
