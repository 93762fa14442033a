# r05g: as r05f with the near scan as 16-tile blocks, plus the host-buffer legs (pinned ring,
# trim hysteresis) twice
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05g; mkdir -p $OUT
L=$PWD/brotli-lib_amd
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
for w in c4 c3; do
  BROTLI_AMD_LIB=$L/libbrotli_amd_head.so timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline > $OUT/${w}_head.json 2> $OUT/${w}_head.err || { echo "$w head failed"; tail $OUT/${w}_head.err; exit 1; }
  MIB_NEAR=0 BROTLI_AMD_LIB=$L/libbrotli_amd_exp.so timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline > $OUT/${w}_nonear.json 2> $OUT/${w}_nonear.err || { echo "$w nonear failed"; tail $OUT/${w}_nonear.err; exit 1; }
  timeout -k 10 300 python3 bench.py --workload $w > $OUT/${w}_new.json 2> $OUT/${w}_new.err || { echo "$w new failed"; tail $OUT/${w}_new.err; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o c4 -- python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/prof_c4.json 2> $OUT/prof_c4.err || { echo "prof failed"; tail $OUT/prof_c4.err; exit 1; }
timeout -k 10 300 python3 bench.py --gpus-in-lib 4 --no-cpu-baseline > $OUT/inlib4.json 2> $OUT/inlib4.err || { echo "inlib failed"; tail $OUT/inlib4.err; exit 1; }
timeout -k 10 300 python3 bench.py --gpus-in-lib 4 --no-cpu-baseline > $OUT/inlib4b.json 2> $OUT/inlib4b.err || { echo "inlib b failed"; exit 1; }
echo "exit=0"
