# r05h: GPU tests; c4 / c3: HEAD build vs product (near scan as branch-free candidate masks);
# rocprofv3 kernel trace of c4 and c3 (product)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05h; mkdir -p $OUT
L=$PWD/brotli-lib_amd
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
for w in c4 c3; do
  BROTLI_AMD_LIB=$L/libbrotli_amd_head.so timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline > $OUT/${w}_head.json 2> $OUT/${w}_head.err || { echo "$w head failed"; tail $OUT/${w}_head.err; exit 1; }
  timeout -k 10 300 python3 bench.py --workload $w > $OUT/${w}_new.json 2> $OUT/${w}_new.err || { echo "$w new failed"; tail $OUT/${w}_new.err; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o $w -- python3 bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline > $OUT/prof_$w.json 2> $OUT/prof_$w.err || { echo "prof failed"; tail $OUT/prof_$w.err; exit 1; }
done
echo "exit=0"
