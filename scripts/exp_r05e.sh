# r05e: GPU tests (product: near scan with 4-byte words, last-distance parse candidates,
# pinned-ring host copies), then c4 / c3 legs: HEAD build (before the compression changes),
# the experiment build with each change alone, and the product
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05e; mkdir -p $OUT
L=$PWD/brotli-lib_amd
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
for w in c4 c3; do
  BROTLI_AMD_LIB=$L/libbrotli_amd_head.so timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline > $OUT/${w}_head.json 2> $OUT/${w}_head.err || { echo "$w head failed"; tail $OUT/${w}_head.err; exit 1; }
  MIB_NEAR=1 MIB_DP_REP=0 BROTLI_AMD_LIB=$L/libbrotli_amd_exp.so timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline > $OUT/${w}_near.json 2> $OUT/${w}_near.err || { echo "$w near failed"; tail $OUT/${w}_near.err; exit 1; }
  MIB_NEAR=0 MIB_DP_REP=1 BROTLI_AMD_LIB=$L/libbrotli_amd_exp.so timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline > $OUT/${w}_rep.json 2> $OUT/${w}_rep.err || { echo "$w rep failed"; tail $OUT/${w}_rep.err; exit 1; }
  timeout -k 10 300 python3 bench.py --workload $w > $OUT/${w}_new.json 2> $OUT/${w}_new.err || { echo "$w new failed"; tail $OUT/${w}_new.err; exit 1; }
done
echo "exit=0"
