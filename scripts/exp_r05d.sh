# r05d: GPU tests on the product build (near scan + last-distance candidates in the parse +
# pinned-ring host copies), then c4 / c3 bench legs: product vs the experiment build with both
# compression changes off (MIB_NEAR=0 MIB_DP_REP=0), and the in-library host-buffer leg
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05d; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
for w in c4 c3; do
  timeout -k 10 300 python3 bench.py --workload $w > $OUT/${w}_new.json 2> $OUT/${w}_new.err || { echo "$w new failed"; tail $OUT/${w}_new.err; exit 1; }
  MIB_NEAR=0 MIB_DP_REP=0 BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_exp.so timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline > $OUT/${w}_base.json 2> $OUT/${w}_base.err || { echo "$w base failed"; tail $OUT/${w}_base.err; exit 1; }
done
timeout -k 10 300 python3 bench.py --gpus-in-lib 4 --no-cpu-baseline > $OUT/inlib4.json 2> $OUT/inlib4.err || { echo "inlib failed"; tail $OUT/inlib4.err; exit 1; }
echo "exit=0"
