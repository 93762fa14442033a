# r05c: the test that hung in r05b (test_streaming_batch_matches_single), with the parse's
# last-distance candidates off (experiment build, MIB_DP_REP=0) and then on (product build);
# then the CPU-visible host-path legs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05c; mkdir -p $OUT
T="tests/test_gpu_encode.py::test_streaming_batch_matches_single"
MIB_DP_REP=0 BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_exp.so timeout -k 10 150 python3 -u -m pytest $T -x -v --timeout 120 --timeout-method thread > $OUT/norep.log 2>&1 || { echo "norep failed"; tail -30 $OUT/norep.log; exit 1; }
timeout -k 10 150 python3 -u -m pytest $T -x -v --timeout 120 --timeout-method thread > $OUT/rep.log 2>&1 || { echo "rep failed"; tail -30 $OUT/rep.log; exit 1; }
echo "exit=0"
