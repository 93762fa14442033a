# bench legs with and without parse pieces (MIB_DP_PIECES=0), then the encoder GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abp
run() { tag=$1; shift; env "$@" timeout -k 10 400 python3 bench.py --workload ${W} --no-cpu-baseline > gpurun_out/abp/${W}_$tag.json 2> gpurun_out/abp/${W}_$tag.err || { echo "$W $tag failed"; tail -5 gpurun_out/abp/${W}_$tag.err; exit 1; }; }
W=c4 run def X=1 && W=c2 run def X=1 && W=c2 run nop MIB_DP_PIECES=0 && W=c3 run def X=1 && W=c3 run nop MIB_DP_PIECES=0 || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_configs.py tests/test_gpu_custom_dict.py tests/test_gpu_encode.py tests/test_gpu_parts.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/abp/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/abp/tests.log; exit 1; }
echo "exit=0"
