set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abd
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decode.py tests/test_gpu_parts.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/abd/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/abd/tests.log; exit 1; }
for lib in libbrotli_amd_head libbrotli_amd; do BROTLI_AMD_LIB=$PWD/brotli-lib_amd/$lib.so timeout -k 10 400 python3 bench.py --workload c4 --no-cpu-baseline > gpurun_out/abd/c4_$lib.json 2> gpurun_out/abd/c4_$lib.err || exit 1; done
for lib in libbrotli_amd_head libbrotli_amd; do BROTLI_AMD_LIB=$PWD/brotli-lib_amd/$lib.so timeout -k 10 400 python3 bench.py --workload c3 --no-cpu-baseline > gpurun_out/abd/c3_$lib.json 2> gpurun_out/abd/c3_$lib.err || exit 1; done
echo "exit=0"
