# encoder iteration: encode parity tests, dp per-phase timing (MIB_PROF build), bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_encode.py -x -q --timeout 200 --timeout-method thread > gpurun_out/iter_tests.log 2>&1 && \
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_prof.so timeout -k 10 200 python3 scripts/dp_timing.py > gpurun_out/dptime.log 2>&1 && \
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "exit=$?"
