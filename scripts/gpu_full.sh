# full check: every GPU test, the default bench (with the CPU baseline), then the
# per-phase decode and parse timings (MIB_PROF build)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/full_tests.log 2>&1 && \
timeout -k 10 400 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_prof.so timeout -k 10 200 python3 scripts/decode_timing.py > gpurun_out/dectime.log 2>&1 && \
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_prof.so timeout -k 10 200 python3 scripts/dp_timing.py > gpurun_out/dptime.log 2>&1
echo "exit=$?"
