# decoder iteration: decode timing with per-phase cycle counters (MIB_PROF build)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_prof.so timeout -k 10 300 python3 scripts/decode_timing.py > gpurun_out/dectime.log 2>&1
echo "exit=$?"
