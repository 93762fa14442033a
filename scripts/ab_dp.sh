# DP variants on C4: the working build against the HEAD build (same box, same call)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abdp
B="timeout -k 10 400 python3 bench.py --workload c4 --no-cpu-baseline"
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_head.so $B > gpurun_out/abdp/head.json 2> gpurun_out/abdp/head.err || exit 1
$B > gpurun_out/abdp/work.json 2> gpurun_out/abdp/work.err || exit 1
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_head.so $B > gpurun_out/abdp/head2.json 2> gpurun_out/abdp/head2.err || exit 1
$B > gpurun_out/abdp/work2.json 2> gpurun_out/abdp/work2.err || exit 1
echo "exit=0"
