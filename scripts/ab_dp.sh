# DP variants on C4: the working build (node reads by readlane) with 2 and 1 segments per wave,
# against the HEAD build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abdp
B="timeout -k 10 400 python3 bench.py --workload c4 --no-cpu-baseline"
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_head.so $B > gpurun_out/abdp/head.json 2> gpurun_out/abdp/head.err || exit 1
$B > gpurun_out/abdp/ks2.json 2> gpurun_out/abdp/ks2.err || exit 1
MIB_DP_KS=1 $B > gpurun_out/abdp/ks1.json 2> gpurun_out/abdp/ks1.err || exit 1
echo "exit=0"
