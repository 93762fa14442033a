# r05u: where the host batch path's time goes (MIB_HOST_TIMING, experiment build)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05u; mkdir -p $OUT
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_exp.so MIB_HOST_TIMING=1 PROBE_GPUS=${PROBE_GPUS:-0} timeout -k 10 300 python3 scripts/host_xfer_probe.py > $OUT/probe.json 2> $OUT/probe.err || { echo "probe failed"; tail $OUT/probe.err; exit 1; }
echo "exit=0"
