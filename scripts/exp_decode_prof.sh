# Decoder phase counters (MIB_PROF build) on C4 and the reference streams: decode_diag.py
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-prof}
mkdir -p $OUT
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_prof.so timeout -k 10 300 python3 scripts/decode_diag.py > $OUT/diag.log 2>&1 || { echo "diag failed"; tail $OUT/diag.log; exit 1; }
echo "exit=0"
