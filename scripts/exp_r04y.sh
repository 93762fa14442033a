# r04y: where a C1 (45,000 B) brotliDecode's time goes: wall vs kernel time per call
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04y
mkdir -p $OUT
timeout -k 10 300 python3 scripts/c1_decode_diag.py > $OUT/c1.log 2>&1 || { echo "diag failed"; tail $OUT/c1.log; exit 1; }
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_prof.so timeout -k 10 300 python3 scripts/c1_decode_diag.py > $OUT/c1_prof.log 2>&1 || { echo "diag prof failed"; tail $OUT/c1_prof.log; exit 1; }
echo "exit=0"
