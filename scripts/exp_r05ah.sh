# r05ah: Huffman kernel phase maxima at the reference's cadence (MIB_PROF build)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05ah; mkdir -p $OUT
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_prof.so CADENCE=1 timeout -k 10 300 python3 scripts/huff_timing.py > $OUT/huff.txt 2> $OUT/huff.err || { echo "huff failed"; tail $OUT/huff.err; exit 1; }
echo "exit=0"
