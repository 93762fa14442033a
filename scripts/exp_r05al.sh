# r05al: the block split's phase cycles at the reference's cadence (MIB_PROF build)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05al; mkdir -p $OUT
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_prof.so CADENCE=1 timeout -k 10 300 python3 scripts/split_timing.py > $OUT/split.txt 2> $OUT/split.err || { echo "split failed"; tail $OUT/split.err; exit 1; }
echo "exit=0"
