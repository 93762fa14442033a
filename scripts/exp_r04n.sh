# r04n: three builds of find_matches' candidate walk (MIB_FM_WALK 1: one 16-byte LDS record
# per candidate, prefetched; 2: + a byte-mask rejection first; 3: a tight skip loop + a take
# loop), C4 bench each (streams must stay 0.36469)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04n
mkdir -p $OUT
A="--steps 3 --warmup 1 --no-cpu-baseline"
for v in 1 2 3; do
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_fm$v.so timeout -k 10 300 python3 bench.py $A > $OUT/c4_fm$v.json 2> $OUT/c4_fm$v.err || { echo "fm$v failed"; tail $OUT/c4_fm$v.err; exit 1; }
done
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_alt.so timeout -k 10 300 python3 bench.py $A > $OUT/c4_base.json 2> $OUT/c4_base.err || { echo "base failed"; tail $OUT/c4_base.err; exit 1; }
echo "exit=0"
