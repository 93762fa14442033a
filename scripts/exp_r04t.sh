# r04t: find_matches with key and position interleaved in LDS (libbrotli_amd_flat.so) against
# the default build, one encode lane (kernel times not shared)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04t2
mkdir -p $OUT
A="--steps 3 --warmup 1 --no-cpu-baseline"
MIB_ENC_LANES=1 BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_flat.so timeout -k 10 300 python3 bench.py $A > $OUT/c4_flat.json 2> $OUT/c4_flat.err || { echo "flat failed"; tail $OUT/c4_flat.err; exit 1; }
MIB_ENC_LANES=1 timeout -k 10 300 python3 bench.py $A > $OUT/c4_base.json 2> $OUT/c4_base.err || { echo "base failed"; tail $OUT/c4_base.err; exit 1; }
echo "exit=0"
