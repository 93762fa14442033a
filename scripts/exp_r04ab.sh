# r04ab: the DP's per-step rare cases (segment end, long insert codes) under wave-uniform
# branches (libbrotli_amd_dpf2.so) against the committed build (libbrotli_amd_alt.so), one
# encode lane; streams must not change
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04ab
mkdir -p $OUT
A="--steps 3 --warmup 1 --no-cpu-baseline"
MIB_ENC_LANES=1 BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_dpf2.so timeout -k 10 300 python3 bench.py $A > $OUT/c4_new.json 2> $OUT/c4_new.err || { echo "new failed"; tail $OUT/c4_new.err; exit 1; }
MIB_ENC_LANES=1 BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_alt.so timeout -k 10 300 python3 bench.py $A > $OUT/c4_base.json 2> $OUT/c4_base.err || { echo "base failed"; tail $OUT/c4_base.err; exit 1; }
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_dpf2.so timeout -k 10 300 python3 bench.py $A --workload c3 > $OUT/c3_new.json 2> $OUT/c3_new.err || { echo "c3 failed"; tail $OUT/c3_new.err; exit 1; }
echo "exit=0"
