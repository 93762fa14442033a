# r04v: the DP's copy edges under a wave-uniform branch (libbrotli_amd_dpflat.so) against the
# default build, one encode lane; streams must not change
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04v
mkdir -p $OUT
A="--steps 3 --warmup 1 --no-cpu-baseline"
MIB_ENC_LANES=1 BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_dpflat.so timeout -k 10 300 python3 bench.py $A > $OUT/c4_dpflat.json 2> $OUT/c4_dpflat.err || { echo "dpflat failed"; tail $OUT/c4_dpflat.err; exit 1; }
MIB_ENC_LANES=1 timeout -k 10 300 python3 bench.py $A > $OUT/c4_base.json 2> $OUT/c4_base.err || { echo "base failed"; tail $OUT/c4_base.err; exit 1; }
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_dpflat.so timeout -k 10 300 python3 bench.py $A --workload c3 > $OUT/c3_dpflat.json 2> $OUT/c3_dpflat.err || { echo "c3 dpflat failed"; tail $OUT/c3_dpflat.err; exit 1; }
echo "exit=0"
