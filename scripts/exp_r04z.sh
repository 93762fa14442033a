# r04z: the DP's copy edges under a wave-uniform branch (libbrotli_amd_dprl.so) against the
# default build, one encode lane; streams must not change
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04z
mkdir -p $OUT
A="--steps 3 --warmup 1 --no-cpu-baseline"
MIB_ENC_LANES=1 BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_dprl.so timeout -k 10 300 python3 bench.py $A > $OUT/c4_dprl.json 2> $OUT/c4_dprl.err || { echo "dprl failed"; tail $OUT/c4_dprl.err; exit 1; }
MIB_ENC_LANES=1 timeout -k 10 300 python3 bench.py $A > $OUT/c4_base.json 2> $OUT/c4_base.err || { echo "base failed"; tail $OUT/c4_base.err; exit 1; }
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_dprl.so timeout -k 10 300 python3 bench.py $A --workload c3 > $OUT/c3_dprl.json 2> $OUT/c3_dprl.err || { echo "c3 dprl failed"; tail $OUT/c3_dprl.err; exit 1; }
echo "exit=0"
