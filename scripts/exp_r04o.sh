# r04o: two encode lanes (MIB_ENC_LANES 2 vs 1) -- encode tests and C4 / C3 benches; then the
# DP at 4 waves per SIMD (libbrotli_amd_dp4.so; default 5), DP with arithmetic copy codes (dpcc), the three builds of find_matches' walk (single lane builds) against the round's previous build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04o
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_encode.py tests/test_gpu_configs.py tests/test_gpu_multi.py -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
A="--steps 3 --warmup 1 --no-cpu-baseline"
for w in c4 c3; do
timeout -k 10 300 python3 bench.py $A --workload $w > $OUT/${w}_lanes2.json 2> $OUT/${w}_lanes2.err || { echo "$w failed"; tail $OUT/${w}_lanes2.err; exit 1; }
MIB_ENC_LANES=1 timeout -k 10 300 python3 bench.py $A --workload $w > $OUT/${w}_lanes1.json 2> $OUT/${w}_lanes1.err || { echo "$w l1 failed"; tail $OUT/${w}_lanes1.err; exit 1; }
done
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_dp4.so timeout -k 10 300 python3 bench.py $A > $OUT/c4_dp4.json 2> $OUT/c4_dp4.err || { echo "dp4 failed"; tail $OUT/c4_dp4.err; exit 1; }
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_dpcc.so timeout -k 10 300 python3 bench.py $A > $OUT/c4_dpcc.json 2> $OUT/c4_dpcc.err || { echo "dpcc failed"; tail $OUT/c4_dpcc.err; exit 1; }
for v in 1 2 3; do
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_fm$v.so timeout -k 10 300 python3 bench.py $A > $OUT/c4_fm$v.json 2> $OUT/c4_fm$v.err || { echo "fm$v failed"; tail $OUT/c4_fm$v.err; exit 1; }
done
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_alt.so timeout -k 10 300 python3 bench.py $A > $OUT/c4_base.json 2> $OUT/c4_base.err || { echo "base failed"; tail $OUT/c4_base.err; exit 1; }
echo "exit=0"
