# r04p: encode lanes 1-4 (MIB_ENC_LANES) with the original match walk and the DP at 4 waves per
# SIMD: encode tests, C4 / C3 benches per lane count
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04p
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_encode.py tests/test_gpu_configs.py tests/test_gpu_multi.py -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
MIB_ENC_LANES=4 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_encode.py -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/tests4.log 2>&1 || { echo "tests4 failed"; tail -40 $OUT/tests4.log; exit 1; }
A="--steps 3 --warmup 1 --no-cpu-baseline"
for n in 2 3 4 1; do
MIB_ENC_LANES=$n timeout -k 10 300 python3 bench.py $A > $OUT/c4_l$n.json 2> $OUT/c4_l$n.err || { echo "c4 l$n failed"; tail $OUT/c4_l$n.err; exit 1; }
done
for n in 2 4; do
MIB_ENC_LANES=$n timeout -k 10 300 python3 bench.py $A --workload c3 > $OUT/c3_l$n.json 2> $OUT/c3_l$n.err || { echo "c3 l$n failed"; tail $OUT/c3_l$n.err; exit 1; }
done
echo "exit=0"
