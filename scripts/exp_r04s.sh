# r04s: DP stage entries padded per 32 lanes (bank spread) -- C4 / C3 bench; then the
# rocprofv3 kernel stats of the C4 step on this build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04s
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_encode.py tests/test_gpu_lanes.py -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
A="--steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 python3 bench.py $A > $OUT/c4.json 2> $OUT/c4.err || { echo "c4 failed"; tail $OUT/c4.err; exit 1; }
MIB_ENC_LANES=1 timeout -k 10 300 python3 bench.py $A > $OUT/c4_l1.json 2> $OUT/c4_l1.err || { echo "c4 l1 failed"; tail $OUT/c4_l1.err; exit 1; }
timeout -k 10 300 python3 bench.py $A --workload c3 > $OUT/c3.json 2> $OUT/c3.err || { echo "c3 failed"; tail $OUT/c3.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -f csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/trace.log 2>&1 || { echo "trace failed"; tail $OUT/trace.log; exit 1; }
echo "exit=0"
