# r04g: rocprofv3 kernel stats of the C4 step (the bucket sort's kernels), find_matches with
# and without the XCD-aware tile order, the new update() cadence tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04g
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_encode.py -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
A="--steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -f csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/trace.log 2>&1 || { echo "trace failed"; tail $OUT/trace.log; exit 1; }
MIB_FM_XCD=0 timeout -k 10 300 python3 bench.py $A > $OUT/c4_noxcd.json 2> $OUT/c4_noxcd.err || { echo "c4 failed"; tail $OUT/c4_noxcd.err; exit 1; }
timeout -k 10 300 python3 bench.py $A > $OUT/c4.json 2> $OUT/c4.err || { echo "c4 failed"; tail $OUT/c4.err; exit 1; }
timeout -k 10 400 python3 bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.err || { echo "c5 failed"; tail $OUT/c5.err; exit 1; }
timeout -k 10 600 python3 bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline --stream-chunk 0 > $OUT/c5_cadence.json 2> $OUT/c5_cadence.err || { echo "c5 cadence failed"; tail $OUT/c5_cadence.err; exit 1; }
echo "exit=0"
