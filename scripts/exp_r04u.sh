# r04u: the flattened match walk (window-only and streaming builds) -- encode, streaming and
# dictionary tests; C4 and C5 benches (C5 streams through the history-table build)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04u
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_encode.py tests/test_gpu_custom_dict.py tests/test_gpu_lanes.py -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
A="--steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 python3 bench.py $A > $OUT/c4.json 2> $OUT/c4.err || { echo "c4 failed"; tail $OUT/c4.err; exit 1; }
timeout -k 10 500 python3 bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.err || { echo "c5 failed"; tail $OUT/c5.err; exit 1; }
echo "exit=0"
