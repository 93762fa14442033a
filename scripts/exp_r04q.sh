# r04q: the whole GPU suite on the round-4 build so far, then the default C4 bench (with the
# CPU baseline) and C3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04q
mkdir -p $OUT
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
timeout -k 10 400 python3 bench.py > $OUT/c4.json 2> $OUT/c4.err || { echo "c4 failed"; tail $OUT/c4.err; exit 1; }
timeout -k 10 300 python3 bench.py --workload c3 --no-cpu-baseline > $OUT/c3.json 2> $OUT/c3.err || { echo "c3 failed"; tail $OUT/c3.err; exit 1; }
echo "exit=0"
