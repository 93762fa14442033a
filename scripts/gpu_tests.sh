# GPU tests (pytest -k FILTER when given; files in FILES first), then bench legs for the
# given workloads; every step under its own time limit, stop at the first failure
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out/$TAG
if [ -n "$FILES" ]; then
  timeout -k 10 900 python3 -u -m pytest $FILES -m gpu -x -v --timeout 400 --timeout-method thread ${FILTER:+-k "$FILTER"} > gpurun_out/$TAG/tests_first.log 2>&1 || { echo "first tests failed"; tail -40 gpurun_out/$TAG/tests_first.log; exit 1; }
fi
if [ -z "$NOSUITE" ]; then
  timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread ${FILTER:+-k "$FILTER"} > gpurun_out/$TAG/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/$TAG/tests.log; exit 1; }
fi
for w in "$@"; do
  timeout -k 10 500 python3 bench.py --workload $w > gpurun_out/$TAG/bench_$w.json 2> gpurun_out/$TAG/bench_$w.err || { echo "bench $w failed"; tail gpurun_out/$TAG/bench_$w.err; exit 1; }
done
echo "exit=0"
