# GPU tests (optionally a -k filter), then bench legs for the given workloads
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
FILTER=${FILTER:-}
mkdir -p gpurun_out/$TAG
if [ -n "$FILTER" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$FILTER" > gpurun_out/$TAG/tests.log 2>&1 || { echo "tests failed"; exit 1; }
fi
for w in "$@"; do
  timeout -k 10 500 python3 bench.py --workload $w > gpurun_out/$TAG/bench_$w.json 2> gpurun_out/$TAG/bench_$w.err || { echo "bench $w failed"; exit 1; }
done
echo "exit=0"
