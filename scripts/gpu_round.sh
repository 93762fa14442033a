# round check: every GPU test, then bench legs for each workload (default c4 first)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r02}
mkdir -p gpurun_out/$TAG
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 || { echo "tests failed"; exit 1; }
for w in c4 c2 c3 c5; do
  timeout -k 10 500 python3 bench.py --workload $w > gpurun_out/$TAG/bench_$w.json 2> gpurun_out/$TAG/bench_$w.err || { echo "bench $w failed"; exit 1; }
done
echo "exit=0"
