# part-parallel decode: its tests, the rest of the GPU suite, then the C2 / C4 bench legs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-parts}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parts.py -x -v --timeout 200 --timeout-method thread > gpurun_out/$TAG/parts.log 2>&1 || { echo "parts tests failed"; exit 1; }
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 || { echo "tests failed"; exit 1; }
for w in ${WORKLOADS:-c2 c4}; do
  timeout -k 10 500 python3 bench.py --workload $w > gpurun_out/$TAG/bench_$w.json 2> gpurun_out/$TAG/bench_$w.err || { echo "bench $w failed"; exit 1; }
done
echo "exit=0"
