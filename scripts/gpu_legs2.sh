set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-legs}
mkdir -p gpurun_out/$T
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parts.py -x -v --timeout 200 --timeout-method thread > gpurun_out/$T/parts.log 2>&1 || { echo "parts tests failed"; tail -30 gpurun_out/$T/parts.log; exit 1; }
for w in ${WORKLOADS:-c5 ref}; do
  timeout -k 10 500 python3 bench.py --workload $w > gpurun_out/$T/bench_$w.json 2> gpurun_out/$T/bench_$w.err || { echo "bench $w failed"; tail gpurun_out/$T/bench_$w.err; exit 1; }
done
echo exit=0
