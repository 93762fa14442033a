# Round-end evidence in one call: the GPU tests, the smoke entry point, every bench leg (the
# default no-flags run too) into gpurun_out/TAG/; each step under its own limit, stop at the
# first failure.  (rocprofv3 evidence: scripts/gpu_profile_all.sh.)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-final}
O=gpurun_out/$TAG
mkdir -p $O
if [ -z "$NOTESTS" ]; then
  timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.txt; exit 1; }
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail $O/smoke.txt; exit 1; }
fi
run() { n=$1; shift; timeout -k 10 600 python3 bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { echo "bench $n failed"; tail $O/bench_$n.err; exit 1; }; }
for leg in ${LEGS:-default c4 c3 c2 c5 c5_cadence ref latency}; do
  case $leg in
    default) run c4_default_run ;;
    c5_cadence) run c5_cadence --workload c5 --stream-chunk 0 --steps 2 --warmup 1 ;;
    *) run $leg --workload $leg ;;
  esac
done
echo "exit=0"
