# quick iteration: GPU tests, then the default bench (no CPU baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/iter_tests.log 2>&1 && \
timeout -k 10 600 python3 bench.py --no-cpu-baseline "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "exit=$?"
