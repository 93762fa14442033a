# quick iteration: encoder tests, then the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -m pytest tests/test_gpu_encode.py tests/test_gpu_decode.py tests/test_gpu_node.py -x -q -s > gpurun_out/iter_tests.log 2>&1 && \
timeout -k 10 600 python3 bench.py --no-cpu-baseline "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "exit=$?"
