# GPU tests then the default bench line and a kernel-trace profile of one bench step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r02}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 && \
timeout -k 10 400 python3 bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/trace -o run -f csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/trace.log 2>&1
echo "exit=$?"
