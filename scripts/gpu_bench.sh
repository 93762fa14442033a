set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "exit=$?"
