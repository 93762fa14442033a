set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -m pytest tests/test_gpu_encode.py -q -s > gpurun_out/gpu_encode.log 2>&1
echo "exit=$?"
