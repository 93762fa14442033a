set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python3 scripts/gpu_decode_diag.py > gpurun_out/diag_stdout.log 2>&1
echo "exit=$?"
