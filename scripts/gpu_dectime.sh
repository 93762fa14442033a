set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 scripts/decode_timing.py > gpurun_out/dectime.log 2>&1
echo "exit=$?"
