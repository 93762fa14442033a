set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abs
for w in c4 c3 c2; do for p in 3 2; do MIB_DP_PIECES=$p timeout -k 10 400 python3 bench.py --workload $w --no-cpu-baseline > gpurun_out/abs/${w}_p$p.json 2> gpurun_out/abs/${w}_p$p.err || exit 1; done; done
echo "exit=0"
