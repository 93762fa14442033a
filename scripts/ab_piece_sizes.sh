# C4 / C3 / C2 bench legs at parse-piece shifts given in PS (default "3 4")
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abs
for w in ${WL:-c4 c3 c2}; do for p in ${PS:-3 4}; do MIB_DP_PIECES=$p timeout -k 10 400 python3 bench.py --workload $w --no-cpu-baseline > gpurun_out/abs/${w}_p$p.json 2> gpurun_out/abs/${w}_p$p.err || exit 1; done; done
echo "exit=0"
