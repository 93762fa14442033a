# C3 (fonts) and C4 with each literal context mode forced (MIB_CTX_MODE 0 LSB6, 1 MSB6, 2 UTF8, 3 SIGNED)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abcm
for w in ${WL:-c3}; do for m in ${MODES:-def 0 1 2 3}; do
  if [ $m = def ]; then E=X=1; else E=MIB_CTX_MODE=$m; fi
  env $E timeout -k 10 400 python3 bench.py --workload $w --no-cpu-baseline > gpurun_out/abcm/${w}_$m.json 2> gpurun_out/abcm/${w}_$m.err || exit 1
done; done
echo "exit=0"
