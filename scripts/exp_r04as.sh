# r04as: encode lanes (MIB_ENC_LANES 2 / 3 / 4) with the four-segment DP, C4 and C3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04as
mkdir -p $OUT
A="--steps 3 --warmup 1 --no-cpu-baseline"
for w in c4 c3; do
  for n in 2 3 4; do
    MIB_ENC_LANES=$n timeout -k 10 300 python3 bench.py $A --workload $w > $OUT/${w}_l$n.json 2> $OUT/${w}_l$n.err || { echo "$w $n failed"; tail $OUT/${w}_l$n.err; exit 1; }
  done
done
echo "exit=0"
