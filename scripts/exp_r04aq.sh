# r04aq: four segments per DP wave below the default threshold: C2 (8,192 pieces) and C5 with
# MIB_DP_KS=4 against the default
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04aq
mkdir -p $OUT
A="--steps 3 --warmup 1 --no-cpu-baseline"
for w in c2 c5; do
  timeout -k 10 400 python3 bench.py $A --workload $w > $OUT/${w}_def.json 2> $OUT/${w}_def.err || { echo "$w def failed"; tail $OUT/${w}_def.err; exit 1; }
  MIB_DP_KS=4 timeout -k 10 400 python3 bench.py $A --workload $w > $OUT/${w}_ks4.json 2> $OUT/${w}_ks4.err || { echo "$w ks4 failed"; tail $OUT/${w}_ks4.err; exit 1; }
done
echo "exit=0"
