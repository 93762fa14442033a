# r04af: literal block types against the literal code cap: (types, cap) = (8, 32), (8, 48),
# (6, 24), (4, 24) on C2 / C4 / C3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04af
mkdir -p $OUT
A="--steps 3 --warmup 1 --no-cpu-baseline"
for w in c2 c4 c3; do
  for kc in 8:32 8:48 6:24 4:24; do
    k=${kc%:*}; c=${kc#*:}
    MIB_SPLIT_BT=$k,4,4 MIB_LIT_TREES=$c timeout -k 10 300 python3 bench.py $A --workload $w > $OUT/${w}_${k}_$c.json 2> $OUT/${w}_${k}_$c.err || { echo "$w $kc failed"; tail $OUT/${w}_${k}_$c.err; exit 1; }
  done
done
echo "exit=0"
