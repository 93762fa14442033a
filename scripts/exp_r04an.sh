# r04an: the DP at four segments per wave (MIB_DP_KS=4: 16 lanes a segment) against two, on
# C4 and C3, one encode lane (dp_parse alone)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04an
mkdir -p $OUT
A="--steps 3 --warmup 1 --no-cpu-baseline"
for w in c4 c3; do
  for ks in 2 4; do
    MIB_ENC_LANES=1 MIB_DP_KS=$ks timeout -k 10 300 python3 bench.py $A --workload $w > $OUT/${w}_ks$ks.json 2> $OUT/${w}_ks$ks.err || { echo "$w $ks failed"; tail $OUT/${w}_ks$ks.err; exit 1; }
  done
done
echo "exit=0"
