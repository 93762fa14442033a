# r04r: a per-command penalty in the parse's copy prices (MIB_CMD_PENALTY bits: fewer, longer
# commands for the decoder) -- C4 / C3 ratio and decode time; C3 with three encode lanes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04r
mkdir -p $OUT
A="--steps 3 --warmup 1 --no-cpu-baseline"
for p in 0 1 2 4; do
MIB_CMD_PENALTY=$p timeout -k 10 300 python3 bench.py $A > $OUT/c4_p$p.json 2> $OUT/c4_p$p.err || { echo "c4 p$p failed"; tail $OUT/c4_p$p.err; exit 1; }
MIB_CMD_PENALTY=$p timeout -k 10 300 python3 bench.py $A --workload c3 > $OUT/c3_p$p.json 2> $OUT/c3_p$p.err || { echo "c3 p$p failed"; tail $OUT/c3_p$p.err; exit 1; }
done
MIB_ENC_LANES=3 timeout -k 10 300 python3 bench.py $A --workload c3 > $OUT/c3_l3.json 2> $OUT/c3_l3.err || { echo "c3 l3 failed"; tail $OUT/c3_l3.err; exit 1; }
echo "exit=0"
