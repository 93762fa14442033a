# r04j: LDS / readlane / bpermute chain latencies (chain_probe); C4 and C3 with context-free
# literal coding (MIB_LIT_TREES=1: one literal code per block type) against the default
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04j
mkdir -p $OUT
timeout -k 10 120 ./scripts/probe/chain_probe > $OUT/chain.txt 2>&1 || { echo "probe failed"; cat $OUT/chain.txt; exit 1; }
A="--steps 3 --warmup 1 --no-cpu-baseline"
MIB_LIT_TREES=1 timeout -k 10 300 python3 bench.py $A > $OUT/c4_lit1.json 2> $OUT/c4_lit1.err || { echo "c4 lit1 failed"; tail $OUT/c4_lit1.err; exit 1; }
MIB_LIT_TREES=1 timeout -k 10 300 python3 bench.py $A --workload c3 > $OUT/c3_lit1.json 2> $OUT/c3_lit1.err || { echo "c3 lit1 failed"; tail $OUT/c3_lit1.err; exit 1; }

timeout -k 10 400 python3 bench.py --gpus-in-lib 4 --steps 2 --warmup 1 > $OUT/inlib4.json 2> $OUT/inlib4.err || { echo "inlib failed"; tail $OUT/inlib4.err; exit 1; }

for nt in 1 2 3; do
MIB_FM_NT=$nt timeout -k 10 300 python3 bench.py $A > $OUT/c4_nt$nt.json 2> $OUT/c4_nt$nt.err || { echo "c4 nt$nt failed"; tail $OUT/c4_nt$nt.err; exit 1; }
done
timeout -k 10 300 python3 bench.py $A > $OUT/c4.json 2> $OUT/c4.err || { echo "c4 failed"; tail $OUT/c4.err; exit 1; }
echo "exit=0"
