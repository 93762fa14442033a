# r04ad: up to 8 block types per category (MIB_SPLIT_BT = literal,command,distance seeds):
# encode tests with 8,8,8; C4 / C3 at 4,4,4 (the round's streams), 8,4,4, 4,8,8, 8,8,8
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04ad
mkdir -p $OUT
MIB_SPLIT_BT=8,8,8 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_encode.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests888.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests888.log; exit 1; }
A="--steps 3 --warmup 1 --no-cpu-baseline"
for w in c4 c3; do
  for k in 4,4,4 8,4,4 4,8,8 8,8,8; do
    MIB_SPLIT_BT=$k timeout -k 10 300 python3 bench.py $A --workload $w > $OUT/${w}_$k.json 2> $OUT/${w}_$k.err || { echo "$w $k failed"; tail $OUT/${w}_$k.err; exit 1; }
  done
done
echo "exit=0"
