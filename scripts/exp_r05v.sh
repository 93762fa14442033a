# r05v: the host batch leg (one device: the sharded calls run as the one-context batch), three runs; multi tests (shards forced)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05v; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_multi.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -20 $OUT/tests.log; exit 1; }
for r in a b c; do
  timeout -k 10 300 python3 bench.py --gpus-in-lib 4 --no-cpu-baseline > $OUT/inlib4$r.json 2> $OUT/inlib4$r.err || { echo "inlib failed"; tail $OUT/inlib4$r.err; exit 1; }
done
echo "exit=0"
