# r05final: the round's final build: GPU tests; every bench leg with its CPU baseline (c4 default,
# c3, c2, c5, ref, latency), the cadence leg, the in-library host-buffer leg twice
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05final; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
timeout -k 10 400 python3 bench.py > $OUT/c4.json 2> $OUT/c4.err || { echo "c4 failed"; tail $OUT/c4.err; exit 1; }
for w in c3 c2 ref latency; do
  timeout -k 10 400 python3 bench.py --workload $w > $OUT/$w.json 2> $OUT/$w.err || { echo "$w failed"; tail $OUT/$w.err; exit 1; }
done
timeout -k 10 300 python3 bench.py --workload c5 --stream-chunk 0 --size 268435456 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/c5_cadence.json 2> $OUT/c5_cadence.err || { echo "cadence failed"; tail $OUT/c5_cadence.err; exit 1; }
for r in a b; do
  timeout -k 10 300 python3 bench.py --gpus-in-lib 4 --no-cpu-baseline > $OUT/inlib4$r.json 2> $OUT/inlib4$r.err || { echo "inlib failed"; tail $OUT/inlib4$r.err; exit 1; }
done
timeout -k 10 500 python3 bench.py --workload c5 > $OUT/c5.json 2> $OUT/c5.err || { echo "c5 failed"; tail $OUT/c5.err; exit 1; }
echo "exit=0"
