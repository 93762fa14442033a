# r05q: wave-parallel context-map build + LDS-staged block-split codes in the header kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05q; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
for w in c4 latency; do
  timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline > $OUT/$w.json 2> $OUT/$w.err || { echo "$w failed"; tail $OUT/$w.err; exit 1; }
done
timeout -k 10 300 python3 bench.py --workload c5 --stream-chunk 0 --size 268435456 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/c5_cadence.json 2> $OUT/c5_cadence.err || { echo "cadence failed"; tail $OUT/c5_cadence.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o cad -- python3 bench.py --workload c5 --stream-chunk 0 --size 67108864 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/prof_cad.json 2> $OUT/prof_cad.err || { echo "prof failed"; tail $OUT/prof_cad.err; exit 1; }
echo "exit=0"
