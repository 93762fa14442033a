# r05k: near scan v7 (words staged from global, two barriers per tile): tests, c4, c3, latency, ref legs; c4 trace
# GPU tests, c4 (expect the v5 stream bytes: ratio 0.36281), c2, c5, kernel trace of c4
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05k; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
for w in c4 c3 latency ref; do
  timeout -k 10 400 python3 bench.py --workload $w > $OUT/${w}_new.json 2> $OUT/${w}_new.err || { echo "$w new failed"; tail $OUT/${w}_new.err; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o c4 -- python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/prof_c4.json 2> $OUT/prof_c4.err || { echo "prof failed"; tail $OUT/prof_c4.err; exit 1; }
echo "exit=0"
