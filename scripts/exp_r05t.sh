# r05t: find_matches walk in lockstep with a first-word screen (byte mask) before the exact tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05t; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
for w in c4 c3 c4 c3; do
  timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline >> $OUT/$w.json 2>> $OUT/$w.err || { echo "$w failed"; tail $OUT/$w.err; exit 1; }
done
echo "exit=0"
