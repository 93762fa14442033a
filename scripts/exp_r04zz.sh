# r04zz: the round's last tree: smoke(), the full GPU suite, the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04zz
mkdir -p $OUT
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
timeout -k 10 400 python3 bench.py > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { echo "bench failed"; tail $OUT/bench_c4.err; exit 1; }
echo "exit=0"
