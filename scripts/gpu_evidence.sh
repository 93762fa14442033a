# round evidence in one call: every GPU test, bench legs (c4 c2 c3 c5 ref), then rocprofv3
# kernel-trace stats for c4 and c3 and the FETCH_SIZE / WRITE_SIZE passes for c4
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r02}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
for w in c4 c2 c3 c5 ref; do
  timeout -k 10 500 python3 bench.py --workload $w > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { echo "bench $w failed"; tail $OUT/bench_$w.err; exit 1; }
done
ARGS="--steps 1 --warmup 1 --no-cpu-baseline"
for w in c4 c3; do
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/trace_$w -o run -f csv -- python3 bench.py $ARGS --workload $w > $OUT/trace_$w.log 2>&1 || { echo "trace $w failed"; exit 1; }
done
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run -f csv -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1 && \
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run -f csv -- python3 bench.py $ARGS > $OUT/write.log 2>&1 || { echo "pmc failed"; exit 1; }
echo "exit=0"
