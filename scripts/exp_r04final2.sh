# r04final2: the remaining bench legs of the final build (c2, c5, ref, latency) and the
# in-library 4-shard leg
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04final
mkdir -p $OUT
for w in c2 c5 ref latency; do
  timeout -k 10 500 python3 bench.py --workload $w > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { echo "bench $w failed"; tail $OUT/bench_$w.err; exit 1; }
done
timeout -k 10 500 python3 bench.py --gpus-in-lib 4 --no-cpu-baseline > $OUT/inlib4.json 2> $OUT/inlib4.err || { echo "inlib failed"; tail $OUT/inlib4.err; exit 1; }
echo "exit=0"
