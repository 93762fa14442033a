# r05ao: per-kernel stats at the reference's cadence (c5 --stream-chunk 0), one step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05ao; mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -f csv -- python3 bench.py --workload c5 --stream-chunk 0 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo "prof failed"; tail $OUT/bench.err; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/prof
echo "exit=0"
