# r05ab: kernel trace of the cadence leg (64 MiB in 1 MiB update() calls) on the current build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05ab; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o cad -f csv -- python3 bench.py --workload c5 --stream-chunk 0 --size 67108864 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/prof_cad.json 2> $OUT/prof_cad.err || { echo "prof failed"; tail $OUT/prof_cad.err; exit 1; }
echo "exit=0"
