# r05m: the reference-cadence streaming leg (C5 shape, 256 MiB, update() of 1 MiB, every
# update encodes its complete blocks): bench, then kernel + HIP API traces of the same
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05m; mkdir -p $OUT
timeout -k 10 300 python3 bench.py --workload c5 --stream-chunk 0 --size 268435456 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/c5_cadence.json 2> $OUT/c5_cadence.err || { echo "cadence failed"; tail $OUT/c5_cadence.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats -d $OUT/prof -o cad -- python3 bench.py --workload c5 --stream-chunk 0 --size 67108864 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/prof_cad.json 2> $OUT/prof_cad.err || { echo "prof failed"; tail $OUT/prof_cad.err; exit 1; }
echo "exit=0"
