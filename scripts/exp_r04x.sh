# r04x: the latency leg with one literal code per block type (MIB_LIT_TREES=1) -- sizes and
# decode times of the small calls when every literal run takes the 64-at-once path
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04x
mkdir -p $OUT
MIB_LIT_TREES=1 timeout -k 10 300 python3 bench.py --workload latency --steps 1 --warmup 1 --no-cpu-baseline > $OUT/lat_lit1.json 2> $OUT/lat_lit1.err || { echo "lat failed"; tail $OUT/lat_lit1.err; exit 1; }
timeout -k 10 300 python3 bench.py --workload latency --steps 1 --warmup 1 --no-cpu-baseline > $OUT/lat.json 2> $OUT/lat.err || { echo "lat failed"; tail $OUT/lat.err; exit 1; }
echo "exit=0"
