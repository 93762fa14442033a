# rocprofv3 evidence for the bench workload: kernel-trace stats, then one PMC pass per
# counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
ARGS="--steps 1 --warmup 1 --no-cpu-baseline"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -f csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 && \
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run -f csv -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1 && \
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run -f csv -- python3 bench.py $ARGS > $OUT/write.log 2>&1
echo "exit=$?"
find $OUT -name "*.csv" | head -20
