# r05aq: independent launches on a side stream for calls of few metablocks (literal histogram and context mode beside the match search, history update beside the parse, the split pair, prefix codes beside the header): GPU tests, then same-box A/B
# against the last commit on C4 and at the reference's cadence (c5 --stream-chunk 0)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05aq; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.txt; exit 1; }
tail -3 $OUT/gpu_tests.txt
TAG=r05aq/c4 R=2 WL=c4 bash scripts/exp_ab.sh || exit 1
TAG=r05aq/cad R=1 WL=c5 BENCH_ARGS="--stream-chunk 0 --steps 1 --warmup 1" bash scripts/exp_ab.sh || exit 1
TAG=r05aq/c2 R=2 WL=c2 bash scripts/exp_ab.sh || exit 1
echo "exit=0"
