# r05ac: the block split's serial code-building tail in LDS (no scratch): GPU tests, A/B against
# HEAD on c4 and on the cadence leg (c5, 1 MiB update() calls, 256 MiB)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05ac; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
TAG=r05ac/ab R=2 WL=c4 bash scripts/exp_ab.sh || exit 1
TAG=r05ac/cad R=2 WL=c5 BENCH_ARGS="--stream-chunk 0 --size 268435456 --steps 1 --warmup 1" bash scripts/exp_ab.sh
