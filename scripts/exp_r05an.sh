# r05an: sizes by tiles (blocks per segment, bits by atomicAdd): GPU tests, then same-box A/B
# against the last commit on C4 and at the reference's cadence (c5 --stream-chunk 0)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05an; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.txt; exit 1; }
tail -3 $OUT/gpu_tests.txt
TAG=r05an/c4 R=2 WL=c4 bash scripts/exp_ab.sh || exit 1
TAG=r05an/cad R=2 WL=c5 BENCH_ARGS="--stream-chunk 0 --steps 1 --warmup 1" bash scripts/exp_ab.sh || exit 1
echo "exit=0"
