# r05ar: r05aq with the unforked order restored (C4), same-box A/B against d7f528c
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05ar; mkdir -p $OUT
TAG=r05ar/c4 R=2 WL=c4 bash scripts/exp_ab.sh || exit 1
TAG=r05ar/cad R=1 WL=c5 BENCH_ARGS="--stream-chunk 0 --steps 1 --warmup 1" bash scripts/exp_ab.sh || exit 1
echo "exit=0"
