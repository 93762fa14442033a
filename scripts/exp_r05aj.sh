# r05aj: the complex prefix-code store with the wave (scan, histogram, code bits by prefix sum):
# GPU tests, Huffman phase maxima at cadence (MIB_PROF build), A/B against HEAD on c4, c3, cadence
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05aj; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_prof.so CADENCE=1 timeout -k 10 300 python3 scripts/huff_timing.py > $OUT/huff.txt 2> $OUT/huff.err || { echo "huff failed"; tail $OUT/huff.err; exit 1; }
TAG=r05aj/ab R=2 WL="c4 c3" bash scripts/exp_ab.sh || exit 1
TAG=r05aj/cad R=2 WL=c5 BENCH_ARGS="--stream-chunk 0 --size 268435456 --steps 1 --warmup 1" bash scripts/exp_ab.sh
