# r05ak: the header kernel's context-map code by the wave (serial_depths_wave, wave_put_items):
# GPU tests, Huffman phase maxima at cadence (MIB_PROF build), A/B against HEAD on c4, c3, cadence
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05ak; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_prof.so CADENCE=1 timeout -k 10 300 python3 scripts/huff_timing.py > $OUT/huff.txt 2> $OUT/huff.err || { echo "huff failed"; tail $OUT/huff.err; exit 1; }
TAG=r05ak/ab R=2 WL="c4 c3" bash scripts/exp_ab.sh || exit 1
TAG=r05ak/cad R=2 WL=c5 BENCH_ARGS="--stream-chunk 0 --size 268435456 --steps 1 --warmup 1" bash scripts/exp_ab.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o cad -f csv -- python3 bench.py --workload c5 --stream-chunk 0 --size 67108864 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/prof_cad.json 2> $OUT/prof_cad.err || { echo "prof failed"; exit 1; }
