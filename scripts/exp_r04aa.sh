# r04aa: the context-modelled literal loop with a 128-bit bit window moved every 64 bits
# (libbrotli_amd.so) against the committed build (libbrotli_amd_alt.so): decoder parity tests,
# reference streams, latency leg, C4
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04aa
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_decode.py tests/test_gpu_literal_tables.py -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
A="--steps 3 --warmup 1 --no-cpu-baseline"
for lib in "" alt; do
L=$PWD/brotli-lib_amd/libbrotli_amd${lib:+_$lib}.so
BROTLI_AMD_LIB=$L timeout -k 10 300 python3 bench.py $A --workload ref > $OUT/ref$lib.json 2> $OUT/ref$lib.err || { echo "ref $lib failed"; tail $OUT/ref$lib.err; exit 1; }
BROTLI_AMD_LIB=$L timeout -k 10 300 python3 bench.py --workload latency --steps 1 --warmup 1 --no-cpu-baseline > $OUT/lat$lib.json 2> $OUT/lat$lib.err || { echo "lat $lib failed"; tail $OUT/lat$lib.err; exit 1; }
BROTLI_AMD_LIB=$L timeout -k 10 300 python3 bench.py $A > $OUT/c4$lib.json 2> $OUT/c4$lib.err || { echo "c4 $lib failed"; tail $OUT/c4$lib.err; exit 1; }
done
echo "exit=0"
