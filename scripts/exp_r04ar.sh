# r04ar: the Huffman kernel's rank sort over packed (count, symbol) keys read two at a time:
# encode / parts / lanes / dictionary tests, C4 / C3 / C5 / C2 against the committed build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04ar
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_encode.py tests/test_gpu_parts.py tests/test_gpu_lanes.py tests/test_gpu_custom_dict.py -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
A="--steps 3 --warmup 1 --no-cpu-baseline"
ALT=$PWD/brotli-lib_amd/libbrotli_amd_alt.so
for w in c4 c3 c5 c2; do
  timeout -k 10 300 python3 bench.py $A --workload $w > $OUT/${w}_new.json 2> $OUT/${w}_new.err || { echo "$w new failed"; tail $OUT/${w}_new.err; exit 1; }
  BROTLI_AMD_LIB=$ALT timeout -k 10 300 python3 bench.py $A --workload $w > $OUT/${w}_base.json 2> $OUT/${w}_base.err || { echo "$w base failed"; tail $OUT/${w}_base.err; exit 1; }
done
echo "exit=0"
