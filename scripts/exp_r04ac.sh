# r04ac: the match walk's trip count from a segmented max-scan of bucket-run starts (no key
# reads in the walk) against the committed build: encode / streaming / dictionary tests, C4
# (one lane), C5
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04ac
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_encode.py tests/test_gpu_custom_dict.py tests/test_gpu_lanes.py tests/test_gpu_dictionary.py -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
A="--steps 3 --warmup 1 --no-cpu-baseline"
MIB_ENC_LANES=1 timeout -k 10 300 python3 bench.py $A > $OUT/c4_new.json 2> $OUT/c4_new.err || { echo "new failed"; tail $OUT/c4_new.err; exit 1; }
MIB_ENC_LANES=1 BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_alt.so timeout -k 10 300 python3 bench.py $A > $OUT/c4_base.json 2> $OUT/c4_base.err || { echo "base failed"; tail $OUT/c4_base.err; exit 1; }
timeout -k 10 500 python3 bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.err || { echo "c5 failed"; tail $OUT/c5.err; exit 1; }
timeout -k 10 300 python3 bench.py $A --workload c3 > $OUT/c3.json 2> $OUT/c3.err || { echo "c3 failed"; tail $OUT/c3.err; exit 1; }
echo "exit=0"
