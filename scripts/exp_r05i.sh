# r05i: the distance-cache test (product, then the HEAD build for its counts: informational),
# GPU tests, c4 / c3 HEAD vs product (near scan v5 outside FONT mode), kernel traces
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05i; mkdir -p $OUT
L=$PWD/brotli-lib_amd
T=tests/test_gpu_distance_cache.py
timeout -k 10 300 python3 -u -m pytest $T -v -s --timeout 200 --timeout-method thread > $OUT/dc_new.log 2>&1; echo "dc_new rc=$?"
BROTLI_AMD_LIB=$L/libbrotli_amd_head.so timeout -k 10 300 python3 -u -m pytest $T -v -s --timeout 200 --timeout-method thread > $OUT/dc_head.log 2>&1; echo "dc_head rc=$?"
grep -E "copies:" $OUT/dc_new.log $OUT/dc_head.log
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; echo "tests rc=$?"; grep -E "FAILED|passed|failed" $OUT/tests.log | tail -5
for w in c4 c3; do
  BROTLI_AMD_LIB=$L/libbrotli_amd_head.so timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline > $OUT/${w}_head.json 2> $OUT/${w}_head.err || { echo "$w head failed"; tail $OUT/${w}_head.err; exit 1; }
  timeout -k 10 300 python3 bench.py --workload $w > $OUT/${w}_new.json 2> $OUT/${w}_new.err || { echo "$w new failed"; tail $OUT/${w}_new.err; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o $w -- python3 bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline > $OUT/prof_$w.json 2> $OUT/prof_$w.err || { echo "prof failed"; tail $OUT/prof_$w.err; exit 1; }
done
echo "exit=0"
