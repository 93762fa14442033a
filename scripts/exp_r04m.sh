# r04m: find_matches with one 16-byte LDS record per candidate, prefetched a step ahead --
# encoder tests (streams must not change), C4 / C3 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04m
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_encode.py tests/test_gpu_configs.py -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
A="--steps 3 --warmup 1 --no-cpu-baseline"
for w in c4 c3; do
timeout -k 10 300 python3 bench.py $A --workload $w > $OUT/$w.json 2> $OUT/$w.err || { echo "$w failed"; tail $OUT/$w.err; exit 1; }
done

BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_prof.so timeout -k 10 300 python3 scripts/dp_timing.py > $OUT/dp_timing.log 2>&1 || { echo "dp timing failed"; tail $OUT/dp_timing.log; exit 1; }
echo "exit=0"
