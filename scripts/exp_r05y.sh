# r05y: DP window shift by wave-wide selects (no per-step window copies)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05y; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
for w in c4 c3 c4 c3; do
  timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline >> $OUT/$w.json 2>> $OUT/$w.err || { echo "$w failed"; tail $OUT/$w.err; exit 1; }
done
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_exp.so MIB_ENC_LANES=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace1 -o run -f csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/lanes1.json 2> $OUT/lanes1.err || { echo "trace failed"; exit 1; }
echo "exit=0"
