# r04f: decoder phase counters (MIB_PROF), the GPU suite with the new bucket sort, C4 bench
# with the default DP and with 4 segments per DP wave (MIB_DP_KS=4)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04f
mkdir -p $OUT
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_prof.so timeout -k 10 300 python3 scripts/decode_diag.py > $OUT/diag.log 2>&1 || { echo "diag failed"; tail $OUT/diag.log; exit 1; }
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
A="--steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 python3 bench.py $A > $OUT/c4.json 2> $OUT/c4.err || { echo "c4 failed"; tail $OUT/c4.err; exit 1; }
MIB_DP_KS=4 timeout -k 10 300 python3 bench.py $A > $OUT/c4_ks4.json 2> $OUT/c4_ks4.err || { echo "c4 ks4 failed"; tail $OUT/c4_ks4.err; exit 1; }
timeout -k 10 300 python3 bench.py $A --workload c3 > $OUT/c3.json 2> $OUT/c3.err || { echo "c3 failed"; tail $OUT/c3.err; exit 1; }
echo "exit=0"
