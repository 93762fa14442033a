# r04k: the VGPR literal chain in fast_loop -- decoder parity tests, then C4 / C3 / ref /
# latency with it (libbrotli_amd.so) and without (libbrotli_amd_alt.so, MIB_VLIT=0), and
# the phase counters of the MIB_PROF build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04k
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_literal_tables.py tests/test_gpu_decode.py tests/test_gpu_custom_dict.py -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
A="--steps 3 --warmup 1 --no-cpu-baseline"
for w in c4 c3 ref; do
timeout -k 10 300 python3 bench.py $A --workload $w > $OUT/$w.json 2> $OUT/$w.err || { echo "$w failed"; tail $OUT/$w.err; exit 1; }
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_alt.so timeout -k 10 300 python3 bench.py $A --workload $w > $OUT/${w}_alt.json 2> $OUT/${w}_alt.err || { echo "$w alt failed"; tail $OUT/${w}_alt.err; exit 1; }
done
timeout -k 10 300 python3 bench.py --workload latency --steps 1 --warmup 1 --no-cpu-baseline > $OUT/latency.json 2> $OUT/latency.err || { echo "latency failed"; tail $OUT/latency.err; exit 1; }
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_prof.so timeout -k 10 300 python3 scripts/decode_diag.py > $OUT/diag.log 2>&1 || { echo "diag failed"; tail $OUT/diag.log; exit 1; }

# find_matches without its scattered record stores (records in sorted order: the streams are
# wrong and the bench stops at its round-trip check, exit 1 expected; the kernel trace of the
# warmup step is what is read)
MIB_FM_SORTED_STORE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/fmsorted -o run -f csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/fmsorted.log 2>&1
rc=$?; [ $rc -le 1 ] || { echo "fmsorted rc=$rc"; tail $OUT/fmsorted.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/fmbase -o run -f csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/fmbase.log 2>&1 || { echo "fmbase failed"; tail $OUT/fmbase.log; exit 1; }
echo "exit=0"
