# r05w: C4 encode kernels alone (one encode lane, experiment build): kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05w; mkdir -p $OUT
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_exp.so MIB_ENC_LANES=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace1 -o run -f csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/lanes1.json 2> $OUT/lanes1.err || { echo "trace failed"; tail $OUT/lanes1.err; exit 1; }
echo "exit=0"
