# r05af: 1 KiB parse pieces for small one-shot streams? the latency leg with MIB_DP_PIECES 5 / 6
# (experiment build), twice each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05af; mkdir -p $OUT
for r in 1 2; do
  for ps in 5 6; do
    BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_exp.so MIB_DP_PIECES=$ps timeout -k 10 300 python3 bench.py --workload latency --no-cpu-baseline >> $OUT/lat_ps$ps.json 2>> $OUT/lat_ps$ps.err || { echo "ps $ps failed"; tail $OUT/lat_ps$ps.err; exit 1; }
  done
done
echo "exit=0"
