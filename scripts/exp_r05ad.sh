# r05ad: 1 KiB parse pieces for the cadence leg's 1 MiB chunks (experiment build, MIB_DP_PIECES
# 5 = 2 KiB, the default for streaming chunks, against 6 = 1 KiB), twice each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05ad; mkdir -p $OUT
for r in 1 2; do
  for ps in 5 6; do
    BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_exp.so MIB_DP_PIECES=$ps timeout -k 10 300 python3 bench.py --workload c5 --stream-chunk 0 --size 268435456 --steps 1 --warmup 1 --no-cpu-baseline >> $OUT/cad_ps$ps.json 2>> $OUT/cad_ps$ps.err || { echo "ps $ps failed"; tail $OUT/cad_ps$ps.err; exit 1; }
  done
done
echo "exit=0"
