# A/B of the working tree's library against libbrotli_amd_head.so (the last commit), same box,
# interleaved: WL workloads (default c4), R rounds, BENCH_ARGS passed to every bench run
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}; mkdir -p $OUT
for r in $(seq 1 ${R:-3}); do
  for w in ${WL:-c4}; do
    for v in head new; do
      L=$PWD/brotli-lib_amd/libbrotli_amd.so; [ $v = head ] && L=$PWD/brotli-lib_amd/libbrotli_amd_head.so
      BROTLI_AMD_LIB=$L timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline ${BENCH_ARGS:-} >> $OUT/${w}_$v.json 2>> $OUT/${w}_$v.err || { echo "$w $v failed"; tail $OUT/${w}_$v.err; exit 1; }
    done
  done
done
echo "exit=0"
