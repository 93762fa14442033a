# A/B of experiment-build knob settings on one box: CFGS="name:VAR=v+VAR2=w name2:..." (an
# empty setting list is the build's defaults), WL workloads, R rounds; bench lines per
# (workload, setting) under gpurun_out/TAG/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-knobs}; mkdir -p $OUT
L=$PWD/brotli-lib_amd/libbrotli_amd_exp.so
for r in $(seq 1 ${R:-1}); do
  for w in ${WL:-c4}; do
    for c in $CFGS; do
      name=${c%%:*}; envs=${c#*:}
      env $(echo "$envs" | tr '+' ' ') BROTLI_AMD_LIB=$L timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline ${BENCH_ARGS:-} >> $OUT/${w}_$name.json 2>> $OUT/${w}_$name.err || { echo "$w $name failed"; tail $OUT/${w}_$name.err; exit 1; }
    done
  done
done
echo "exit=0"
