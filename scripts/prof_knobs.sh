# rocprofv3 kernel-trace stats of one bench leg per experiment-build knob setting (CFGS as in
# ab_knobs.sh): gpurun_out/TAG/<name>/ holds each run's kernel_stats.csv
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_exp.so
OUT=gpurun_out/${TAG:-profk}; mkdir -p $OUT
for c in $CFGS; do
  name=${c%%:*}; envs=${c#*:}
  for kv in $(echo "$envs" | tr '+' ' '); do export "$kv"; done
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/$name -o run -f csv -- python3 bench.py --workload ${WL:-c4} --steps 2 --warmup 1 --no-cpu-baseline > $OUT/$name.log 2>&1 || { echo "$name failed"; tail $OUT/$name.log; exit 1; }
  for kv in $(echo "$envs" | tr '+' ' '); do unset "${kv%%=*}"; done
done
echo "exit=0"
