# bench legs under each value of one environment override: VAR=MIB_X VALS="a b" WORKLOADS="c4 c3"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-sweep}
mkdir -p gpurun_out/$T
for v in $VALS; do
  f=${v//\//_}
  for w in ${WORKLOADS:-c4 c3}; do
    env $VAR=$v timeout -k 10 300 python3 bench.py --workload $w --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > gpurun_out/$T/b_${w}_$f.json 2> gpurun_out/$T/b_${w}_$f.err || { echo "bench $w $v failed"; tail gpurun_out/$T/b_${w}_$f.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/$T/b_${w}_$f.json'));k=d['kernel_ms_per_step'];print('$w $VAR=$v', d['value'], d['encode_MBps'], d['compressed_ratio'], k.get('dp_parse'), k.get('cost_model'), k.get('backtrack'))"
  done
done
echo exit=0
