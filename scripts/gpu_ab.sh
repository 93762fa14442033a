# A/B of encoder knobs on the c4 bench leg (no CPU baseline): one line per variant
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-ab}
mkdir -p gpurun_out/$T
i=0
for v in "${@:2}"; do
  i=$((i+1))
  env $v timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 ${ABARGS:-} > gpurun_out/$T/v$i.json 2> gpurun_out/$T/v$i.err || { echo "variant $v failed"; tail gpurun_out/$T/v$i.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/$T/v$i.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('$v', d['value'], d['compressed_ratio'], {x:k.get(x) for x in ('find_matches','radix_sort','hash_keys','dp_parse','decode_streams_kernel')})" | tee -a gpurun_out/$T/summary.txt
done
echo exit=0
