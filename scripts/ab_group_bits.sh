# find_matches locality: the sort key's stream-group bits (MIB_GROUP_BITS) on one bench leg
# usage (GPU box): WL=c4 GBS="6 8 10" bash scripts/ab_group_bits.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1
mkdir -p gpurun_out/$TAG
for gb in ${GBS:-6 8 10}; do
  MIB_GROUP_BITS=$gb timeout -k 10 300 python3 bench.py --workload ${WL:-c4} --no-cpu-baseline > gpurun_out/$TAG/${WL:-c4}_g$gb.json 2> gpurun_out/$TAG/${WL:-c4}_g$gb.err || { echo "g$gb failed"; tail gpurun_out/$TAG/${WL:-c4}_g$gb.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print(sys.argv[2], d['value'], d.get('compressed_ratio'), 'fm', k.get('find_matches'), 'sort', k.get('radix_sort'), 'dp', k.get('dp_parse'))" gpurun_out/$TAG/${WL:-c4}_g$gb.json g$gb
done
echo "exit=0"
