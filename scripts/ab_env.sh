# One bench leg per value of an environment knob: VAR=MIB_DEPTH VALS="64 32" WL=c4 bash scripts/ab_env.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1
mkdir -p gpurun_out/$TAG
for v in $VALS; do
  env $VAR=$v timeout -k 10 300 python3 bench.py --workload ${WL:-c4} --no-cpu-baseline > gpurun_out/$TAG/${WL:-c4}_$v.json 2> gpurun_out/$TAG/${WL:-c4}_$v.err || { echo "$v failed"; tail gpurun_out/$TAG/${WL:-c4}_$v.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print(sys.argv[2], d['value'], d.get('compressed_ratio'), ' '.join('%s %.1f' % (n, k[n]) for n in sorted(k, key=lambda n: -k[n])[:8]))" gpurun_out/$TAG/${WL:-c4}_$v.json $VAR=$v
done
echo "exit=0"
