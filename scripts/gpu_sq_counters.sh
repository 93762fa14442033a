# SQ instruction counters for the DP / decode / find_matches kernels (one rocprofv3 --pmc pass)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-sq}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH \
  --kernel-include-regex "${KRE:-dp_kernel|decode_streams|find_matches}" -d $OUT/pmc -o run -f csv -- python3 bench.py --workload ${WL:-c4} --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc.log 2>&1
echo "exit=$?"
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
rows = []
for p in glob.glob(sys.argv[1] + '/pmc/**/*counter_collection.csv', recursive=True):
    rows += list(csv.DictReader(open(p)))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.defaultdict(set)
for r in rows:
    k = r['Kernel_Name'].split('(')[0][-60:]
    agg[k][r['Counter_Name']] += float(r['Counter_Value'])
    n[k].add(r['Dispatch_Id'])
for k, v in agg.items():
    print(k, len(n[k]), {c: '%.4g' % x for c, x in sorted(v.items())})
PY
