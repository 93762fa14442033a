set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-chk}
mkdir -p gpurun_out/$T
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/$T/tests.log; exit 1; }
for w in ${WORKLOADS:-c4 c2}; do
  timeout -k 10 500 python3 bench.py --workload $w --no-cpu-baseline > gpurun_out/$T/bench_$w.json 2> gpurun_out/$T/bench_$w.err || { echo "bench $w failed"; tail gpurun_out/$T/bench_$w.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/$T/bench_$w.json'));print('$w', d['value'], d['encode_MBps'], d['decode_MBps'], d['compressed_ratio'], d['kernel_ms_per_step'].get('find_matches'), d['kernel_ms_per_step'].get('dp_parse'))"
done
echo exit=0
