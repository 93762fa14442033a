set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/parts3
MIB_PART_MIN=65537 MIB_PART_BITS=16 timeout -k 10 120 python3 tests/golden/parts/make_fixture.py gpurun_out/parts3/parts_enwik300k.br > gpurun_out/parts3/fixture.log 2>&1 || { echo fixture failed; exit 1; }
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parts.py -x -v --timeout 200 --timeout-method thread > gpurun_out/parts3/parts.log 2>&1 || { echo "parts tests failed"; exit 1; }
for w in c4 c2; do
  timeout -k 10 500 python3 bench.py --workload $w --no-cpu-baseline > gpurun_out/parts3/bench_$w.json 2> gpurun_out/parts3/bench_$w.err || { echo "bench $w failed"; exit 1; }
done
echo exit=0
