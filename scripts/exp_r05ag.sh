# r05ag: 1 KiB parse pieces for one-segment one-shot streams too: GPU tests, cadence, latency
# and c5 throughput mode
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05ag; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
timeout -k 10 300 python3 bench.py --workload c5 --stream-chunk 0 --size 268435456 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/c5_cadence.json 2> $OUT/c5_cadence.err || { echo "cadence failed"; tail $OUT/c5_cadence.err; exit 1; }
timeout -k 10 300 python3 bench.py --workload latency > $OUT/latency.json 2> $OUT/latency.err || { echo "latency failed"; tail $OUT/latency.err; exit 1; }
echo "exit=0"
