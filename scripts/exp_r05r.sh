# r05r: the decoder's pending-copy queue in lanes (v_writelane / v_readlane) instead of eight
# shifted SGPRs: GPU tests, c4 / c3 / latency, SQ instruction counters of decode_streams_kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05r; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
for w in c4 c3 latency; do
  timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline > $OUT/$w.json 2> $OUT/$w.err || { echo "$w failed"; tail $OUT/$w.err; exit 1; }
done
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
P2="SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT"
timeout -k 10 400 rocprofv3 --pmc $P1 --kernel-include-regex decode_streams_kernel -d $OUT/sq1_decode_streams_kernel -o run -f csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/sq1.log 2>&1 || { echo "sq1 failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc $P2 --kernel-include-regex decode_streams_kernel -d $OUT/sq2_decode_streams_kernel -o run -f csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/sq2.log 2>&1 || { echo "sq2 failed"; exit 1; }
echo "exit=0"
