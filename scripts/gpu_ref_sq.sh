# SQ counters of decode_streams_kernel on the ref leg (one foreign stream per call): the
# lone-wave decode bound measured, not asserted.  Two passes of 8 SQ counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/prof_${1:-r03}
mkdir -p $OUT
K=decode_streams_kernel
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
P2="SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT"
A="--workload ref --steps 1 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc $P1 --kernel-include-regex $K -d $OUT/sqref1_$K -o run -f csv -- python3 bench.py $A > $OUT/sqref1.log 2>&1 || { echo "sqref1 failed"; tail $OUT/sqref1.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc $P2 --kernel-include-regex $K -d $OUT/sqref2_$K -o run -f csv -- python3 bench.py $A > $OUT/sqref2.log 2>&1 || { echo "sqref2 failed"; tail $OUT/sqref2.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_ref -o run -f csv -- python3 bench.py $A > $OUT/trace_ref.log 2>&1 || { echo "trace ref failed"; exit 1; }
echo "exit=0"
