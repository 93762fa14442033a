# SQ counters for one kernel on a reduced bench workload: where do its waves spend time?
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
K=${1:-dp_kernel}
OUT=gpurun_out/pmc_$K
mkdir -p $OUT
ARGS="--steps 1 --warmup 1 --no-cpu-baseline --streams ${STREAMS:-256}"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex $K -d $OUT/a -o run -f csv -- python3 bench.py $ARGS > $OUT/a.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --kernel-include-regex $K -d $OUT/b -o run -f csv -- python3 bench.py $ARGS > $OUT/b.log 2>&1
echo "exit=$?"
