# decoder diagnostics: MIB_PROF phase counters + a sample of C4 streams (decode_diag.py), then
# SQ counters of decode_streams_kernel on the ref leg (one foreign stream per call) and on C4
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-sq}
mkdir -p $OUT
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_prof.so timeout -k 10 300 python3 scripts/decode_diag.py > $OUT/diag.log 2>&1 || { echo "diag failed"; tail $OUT/diag.log; exit 1; }
K=decode_streams_kernel
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
P2="SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM"
for w in ref c4; do
  A="--workload $w --steps 1 --warmup 1 --no-cpu-baseline"
  timeout -k 10 300 rocprofv3 --pmc $P1 --kernel-include-regex $K -d $OUT/${w}_1 -o run -f csv -- python3 bench.py $A > $OUT/${w}_1.log 2>&1 || { echo "pmc1 $w failed"; tail $OUT/${w}_1.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc $P2 --kernel-include-regex $K -d $OUT/${w}_2 -o run -f csv -- python3 bench.py $A > $OUT/${w}_2.log 2>&1 || { echo "pmc2 $w failed"; tail $OUT/${w}_2.log; exit 1; }
done
echo "exit=0"
