# rocprofv3 evidence for the round: kernel-trace stats of c4, c3, c2 (WORKLOADS: also c5 and
# c5cad, C5 at the reference's update() cadence); FETCH_SIZE / WRITE_SIZE
# passes of each (separate runs: they cannot share a pass); SQ counters of the dominant encode
# kernels on c4.  Every step under its own limit; stop at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r03}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
A="--steps 1 --warmup 1 --no-cpu-baseline"
# only the summaries travel back (gpurun copies at most 64 MiB of gpurun_out)
keep() { find "$1" -type f ! -name "*kernel_stats.csv" ! -name "*counter_collection.csv" -delete; }
for w in ${WORKLOADS-c4 c3 c2}; do
  WA="--workload $w"; [ $w = c5cad ] && WA="--workload c5 --stream-chunk 0"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace_$w -o run -f csv -- python3 bench.py $A $WA > $OUT/trace_$w.log 2>&1 || { echo "trace $w failed"; tail $OUT/trace_$w.log; exit 1; }
  keep $OUT/trace_$w
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch_$w -o run -f csv -- python3 bench.py $A $WA > $OUT/fetch_$w.log 2>&1 || { echo "fetch $w failed"; exit 1; }
  keep $OUT/fetch_$w
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/write_$w -o run -f csv -- python3 bench.py $A $WA > $OUT/write_$w.log 2>&1 || { echo "write $w failed"; exit 1; }
  keep $OUT/write_$w
done
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
P2="SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT"
for k in ${SQ_KERNELS-dp_kernel find_matches_kernel decode_streams_kernel}; do
  timeout -k 10 400 rocprofv3 --pmc $P1 --kernel-include-regex $k -d $OUT/sq1_$k -o run -f csv -- python3 bench.py $A > $OUT/sq1_$k.log 2>&1 || { echo "sq1 $k failed"; exit 1; }
  keep $OUT/sq1_$k
  timeout -k 10 400 rocprofv3 --pmc $P2 --kernel-include-regex $k -d $OUT/sq2_$k -o run -f csv -- python3 bench.py $A > $OUT/sq2_$k.log 2>&1 || { echo "sq2 $k failed"; exit 1; }
  keep $OUT/sq2_$k
done
echo "exit=0"
