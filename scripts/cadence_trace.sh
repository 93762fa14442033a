# rocprofv3 kernel trace of the reference-cadence leg on 64 MiB (64 update() calls), for
# scripts/chunk_timeline.py: which kernels one 1 MiB update waits on
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && OUT=gpurun_out/${TAG:-cad_trace} && mkdir -p $OUT && \
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o run -f csv -- python3 bench.py --workload c5 --stream-chunk 0 --size 67108864 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/trace.log 2>&1
echo "exit=$?"
find $OUT -name "*kernel_trace.csv" | head
