# r04l: find_matches taken apart (kernel traces of one warmup step; the experiment builds
# write wrong streams, so the bench stops at its round-trip check, exit 1 expected):
# staging only (MIB_FM_EXP=32), staging without the prefix gather (96), the walk without
# the gather (64)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04l
mkdir -p $OUT
for x in 32 96 64; do
MIB_FM_EXP=$x timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/fm$x -o run -f csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/fm$x.log 2>&1
rc=$?; [ $rc -le 1 ] || { echo "fm$x rc=$rc"; tail $OUT/fm$x.log; exit 1; }
done
echo "exit=0"
