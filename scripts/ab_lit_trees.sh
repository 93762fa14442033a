# literal prefix codes per metablock (MIB_LIT_TREES caps them) against compressed size and
# decode speed: past the decoder's LDS table area a metablock's tables stay in HBM
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ablt
for w in ${WL:-c3 c4}; do for c in ${CAPS:-64 32 24}; do
  MIB_LIT_TREES=$c timeout -k 10 400 python3 bench.py --workload $w --no-cpu-baseline > gpurun_out/ablt/${w}_$c.json 2> gpurun_out/ablt/${w}_$c.err || exit 1
done; done
echo "exit=0"
