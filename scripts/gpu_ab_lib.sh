# A/B of library builds on one bench leg: bench.py with BROTLI_AMD_LIB=<each .so given>
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; W=$2; shift 2
mkdir -p gpurun_out/$TAG
for lib in "$@"; do
  n=$(basename $lib .so)
  BROTLI_AMD_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --workload $W --no-cpu-baseline > gpurun_out/$TAG/${W}_$n.json 2> gpurun_out/$TAG/${W}_$n.err || { echo "$n failed"; tail gpurun_out/$TAG/${W}_$n.err; exit 1; }
done
echo "exit=0"
