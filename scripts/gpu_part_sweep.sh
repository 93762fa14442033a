# C2 ratio / speed against the part size and source lag (MIB_PART_BITS / MIB_PART_LAG)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep
for cfg in "0 16 4096" "1 16 4096" "1 16 1024" "1 16 256" "1 17 1024" "1 18 1024" "1 18 4096" "1 20 4096"; do
  set -- $cfg
  if [ "$1" = "0" ]; then export MIB_PART_MIN=0; else unset MIB_PART_MIN; fi
  export MIB_PART_BITS=$2 MIB_PART_LAG=$3
  timeout -k 10 300 python3 bench.py --workload c2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sweep/c2_$1_$2_$3.json 2>/dev/null || { echo "failed $cfg"; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/sweep/c2_$1_$2_$3.json'));print('$cfg', d['value'], d['encode_MBps'], d['decode_MBps'], d['compressed_ratio'])"
done
