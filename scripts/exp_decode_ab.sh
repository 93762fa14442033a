# Decoder A/B experiments on the C4 leg (bench.py, no CPU baseline): the same build under
# encoder / launch knobs.  Usage: exp_decode_ab.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
A="--steps 3 --warmup 1 --no-cpu-baseline"
run() {   # name, env..., -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py $A > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail $OUT/$name.err; exit 1; }
  echo "$name done"
}
run base MIB_X=0
run lit4 MIB_LIT_TREES=4
run grid512 MIB_DEC_GRID=512
run grid256 MIB_DEC_GRID=256
echo "exit=0"
