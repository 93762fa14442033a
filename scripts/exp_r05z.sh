# r05z: the streaming build's match walk in lockstep too: GPU tests, then c5 A/B against HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05z; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
TAG=r05z/ab R=2 WL=c5 bash scripts/exp_ab.sh
