# r05aa: the short scan's masks by packed 16-bit min (v_pk_min_u16): GPU tests, c4 A/B against HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05aa; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
TAG=r05aa/ab R=3 WL=c4 bash scripts/exp_ab.sh
