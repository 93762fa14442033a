# Run one gpurun call, retrying (every 2 minutes, at most 8 times) only while the pool has no
# free slot or box (gpurun exit 3 / "transient": nothing ran, nothing charged).  Never retries a
# call that ran.  usage: scripts/gpurun_retry.sh <log> <timeout> <command>
LOG=$1; TO=$2; shift 2
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
  rc=$?
  if grep -q "status=transient" $LOG; then sleep 120; continue; fi
  exit $rc
done
exit 3
