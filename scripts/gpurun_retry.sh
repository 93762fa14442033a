# Run one gpurun call, retrying only while the pool has no free slot or box or access is backing
# off (gpurun "transient": nothing ran, nothing charged) -- after the wait gpurun names, else 2
# minutes; at most 10 tries.  Never retries a call that ran.
# usage: scripts/gpurun_retry.sh <log> <timeout> <command>
LOG=$1; TO=$2; shift 2
for i in 1 2 3 4 5 6 7 8 9 10; do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
  rc=$?
  if grep -q "status=transient" $LOG; then
    w=$(grep -o "retry in [0-9]*s" $LOG | grep -o "[0-9]*" | tail -1)
    sleep $(( ${w:-110} + 10 ))
    continue
  fi
  exit $rc
done
exit 3
