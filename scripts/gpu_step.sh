# Run one GPU step under its own time limit; exit 0 when it passed or only failed tests /
# assertions (rc 1), otherwise (fault, abort, segfault, time limit) stop with its code so the
# caller's && chain starts nothing more on the GPU.   usage: gpu_step.sh SECONDS LOG cmd...
T=$1; LOG=$2; shift 2
mkdir -p "$(dirname "$LOG")"
timeout -k 10 "$T" "$@" > "$LOG" 2>&1
rc=$?
echo "step rc=$rc: $*" >> "$LOG"
tail -5 "$LOG"
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then exit 0; fi
exit $rc
