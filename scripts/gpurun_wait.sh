#!/bin/bash
# Submit one gpurun call, waiting out infrastructure back-off / no-box answers (exit 3, "backing off",
# "stopped responding while being prepared": nothing ran, nothing charged).  A call that actually ran is
# never resubmitted, whatever its exit status.
#   scripts/gpurun_wait.sh <timeout-seconds> '<command>'  > log
T=$1
shift
for attempt in $(seq 1 ${GPURUN_ATTEMPTS:-30}); do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1)
  rc=$?
  echo "$out"
  if echo "$out" | grep -q "status=transient\|backing off\|no box\|slot free"; then
    wait_s=$(echo "$out" | grep -o "retry in [0-9]*s" | grep -o "[0-9]*" | tail -1)
    wait_s=${wait_s:-60}
    echo "[gpurun_wait] infrastructure not ready (attempt $attempt); sleeping $((wait_s + 10))s"
    sleep $((wait_s + 10))
    continue
  fi
  exit $rc
done
exit 3
