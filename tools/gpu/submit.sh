#!/bin/bash
# Submit one gpurun call, retrying only while no box / slot is free (gpurun exit 3 or its "no free
# box" / "stopped responding while being prepared" notes: nothing ran, nothing was charged).
#   tools/gpu/submit.sh <log> <timeout_s> '<command>'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 30); do
  timeout $((TO + 1500)) /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -qE "no free box|slot\(s\) on this pod are busy|stopped responding while being prepared|backing off|status=transient" "$LOG"; then
    sleep 90; continue
  fi
  exit $rc
done
exit $rc
