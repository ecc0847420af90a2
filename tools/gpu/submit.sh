#!/bin/bash
# Submit one gpurun call, waiting for a free slot: re-submits ONLY while gpurun reports
# status=transient (no box / all slots busy / backing off: nothing ran, nothing charged);
# any call that ran on a box is final, whatever its exit code.
#   tools/gpu/submit.sh LOG TIMEOUT_S 'command'
LOG=$1; TO=$2; CMD=$3
for attempt in $(seq 1 60); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient" "$LOG"; then
    sleep 60
    continue
  fi
  exit $rc
done
exit 3
