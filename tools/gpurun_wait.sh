#!/bin/bash
# Queue a gpurun call until a box is free: re-issues the SAME call only when gpurun reports
# that no box was free (exit 3 / "transient", nothing ran, nothing charged); any call that
# ran -- whatever its result -- ends the loop.  usage: tools/gpurun_wait.sh LOG TIMEOUT CMD
log=$1; to=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient rc=None" "$log"; then
    sleep 150
    continue
  fi
  exit $rc
done
exit 3
