#!/bin/bash
# Submit one gpurun call, re-submitting it only while the pool reports "no box / slot free" (exit 3: nothing ran,
# nothing charged) or a transient infrastructure back-off; any other outcome (the command ran, or was refused) ends
# the loop. Usage: scripts/mi355x/gpurun_when_free.sh <logfile> <max_attempts> <gpurun args...>
log=$1; max=$2; shift 2
for i in $(seq 1 "$max"); do
  /usr/local/graft/bin/gpurun "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$log"; then
    echo "attempt $i: no box (rc=$rc)" >> "$log.attempts"
    sleep 150
    continue
  fi
  echo "attempt $i: rc=$rc" >> "$log.attempts"
  exit $rc
done
exit 3
