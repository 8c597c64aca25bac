#!/bin/bash
# GPU-box step runner for gpurun calls: `source scripts/mi355x/steps.sh <outdir>` then `step <name> <seconds> cmd...`.
# Every step runs under its own time limit, logs to gpurun_out/<outdir>/<name>.log and appends "<name> rc=<rc>
# <seconds>s" to steps.txt. rc 0/1 (pass / test failure / Python error) go on to the next step; anything else (a
# time limit 124/137, an abort 134, a segfault 139, ...) ends the call there, so nothing more touches a GPU that may
# be in a bad state.
OUT=gpurun_out/${1:-run}
mkdir -p "$OUT"
step() {
  local name=$1 t=$2
  shift 2
  local t0=$SECONDS
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $((SECONDS - t0))s" >> "$OUT/steps.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after $name (rc=$rc)" >> "$OUT/steps.txt"
    exit $rc
  fi
}
