#!/usr/bin/env bash
# usage: gpurun_retry.sh LOG TIMEOUT CMD  -- retries only while the pool has no free box
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient" "$LOG" && ! grep -q "status=ok" "$LOG"; then sleep 90; continue; fi
  echo "final rc=$rc try=$i" >> "$LOG"; exit $rc
done
