#!/usr/bin/env bash
# usage: gpurun_retry.sh LOG TIMEOUT CMD  -- retries only while the pool has no free box
# (exit 3 or a transient infrastructure status: nothing ran, nothing was charged)
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ]; then sleep 60; continue; fi
  if grep -q "status=transient" "$LOG" && ! grep -q "status=ok" "$LOG"; then sleep 60; continue; fi
  echo "final rc=$rc try=$i" >> "$LOG"; exit $rc
done
