#!/bin/bash
# (run from the build container: gpurun only when nothing ran because no box or slot was free)
# usage: gpu_retry.sh LOG TIMEOUT CMD  — retries only when no box/slot was obtained (nothing ran)
LOG=$1; TO=$2; shift 2
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > "$LOG" 2>&1
  if grep -q "status=transient" "$LOG" && ! grep -q "charged=[1-9]" "$LOG"; then
    sleep 120; continue
  fi
  break
done
echo "__DONE__" >> "$LOG"
