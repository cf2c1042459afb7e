#!/bin/bash
# Submit one gpurun call; when the pool has no free box / slot (exit 3: nothing ran, nothing
# charged) wait and submit the same call again, at most $GPURUN_TRIES times. Any other exit
# (including a failing command) is final. Usage: tools/gpurun_wait.sh <log> <timeout_s> '<cmd>'
log=$1; t=$2; shift 2
tries=${GPURUN_TRIES:-12}
for i in $(seq 1 "$tries"); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$log"; then exit $rc; fi
  echo "[gpurun_wait] try $i: no box/slot (rc=$rc), retrying in 150 s" >> "$log.retries"
  sleep 150
done
exit 3
