#!/bin/bash
# Host side only: re-submit a gpurun call while the pool reports a transient (infrastructure)
# status -- no box taken, nothing of the command ran.  Any other outcome is returned as is.
# usage: tools/gpurun_retry.sh OUTFILE TIMEOUT 'command'
OUT=$1; TMO=$2; CMD=$3
for i in $(seq 1 ${GPURUN_TRIES:-20}); do
  /usr/local/graft/bin/gpurun --timeout "$TMO" -- "$CMD" > "$OUT" 2>&1
  rc=$?
  if grep -q '"status": "transient"' gpurun_out/.last_call.json 2>/dev/null; then
    echo "transient ($i), retrying in 90 s" >> "$OUT.retries"
    sleep 90
    continue
  fi
  exit $rc
done
exit 3
