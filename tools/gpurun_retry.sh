#!/bin/bash
# Re-submit a gpurun call only when the infrastructure reports a transient failure
# (box not acquired / stopped responding before the command ran: nothing executed,
# nothing charged).  Any real outcome of the command — pass, fail, fault — ends it.
# usage: tools/gpurun_retry.sh <timeout_s> '<command>'
T=$1; shift
for i in 1 2 3 4 5 6; do
  out=$(timeout $((T + 900)) /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1); rc=$?
  echo "$out" | tail -60
  if echo "$out" | grep -q "status=transient\|backing off" || [ $rc -eq 3 ]; then
    echo "[retry] transient infrastructure failure, attempt $i"; sleep 45; continue
  fi
  exit $rc
done
exit 3
