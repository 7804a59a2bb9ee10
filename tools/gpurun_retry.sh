#!/bin/bash
# host-side retry of gpurun while no box/slot is available (nothing ran, nothing charged)
cmd="$1"; limit="${2:-1000}"
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$limit" -- "$cmd" > /tmp/np8_gpurun_last.out 2>&1
  rc=$?
  if grep -q "status=transient" /tmp/np8_gpurun_last.out || [ $rc -eq 3 ]; then
    echo "attempt $i: transient/no slot (rc=$rc), retrying" >&2; sleep 60; continue
  fi
  cat /tmp/np8_gpurun_last.out | tail -12
  exit $rc
done
echo "gave up"; exit 3
