#!/bin/bash
# Submit one gpurun call, re-submitting ONLY while the pool has no free box / slot (nothing ran,
# nothing charged: exit 3 or a "transient" status).  A call that ran is never repeated.
#   tools/gpurun_retry.sh OUTFILE TIMEOUT 'command'
OUT=$1; TMO=$2; CMD=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$TMO" -- "$CMD" > "$OUT" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$OUT"; then sleep 120; continue; fi
  exit $rc
done
exit 3
