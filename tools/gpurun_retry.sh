#!/bin/bash
# Submit one gpurun call, resubmitting only while the pool has no free slot or
# box (gpurun exit 3 / a transient status: nothing ran, nothing charged).
# Usage: tools/gpurun_retry.sh OUTFILE TIMEOUT 'command'
out=$1; to=$2; cmd=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$out" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient\|no free box\|slot(s) on this pod are busy" "$out"; then
    sleep 90; continue
  fi
  echo "rc=$rc" >> "$out"; exit $rc
done
exit 3
