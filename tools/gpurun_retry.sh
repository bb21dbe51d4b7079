#!/bin/bash
# Host-side helper: run one gpurun call, re-submitting it (up to 12 times,
# 2 minutes apart) only when gpurun reports that no box was obtained (exit 3 /
# "transient"), i.e. when nothing ran on a GPU.  Usage: tools/gpurun_retry.sh LOG TIMEOUT CMD...
log=$1; shift; to=$1; shift
for i in $(seq 1 ${RETRIES:-12}); do
  timeout $((to + 1500)) /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$log"; then
    echo "attempt $i: no box ($rc), retrying" >> "$log.retries"; sleep ${RETRY_SLEEP:-120}; continue
  fi
  exit $rc
done
exit $rc
