#!/bin/bash
# Run one gpurun call, retrying only while the pool has no free box (exit 3 /
# "transient": nothing ran, nothing charged).  Usage: tools/gpurun_retry.sh OUT TIMEOUT 'command'
out=$1; to=$2; shift 2
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $out 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" $out; then sleep 120; continue; fi
  exit $rc
done
exit 3
