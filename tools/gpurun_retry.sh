#!/bin/bash
# (local helper: run gpurun again only when the pool reported no free box / slot — nothing ran, nothing was charged)
# retry gpurun only while the pool has no free box / slot (nothing ran, nothing charged)
log=$1; shift
for i in 1 2 3 4 5 6 7 8 9 10; do
  timeout 2700 /usr/local/graft/bin/gpurun "$@" > $log 2>&1
  rc=$?
  if grep -q "status=transient" $log && ! grep -q "status=ok\|status=fail" $log; then
    sleep 150; continue
  fi
  exit $rc
done
exit 99
