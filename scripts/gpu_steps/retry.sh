#!/bin/bash
# retry a gpurun call while the pool has no free box (exit 3: nothing ran, nothing charged)
out=$1; shift
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun "$@" > "$out" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$out"; then echo "rc=$rc" >> "$out"; exit $rc; fi
  sleep 90
done
