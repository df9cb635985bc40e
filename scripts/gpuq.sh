#!/bin/bash
# (host-side helper, runs in this container: it only resubmits a call the pool did not start)
# submit a gpurun call; resubmit only while the pool reports no free slot/box (exit 3: nothing ran, nothing charged)
T=$1; shift
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout $T -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[gpuq] no slot (attempt $i), waiting 90 s"; sleep 90
done
exit 3
