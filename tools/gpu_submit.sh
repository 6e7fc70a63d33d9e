#!/bin/bash
# (run here, not on the box) submit a gpurun command; resubmit only when the pool had no box / the box was lost before
# the command ran (nothing ran, nothing charged); at most 8 tries
OUT=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun "$@" > $OUT 2>&1
  if grep -q "no free box\|status=transient" $OUT && ! grep -q "status=ok\|status=fail" $OUT; then sleep 90; continue; fi
  break
done
