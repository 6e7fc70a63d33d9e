#!/bin/bash
# classify_kernel ablations on one config (profiling switches, results are not joins):
# 11 = no pixel loads, 12 = no code stores, 14 = no LDS block table, 15 = LDS table only
set -o pipefail
CFG=${1:-c2}
mkdir -p gpurun_out
export TMPDIR=/tmp
for ab in 0 11 12 14 15; do
  MGPU_ABLATE=$ab timeout -k 10 200 python3 -u tools/ab_time.py --configs $CFG --reps 5 > gpurun_out/ablate_${CFG}_$ab.json 2> gpurun_out/ablate_${CFG}_$ab.err || { tail -3 gpurun_out/ablate_${CFG}_$ab.err; exit 1; }
  sed "s/^/ablate $ab /" gpurun_out/ablate_${CFG}_$ab.json
done
