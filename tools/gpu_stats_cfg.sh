#!/bin/bash
# The MGPU_STATS variant's counters on each bench config (candidates, mixed, edges walked).
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-s}
for c in c2 c4 c5; do
  MGPU_DEBUG_COUNTERS=1 MOSAIC_AMD_LIB=$PWD/build/variants/stats/libmosaic_gpu.so timeout -k 10 200 python3 -u tools/join_once.py --reps 1 --config $c > gpurun_out/stats_${c}_$TAG.log 2>&1 || exit 1
  echo "$c: $(grep 'mgpu counters' gpurun_out/stats_${c}_$TAG.log)"
done
