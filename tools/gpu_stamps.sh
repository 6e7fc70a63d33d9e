#!/bin/bash
# Per-phase tile time (MGPU_STAMPS variant, counters[11..14] in 100 MHz ticks, summed
# over tiles) on each bench config.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-st}
for c in ${CONFIGS:-c2 c4 c5}; do
 for r in ${RASTER:-1}; do
  MGPU_RASTER=$r MGPU_DEBUG_COUNTERS=1 MOSAIC_AMD_LIB=$PWD/build/variants/stamps/libmosaic_gpu.so timeout -k 10 200 python3 -u tools/join_once.py --reps 1 --config $c > gpurun_out/stamps_${c}_${r}_$TAG.log 2>&1 || exit 1
  echo "$c raster=$r: $(grep 'mgpu counters' gpurun_out/stamps_${c}_${r}_$TAG.log)"
 done
done
