#!/bin/bash
# Parity tests, time breakdown, and the MGPU_STATS variant's counters.
set -o pipefail
TAG=${1:-s}
bash tools/gpu_quick.sh $TAG || exit 1
MGPU_DEBUG_COUNTERS=1 MOSAIC_AMD_LIB=$PWD/build/variants/stats/libmosaic_gpu.so timeout -k 10 200 python3 -u tools/join_once.py --reps 1 > gpurun_out/stats_$TAG.log 2>&1
rc=$?
cat gpurun_out/stats_$TAG.log | grep -v amdgpu.ids
exit $rc
