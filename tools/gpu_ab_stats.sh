#!/bin/bash
set -o pipefail
bash tools/gpu_ab.sh ${1:-abs} || exit 1
MGPU_DEBUG_COUNTERS=1 MOSAIC_AMD_LIB=$PWD/build/variants/stats/libmosaic_gpu.so timeout -k 10 200 python3 -u tools/join_once.py --reps 1 2>&1 | grep -v amdgpu.ids
