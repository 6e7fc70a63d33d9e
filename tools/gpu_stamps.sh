#!/bin/bash
set -o pipefail
MGPU_DEBUG_COUNTERS=1 MOSAIC_AMD_LIB=$PWD/build/variants/stamps/libmosaic_gpu.so timeout -k 10 200 python3 -u tools/join_once.py --reps 2 2>&1 | grep -v amdgpu.ids
