#!/bin/bash
# Per-phase clock shares of the join tiles (tools/phase_stamps.py) from the stamps variant
# (tools/build_variants.sh "stamps:-DMGPU_STAMPS"): gpurun_out/stamps_TAG.json
set -o pipefail
TAG=${1:-s}; CFGS=${2:-c3,c2}; shift 2; EXTRA="$@"
mkdir -p gpurun_out
MOSAIC_AMD_LIB=$PWD/build/ab/stamps/libmosaic_gpu.so timeout -k 10 300 python3 -u tools/phase_stamps.py --configs $CFGS $EXTRA > gpurun_out/stamps_$TAG.json 2> gpurun_out/stamps_$TAG.err || { echo "stamps failed"; tail -5 gpurun_out/stamps_$TAG.err; exit 1; }
cat gpurun_out/stamps_$TAG.json
