#!/bin/bash
# Time-breakdown of each build/variants/* library (plus the in-tree one), one process each.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-v}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
for d in build/variants/*/; do
  n=$(basename $d)
  MOSAIC_AMD_LIB=$PWD/$d/libmosaic_gpu.so timeout -k 10 200 python3 -u tools/breakdown.py > gpurun_out/bd_${TAG}_$n.json 2> gpurun_out/bd_${TAG}_$n.err || { echo "variant $n failed"; cat gpurun_out/bd_${TAG}_$n.err | tail -5; exit 1; }
  echo "$n $(cat gpurun_out/bd_${TAG}_$n.json)"
done
