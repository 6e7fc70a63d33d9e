#!/bin/bash
# Interleaved A/B timing of build/variants/* (two rounds each), after the GPU tests.
set -o pipefail
TAG=${1:-ab}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
for round in 1 2; do
  for d in build/variants/*/; do
    n=$(basename $d)
    MOSAIC_AMD_LIB=$PWD/$d/libmosaic_gpu.so timeout -k 10 200 python3 -u tools/breakdown.py > gpurun_out/ab_${TAG}_${n}_$round.json 2> gpurun_out/ab_${TAG}_${n}_$round.err || { echo "variant $n failed"; tail -5 gpurun_out/ab_${TAG}_${n}_$round.err; exit 1; }
    echo "$round $n $(cat gpurun_out/ab_${TAG}_${n}_$round.json)"
  done
done
