#!/bin/bash
# Interleaved A/B timing of build/variants/* on the bench configs (rounds x variants).
set -o pipefail
TAG=${1:-ab}
mkdir -p gpurun_out
for round in 1 2; do
  for d in build/variants/*/; do
    n=$(basename $d)
    MOSAIC_AMD_LIB=$PWD/$d/libmosaic_gpu.so timeout -k 10 200 python3 -u tools/ab_time.py ${AB_ARGS:-} > gpurun_out/ab_${TAG}_${n}_$round.json 2> gpurun_out/ab_${TAG}_${n}_$round.err || { echo "variant $n failed"; tail -5 gpurun_out/ab_${TAG}_${n}_$round.err; exit 1; }
    echo "== $round $n"; cat gpurun_out/ab_${TAG}_${n}_$round.json
  done
done
