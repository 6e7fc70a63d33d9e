#!/bin/bash
# cells_kernel timing per build/variants/* (H3 res 9 and BNG res 4 on 1e8 points).
set -o pipefail
for d in build/variants/*/; do
  n=$(basename $d)
  MOSAIC_AMD_LIB=$PWD/$d/libmosaic_gpu.so timeout -k 10 200 python3 -u tools/cells_bench.py > gpurun_out/cells_$n.json 2> gpurun_out/cells_$n.err || { tail -3 gpurun_out/cells_$n.err; exit 1; }
  echo "$n $(cat gpurun_out/cells_$n.json)"
done
