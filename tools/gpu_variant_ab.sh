#!/bin/bash
# Interleaved auto-pipeline timings (tools/bin_ab.py --variants auto) of the tree's library
# and each build/variants/*: tools/gpu_variant_ab.sh CONFIGS
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for c in ${1//,/ }; do
    timeout -k 10 300 python3 -u tools/bin_ab.py --config $c --variants auto > gpurun_out/vab_base_${c}_$rep.json 2>/dev/null || exit 1
    echo "base $rep $(cat gpurun_out/vab_base_${c}_$rep.json | cut -c1-220)"
    for d in build/variants/*/; do
      n=$(basename $d)
      MOSAIC_AMD_LIB=$PWD/$d/libmosaic_gpu.so timeout -k 10 300 python3 -u tools/bin_ab.py --config $c --variants auto > gpurun_out/vab_${n}_${c}_$rep.json 2>/dev/null || exit 1
      echo "$n $rep $(cat gpurun_out/vab_${n}_${c}_$rep.json | cut -c1-220)"
    done
  done
done
