#!/bin/bash
# kRing batch-divergence check: tools/kring_debug.py on the tree's library and each build/variants/*
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 -u tools/kring_debug.py > gpurun_out/kdbg_base.log 2>&1; grep "^res" gpurun_out/kdbg_base.log | cut -c1-60
for d in build/variants/*/; do
  n=$(basename $d)
  MOSAIC_AMD_LIB=$PWD/$d/libmosaic_gpu.so timeout -k 10 200 python3 -u tools/kring_debug.py > gpurun_out/kdbg_$n.log 2>&1; echo "== $n"; grep "^res" gpurun_out/kdbg_$n.log | cut -c1-60
done
