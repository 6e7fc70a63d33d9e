#!/bin/bash
# Build profiling variants of libmosaic_gpu.so: tools/variants.sh NAME "-DFOO=1" [NAME "-D..."]...
# Each lands in build/variants/NAME/libmosaic_gpu.so (select with MOSAIC_AMD_LIB).
set -e
cd "$(dirname "$0")/../mosaic_amd/csrc"
while [ $# -ge 2 ]; do
  d=../../build/variants/$1; mkdir -p $d
  rm -f kernels.o
  make -s OUT=$d/libmosaic_gpu.so KFLAGS="$2" $d/libmosaic_gpu.so
  rm -f kernels.o
  shift 2
done
make -s
