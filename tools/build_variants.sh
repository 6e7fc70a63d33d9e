#!/bin/bash
# Build library variants of the working tree with extra kernel flags, for interleaved
# A/B timings (tools/gpu_ab_split.sh): tools/build_variants.sh "name1:-DFLAG=1 -DX=2" "name2:" ...
# -> build/ab/NAME/libmosaic_gpu.so (each from its own copy of csrc: no shared objects)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
rm -rf $ROOT/build/ab
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  W=/tmp/mgpu_var_$name
  rm -rf $W; mkdir -p $W/mosaic_amd $W/include
  cp -r $ROOT/mosaic_amd/csrc $W/mosaic_amd/csrc; cp $ROOT/include/*.h $W/include/
  rm -f $W/mosaic_amd/csrc/*.o
  mkdir -p $ROOT/build/ab/$name
  ( make -s -j8 -C $W/mosaic_amd/csrc KFLAGS="$flags" OUT=$ROOT/build/ab/$name/libmosaic_gpu.so $ROOT/build/ab/$name/libmosaic_gpu.so ) &
done
wait
ls -la $ROOT/build/ab/*/libmosaic_gpu.so
