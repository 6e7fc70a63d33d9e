#!/bin/bash
# Interleaved join timings (tools/ab_time.py) of build/ab/* on the configs given.
set -o pipefail
TAG=${1:-abs}; shift
CFGS=${1:-c2,c5}; shift; EXTRA="$@"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for d in build/ab/*/; do
    n=$(basename $d)
    MOSAIC_AMD_LIB=$PWD/$d/libmosaic_gpu.so timeout -k 10 300 python3 -u tools/ab_time.py --configs $CFGS $EXTRA > gpurun_out/abs_${TAG}_${n}_$rep.json 2> gpurun_out/abs_${TAG}_${n}_$rep.err || { echo "variant $n failed"; tail -5 gpurun_out/abs_${TAG}_${n}_$rep.err; exit 1; }
    sed "s/^/$n $rep /" gpurun_out/abs_${TAG}_${n}_$rep.json
  done
done
