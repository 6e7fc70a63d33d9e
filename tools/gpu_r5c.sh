#!/bin/bash
# round 5: the GPU suite, an interleaved A/B of build/ab/{base,pair,wave,both} on C2 / C5,
# per-phase stamps of C3 (build/ab/stamps)
set -o pipefail
TAG=${1:-r5c}
mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_tests.sh $TAG || exit 1
for rep in 1 2; do for v in base pair wave both; do
  MOSAIC_AMD_LIB=$PWD/build/ab/$v/libmosaic_gpu.so timeout -k 10 300 python3 -u tools/ab_time.py --configs c2,c5 > gpurun_out/ab_${TAG}_${v}_$rep.json 2> gpurun_out/ab_${TAG}_${v}_$rep.err || { echo "ab $v failed"; tail -5 gpurun_out/ab_${TAG}_${v}_$rep.err; exit 1; }
  sed "s/^/$v $rep /" gpurun_out/ab_${TAG}_${v}_$rep.json
done; done
bash tools/gpu_stamps.sh $TAG c3
