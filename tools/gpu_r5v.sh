#!/bin/bash
# Round-5 binned output A/B, sixth round: the gathering emit with its LDS answers swizzled (swz) vs not (noswz)
# the binned tests on swz first.

set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
MOSAIC_AMD_LIB=$PWD/build/ab/swz/libmosaic_gpu.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_binned.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_bincount6.log 2>&1 || { tail -30 gpurun_out/pytest_bincount6.log; exit 1; }
tail -1 gpurun_out/pytest_bincount6.log
run() {
  MOSAIC_AMD_LIB=$PWD/build/ab/$1/libmosaic_gpu.so timeout -k 10 300 python3 -u tools/ab_time.py --configs c3 --points 125000000 --reps 5 > gpurun_out/bc6_$2_$1.json 2> gpurun_out/bc6_$2_$1.err || { echo "variant $1 failed"; tail -5 gpurun_out/bc6_$2_$1.err; exit 1; }
  sed "s/^/$1 $2 /" gpurun_out/bc6_$2_$1.json
}
for rep in 1 2; do for v in noswz swz; do run $v b$rep || exit 1; done; done
