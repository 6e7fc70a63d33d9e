#!/bin/bash
# Round-5 binned output A/B: the join counts each input chunk's pairs and the emit gathers
# the answers itself (base, MGPU_BIN_JOIN_COUNTS) vs gather + scan + emit (prev); the
# binned / override / capacity GPU tests on base first.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
MOSAIC_AMD_LIB=$PWD/build/ab/base/libmosaic_gpu.so timeout -k 10 900 python3 -u -m pytest tests/test_gpu_binned.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "binned or override or capacity or fetch or c3" > gpurun_out/pytest_bincount.log 2>&1 || { tail -30 gpurun_out/pytest_bincount.log; exit 1; }
tail -2 gpurun_out/pytest_bincount.log
run() {
  MOSAIC_AMD_LIB=$PWD/build/ab/$1/libmosaic_gpu.so timeout -k 10 300 python3 -u tools/ab_time.py --configs c3 --points 125000000 --reps 5 > gpurun_out/bc_$2_$1.json 2> gpurun_out/bc_$2_$1.err || { echo "variant $1 failed"; tail -5 gpurun_out/bc_$2_$1.err; exit 1; }
  sed "s/^/$1 $2 /" gpurun_out/bc_$2_$1.json
}
for rep in 1 2; do for v in prev base; do run $v b$rep || exit 1; done; done
