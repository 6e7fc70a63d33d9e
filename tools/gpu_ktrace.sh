#!/bin/bash
# Kernel-trace stats of tools/join_once.py for each build/variants/* library.
set -o pipefail
TAG=${1:-kt}
export TMPDIR=/tmp
for d in build/variants/*/; do
  n=$(basename $d)
  MOSAIC_AMD_LIB=$PWD/$d/libmosaic_gpu.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_${TAG}_$n -o run -- python3 -u tools/join_once.py --reps 5 > gpurun_out/kt_${TAG}_$n.log 2>&1 || { echo "variant $n failed"; tail -3 gpurun_out/kt_${TAG}_$n.log; exit 1; }
  echo "== $n"; grep mgpu gpurun_out/kt_${TAG}_$n/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-120
done
