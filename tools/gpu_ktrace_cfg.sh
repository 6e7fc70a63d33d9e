#!/bin/bash
# rocprofv3 kernel-trace stats of bench.py on the given configs (default c2), current tree lib
set -o pipefail
TAG=${1:-kt}; shift
CFGS=${@:-c2}
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in $CFGS; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_${TAG}_$c -o run -- python3 -u bench.py --config $c --no-cpu-baseline --steps 5 > gpurun_out/kt_${TAG}_$c.json 2> gpurun_out/kt_${TAG}_$c.err || exit 1
  echo "== $c"; cut -d, -f1-4 gpurun_out/kt_${TAG}_$c/run_kernel_stats.csv | grep -v "at::native" | head -8
done
