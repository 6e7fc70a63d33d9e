#!/bin/bash
# Bench lines + kernel-trace profile: tools/gpu_bench.sh TAG [CONFIGS]
set -o pipefail
TAG=${1:-b}
CFGS=${2:-c2}
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in $CFGS; do
  timeout -k 10 400 python3 -u bench.py --config $c --steps 10 --warmup 3 > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err || { echo "bench $c failed"; tail -5 gpurun_out/bench_${TAG}_$c.err; exit 1; }
  cat gpurun_out/bench_${TAG}_$c.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_$TAG -o run -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/kt_$TAG.log 2>&1 || { echo "ktrace failed"; tail -5 gpurun_out/kt_$TAG.log; exit 1; }
grep -E "mgpu" gpurun_out/kt_$TAG/run_kernel_stats.csv | cut -d, -f1-8 | cut -c1-160
