#!/bin/bash
# Round-3 measurement record on one MI355X: bench lines of C2-C5 (with CPU baseline and the
# PCIe-inclusive rate), kernel-trace stats of the C2, C3 and C4 bench runs, and C4 at BASELINE's
# 500M points (res 3 and 4): tools/gpu_round2.sh TAG [part]
set -o pipefail
TAG=${1:-r3f}
PART=${2:-a}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "$PART" == "a" ]; then
  for c in c2 c3 c4 c5; do
    timeout -k 10 400 python3 -u bench.py --config $c > gpurun_out/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.err || { echo "bench $c failed"; tail -5 gpurun_out/${TAG}_bench_$c.err; exit 1; }
    cat gpurun_out/${TAG}_bench_$c.json
  done
  for c in c2 c3 c4; do
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_$c -o run -- python3 -u bench.py --config $c --no-cpu-baseline --no-pcie --steps 10 > gpurun_out/${TAG}_kt_$c.json 2> gpurun_out/${TAG}_kt_$c.err || { echo "ktrace $c failed"; exit 1; }
    cut -d, -f1-4 gpurun_out/${TAG}_kt_$c/run_kernel_stats.csv | grep -v "at::native" | head -12
  done
else
  for r in 3 4; do
    timeout -k 10 500 python3 -u bench.py --config c4 --points 500000000 --res $r --steps 5 --warmup 2 > gpurun_out/${TAG}_bench_c4_500m_r$r.json 2> gpurun_out/${TAG}_bench_c4_500m_r$r.err || { echo "bench c4 500m r$r failed"; tail -5 gpurun_out/${TAG}_bench_c4_500m_r$r.err; exit 1; }
    cat gpurun_out/${TAG}_bench_c4_500m_r$r.json
  done
fi
