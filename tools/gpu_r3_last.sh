#!/bin/bash
# End of round 3: the -m gpu suite, the NT-store A/B (build/variants), bench lines of C2-C5
# and the C2 kernel trace with the tree's library: tools/gpu_r3_last.sh TAG
set -o pipefail
TAG=${1:-r3g}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "gpu suite failed"; tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
bash tools/gpu_ab_split.sh ntc c3,c4,c2 || exit 1
for c in c2 c3 c4 c5; do
  timeout -k 10 400 python3 -u bench.py --config $c > gpurun_out/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.err || { echo "bench $c failed"; tail -5 gpurun_out/${TAG}_bench_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_$c.json'));print('$c', '%.3e'%d['value'], '%.3f'%d['ms_per_step'], d['kernels_ms'], d['roofline']['frac'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_c2 -o run -- python3 -u bench.py --config c2 --no-cpu-baseline --no-pcie --steps 10 > gpurun_out/${TAG}_kt_c2.json 2> gpurun_out/${TAG}_kt_c2.err || { echo "ktrace failed"; exit 1; }
cut -d, -f1-4 gpurun_out/${TAG}_kt_c2/run_kernel_stats.csv | grep -v "at::native" | head -8
