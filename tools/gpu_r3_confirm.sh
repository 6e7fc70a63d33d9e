#!/bin/bash
# Confirmation run: the -m gpu suite, then bench lines of the given configs: tools/gpu_r3_confirm.sh TAG CONFIGS...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "gpu suite failed"; tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
for c in "$@"; do
  timeout -k 10 400 python3 -u bench.py --config $c > gpurun_out/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.err || { echo "bench $c failed"; tail -5 gpurun_out/${TAG}_bench_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_$c.json'));print('$c', '%.3e'%d['value'], '%.3f'%d['ms_per_step'], d['kernels_ms'], d['roofline']['frac'])"
done
