#!/bin/bash
# C4 at BASELINE size (500M points), res 3 and 4, auto pipeline: gpurun_out/c4_500m_r{3,4}_TAG.json
set -o pipefail
TAG=${1:-a}
mkdir -p gpurun_out
export TMPDIR=/tmp
for res in 3 4; do
  tag=c4_500m_r${res}_$TAG
  timeout -k 10 400 python3 -u bench.py --config c4 --points 500000000 --res $res --steps 5 --warmup 2 --no-cpu-baseline --no-pcie > gpurun_out/$tag.json 2> gpurun_out/$tag.err || { echo "bench $tag failed"; tail -5 gpurun_out/$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/$tag.json'));print('$tag', d['pipeline'], '%.3e'%d['value'], '%.3f ms'%d['ms_per_step'], d['kernels_ms'], d['roofline']['frac'])"
done
