#!/bin/bash
# Host-wait A/B of the C2 bench step (MGPU_SPIN=1 spin on hipStreamQuery vs 0 blocking
# synchronize), interleaved, then the 2-rank rehearsal of bench.py
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for sp in 1 0; do
    MGPU_SPIN=$sp timeout -k 10 300 python3 -u bench.py --config c2 --no-cpu-baseline --no-pcie --steps 20 > gpurun_out/spin_${sp}_$rep.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/spin_${sp}_$rep.json'));print('spin $sp rep $rep: %.4f ms/step, pipeline %.4f ms, %.4g points/s'%(d['ms_per_step'],d['roofline']['pipeline_ms'],d['value']))"
  done
done
bash tools/gpu_dist_rehearsal.sh c2 | cut -c1-300 && bash tools/gpu_dist_rehearsal.sh c3 | cut -c1-300
