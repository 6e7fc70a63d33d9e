#!/bin/bash
# C4 at BASELINE size (500M points): fused vs the BNG pixel-index split pipeline, res 3
# and 4, then FETCH / WRITE / SQ counters of the fused join kernel at res 3 and 4.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for res in 3 4; do
  for opt in "raster_bng=0" "raster_bng=1"; do
    tag=c4_500m_r${res}_${opt/=/}
    timeout -k 10 400 python3 -u bench.py --config c4 --points 500000000 --res $res --steps 5 --warmup 2 --no-cpu-baseline --no-pcie --option $opt > gpurun_out/$tag.json 2> gpurun_out/$tag.err || { echo "bench $tag failed"; tail -5 gpurun_out/$tag.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/$tag.json'));print('$tag', d['pipeline'], '%.3e'%d['value'], '%.3f ms'%d['ms_per_step'], d['kernels_ms'])"
  done
done
for res in 3 4; do
  bash tools/gpu_pmc3.sh c4r$res "--config c4 --res $res" "2 4 5" > gpurun_out/pmc_c4r$res.txt 2>&1 || { echo "pmc c4 r$res failed"; tail -5 gpurun_out/pmc_c4r$res.txt; exit 1; }
  grep -A 3 "pip_join_kernel<1>" gpurun_out/pmc_c4r$res.txt | head -4
done
