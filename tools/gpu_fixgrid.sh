#!/bin/bash
# C4 at 500M points res 3 (candidate-heavy) and the fused / split joins of C2, C4, C5 (regression check)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python3 -u bench.py --config c4 --points 500000000 --res 3 --steps 5 --warmup 2 --no-cpu-baseline --no-pcie > gpurun_out/fix_c4r3.json 2> gpurun_out/fix_c4r3.err || exit 1
python3 -c "
import json;d=json.load(open('gpurun_out/fix_c4r3.json'));print(d['value'],d['ms_per_step'],d['kernels_ms'])"
for c in c2 c4 c5; do
  timeout -k 10 300 python3 -u tools/bin_ab.py --config $c --variants auto,fused > gpurun_out/fix_$c.json 2>gpurun_out/fix_$c.err || exit 1
  cat gpurun_out/fix_$c.json
done
