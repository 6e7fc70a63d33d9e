#!/bin/bash
# Round-5 final lines: bench.py per config (CPU baseline and PCIe-inclusive included) and a
# rocprofv3 kernel trace of the same bench command: gpurun_out/final_TAG_<cfg>.json, kt_TAG_<cfg>/
set -o pipefail
TAG=${1:-f5}; CFGS=${2:-"c2 c3 c4 c5"}
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in $CFGS; do
  timeout -k 10 600 python3 -u bench.py --config $c > gpurun_out/final_${TAG}_$c.json 2> gpurun_out/final_${TAG}_$c.err || { echo "bench $c failed"; tail -5 gpurun_out/final_${TAG}_$c.err; exit 1; }
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_${TAG}_$c -o run -- python3 -u bench.py --config $c --no-cpu-baseline --no-pcie > gpurun_out/kt_${TAG}_$c.json 2> gpurun_out/kt_${TAG}_$c.err || { echo "trace $c failed"; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], '%.3e'%d['value'], '%.3f ms'%d['ms_per_step'], d.get('kernels_ms'), 'frac %.3f'%d['roofline']['frac'], 'cpu', (d.get('cpu_baseline') or {}).get('value'))" gpurun_out/final_${TAG}_$c.json $c
done
