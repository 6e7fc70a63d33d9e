#!/bin/bash
# Kernel-trace stats of bench.py on C2, C3, C4 and the C4 res-3 500M line (current tree lib):
# tools/gpu_bench_r4.sh TAG
set -o pipefail
TAG=${1:-b4}
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_ktrace_cfg.sh $TAG c2 c3 c4 || exit 1
timeout -k 10 400 python3 -u bench.py --config c4 --res 3 --points 500000000 --no-cpu-baseline --no-pcie --steps 5 > gpurun_out/${TAG}_c4r3.json 2> gpurun_out/${TAG}_c4r3.err || { tail -5 gpurun_out/${TAG}_c4r3.err; exit 1; }
for f in gpurun_out/kt_${TAG}_c2.json gpurun_out/kt_${TAG}_c3.json gpurun_out/kt_${TAG}_c4.json gpurun_out/${TAG}_c4r3.json; do
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], '%.3e'%d['value'], '%.3f'%d['ms_per_step'], d.get('kernels_ms'), d['roofline'].get('frac'), d.get('setup_s'))" $f
done
