#!/bin/bash
# Round 4 driver: the -m gpu suite, the C2 bench line, then the interleaved A/B of
# build/variants/* on the configs given: tools/gpu_r4.sh TAG [CONFIGS] [tests|notests]
set -o pipefail
TAG=${1:-r4}; CFGS=${2:-c2}; T=${3:-tests}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "$T" = tests ]; then
  bash tools/gpu_tests.sh $TAG || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
fi
timeout -k 10 300 python3 -u bench.py --config c2 --no-cpu-baseline --no-pcie > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err || { tail -5 gpurun_out/${TAG}_c2.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_c2.json'));print('c2', '%.3e'%d['value'], '%.3f'%d['ms_per_step'], d['kernels_ms'], d['roofline']['frac'])"
if [ -d build/variants ]; then bash tools/gpu_ab_split.sh $TAG $CFGS; fi
