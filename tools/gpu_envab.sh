#!/bin/bash
# GPU parity tests, then join timings (tools/ab_time.py) with an environment switch off/on:
# tools/gpu_envab.sh TAG VAR CONFIGS
set -o pipefail
TAG=${1:-env}; VAR=$2; CFGS=${3:-c2,c5}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
for v in 0 1 0 1; do
  env $VAR=$v timeout -k 10 300 python3 -u tools/ab_time.py --configs $CFGS --reps 7 > gpurun_out/env_${TAG}_$v.json 2> gpurun_out/env_${TAG}_$v.err || { tail -5 gpurun_out/env_${TAG}_$v.err; exit 1; }
  sed "s/^/$VAR=$v /" gpurun_out/env_${TAG}_$v.json | cut -c1-160
done
