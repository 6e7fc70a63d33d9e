#!/bin/bash
# GPU parity tests of the working tree, then interleaved join timings of build/variants/*.
set -o pipefail
TAG=${1:-tab}; CFGS=${2:-c2,c5}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
bash tools/gpu_ab_split.sh $TAG $CFGS
