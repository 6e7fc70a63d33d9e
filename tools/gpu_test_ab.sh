#!/bin/bash
# GPU parity tests on the working tree, then the interleaved A/B of build/variants/*.
set -o pipefail
TAG=${1:-ab}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
bash tools/gpu_ab2.sh $TAG
