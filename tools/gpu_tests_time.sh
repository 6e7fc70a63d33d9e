#!/bin/bash
# The -m gpu suite, then join timings of the working tree on CONFIGS (tools/ab_time.py):
#   tools/gpu_tests_time.sh TAG [CONFIGS]   -> gpurun_out/pytest_gpu_TAG.log, time_TAG.json
set -o pipefail
TAG=${1:-t}; CFGS=${2:-c2,c5,c4}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "gpu suite failed"; tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 400 python3 -u tools/ab_time.py --configs $CFGS > gpurun_out/time_$TAG.json 2> gpurun_out/time_$TAG.err || { echo "timing failed"; tail -5 gpurun_out/time_$TAG.err; exit 1; }
cat gpurun_out/time_$TAG.json
