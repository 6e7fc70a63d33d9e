#!/bin/bash
# Parity tests, then the HBM traffic passes of one config's join (tools/gpu_traffic.sh).
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-tt}
CFG=${2:-c2}
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 &&
bash tools/gpu_traffic.sh $TAG $CFG
rc=$?
tail -3 gpurun_out/pytest_gpu_$TAG.log
echo "exit $rc"
exit $rc
