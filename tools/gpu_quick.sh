#!/bin/bash
# GPU parity tests + time breakdown (fast iteration loop).
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-q}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 &&
timeout -k 10 300 python3 -u tools/breakdown.py > gpurun_out/breakdown_$TAG.json 2> gpurun_out/breakdown_$TAG.err
rc=$?
tail -3 gpurun_out/pytest_gpu_$TAG.log
cat gpurun_out/breakdown_$TAG.json
echo "exit $rc"
exit $rc
