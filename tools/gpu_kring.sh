#!/bin/bash
# GPU parity tests, then the device kRing / kLoop and string-id throughput.
set -o pipefail
TAG=${1:-kr}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 200 python3 -u tools/kring_bench.py > gpurun_out/kring_$TAG.json 2> gpurun_out/kring_$TAG.err &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kring_prof_$TAG -o run -- python3 -u tools/kring_bench.py > gpurun_out/kring_prof_$TAG.json 2> gpurun_out/kring_prof_$TAG.err
rc=$?
cat gpurun_out/kring_$TAG.json
exit $rc
