#!/bin/bash
# Parity tests, then the bench on each BASELINE config (c2 default, c4 BNG, c5 skewed).
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r1}
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c2 > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err &&
timeout -k 10 300 python -u bench.py --config c4 > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err &&
timeout -k 10 300 python -u bench.py --config c5 > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err
rc=$?
tail -3 gpurun_out/pytest_gpu_$TAG.log
cat gpurun_out/bench_c*_$TAG.json
echo "exit $rc"
exit $rc
