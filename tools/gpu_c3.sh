#!/bin/bash
# Parity tests, then the C3 bench (74k tracts, res 10, 1.25e8 points) and its kernel trace.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-c3}
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 &&
timeout -k 10 500 python -u bench.py --config c3 > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3_$TAG -o run -- python3 -u bench.py --config c3 --no-cpu-baseline --steps 5 > gpurun_out/bench_c3_prof_$TAG.json 2> gpurun_out/bench_c3_prof_$TAG.err
rc=$?
tail -3 gpurun_out/pytest_gpu_$TAG.log
cat gpurun_out/bench_c3_$TAG.json
echo "exit $rc"
exit $rc
