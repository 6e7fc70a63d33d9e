#!/bin/bash
# One GPU-box session: parity tests, bench, rocprof kernel stats of the bench command,
# HBM traffic passes.  Each GPU step has its own time limit; steps are chained with &&.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r1}
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 -u bench.py --no-cpu-baseline > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/bench_prof_$TAG.err &&
bash tools/gpu_traffic.sh $TAG
rc=$?
tail -2 gpurun_out/pytest_gpu_$TAG.log
cat gpurun_out/bench_$TAG.json
echo "exit $rc"
exit $rc
