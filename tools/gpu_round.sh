#!/bin/bash
# One GPU-box session: parity tests, bench, rocprof kernel stats.  Each GPU step has
# its own time limit; steps are chained with && so the first failure ends the call.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r1}
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
rc=$?
echo "exit $rc"
exit $rc
