#!/bin/bash
# One check of the current tree on the box: the -m gpu suite, smoke(), the default bench line.
# Outputs: gpurun_out/pytest_gpu_TAG.log, smoke_TAG.log, bench_TAG.json
set -o pipefail
TAG=${1:-t}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "gpu suite failed"; tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log | cut -c1-200
timeout -k 10 300 python3 -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -5 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-600 gpurun_out/bench_$TAG.json
