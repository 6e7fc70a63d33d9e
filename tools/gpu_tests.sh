#!/bin/bash
# The GPU parity suite (or the tests matching $2) on the box: gpurun_out/pytest_gpu_TAG.log.
set -o pipefail
TAG=${1:-t}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$2" ]; then SEL=(-k "$2"); else SEL=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread "${SEL[@]}" > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu_$TAG.log
exit $rc
