#!/bin/bash
# Last check of the round: the -m gpu suite, smoke(), the C3 2-rank rehearsal
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_last.log 2>&1 || { echo "gpu suite failed"; tail -30 gpurun_out/pytest_gpu_last.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_last.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_last.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/smoke_last.log; exit 1; }
tail -1 gpurun_out/smoke_last.log | cut -c1-200
bash tools/gpu_dist_rehearsal.sh c3 | cut -c1-400
