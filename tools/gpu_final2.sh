#!/bin/bash
# End-of-round record: the -m gpu suite, then bench lines of C2-C5 and kernel traces (gpu_round2.sh a)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_final2.log 2>&1 || { echo "gpu suite failed"; tail -30 gpurun_out/pytest_gpu_final2.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_final2.log
bash tools/gpu_round2.sh r2g a
