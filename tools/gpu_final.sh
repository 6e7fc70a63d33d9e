#!/bin/bash
# Full GPU suite + the C4 res-3 500M bench line (with CPU baseline and PCIe rate)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1 || { echo "gpu suite failed"; tail -40 gpurun_out/pytest_gpu_final.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_final.log
timeout -k 10 500 python3 -u bench.py --config c4 --points 500000000 --res 3 --steps 5 --warmup 2 > gpurun_out/final_c4_500m_r3.json 2> gpurun_out/final_c4_500m_r3.err || exit 1
cut -c1-300 gpurun_out/final_c4_500m_r3.json
