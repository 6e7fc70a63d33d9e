#!/bin/bash
# Quick check after a kernel change: the join tests, then auto-pipeline timings of C2, C5, C3
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pip_join or binned or split or pixel" > gpurun_out/pytest_quick.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_quick.log; exit 1; }
tail -1 gpurun_out/pytest_quick.log
for c in ${1:-c2,c5}; do :; done
for c in ${1//,/ }; do
  timeout -k 10 300 python3 -u tools/bin_ab.py --config $c --variants auto > gpurun_out/quick_$c.json 2> gpurun_out/quick_$c.err || exit 1
  cat gpurun_out/quick_$c.json
done
