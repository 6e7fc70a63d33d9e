#!/bin/bash
# The binned pipeline on the box: its GPU tests, then binned-vs-fused timings on C3 (and
# the other configs given): tools/gpu_binned.sh TAG [CONFIGS] [all]
set -o pipefail
TAG=${1:-t}
CFGS=${2:-c3}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_binned.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_binned_$TAG.log 2>&1 || { echo "binned tests failed"; tail -40 gpurun_out/pytest_binned_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_binned_$TAG.log
if [ "$3" == "all" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "gpu suite failed"; tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu_$TAG.log
fi
for c in ${CFGS//,/ }; do
  timeout -k 10 400 python3 -u tools/bin_ab.py --config $c > gpurun_out/binab_${TAG}_$c.json 2> gpurun_out/binab_${TAG}_$c.err || { echo "bin_ab $c failed"; tail -5 gpurun_out/binab_${TAG}_$c.err; exit 1; }
  cat gpurun_out/binab_${TAG}_$c.json
done
