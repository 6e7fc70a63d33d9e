#!/bin/bash
# One GPU iteration: parity suite, then join timings with the pixel index off / on
# (tools/ab_time.py), each step under its own limit: tools/gpu_check.sh TAG [CONFIGS]
set -o pipefail
TAG=${1:-x}
CFGS=${2:-c2,c4,c5}
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu_$TAG.log | head -20; exit $rc; }
fi
rc=0
for v in ${VARIANTS:-"norast:MGPU_RASTER=0" "fused:MGPU_SPLIT=0" "split:MGPU_SPLIT=1"}; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 300 python3 -u tools/ab_time.py --configs $CFGS > gpurun_out/ab_${TAG}_$name.json 2> gpurun_out/ab_${TAG}_$name.err || { rc=$?; tail -5 gpurun_out/ab_${TAG}_$name.err; break; }
  echo "== $name ($envs)"; cat gpurun_out/ab_${TAG}_$name.json
done
exit $rc
