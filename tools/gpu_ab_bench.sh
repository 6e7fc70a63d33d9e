#!/bin/bash
# GPU parity tests on the working tree, then interleaved bench runs of build/variants/*
# (MOSAIC_AMD_LIB) on the configs given (default: c2 c5 c3), no CPU baseline.
set -o pipefail
TAG=${1:-abb}; shift
CFGS=${@:-c2 c5 c3}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
for c in $CFGS; do
  for d in build/variants/*/; do
    n=$(basename $d)
    MOSAIC_AMD_LIB=$PWD/$d/libmosaic_gpu.so timeout -k 10 300 python3 -u bench.py --config $c --no-cpu-baseline > gpurun_out/abb_${TAG}_${c}_${n}.json 2> gpurun_out/abb_${TAG}_${c}_${n}.err || { echo "variant $n $c failed"; tail -5 gpurun_out/abb_${TAG}_${c}_${n}.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], sys.argv[3], '%.4g pts/s  step %.3f ms  join %.3f ms  pipeline %.3f ms' % (d['value'], d['ms_per_step'], r['kernel_ms'], r['pipeline_ms']), d['pairs_per_gpu'])" gpurun_out/abb_${TAG}_${c}_${n}.json $c $n
  done
done
