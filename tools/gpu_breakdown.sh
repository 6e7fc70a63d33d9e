#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-b}
for c in ${CONFIGS:-c2 c4 c5}; do
  timeout -k 10 300 python3 -u tools/breakdown.py --config $c > gpurun_out/breakdown_${c}_$TAG.json 2> gpurun_out/breakdown_${c}_$TAG.err || exit 1
  cat gpurun_out/breakdown_${c}_$TAG.json
done
