#!/bin/bash
# HBM traffic of the split pipeline's kernels (rocprofv3 FETCH_SIZE / WRITE_SIZE, one
# counter per pass), on the workload and on its pure-stream ablation (MGPU_ABLATE=11:
# no pixel loads -- a 16 B read + 2 B write stream of known size that calibrates the
# counters for this access pattern): tools/gpu_traffic2.sh TAG [CONFIG]
set -o pipefail
TAG=${1:-t}
CFG=${2:-c2}
OUT=gpurun_out/traffic_$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for ab in 0 11; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/${c}_$ab -o run -- python3 -u tools/join_once.py --config $CFG --ablate $ab > $OUT/${c}_$ab.log 2>&1 || { echo "pass $c $ab failed"; tail -3 $OUT/${c}_$ab.log; exit 1; }
  done
done
echo done
