#!/bin/bash
# FETCH_SIZE of pip_join_kernel under each MGPU_ABLATE mode (where the re-fetches come from).
set -o pipefail
TAG=${1:-fa}
OUT=gpurun_out/fetch_$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for ab in 0 1 3 4 5; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/ab$ab -o run -- python3 -u tools/join_once.py --ablate $ab > $OUT/ab$ab.log 2>&1 || { echo "ablate $ab failed"; tail -3 $OUT/ab$ab.log; exit 1; }
done
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/hit -o run -- python3 -u tools/join_once.py > $OUT/hit.log 2>&1
python3 - <<'PY'
import csv, collections, glob, os
d = "gpurun_out/fetch_" + os.environ.get("TAG", "fa")
PY
echo done
