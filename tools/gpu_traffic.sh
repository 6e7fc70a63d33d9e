#!/bin/bash
# HBM traffic of pip_join_kernel from rocprofv3 FETCH_SIZE / WRITE_SIZE (separate passes),
# calibrated on the BNG cells kernel (a pure stream of known bytes with the same 8-byte
# per-lane accesses): writes gpurun_out/traffic_TAG/*.  Each pass has its own limit.
set -o pipefail
TAG=${1:-t}
CFG=${2:-c2}
RES=${3:+--res $3}   # (optional: a resolution other than the config's default)
OUT=gpurun_out/traffic_$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/join_fetch -o run -- python3 -u tools/join_once.py --config $CFG $RES --cache /tmp/mgpu_cache_$CFG$3.npz > $OUT/join_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/join_write -o run -- python3 -u tools/join_once.py --config $CFG $RES --cache /tmp/mgpu_cache_$CFG$3.npz > $OUT/join_write.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/bng_fetch -o run -- python3 -u tools/join_once.py --cells --bng > $OUT/bng_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/bng_write -o run -- python3 -u tools/join_once.py --cells --bng > $OUT/bng_write.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
