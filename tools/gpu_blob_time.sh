#!/bin/bash
# C3 chip-table upload phases on the box (a -DMGPU_BLOB_TIMING build in build/timing/timing),
# after the upload-path GPU tests.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "blob_roundtrip or c3_full_table or nyc" > gpurun_out/pytest_blob.log 2>&1 || { tail -30 gpurun_out/pytest_blob.log; exit 1; }
tail -3 gpurun_out/pytest_blob.log
MOSAIC_AMD_LIB=$PWD/build/timing/timing/libmosaic_gpu.so timeout -k 10 300 python3 -u tools/blob_time.py c3 --upload > gpurun_out/blob_c3b.out 2> gpurun_out/blob_c3b.err || { tail -20 gpurun_out/blob_c3b.err; exit 1; }
cat gpurun_out/blob_c3b.out; grep blob gpurun_out/blob_c3b.err
