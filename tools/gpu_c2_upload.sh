#!/bin/bash
# C2 chip-table upload on the box: builder phases (a -DMGPU_BLOB_TIMING build in
# build/ab/timing), then the C2 bench line with the product library.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
MOSAIC_AMD_LIB=$PWD/build/ab/timing/libmosaic_gpu.so timeout -k 10 300 python3 -u tools/blob_time.py c2 --upload > gpurun_out/blob_c2.out 2> gpurun_out/blob_c2.err || { tail -20 gpurun_out/blob_c2.err; exit 1; }
cat gpurun_out/blob_c2.out; grep -E "blob\]|raster\]" gpurun_out/blob_c2.err
timeout -k 10 600 python3 -u bench.py --config c2 --no-cpu-baseline --no-pcie > gpurun_out/c2_upl.json 2> gpurun_out/c2_upl.err || { tail -5 gpurun_out/c2_upl.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/c2_upl.json'));print('c2', d['ms_per_step'], d['setup_s']['upload_s'])"
