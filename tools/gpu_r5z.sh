#!/bin/bash
# Round-5 closing check of the final build: the GPU suite, smoke(), then the C3 upload's
# phases on the box (a -DMGPU_BLOB_TIMING build of the same sources in build/timing).
set -o pipefail
bash tools/gpu_tests.sh r5z || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r5z.log 2>&1 || { tail -20 gpurun_out/smoke_r5z.log; exit 1; }
tail -1 gpurun_out/smoke_r5z.log
MOSAIC_AMD_LIB=$PWD/build/timing/timing/libmosaic_gpu.so timeout -k 10 300 python3 -u tools/blob_time.py c3 --upload > gpurun_out/blob_c3z.out 2> gpurun_out/blob_c3z.err || { tail -20 gpurun_out/blob_c3z.err; exit 1; }
cat gpurun_out/blob_c3z.out; grep blob gpurun_out/blob_c3z.err | tail -12
