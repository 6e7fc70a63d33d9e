#!/bin/bash
# Round-5 final C3 / C2 lines after the builder's huge-page arrays (setup time), with the
# upload-path tests first (device blob byte-equal to the host blob).
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "blob_roundtrip or c3_full_table" > gpurun_out/pytest_r5y.log 2>&1 || { tail -30 gpurun_out/pytest_r5y.log; exit 1; }
tail -1 gpurun_out/pytest_r5y.log
bash tools/gpu_final_r5.sh f5y "c3 c2"
