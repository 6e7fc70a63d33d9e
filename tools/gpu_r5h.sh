#!/bin/bash
# Round-5 check of the final build: the GPU suite, smoke(), then the C2 / C5 final lines
# and their kernel traces (tools/gpu_final_r5.sh).
set -o pipefail
bash tools/gpu_tests.sh r5h || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r5h.log 2>&1 || { tail -20 gpurun_out/smoke_r5h.log; exit 1; }
tail -1 gpurun_out/smoke_r5h.log
bash tools/gpu_final_r5.sh f5a "c2 c5"
