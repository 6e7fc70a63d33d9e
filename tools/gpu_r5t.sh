#!/bin/bash
# Round-5 final build, part 1: the GPU suite, smoke(), then the C2 / C5 final lines with
# kernel traces (tools/gpu_final_r5.sh).
set -o pipefail
bash tools/gpu_tests.sh r5t || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r5t.log 2>&1 || { tail -20 gpurun_out/smoke_r5t.log; exit 1; }
tail -1 gpurun_out/smoke_r5t.log
bash tools/gpu_final_r5.sh f5t "c2 c5"
