#!/bin/bash
# Round-5 counters of the final build, part 2 (tools/gpu_pmc_r5.sh): C3, C4 res 3.
set -o pipefail
bash tools/gpu_pmc_r5.sh r5 "c3 c4:3"
