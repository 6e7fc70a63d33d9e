#!/bin/bash
# Round-5 counters of the final build, part 1 (tools/gpu_pmc_r5.sh): C2, C5, C4 res 4.
set -o pipefail
bash tools/gpu_pmc_r5.sh r5 "c2 c5 c4"
