#!/bin/bash
# Round-5 final bench lines on the final build, part 1, after its counters are in profiles/
# (each line attaches its keyed traffic and VALU profile): C2, C5, C4 with kernel traces.
set -o pipefail
bash tools/gpu_final_r5.sh f5w "c2 c5 c4"
