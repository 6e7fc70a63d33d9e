#!/bin/bash
# Round-5 upload + emit-block check: upload-path GPU tests, C3 upload phases
# (tools/gpu_blob_time.sh), then the split A/B of build/ab/* on C2 / C5.
set -o pipefail
bash tools/gpu_blob_time.sh && bash tools/gpu_ab_split.sh cls c2,c5
