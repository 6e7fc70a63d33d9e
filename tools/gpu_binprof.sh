#!/bin/bash
# Kernel-trace stats of the binned pipeline on C3 (tools/bin_ab.py, one variant):
# tools/gpu_binprof.sh TAG [VARIANT] [CONFIG]
set -o pipefail
TAG=${1:-t}
V=${2:-bin256}
CFG=${3:-c3}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/binprof_$TAG -o run -- python3 -u tools/bin_ab.py --config $CFG --variants $V --reps 3 > gpurun_out/binprof_$TAG.log 2>&1 || { echo "profile failed"; tail -5 gpurun_out/binprof_$TAG.log; exit 1; }
f=$(find gpurun_out/binprof_$TAG -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 "$f" | grep -v "at::native" | head -20
