#!/bin/bash
# rocprofv3 kernel-trace stats of the default bench command, then the HBM traffic passes.
set -o pipefail
TAG=${1:-p}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 -u bench.py --no-cpu-baseline > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/bench_prof_$TAG.err &&
bash tools/gpu_traffic.sh $TAG
rc=$?
grep mgpu gpurun_out/prof_$TAG/run_kernel_stats.csv | cut -c1-160
cat gpurun_out/bench_prof_$TAG.json | cut -c1-300
exit $rc
