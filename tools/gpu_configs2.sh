#!/bin/bash
# SQ/cache counter passes on the C2 join (all split-pipeline kernels), then the C3/C4/C5
# bench lines and C3's kernel-trace stats.  Each GPU step has its own limit.
set -o pipefail
TAG=${1:-r2c}
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_pmc2.sh ${TAG}_c2 "--config c2" &&
for c in c3 c4 c5; do
  timeout -k 10 400 python -u bench.py --config $c > gpurun_out/bench_${c}_$TAG.json 2> gpurun_out/bench_${c}_$TAG.err || exit 1
done &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3_$TAG -o run -- python3 -u bench.py --config c3 --no-cpu-baseline --steps 5 > gpurun_out/bench_prof_c3_$TAG.json 2> gpurun_out/bench_prof_c3_$TAG.err
rc=$?
cat gpurun_out/bench_c*_$TAG.json
echo "exit $rc"
exit $rc
