#!/bin/bash
# Round-end measurements: 2-rank C3 protocol rehearsal, the default bench line (C2, CPU
# baseline), its rocprofv3 kernel-trace stats, and the other configs' bench lines.
set -o pipefail
TAG=${1:-fin}
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_dist_rehearsal.sh c3 &&
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 -u bench.py --no-cpu-baseline > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/bench_prof_$TAG.err &&
for c in c3 c4 c5; do
  timeout -k 10 400 python -u bench.py --config $c > gpurun_out/bench_${c}_$TAG.json 2> gpurun_out/bench_${c}_$TAG.err || exit 1
done
rc=$?
cat gpurun_out/bench_$TAG.json
echo "exit $rc"
exit $rc
