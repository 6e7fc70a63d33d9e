#!/bin/bash
# round 5: interleaved A/B of build/ab/* on C2 / C5, then the default bench line (C2) and C3
set -o pipefail
TAG=${1:-r5e}
mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_tests.sh ${TAG} "binned or ring_join or negative or override" || exit 1
for rep in 1 2; do for d in build/ab/*/; do v=$(basename $d)
  MOSAIC_AMD_LIB=$PWD/$d/libmosaic_gpu.so timeout -k 10 300 python3 -u tools/ab_time.py --configs c2,c5 > gpurun_out/ab_${TAG}_${v}_$rep.json 2> gpurun_out/ab_${TAG}_${v}_$rep.err || { echo "ab $v failed"; tail -5 gpurun_out/ab_${TAG}_${v}_$rep.err; exit 1; }
  sed "s/^/$v $rep /" gpurun_out/ab_${TAG}_${v}_$rep.json
done; done
timeout -k 10 300 python3 -u bench.py > gpurun_out/bench_${TAG}_c2.json 2> gpurun_out/bench_${TAG}_c2.err || { echo "bench c2 failed"; tail -5 gpurun_out/bench_${TAG}_c2.err; exit 1; }
cat gpurun_out/bench_${TAG}_c2.json
timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu-baseline --no-pcie > gpurun_out/bench_${TAG}_c3.json 2> gpurun_out/bench_${TAG}_c3.err || { echo "bench c3 failed"; tail -5 gpurun_out/bench_${TAG}_c3.err; exit 1; }
cat gpurun_out/bench_${TAG}_c3.json
