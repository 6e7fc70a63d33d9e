#!/bin/bash
# C3 join A/B of library variants build/ab/* (interleaved, two repetitions): ms per
# 1.25e8 points per pipeline part (tools/ab_time.py), then bench.py C3 options given
#   tools/gpu_c3_vab.sh TAG ["opt=v ..." ...]
set -o pipefail
TAG=${1:-c3v}; shift
mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do for d in build/ab/*/; do v=$(basename $d)
  MOSAIC_AMD_LIB=$PWD/$d/libmosaic_gpu.so timeout -k 10 300 python3 -u tools/ab_time.py --configs c3 --points 125000000 --reps 5 > gpurun_out/ab_${TAG}_${v}_$rep.json 2> gpurun_out/ab_${TAG}_${v}_$rep.err || { echo "ab $v failed"; tail -5 gpurun_out/ab_${TAG}_${v}_$rep.err; exit 1; }
  sed "s/^/$v $rep /" gpurun_out/ab_${TAG}_${v}_$rep.json
done; done
for o in "$@"; do
  OPTS=""; for kv in $o; do OPTS="$OPTS --option $kv"; done
  timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu-baseline --no-pcie $OPTS > gpurun_out/c3o_${TAG}.json 2> gpurun_out/c3o_${TAG}.err || { echo "bench $o failed"; tail -5 gpurun_out/c3o_${TAG}.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], '%.3e'%d['value'], '%.3f ms'%d['ms_per_step'], {k:round(v,3) for k,v in d['kernels_ms'].items()})" gpurun_out/c3o_${TAG}.json "$o"
done
