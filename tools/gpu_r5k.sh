#!/bin/bash
# Round-5 A/B: prev (HEAD) vs base (the cell-id path's resolution made opaque, so its
# per-resolution predicates no longer spill across the join loops), interleaved, two passes.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
run() {  # variant configs points tag
  MOSAIC_AMD_LIB=$PWD/build/ab/$1/libmosaic_gpu.so timeout -k 10 300 python3 -u tools/ab_time.py --configs $2 --points $3 --reps 5 > gpurun_out/res_$4_$1.json 2> gpurun_out/res_$4_$1.err || { echo "variant $1 $2 failed"; tail -5 gpurun_out/res_$4_$1.err; exit 1; }
  sed "s/^/$1 $4 /" gpurun_out/res_$4_$1.json
}
for rep in 1 2; do
  for v in prev base; do run $v c2,c5,c4 100000000 s$rep || exit 1; done
  for v in prev base; do run $v c3 125000000 b$rep || exit 1; done
done
