#!/bin/bash
# Round-5 probe: the split pipeline's mixed-tile launch with every listed point answered
# "no match" at once (mabl, a -DMGPU_MIXED_ABLATE build of a profiling-only change to
# pip_mixed_kernel: wrong pairs, nothing read out of range) vs base -- how much of
# pip_mixed_kernel's time is the dispatch of its one-wave workgroups
# (profiles/r5/probe_mixed_dispatch.txt).
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do for v in base mabl; do
  MOSAIC_AMD_LIB=$PWD/build/ab/$v/libmosaic_gpu.so timeout -k 10 300 python3 -u tools/ab_time.py --configs c2,c5 --reps 7 > gpurun_out/mabl_${rep}_$v.json 2> gpurun_out/mabl_${rep}_$v.err || { echo "variant $v failed"; tail -5 gpurun_out/mabl_${rep}_$v.err; exit 1; }
  sed "s/^/$v $rep /" gpurun_out/mabl_${rep}_$v.json
done; done
