#!/bin/bash
# Round-5 split emit A/B: one-match items staged in one branch each, the rest in a second
# walk (e2p, MGPU_EMIT_2P) vs the single walk (jc2); the parity suite on e2p first.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
MOSAIC_AMD_LIB=$PWD/build/ab/e2p/libmosaic_gpu.so timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_e2p.log 2>&1 || { tail -30 gpurun_out/pytest_e2p.log; exit 1; }
tail -1 gpurun_out/pytest_e2p.log
for rep in 1 2; do for v in jc2 e2p; do
  MOSAIC_AMD_LIB=$PWD/build/ab/$v/libmosaic_gpu.so timeout -k 10 300 python3 -u tools/ab_time.py --configs c2,c5 --reps 7 > gpurun_out/e2p_${rep}_$v.json 2> gpurun_out/e2p_${rep}_$v.err || { echo "variant $v failed"; tail -5 gpurun_out/e2p_${rep}_$v.err; exit 1; }
  sed "s/^/$v $rep /" gpurun_out/e2p_${rep}_$v.json
done; done
