#!/bin/bash
# Multi-rank protocol rehearsal of bench.py on a 1-GPU box: 2 ranks on the same GPU
# over gloo (chip-table broadcast staged through the host, count all-gather).
set -o pipefail
mkdir -p gpurun_out
MGPU_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 3 --warmup 1 --points 20000000 \
  --no-cpu-baseline > gpurun_out/dist_rehearsal.json 2> gpurun_out/dist_rehearsal.err
rc=$?
cat gpurun_out/dist_rehearsal.json; tail -5 gpurun_out/dist_rehearsal.err
exit $rc
