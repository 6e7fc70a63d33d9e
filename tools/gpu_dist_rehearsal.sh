#!/bin/bash
# Multi-rank protocol rehearsal of bench.py on a 1-GPU box: 2 ranks on the same GPU
# over gloo (chip-table broadcast staged through the host, count all-gather).
set -o pipefail
CFG=${1:-c2}
mkdir -p gpurun_out
MGPU_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 3 --warmup 1 --points 20000000 \
  --config $CFG --no-cpu-baseline > gpurun_out/dist_rehearsal_$CFG.out 2> gpurun_out/dist_rehearsal_$CFG.err
rc=$?
# the record is rank 0's JSON line only (gloo's connection logs share stdout)
grep '^{' gpurun_out/dist_rehearsal_$CFG.out > gpurun_out/dist_rehearsal_$CFG.json
cat gpurun_out/dist_rehearsal_$CFG.json; tail -5 gpurun_out/dist_rehearsal_$CFG.err
exit $rc
