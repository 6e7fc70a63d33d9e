#!/bin/bash
# SQ / TCC / traffic counter passes of one join workload, per kernel:
#   tools/gpu_pmc3.sh TAG "JOIN_ONCE_ARGS" [PASSES]     (default passes: 1 2 3 4 5)
# Each pass is its own rocprofv3 run of tools/join_once.py (chip table cached in /tmp);
# summary: python3 tools/pmc_kernels.py gpurun_out/pmc_TAG
set -o pipefail
TAG=$1; ARGS=$2; PASSES=${3:-"1 2 3 4 5"}
OUT=gpurun_out/pmc_$TAG; mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH"
P2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum GRBM_GUI_ACTIVE"
P4="FETCH_SIZE"
P5="WRITE_SIZE"
echo "$ARGS" > $OUT/args
# warm the chip-table cache outside the profiler
timeout -k 10 600 python3 -u tools/join_once.py $ARGS --reps 1 --cache /tmp/chips_$TAG.npz > $OUT/warm.log 2>&1 || { echo "warm run failed"; tail -5 $OUT/warm.log; exit 1; }
for pn in $PASSES; do
  eval "P=\$P$pn"
  timeout -s KILL 180 rocprofv3 --pmc $P --output-format csv -d $OUT/p$pn -o run -- python3 -u tools/join_once.py $ARGS --cache /tmp/chips_$TAG.npz > $OUT/p$pn.log 2>&1 || { echo "pass $pn failed"; tail -5 $OUT/p$pn.log; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 -u tools/join_once.py $ARGS --cache /tmp/chips_$TAG.npz > $OUT/kt.log 2>&1 || { echo "ktrace failed"; exit 1; }
python3 tools/pmc_kernels.py $OUT
