#!/bin/bash
# PMC passes (SQ + cache counters) over tools/join_once.py: tools/gpu_pmc2.sh TAG "ARGS"
set -o pipefail
TAG=$1; ARGS=$2
OUT=gpurun_out/pmc_$TAG; mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH"
P2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
P3="TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_EA0_RDREQ_sum"
P4="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TA_TA_BUSY_sum"
P5="FETCH_SIZE"
P6="WRITE_SIZE"
for pn in 1 2 3 4 5 6; do
  eval "P=\$P$pn"
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/c1_p$pn -o run -- python3 -u tools/join_once.py $ARGS > $OUT/c1_p$pn.log 2>&1 || { echo "pass $pn failed"; tail -5 $OUT/c1_p$pn.log; }
done
echo "$ARGS" > $OUT/c1.args
echo done
