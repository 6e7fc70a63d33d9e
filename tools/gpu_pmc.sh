#!/bin/bash
# SQ counter passes over tools/join_once.py configurations: tools/gpu_pmc.sh TAG "ARGS1" "ARGS2" ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/pmc_$TAG; mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64"
P2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INST_CYCLES_SALU"
P4="SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_FLAT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC"
P3="SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS_ATOMIC"
i=0
for args in "$@"; do
  i=$((i+1))
  for pn in 1 2 3 4; do
    eval "P=\$P$pn"
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/c${i}_p$pn -o run -- python3 -u tools/join_once.py $args > $OUT/c${i}_p$pn.log 2>&1 || { echo "pass $i/$pn failed"; tail -5 $OUT/c${i}_p$pn.log; exit 1; }
  done
  echo "$args" > $OUT/c${i}.args
done
echo done
