#!/bin/bash
# Round-5 counters: per config, the SQ instruction / wave-cycle passes (gpu_pmc3.sh passes 1 2)
# and the FETCH_SIZE / WRITE_SIZE traffic passes (gpu_traffic.sh):
#   tools/gpu_pmc_r5.sh TAG "CFG[:RES] ..."      e.g. "c2 c4:3 c4"
set -o pipefail
TAG=$1; CFGS=$2
for cr in $CFGS; do
  c=${cr%%:*}; r=${cr#*:}; [ "$r" = "$cr" ] && r=""
  n=${c}${r:+r$r}
  bash tools/gpu_pmc3.sh ${TAG}_$n "--config $c ${r:+--res $r}" "1 2" > gpurun_out/pmc_${TAG}_$n.txt 2>&1 || { echo "pmc $n failed"; tail -5 gpurun_out/pmc_${TAG}_$n.txt; exit 1; }
  bash tools/gpu_traffic.sh ${TAG}_$n $c $r > gpurun_out/traffic_${TAG}_$n.txt 2>&1 || { echo "traffic $n failed"; tail -5 gpurun_out/traffic_${TAG}_$n.txt; exit 1; }
  echo "== $n done"
done
