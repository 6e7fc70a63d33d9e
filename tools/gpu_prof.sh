#!/bin/bash
# Kernel trace + PMC passes of the bench command (one counter group per pass, each
# pass its own time limit; the first failure ends the script).
set -o pipefail
TAG=${1:-r1}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/trace_bench.json 2> $OUT/trace.err &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- $CMD > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- $CMD > $OUT/pmc_write.json 2> $OUT/pmc_write.err &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/pmc_sq -o run -- $CMD > $OUT/pmc_sq.json 2> $OUT/pmc_sq.err &&
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/pmc_grbm -o run -- $CMD > $OUT/pmc_grbm.json 2> $OUT/pmc_grbm.err &&
timeout -k 10 300 python3 -u tools/breakdown.py > $OUT/breakdown.json 2> $OUT/breakdown.err
rc=$?
echo "exit $rc"
exit $rc
