#!/bin/bash
# The one GPU-box driver (run through gpurun; writes under gpurun_out/).  Steps are joined
# with "+" and run in order; the first failing step ends the call (no GPU step after it):
#
#   bash tools/gpu.sh tests TAG [K_EXPR] + smoke TAG + bench TAG "c2 c3" [BENCH_ARGS...]
#
# Steps:
#   tests TAG [K_EXPR]              the -m gpu suite (or the tests matching K_EXPR)
#   smoke TAG                       __graft_entry__.smoke()
#   bench TAG "CFGS" [ARGS]         bench.py per config (CPU baseline + PCIe line) and a
#                                   rocprofv3 kernel trace of the same command (kt_TAG_<cfg>/)
#   ktrace TAG "CFGS" [ARGS]        kernel-trace stats of bench.py only
#   opts TAG CFG "k=v ..." ...      bench.py on CFG once per option set (two interleaved reps)
#   ab TAG CFGS [AB_ARGS]           tools/ab_time.py over every build/ab/*/ library variant,
#                                   interleaved, two reps (variants: tools/variants.sh)
#   counters TAG "CFG[:RES] ..."    SQ passes (pmc) + FETCH/WRITE traffic passes per config
#   pmc TAG "JOIN_ONCE_ARGS" [P]    counter passes P (default "1 2 3 4 5") of one join, per kernel
#   traffic TAG CFG [RES]           FETCH_SIZE / WRITE_SIZE passes + the BNG-cells calibration
#   stamps TAG CFGS [ARGS]          per-phase clock shares (the build/ab/stamps variant)
#   blob TAG CFG                    chip-table builder phases (the build/ab/timing variant) + upload
#   kring TAG | bngfmt TAG          kRing / StringType throughput + kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out

line() {  # one summary line of a bench JSON
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d.get('roofline') or {};print(sys.argv[2], '%.3e'%d['value'], '%.3f ms'%d['ms_per_step'], {k:round(v,3) for k,v in (d.get('kernels_ms') or {}).items()}, 'frac', r.get('frac'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))" "$1" "$2"
}

step_tests() {
  local TAG=$1; local SEL=(); [ -n "$2" ] && SEL=(-k "$2")
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread "${SEL[@]}" > $O/pytest_gpu_$TAG.log 2>&1
  local rc=$?; tail -3 $O/pytest_gpu_$TAG.log; return $rc
}

step_smoke() {
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_$1.log 2>&1 || { tail -20 $O/smoke_$1.log; return 1; }
  tail -1 $O/smoke_$1.log
}

step_bench() {
  local TAG=$1 CFGS=$2; shift 2
  for c in $CFGS; do
    timeout -k 10 600 python3 -u bench.py --config $c "$@" > $O/final_${TAG}_$c.json 2> $O/final_${TAG}_$c.err || { echo "bench $c failed"; tail -5 $O/final_${TAG}_$c.err; return 1; }
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${TAG}_$c -o run -- python3 -u bench.py --config $c --no-cpu-baseline --no-pcie "$@" > $O/kt_${TAG}_$c.json 2> $O/kt_${TAG}_$c.err || { echo "trace $c failed"; return 1; }
    line $O/final_${TAG}_$c.json $c
  done
}

step_ktrace() {
  local TAG=$1 CFGS=$2; shift 2
  for c in $CFGS; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${TAG}_$c -o run -- python3 -u bench.py --config $c --no-cpu-baseline --no-pcie --steps 5 "$@" > $O/kt_${TAG}_$c.json 2> $O/kt_${TAG}_$c.err || { echo "trace $c failed"; return 1; }
    echo "== $c"; cut -d, -f1-4 $O/kt_${TAG}_$c/run_kernel_stats.csv | grep -v "at::native" | head -8
  done
}

step_opts() {
  local TAG=$1 CFG=$2; shift 2
  for rep in 1 2; do
    local i=0
    for o in "$@"; do
      i=$((i+1)); local OPTS=""; for kv in $o; do OPTS="$OPTS --option $kv"; done
      timeout -k 10 300 python3 -u bench.py --config $CFG --no-cpu-baseline --no-pcie $OPTS > $O/opts_${TAG}_${i}_$rep.json 2> $O/opts_${TAG}_${i}_$rep.err || { echo "bench $o failed"; tail -5 $O/opts_${TAG}_${i}_$rep.err; return 1; }
      line $O/opts_${TAG}_${i}_$rep.json "[$o] rep $rep"
    done
  done
}

step_ab() {
  local TAG=$1 CFGS=$2; shift 2
  for rep in 1 2; do
    for d in build/ab/*/; do
      local n=$(basename $d)
      MOSAIC_AMD_LIB=$PWD/$d/libmosaic_gpu.so timeout -k 10 300 python3 -u tools/ab_time.py --configs $CFGS "$@" > $O/ab_${TAG}_${n}_$rep.json 2> $O/ab_${TAG}_${n}_$rep.err || { echo "variant $n failed"; tail -5 $O/ab_${TAG}_${n}_$rep.err; return 1; }
      sed "s/^/$n $rep /" $O/ab_${TAG}_${n}_$rep.json
    done
  done
}

step_traffic() {
  local TAG=$1 CFG=$2 R=$3; local RES=${R:+--res $R}
  local OUT=$O/traffic_$TAG; mkdir -p $OUT
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/join_fetch -o run -- python3 -u tools/join_once.py --config $CFG $RES --cache /tmp/mgpu_cache_$CFG$R.npz > $OUT/join_fetch.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/join_write -o run -- python3 -u tools/join_once.py --config $CFG $RES --cache /tmp/mgpu_cache_$CFG$R.npz > $OUT/join_write.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/bng_fetch -o run -- python3 -u tools/join_once.py --cells --bng > $OUT/bng_fetch.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/bng_write -o run -- python3 -u tools/join_once.py --cells --bng > $OUT/bng_write.log 2>&1
}

step_pmc() {
  local TAG=$1 ARGS=$2 PASSES=${3:-"1 2 3 4 5"}
  local OUT=$O/pmc_$TAG; mkdir -p $OUT
  local P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH"
  local P2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
  local P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum GRBM_GUI_ACTIVE"
  local P4="FETCH_SIZE" P5="WRITE_SIZE"
  echo "$ARGS" > $OUT/args
  timeout -k 10 600 python3 -u tools/join_once.py $ARGS --reps 1 --cache /tmp/chips_$TAG.npz > $OUT/warm.log 2>&1 || { echo "warm run failed"; tail -5 $OUT/warm.log; return 1; }
  for pn in $PASSES; do
    eval "local P=\$P$pn"
    timeout -s KILL 180 rocprofv3 --pmc $P --output-format csv -d $OUT/p$pn -o run -- python3 -u tools/join_once.py $ARGS --cache /tmp/chips_$TAG.npz > $OUT/p$pn.log 2>&1 || { echo "pass $pn failed"; tail -5 $OUT/p$pn.log; return 1; }
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 -u tools/join_once.py $ARGS --cache /tmp/chips_$TAG.npz > $OUT/kt.log 2>&1 || { echo "ktrace failed"; return 1; }
  python3 tools/pmc_kernels.py $OUT
}

step_counters() {
  local TAG=$1 CFGS=$2
  for cr in $CFGS; do
    local c=${cr%%:*} r=${cr#*:}; [ "$r" = "$cr" ] && r=""
    local n=${c}${r:+r$r}
    step_pmc ${TAG}_$n "--config $c ${r:+--res $r}" "1 2" > $O/pmc_${TAG}_$n.txt 2>&1 || { echo "pmc $n failed"; tail -5 $O/pmc_${TAG}_$n.txt; return 1; }
    step_traffic ${TAG}_$n $c $r > $O/traffic_${TAG}_$n.txt 2>&1 || { echo "traffic $n failed"; tail -5 $O/traffic_${TAG}_$n.txt; return 1; }
    echo "== $n done"
  done
}

step_stamps() {
  local TAG=$1 CFGS=$2; shift 2
  MOSAIC_AMD_LIB=$PWD/build/ab/stamps/libmosaic_gpu.so timeout -k 10 300 python3 -u tools/phase_stamps.py --configs $CFGS "$@" > $O/stamps_$TAG.json 2> $O/stamps_$TAG.err || { echo "stamps failed"; tail -5 $O/stamps_$TAG.err; return 1; }
  cat $O/stamps_$TAG.json
}

step_blob() {
  local TAG=$1 CFG=${2:-c3}
  MOSAIC_AMD_LIB=$PWD/build/ab/timing/libmosaic_gpu.so timeout -k 10 300 python3 -u tools/blob_time.py $CFG --upload > $O/blob_${TAG}.out 2> $O/blob_${TAG}.err || { tail -20 $O/blob_${TAG}.err; return 1; }
  cat $O/blob_${TAG}.out; grep -E "blob\]|raster\]" $O/blob_${TAG}.err | tail -16
}

step_kring() {
  timeout -k 10 200 python3 -u tools/kring_bench.py > $O/kring_$1.json 2> $O/kring_$1.err &&
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kring_prof_$1 -o run -- python3 -u tools/kring_bench.py > $O/kring_prof_$1.json 2> $O/kring_prof_$1.err || return 1
  cat $O/kring_$1.json
}

step_bngfmt() {
  timeout -k 10 200 python3 -u tools/bng_format_bench.py > $O/bngfmt_$1.json 2> $O/bngfmt_$1.err &&
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bngfmt_prof_$1 -o run -- python3 -u tools/bng_format_bench.py > $O/bngfmt_prof_$1.json 2> $O/bngfmt_prof_$1.err || return 1
  cat $O/bngfmt_$1.json
}

# split the arguments at "+" and run the steps in order
args=()
run_step() {
  [ ${#args[@]} -eq 0 ] && return 0
  local name=${args[0]}
  echo "## ${args[*]}"
  if ! declare -F step_$name > /dev/null; then echo "unknown step $name"; exit 2; fi
  step_$name "${args[@]:1}" || { echo "step $name failed"; exit 1; }
  args=()
}
for a in "$@"; do
  if [ "$a" = "+" ]; then run_step; else args+=("$a"); fi
done
run_step
