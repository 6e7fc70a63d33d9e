#!/bin/bash
# C4 (1e8 points) under context options: tools/gpu_c4_opts.sh TAG RES "opt1 opt2" "opt3" ... (each quoted
# group = one run's --option KEY=VALUE list) -> gpurun_out/c4opt_TAG_*.json
set -o pipefail
TAG=$1; RES=$2; shift 2
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for grp in "$@"; do
  i=$((i+1)); args=""
  for kv in $grp; do args="$args --option $kv"; done
  out=gpurun_out/c4opt_${TAG}_$i
  timeout -k 10 300 python3 -u bench.py --config c4 --res $RES --steps 10 --warmup 3 --no-cpu-baseline --no-pcie $args > $out.json 2> $out.err || { echo "run $i ($grp) failed"; tail -5 $out.err; exit 1; }
  python3 -c "import json;d=json.load(open('$out.json'));print('r$RES [$grp]', d['pipeline'], '%.3e'%d['value'], '%.3f ms'%d['ms_per_step'], d['kernels_ms'])"
done
