#!/bin/bash
# C3 A/B on one box: the binned GPU tests, then bench.py --config c3 with each option set
# given (interleaved, two repetitions): gpurun_out/c3ab_TAG_<i>_<rep>.json
#   tools/gpu_c3_ab.sh TAG "bin_keys=0" "bin_keys=1"
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_binned.py -x -q --timeout 300 --timeout-method thread > gpurun_out/c3ab_${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/c3ab_${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/c3ab_${TAG}_tests.log
for rep in 1 2; do
  i=0
  for o in "$@"; do
    i=$((i+1))
    OPTS=""; for kv in $o; do OPTS="$OPTS --option $kv"; done
    timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu-baseline --no-pcie $OPTS > gpurun_out/c3ab_${TAG}_${i}_$rep.json 2> gpurun_out/c3ab_${TAG}_${i}_$rep.err || { echo "bench $o failed"; tail -5 gpurun_out/c3ab_${TAG}_${i}_$rep.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], '%.3e'%d['value'], '%.3f ms'%d['ms_per_step'], {k:round(v,3) for k,v in d['kernels_ms'].items()}, 'setup', {k:(round(v,2) if isinstance(v,float) else v) for k,v in d['setup_s'].items() if k.endswith('_s')})" gpurun_out/c3ab_${TAG}_${i}_$rep.json "$o"
  done
done
