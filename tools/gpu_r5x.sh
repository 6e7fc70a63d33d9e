#!/bin/bash
# Round-5 final bench lines, part 2: C3 with its kernel trace, C4 at BASELINE's 500M points.
set -o pipefail
bash tools/gpu_final_r5.sh f5w "c3" || exit 1
timeout -k 10 600 python3 -u bench.py --config c4 --points 500000000 --res 3 > gpurun_out/final_f5w_c4_500m_r3.json 2> gpurun_out/final_f5w_c4_500m_r3.err || { echo "c4 500m failed"; tail -5 gpurun_out/final_f5w_c4_500m_r3.err; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('c4 500M r3', '%.3e'%d['value'], '%.3f ms'%d['ms_per_step'], d.get('kernels_ms'), 'frac %.3f'%d['roofline']['frac'], 'traffic', d['roofline'].get('traffic'))" gpurun_out/final_f5w_c4_500m_r3.json
