#!/usr/bin/env python3
"""profiles/r4_pmc/<cfg>_kernels.json (tools/pmc_kernels.py of a tools/gpu_pmc_r4.sh run)
-> profiles/pmc_valu.json: the dominant join kernel's VALU / SALU wave-instructions per
point, which bench.py turns into a VALU-issue fraction of its own measured kernel time.
Usage: tools/valu_summary.py ROUND CFG:RES:FILE:PASS_LOG ...   (1e8 points per join_once launch;
PASS_LOG: the SQ pass's join_once log, whose KEY line keys the entry to its build and table)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOM = ("classify_wave_kernel", "classify_pair_kernel", "pip_binned_kernel", "pip_join_kernel")
out_path = os.path.join(ROOT, "profiles", "pmc_valu.json")
out = json.load(open(out_path)) if os.path.exists(out_path) else {}
rnd = sys.argv[1]
def run_key(log):
    """The KEY line tools/join_once.py printed in the counter pass (bench.py traffic_key)."""
    for line in open(log):
        if line.startswith("KEY "):
            return json.loads(line[4:])
    raise SystemExit("no KEY line in %s" % log)


for spec in sys.argv[2:]:
    cfg, res, f, log = spec.split(":", 3)
    d = json.load(open(f))
    k = next(k for k in d if any(x in k for x in DOM) and "SQ_INSTS_VALU" in d[k])
    m = d[k]
    n = 100_000_000
    out["%s_r%s" % (cfg, res)] = {
        "round": rnd, "kernel": k.replace("void mgpu::", "").replace("mgpu::", ""), "points": n,
        "valu_insts_per_point": m["SQ_INSTS_VALU"] / n, "salu_insts_per_point": m["SQ_INSTS_SALU"] / n,
        "lds_insts_per_point": m.get("SQ_INSTS_LDS", 0.0) / n,
        "lds_conflict_cycles_per_point": m.get("SQ_LDS_BANK_CONFLICT", 0.0) / n,
        "wait_share": m.get("SQ_WAIT_ANY/WAVE_CYCLES"), "duration_ns": m.get("duration_ns"),
        "source": os.path.relpath(f, ROOT), "key": run_key(log)}
json.dump(out, open(out_path, "w"), indent=1, sort_keys=True)
print(json.dumps(out, indent=1, sort_keys=True))
