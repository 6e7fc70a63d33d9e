#!/usr/bin/env python3
"""gpurun_out/traffic_TAG -> profiles/pmc_join_traffic.json.

FETCH_SIZE / WRITE_SIZE are KB per dispatch (summed over the counter's instances).  On
gfx950 FETCH_SIZE under-reports wide coalesced reads (MI355X_MICROARCH.md, HBM), and
other access widths are uncalibrated, so both are calibrated on cells_kernel<BNG>: a
stream of exactly 16 B read + 8 B written per point with the same 8-byte per-lane
accesses as the join's point reads and record writes."""
import collections
import csv
import json
import os
import sys

d, tag = sys.argv[1], sys.argv[2]
CFG = sys.argv[3] if len(sys.argv) > 3 else "c2"   # the join_once --config of the join passes
N = 100_000_000
DESC = {"c2": ("uniform NYC-bbox points, H3 res 9, 263 zones", 9),
        "c3": ("uniform points in the C3 extent, H3 res 10, 74k tract-like polygons (9.4M chips)", 10),
        "c4": ("UPRN-like London points, BNG res 4, 180 districts", 4),
        "c5": ("skewed points near 4 fractal polygons, H3 res 9", 9)}[CFG]
RES = int(sys.argv[4]) if len(sys.argv) > 4 else DESC[1]   # the join_once --res, if not the default
if RES != DESC[1]:
    DESC = (DESC[0].replace("res %d" % DESC[1], "res %d" % RES), RES)


def per_kernel(sub):
    """{kernel short name: (mean counter bytes per dispatch, dispatches)} for mgpu kernels."""
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(os.path.join(d, sub, "run_counter_collection.csv"))):
        name = r["Kernel_Name"]
        if "mgpu::" not in name:
            continue
        short = name.split("mgpu::", 1)[1].split("(", 1)[0]
        tot[short][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: (sum(v.values()) / len(v) * 1024.0, len(v)) for k, v in tot.items()}


def traffic_name(cfg, res):
    """(bench.py reads the same names)"""
    default = {"c2": 9, "c3": 10, "c4": 4, "c5": 9}[cfg]
    base = "pmc_join_traffic" if cfg == "c2" else "pmc_join_traffic_%s" % cfg
    return base + ("" if res == default else "_r%d" % res) + ".json"


def run_key(sub):
    for line in open(os.path.join(d, sub + ".log")):
        if line.startswith("KEY "):
            return json.loads(line[4:])
    raise SystemExit("no KEY line in %s.log (tools/join_once.py)" % sub)


key = run_key("join_fetch")
assert key == run_key("join_write"), "the two passes ran different builds / tables"
jf_all, jw_all = per_kernel("join_fetch"), per_kernel("join_write")
bf, nb = per_kernel("bng_fetch")["cells_kernel<1>"]
bw, _ = per_kernel("bng_write")["cells_kernel<1>"]
f_read = bf / (16.0 * N)
f_write = bw / (8.0 * N)
# the dominant kernel: classify_kernel in the split pipeline, pip_binned_kernel in the binned
# one, else the fused pip_join_kernel
dom = next(k for k in jf_all if k.split("<")[0] in ("classify_kernel", "classify_wave_kernel", "classify_pair_kernel", "pip_join_kernel",
                                                     "pip_binned_kernel"))
jf, nj = jf_all[dom]
jw, _ = jw_all[dom]
out = {
    "round": tag, "config": CFG, "points": N, "res": DESC[1], "kernel": dom, "key": key,
    "join_fetch_bytes_raw": jf, "join_write_bytes_raw": jw, "dispatches": nj,
    "calib_bng_fetch_bytes_raw": bf, "calib_bng_write_bytes_raw": bw,
    "calib_read_factor": f_read, "calib_write_factor": f_write,
    "hbm_read_bytes_per_launch": jf / f_read, "hbm_write_bytes_per_launch": jw / f_write,
    "hbm_bytes_per_launch": jf / f_read + jw / f_write,
    "per_kernel": {k: {"hbm_read_bytes": jf_all[k][0] / f_read,
                       "hbm_write_bytes": jw_all.get(k, (0.0, 0))[0] / f_write} for k in sorted(jf_all)},
    "note": dom + ", 1e8 " + DESC[0] + "; FETCH_SIZE and WRITE_SIZE "
            "in separate rocprofv3 --pmc passes, each divided by its factor measured on cells_kernel<BNG> "
            "(16 B read + 8 B written per point)",
}
json.dump(out, open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles",
                                 traffic_name(CFG, RES)), "w"),
          indent=1)
print(json.dumps(out, indent=1))
