#!/usr/bin/env python3
"""Per-kernel summary of a tools/gpu_pmc3.sh directory: counter means per dispatch, the
kernel-trace mean duration, and derived ratios (wait share, L2 hit rate, bytes)."""
import collections
import csv
import glob
import json
import os
import sys


def main(d, out_json=None):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            per[(k, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (k, _, name), v in per.items():
            vals[k][name].append(v)
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "kt", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[r["Kernel_Name"].split("(")[0]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    res = {}
    for k in sorted(vals, key=lambda k: -sum(dur.get(k, [0])) / max(1, len(dur.get(k, [1])))):
        m = {c: sum(v) / len(v) for c, v in vals[k].items()}
        if k in dur:
            m["duration_ns"] = sum(dur[k]) / len(dur[k])
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS"):
                if c in m:
                    m[c + "/WAVE_CYCLES"] = m[c] / wc
        if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
            m["L2_hit_rate"] = m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
        if "GRBM_GUI_ACTIVE" in m and "duration_ns" in m:
            m["clock_GHz_est"] = m["GRBM_GUI_ACTIVE"] / 8 / m["duration_ns"]
        if "SQ_WAVES" in m and "SQ_WAVE_CYCLES" in m and "duration_ns" in m and "clock_GHz_est" in m:
            # average resident waves per CU: wave-cycles (quad-cycles x4) over kernel cycles x 256 CUs
            m["avg_waves_per_CU"] = m["SQ_WAVE_CYCLES"] * 4 / (m["duration_ns"] * m["clock_GHz_est"] * 256)
        res[k] = m
        print("== %s" % k)
        for c in sorted(m):
            print("  %-34s %16.6g" % (c, m[c]))
    if out_json:
        json.dump(res, open(out_json, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
