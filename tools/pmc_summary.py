#!/usr/bin/env python3
"""Summarise gpurun_out/pmc_TAG: per configuration, per-dispatch counter means of the
mgpu kernels, normalised per wave."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "mgpu::"
for args in sorted(glob.glob(os.path.join(d, "c*.args"))):
    c = os.path.basename(args)[:-5]
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, c + "_p*", "run_counter_collection.csv")):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if kern not in r["Kernel_Name"]:
                continue
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (disp, name), v in per.items():
            vals[name].append(v)
    m = {k: sum(v) / len(v) for k, v in vals.items()}
    w = m.get("SQ_WAVES", 1)
    print("==", open(args).read().strip())
    for k in sorted(m):
        print("  %-28s %14.4g  per-wave %10.1f" % (k, m[k], m[k] / w))
