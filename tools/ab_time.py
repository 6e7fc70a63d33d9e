#!/usr/bin/env python3
"""Join timings of the library MOSAIC_AMD_LIB points at, on each bench config: one JSON
line per config {config, stream_ms (pip_join_kernel), pipeline_ms (all join launches)}."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c2,c4,c5")
    ap.add_argument("--points", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--res", type=int, default=None)
    a = ap.parse_args()
    import mosaic_amd as M
    import bench as B
    import bench_workloads as W
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = M.default_context(dev)
    ctx.reserve(a.points)
    for c in a.configs.split(","):
        ns = argparse.Namespace(config=c, res=a.res, seed=0x20250314, points=a.points)
        wl = B.workload(ns, W, M)
        chips = M.tessellate(wl["polygons"], wl["isys"], ns.res).upload(ctx)
        x, y = wl["points"](a.points, 0, dev)
        cap = int(a.points * wl["pairs_per_point"]) + 1024
        op = torch.empty(cap, dtype=torch.int64, device=dev)
        oq = torch.empty(cap, dtype=torch.int32, device=dev)
        s, p, mx, em = [], [], [], []
        for _ in range(a.reps + 1):
            r = M.pip_join(x, y, chips, ns.res, out=(op, oq), capacity=cap, index_system=wl["isys"])
            s.append(r.stats["stream_kernel_ms"])
            p.append(r.stats["kernel_ms"])
            mx.append(r.stats["mixed_kernel_ms"])
            em.append(r.stats["emit_kernel_ms"])
        print(json.dumps({"config": c, "stream_ms": float(np.median(s[1:])), "pipeline_ms": float(np.median(p[1:])),
                          "mixed_ms": float(np.median(mx[1:])), "emit_ms": float(np.median(em[1:])),
                          "pipeline": r.stats["pipeline"], "pairs": len(r), "near_ties": r.stats["n_near_ties"],
                          "candidates": r.stats["n_candidates"]}), flush=True)
        del x, y, op, oq, chips
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
