#!/usr/bin/env python3
"""Binned vs fused/split join timings on one bench config (the chip table and the points
built once; the pipeline chosen per call by the context options): one JSON line per
variant {config, variant, stream_ms, bin_ms, emit_ms, pipeline_ms, pipeline, pairs}.
tools/bin_ab.py --config c3 [--points N] [--variants fused,bin1024,...]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

VARIANTS = {
    "auto": {},
    "fused": {"pipeline": 0},
    "split": {"pipeline": 1},
    "bin16": {"pipeline": 2, "bin_count": 16},
    "bin32": {"pipeline": 2, "bin_count": 32},
    "bin64": {"pipeline": 2, "bin_count": 64},
    "bin128": {"pipeline": 2, "bin_count": 128},
    "bin256": {"pipeline": 2, "bin_count": 256},
    "bin512": {"pipeline": 2, "bin_count": 512},
    "bin256_noxcd": {"pipeline": 2, "bin_count": 256, "bin_xcd": 0},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--points", type=int, default=None)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", default="fused,bin16,bin32,bin64,bin128,bin256,auto")
    a = ap.parse_args()
    import mosaic_amd as M
    import bench as B
    import bench_workloads as W
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = M.default_context(dev)
    ns = argparse.Namespace(config=a.config, res=None, seed=0x20250314, points=a.points)
    wl = B.workload(ns, W, M)
    chips = M.tessellate(wl["polygons"], wl["isys"], ns.res, keep_core_geometries=wl.get("keep_core", True)).upload(ctx)
    x, y = wl["points"](ns.points, 0, dev)
    ctx.reserve(ns.points)
    cap = int(ns.points * wl["pairs_per_point"]) + 1024
    op = torch.empty(cap, dtype=torch.int64, device=dev)
    oq = torch.empty(cap, dtype=torch.int32, device=dev)
    ref = None
    for v in a.variants.split(","):
        with ctx.options(**VARIANTS[v]):
            s, p, mx, em = [], [], [], []
            for _ in range(a.reps + 1):
                r = M.pip_join(x, y, chips, ns.res, out=(op, oq), capacity=cap, index_system=wl["isys"])
                s.append(r.stats["stream_kernel_ms"])
                p.append(r.stats["kernel_ms"])
                mx.append(r.stats["mixed_kernel_ms"])
                em.append(r.stats["emit_kernel_ms"])
        # every variant's pairs equal the first one's (checksums over the full output)
        m = len(r)
        ck = (int(op[:m].sum().item()), int((oq[:m].to(torch.int64) * (torch.arange(m, device=dev) % 7919)).sum().item()))
        ref = ck if ref is None else ref
        print(json.dumps({"config": a.config, "variant": v, "stream_ms": float(np.median(s[1:])),
                          "bin_ms": float(np.median(mx[1:])), "emit_ms": float(np.median(em[1:])),
                          "pipeline_ms": float(np.median(p[1:])), "pipeline": r.stats["pipeline"], "pairs": m,
                          "candidates": r.stats["n_candidates"], "near_ties": r.stats["n_near_ties"],
                          "same_as_first": ck == ref}), flush=True)


if __name__ == "__main__":
    main()
