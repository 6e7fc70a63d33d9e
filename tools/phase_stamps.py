#!/usr/bin/env python3
"""Per-phase clock shares of the join tiles, from a -DMGPU_STAMPS build of the library
(tools/build_variants.sh "stamps:-DMGPU_STAMPS"; run with MOSAIC_AMD_LIB pointing at it).
Thread 0 of every tile adds the wall-clock ticks (100 MHz) of each phase to the workspace
counters [10..14] (kernels.hip MGPU_STAMP): 1 = phase 1 (cells, probes, candidates),
2 = phase 2 (envelope / classification grid), 3 = phase 2b (strip walks), 4 = phase 3
(output), 5 = pixel-index pass A.  With -DMGPU_STATS also: candidates, strip walks
(phase 2b candidates) and the strip edges they visited.  One JSON line per config: ticks per phase summed over
the tiles of one join, and their shares."""
import ctypes
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
    ap.add_argument("--configs", default="c3,c2")
    ap.add_argument("--points", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--res", type=int, default=None)
    a = ap.parse_args()
    import mosaic_amd as M
    from mosaic_amd import _native as N
    import bench as B
    import bench_workloads as W
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = M.default_context(dev)
    ctx.reserve(a.points)
    names = {1: "phase1", 2: "phase2", 3: "phase2b", 4: "phase3", 5: "passA"}
    for c in a.configs.split(","):
        ns = argparse.Namespace(config=c, res=a.res, seed=0x20250314, points=a.points)
        wl = B.workload(ns, W, M)
        chips = M.tessellate(wl["polygons"], wl["isys"], ns.res).upload(ctx)
        x, y = wl["points"](a.points, 0, dev)
        cap = int(a.points * wl["pairs_per_point"]) + 1024
        op = torch.empty(cap, dtype=torch.int64, device=dev)
        oq = torch.empty(cap, dtype=torch.int32, device=dev)
        ticks = []
        for _ in range(a.reps):
            r = M.pip_join(x, y, chips, ns.res, out=(op, oq), capacity=cap, index_system=wl["isys"])
            cnt = (ctypes.c_uint64 * 16)()
            N.check(N.lib().mgpu_test_join_counters(ctx.handle, cnt))
            ticks.append([int(cnt[9 + k]) for k in range(1, 6)])
            extra = {"candidates": int(cnt[3]), "strip_walks": int(cnt[8]), "strip_edges": int(cnt[9])}
        t = np.median(np.array(ticks, dtype=np.float64), axis=0)
        tot = float(t.sum()) or 1.0
        print(json.dumps({"config": c, "res": a.res, "pipeline": r.stats["pipeline"], "kernel_ms": r.stats["kernel_ms"],
                          "ticks": {names[k + 1]: float(t[k]) for k in range(5)},
                          "share": {names[k + 1]: round(float(t[k]) / tot, 4) for k in range(5)}, **extra}), flush=True)
        del x, y, op, oq, chips
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
