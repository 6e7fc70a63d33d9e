#!/usr/bin/env python3
"""Run the bench workload's join (or cells) kernel a few times -- a short target for
rocprofv3 PMC passes.  --pipeline forces one of the join's pipelines (context option)."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=100_000_000)
    ap.add_argument("--res", type=int, default=None)
    ap.add_argument("--config", choices=["c2", "c3", "c4", "c5"], default="c2")
    ap.add_argument("--seed", type=int, default=0x20250314)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--pipeline", type=int, default=-1)
    ap.add_argument("--option", action="append", default=[], help="context option key=value (as bench.py)")
    ap.add_argument("--cells", action="store_true")
    ap.add_argument("--cache", default=None, help="npz of the tessellated chip table (written when absent): "
                    "PMC passes of a large config tessellate once")
    ap.add_argument("--bng", action="store_true", help="with --cells: BNG res 4 on eastings/northings "
                    "(a pure 16 B read + 8 B write stream, used to calibrate FETCH_SIZE / WRITE_SIZE)")
    a = ap.parse_args()
    import mosaic_amd as M
    import bench as B
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = M.default_context(dev)
    ctx.set_option("pipeline", a.pipeline)
    for kv in a.option:
        k, v = kv.split("=", 1)
        ctx.set_option(k, int(v))
    import bench_workloads as W
    wl = B.workload(a, W, M)
    isys = wl["isys"]
    import numpy as np
    if a.cache and os.path.exists(a.cache):
        z = np.load(a.cache)
        table = M.ChipTable(z["cell"], z["polygon_id"], z["is_core"], z["wkb_offsets"], z["wkb"], isys.code)
    else:
        table = M.tessellate(wl["polygons"], isys, a.res, keep_core_geometries=wl.get("keep_core", True))
        if a.cache:
            np.savez(a.cache, cell=table.cell, polygon_id=table.polygon_id, is_core=table.is_core,
                     wkb_offsets=table.wkb_offsets, wkb=table.wkb)
    chips = table.upload(ctx)
    if not a.cells:
        import json
        # what a bench line must match to carry this run's counters (bench.py traffic_key)
        print("KEY " + json.dumps(B.traffic_key(a.option, chips.info())), flush=True)
    x, y = wl["points"](a.points, 0, dev)
    cap = int(a.points * wl["pairs_per_point"]) + 1024
    op = torch.empty(cap, dtype=torch.int64, device=dev)
    oq = torch.empty(cap, dtype=torch.int32, device=dev)
    ctx.reserve(a.points)
    if a.bng:
        x = x.mul(0).add_(torch.rand_like(x).mul_(58000.0).add_(503000.0))
        y = y.mul(0).add_(torch.rand_like(y).mul_(46000.0).add_(155000.0))
    for _ in range(a.reps):
        if a.cells and a.bng:
            M.grid_longlatascellid(x, y, 4, index_system=M.BNGIndexSystem())
        elif a.cells:
            M.grid_longlatascellid(x, y, a.res, index_system=isys)
        else:
            M.pip_join(x, y, chips, a.res, out=(op, oq), capacity=cap, index_system=isys)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
