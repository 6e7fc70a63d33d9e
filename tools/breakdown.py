#!/usr/bin/env python3
"""Where the fused join's time goes (profiling aid, GPU box only).

Times, on the bench workload (uniform NYC-bbox points x 263 zones, H3 res 9):
  cells      mgpu_points_to_cells alone (H3 geoToH3 of every point, 24 B/pt)
  join       the fused kernel
  join/noPIP border chips counted as misses (MGPU_ABLATE=1)
  join/noprobe  H3 projection, no chip-table probe (MGPU_ABLATE=2)
  join/noproj   no projection either: point loads + tile protocol only (MGPU_ABLATE=3)
  join/listonly candidates listed, none evaluated (MGPU_ABLATE=4)
  join/envonly  candidates evaluated by the chip envelope only (MGPU_ABLATE=5)
  join/nogridload  dense probe replaced by one synthetic core chip (MGPU_ABLATE=6)
Prints one JSON object.  Times: the streaming kernel (pip_join_kernel), HIP events on its stream.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=100_000_000)
    ap.add_argument("--res", type=int, default=None)
    ap.add_argument("--config", choices=["c2", "c4", "c5"], default="c2")
    ap.add_argument("--seed", type=int, default=0x20250314)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import mosaic_amd as M
    import bench as B
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = M.default_context(dev)
    import bench_workloads as W
    wl = B.workload(a, W, M)
    isys = wl["isys"]
    chips = M.tessellate(wl["polygons"], isys, a.res).upload(ctx)
    x, y = wl["points"](a.points, 0, dev)
    cap = max(int(a.points * wl["pairs_per_point"]), a.points) + 1024
    op = torch.empty(cap, dtype=torch.int64, device=dev)
    oq = torch.empty(cap, dtype=torch.int32, device=dev)
    ctx.reserve(a.points)
    out = {"points": a.points, "res": a.res, "config": a.config}

    def t_cells():
        ms = []
        for _ in range(a.reps + 1):
            _, st = M.grid_longlatascellid(x, y, a.res, index_system=isys, stats=True)
            ms.append(st["kernel_ms"])
        return float(np.median(ms[1:]))

    def t_join(ablate):
        if ablate:
            os.environ["MGPU_ABLATE"] = str(ablate)
        else:
            os.environ.pop("MGPU_ABLATE", None)
        ms = []
        for _ in range(a.reps + 1):
            r = M.pip_join(x, y, chips, a.res, out=(op, oq), capacity=cap, index_system=isys)
            ms.append(r.stats["stream_kernel_ms"])
        os.environ.pop("MGPU_ABLATE", None)
        return float(np.median(ms[1:])), len(r)

    out["cells_ms"] = t_cells()
    out["join_ms"], out["pairs"] = t_join(0)
    out["join_nopip_ms"], out["pairs_nopip"] = t_join(1)
    out["join_noprobe_ms"], _ = t_join(2)
    out["join_noproj_ms"], _ = t_join(3)
    out["join_listonly_ms"], _ = t_join(4)
    out["join_envonly_ms"], _ = t_join(5)
    out["join_nogridload_ms"], out["pairs_nogridload"] = t_join(6)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
