"""north_star's cell-ordered join measured on C3 (one GPU's 1.25e8 points x 74,000 tracts,
H3 r10) against the binned pipeline the planner picks.  The cell-key sort here is torch.sort
(rocPRIM's device radix sort) over the points' H3 cells -- a stand-in for a hand-written
LSD radix sort, measuring what a sort of that size costs on this GPU, not a product path.
Steps, each timed with events on one stream (median of --reps):
  cells     mgpu_points_to_cells (the cell-id kernel: projection + near-ties)
  sort      torch.sort(cells, stable) -> order (the cell-key sort)
  gather    x[order], y[order] (the points in cell order)
  join      mgpu_pip_join over the cell-ordered points (point ids = order), per pipeline:
            fused (tiles walk cell runs: chips shared inside a tile, L2-local) and binned
  unsort    the pairs back into input order (torch.sort of the point ids + two gathers)
and the binned pipeline on the input order (what the planner runs).
    python3 tools/cell_order_ab.py > gpurun_out/cell_order_ab.json
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(fn, reps, stream):
    ts = []
    out = None
    for _ in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        out = fn()
        e1.record(stream)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts[1:])), out


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=125_000_000)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import mosaic_amd as M
    import bench as B
    import bench_workloads as W
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = M.default_context(dev)
    ctx.reserve(a.points)
    ns = argparse.Namespace(config="c3", res=None, seed=0x20250314, points=a.points)
    wl = B.workload(ns, W, M)
    isys, res = wl["isys"], ns.res
    chips = M.tessellate(wl["polygons"], isys, res, keep_core_geometries=False).upload(ctx)
    x, y = wl["points"](a.points, 0, dev)
    n = x.numel()
    s = torch.cuda.current_stream(dev)
    cap = int(n * wl["pairs_per_point"]) + 1024
    op = torch.empty(cap, dtype=torch.int64, device=dev)
    oq = torch.empty(cap, dtype=torch.int32, device=dev)
    out = {"workload": wl["workload"] % (n, res), "points": n}

    def join(px, py, pid, pipeline):
        with ctx.options(pipeline=pipeline):
            r = M.pip_join(px, py, chips, res, point_id=pid, out=(op, oq), capacity=cap, index_system=isys)
        return r

    # the planner's run on the input order (ctx option pipeline -1 = the planner's choice)
    t, r = timed(lambda: join(x, y, None, -1), a.reps, s)
    out["input_order"] = {"pipeline": r.stats["pipeline"], "ms": t, "kernel_ms": r.stats["kernel_ms"],
                          "join_kernel_ms": r.stats["stream_kernel_ms"], "pairs": len(r)}
    ref_p, ref_q = r.point_id.clone(), r.polygon_id.clone()
    cells = torch.empty(n, dtype=torch.int64, device=dev)
    t, _ = timed(lambda: isys.points_to_index(x, y, res, out=cells), a.reps, s)
    out["cells_ms"] = t
    t, (srt, order) = timed(lambda: torch.sort(cells, stable=True), a.reps, s)
    out["sort_ms"] = t
    del srt, cells
    t, (sx, sy) = timed(lambda: (x[order], y[order]), a.reps, s)
    out["gather_ms"] = t
    for name, pl in (("fused", 0), ("binned", 2)):
        t, r = timed(lambda: join(sx, sy, order, pl), a.reps, s)
        m = len(r)
        rec = {"pipeline": r.stats["pipeline"], "ms": t, "kernel_ms": r.stats["kernel_ms"],
               "join_kernel_ms": r.stats["stream_kernel_ms"], "pairs": m}

        def unsort():
            k, perm = torch.sort(op[:m], stable=True)
            return k, oq[:m][perm]
        tu, (up, uq) = timed(unsort, a.reps, s)
        rec["unsort_ms"] = tu
        rec["equal_to_input_order"] = bool(m == len(ref_p) and torch.equal(up, ref_p) and torch.equal(uq, ref_q))
        out["cell_order_" + name] = rec
    co = out["cell_order_fused"]
    out["cell_order_total_ms"] = out["cells_ms"] + out["sort_ms"] + out["gather_ms"] + co["ms"] + co["unsort_ms"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
