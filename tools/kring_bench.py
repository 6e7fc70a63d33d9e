#!/usr/bin/env python3
"""Throughput of grid_cellkring / grid_cellkloop on the device (mgpu_grid_kring):
BNG: 2e7 res-4 cells of C4's UPRN-like London points; H3 (``h3`` argument): 2e7 res-9
cells of C2's uniform NYC points; k = 1 and 2 (rings) and 2 (loop).
HIP events around the call; one JSON line.  Algorithmic bytes: 8 B read per cell in
each of the two passes + 8 B offset + 8 B per id written."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench_workloads as W
    import mosaic_amd as M
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n = 20_000_000
    if len(sys.argv) > 1 and sys.argv[1] == "h3":
        I = M.H3IndexSystem()
        g = torch.Generator(device=dev).manual_seed(20250314)
        x = torch.rand(n, dtype=torch.float64, device=dev, generator=g) * (-73.7000090639354 + 74.25559136315209) - 74.25559136315209
        y = torch.rand(n, dtype=torch.float64, device=dev, generator=g) * (40.91553277700258 - 40.496115395170364) + 40.496115395170364
        cells = M.grid_longlatascellid(x, y, 9)
        what = "mgpu_grid_kring, H3 res 9 cells of uniform C2 (NYC bbox) points"
    else:
        I = M.BNGIndexSystem()
        x, y = W.london_points(n, 9, dev)
        cells = I.points_to_index(x, y, 4)
        what = "mgpu_grid_kring, BNG res 4 cells of C4 points"
    del x, y
    out = {"what": what, "cells": n}
    for k, loop in ((1, False), (2, False), (2, True)):
        for _ in range(2):
            ids, off = M.grid_cellkring(cells, k, I, loop_only=loop)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(3):
            ids, off = M.grid_cellkring(cells, k, I, loop_only=loop)
        b.record()
        torch.cuda.synchronize(dev)
        ms = a.elapsed_time(b) / 3
        alg = 24.0 * n + 8.0 * ids.numel()
        out["%s%d" % ("loop" if loop else "ring", k)] = {"ms": ms, "ids": int(ids.numel()),
                                                        "cells_per_s": n / (ms * 1e-3),
                                                        "alg_GBps": alg / (ms * 1e-3) / 1e9}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
