#!/usr/bin/env python3
"""Time mgpu_points_to_cells (grid_longlatascellid) on 1e8 points: H3 res 9 (NYC bbox
and global) and BNG res 4.  Prints one JSON object (kernel ms from HIP events)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import mosaic_amd as M
    import bench as B
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n = 100_000_000
    x, y = B.gen_points(n, 0, 0x20250314, dev)
    out = {"points": n}

    def t(xx, yy, res, isys, reps=5):
        ms = []
        for _ in range(reps + 1):
            _, st = M.grid_longlatascellid(xx, yy, res, index_system=isys, stats=True)
            ms.append(st["kernel_ms"])
        return float(np.median(ms[1:]))

    out["h3_nyc_r9_ms"] = t(x, y, 9, M.H3IndexSystem())
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    gx = torch.rand(n, dtype=torch.float64, device=dev, generator=g).mul_(360.0).sub_(180.0)
    gy = torch.rand(n, dtype=torch.float64, device=dev, generator=g).mul_(180.0).sub_(90.0)
    out["h3_global_r9_ms"] = t(gx, gy, 9, M.H3IndexSystem())
    bx = x.mul(0).add_(torch.rand_like(x).mul_(58000.0).add_(503000.0))
    by = y.mul(0).add_(torch.rand_like(y).mul_(46000.0).add_(155000.0))
    out["bng_r4_ms"] = t(bx, by, 4, M.BNGIndexSystem())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
