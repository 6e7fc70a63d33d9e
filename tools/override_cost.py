#!/usr/bin/env python3
"""Cost of the libm override pass: the C2 join of 1e8 uniform points,
clean, and with the NYC r9 adversarial points (cell corners: the host's libm moves some
of their cells) written over as many of them -- wall time of the synchronous call,
median of --reps, one JSON line."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=9)
    ap.add_argument("--adv", type=int, default=0, help="adversarial points written in (0: all of them)")
    a = ap.parse_args()
    import mosaic_amd as M
    from test_gpu_parity import adversarial_points
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    zones = M.Polygons.from_npz(os.path.join(ROOT, "tests", "golden", "nyc_taxi_zones.npz"))
    c = M.tessellate(zones, M.H3IndexSystem(), 9)
    chips = c.upload(M.default_context(dev))
    ax, ay = adversarial_points(c)
    if a.adv:
        pick = np.random.default_rng(3).choice(len(ax), min(a.adv, len(ax)), replace=False)
        ax, ay = ax[pick], ay[pick]
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    x = torch.rand(a.points, dtype=torch.float64, device=dev, generator=g) * 0.5555 - 74.2555
    y = torch.rand(a.points, dtype=torch.float64, device=dev, generator=g) * 0.4194 + 40.4961
    x2, y2 = x.clone(), y.clone()
    at = torch.randperm(a.points, device=dev, generator=g)[:len(ax)].sort().values
    x2[at] = torch.tensor(ax, dtype=torch.float64, device=dev)
    y2[at] = torch.tensor(ay, dtype=torch.float64, device=dev)
    cap = int(a.points * 0.5) + 1024
    op = torch.empty(cap, dtype=torch.int64, device=dev)
    oq = torch.empty(cap, dtype=torch.int32, device=dev)
    out = {}
    for name, (xx, yy) in (("clean", (x, y)), ("adversarial", (x2, y2))):
        ts, st = [], None
        for _ in range(a.reps + 1):
            torch.cuda.synchronize()
            t = time.perf_counter()
            r = M.pip_join(xx, yy, chips, 9, out=(op, oq), capacity=cap)
            ts.append(time.perf_counter() - t)
            st = r.stats
        out[name] = {"ms": float(np.median(ts[1:])) * 1e3, "near_ties": st["n_near_ties"],
                     "libm_overrides": st["libm_overrides"], "pairs": len(r)}
    out["ratio"] = out["adversarial"]["ms"] / out["clean"]["ms"]
    out["adversarial_points"] = len(ax)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
