#!/usr/bin/env python3
"""Throughput of the BNG StringType formatter on the device (mgpu_bng_format_device):
1e8 BNG res-4 ids of UPRN-like London points (C4's workload), HIP events around the call.
Prints one JSON line: ids/s, algorithmic GB/s (8 B read + 8 B offset + the chars written
per id, plus the count pass's 8 B read) against 8 TB/s."""
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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    bng = M.BNGIndexSystem()
    x, y = W.london_points(n, 7, dev)
    cells = bng.points_to_index(x, y, 4)
    del x, y
    for _ in range(2):
        chars, off = bng.format_device(cells)
    torch.cuda.synchronize(dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    a.record()
    for _ in range(reps):
        chars, off = bng.format_device(cells)
    b.record()
    torch.cuda.synchronize(dev)
    ms = a.elapsed_time(b) / reps
    nbytes = int(chars.numel())
    # count pass 8 B read; write pass 8 B read + 8 B offset + the characters
    alg = 8.0 * n + 8.0 * n + 8.0 * n + nbytes
    print(json.dumps({"what": "mgpu_format_cells_device, BNG res 4 ids of C4 points", "ids": n, "chars": nbytes,
                      "ms": ms, "ids_per_s": n / (ms * 1e-3), "alg_GBps": alg / (ms * 1e-3) / 1e9,
                      "frac_of_8TBps": alg / (ms * 1e-3) / 8e12,
                      "sample": bytes(chars[:off[3]].cpu().numpy()).decode()}), flush=True)


if __name__ == "__main__":
    main()
