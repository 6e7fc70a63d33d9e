#!/usr/bin/env python3
"""What LDS staging of border-chip geometry could save in C3's binned join (host only).

The binned join's tile is kTile = 256 consecutive slots of one of the 8 x 8 bins (64 bins
over the table's bounding box, capi.cpp plan_bins).  One bin of C3 holds 1.25e8 / 64 points
in input order; this draws that many uniform points inside one interior bin, takes their
H3 res-10 cells (oracle), and counts per tile the border-chip candidates (chips of the
point's cell that are not core: phase 1's candidate list; the whole-cell shortcut is
ignored, so this over-counts candidates slightly), the distinct chips among them and the
bytes of their headers + strip edges.  Staging only pays where a chip is read by several
candidates of one tile: the reuse factor (candidates / distinct chips) is the most a tile's
LDS copy could divide the edge reads by.  For comparison the same points in cell order
(north_star's sort + merge join) are tiled the same way.

  python3 tools/c3_tile_reuse.py [--cache=/tmp/c3_table.npz] [--bin=3,4]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

K_TILE = 256
HDR_BYTES = 128  # mgpu::ChipHdr (chip_table.h)
EDGE_BYTES = 32  # one strip edge record (x1, y1, x2, y2)


def chip_table(cache):
    if cache and os.path.exists(cache):
        z = np.load(cache)
        return {k: z[k] for k in ("cell", "polygon_id", "is_core", "wkb_offsets", "wkb")}
    import bench_workloads as W
    import mosaic_amd as M
    c = M.tessellate(W.tract_polygons(), M.H3IndexSystem(), 10, keep_core_geometries=False)
    d = {"cell": c.cell, "polygon_id": c.polygon_id, "is_core": c.is_core, "wkb_offsets": c.wkb_offsets, "wkb": c.wkb}
    if cache:
        np.savez(cache, **d)
    return d


def edge_count(b):
    """edges (vertices - 1 per ring) of one chip's WKB (Polygon / MultiPolygon)"""
    import struct
    if not b:
        return 0
    f = "<" if b[0] == 1 else ">"
    t = struct.unpack(f + "I", b[1:5])[0] % 1000
    p, parts = 5, 1
    if t == 6:
        parts = struct.unpack(f + "I", b[p:p + 4])[0]
        p += 4
    e = 0
    for _ in range(parts):
        if t == 6:
            p += 5
        nr = struct.unpack(f + "I", b[p:p + 4])[0]
        p += 4
        for _ in range(nr):
            nv = struct.unpack(f + "I", b[p:p + 4])[0]
            p += 4 + 16 * nv
            e += max(nv - 1, 0)
    return e


def tiles(order, first, cnt, border, chip_bytes):
    """per tile of K_TILE points in `order`: candidates, distinct chips, their bytes"""
    cand, dist, byts = [], [], []
    for t0 in range(0, len(order) - K_TILE + 1, K_TILE):
        pts = order[t0:t0 + K_TILE]
        chips = []
        for p in pts:
            f, c = first[p], cnt[p]
            if c:
                chips.extend(int(f + j) for j in range(c) if border[f + j])
        u = set(chips)
        cand.append(len(chips))
        dist.append(len(u))
        byts.append(int(sum(chip_bytes(j) for j in u)))
    return np.array(cand), np.array(dist), np.array(byts)


def main():
    import oracle as O
    cache = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--cache=")), "/tmp/c3_table.npz")
    bx, by = map(int, next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--bin=")), "3,4").split(","))
    T = chip_table(cache)
    cell = T["cell"].astype(np.int64)
    order = np.lexsort((T["polygon_id"], cell))  # the blob's chip order (cell, polygon id)
    cs, core = cell[order], T["is_core"][order].astype(bool)
    wkb, off, memo = T["wkb"], T["wkb_offsets"], {}

    def chip_bytes(j):  # (strips duplicate an edge into each strip it spans: ~1.5x, capi.cpp build_strips)
        if j not in memo:
            r = order[j]
            memo[j] = HDR_BYTES + int(1.5 * EDGE_BYTES * edge_count(bytes(wkb[off[r]:off[r + 1]])))
        return memo[j]
    ucell, ufirst, ucnt = np.unique(cs, return_index=True, return_counts=True)
    x0, y0, x1, y1 = -77.5, 39.5, -73.5, 42.5
    W, H = (x1 - x0) / 8, (y1 - y0) / 8
    n = 125_000_000 // 64
    rng = np.random.default_rng(7)
    lon = rng.uniform(x0 + bx * W, x0 + (bx + 1) * W, n)
    lat = rng.uniform(y0 + by * H, y0 + (by + 1) * H, n)
    pc = np.asarray(O.h3_points_to_cells(lon, lat, 10, threads=os.cpu_count()), dtype=np.int64)
    k = np.searchsorted(ucell, pc)
    k = np.minimum(k, len(ucell) - 1)
    hit = ucell[k] == pc
    first = np.where(hit, ufirst[k], 0)
    cnt = np.where(hit, ucnt[k], 0)
    border = ~core
    res = {"bin": [bx, by], "points": n, "tile": K_TILE, "border_candidates_per_point": float(
        np.sum([border[f:f + c].sum() for f, c in zip(first[:200000], cnt[:200000])]) / 200000)}
    for name, ordr in (("binned (input order within the bin)", np.arange(n)),
                       ("cell order (sort + merge)", np.argsort(pc, kind="stable"))):
        sample = ordr[:K_TILE * 2000]  # 2000 tiles
        c, d, b = tiles(sample, first, cnt, border, chip_bytes)
        res[name] = {"candidates_per_tile": float(c.mean()), "distinct_chips_per_tile": float(d.mean()),
                     "reuse": float(c.sum() / max(d.sum(), 1)), "distinct_chip_kb_per_tile": float(b.mean() / 1024)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
