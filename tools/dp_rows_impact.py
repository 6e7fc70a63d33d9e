"""The C3 chip table's rows mosaicFill's rule leaves undecided (core_stats "ambiguous": band
membership within the band's DouglasPeuckerSimplifier(0.01 r) margin, core/Mosaic.scala:75-84,
whose kept vertices depend on the start vertex of JTS BufferBuilder's output ring -- not
restated) and the pairs at stake: the C3 workload's points (1.25e8 uniform in the tract
extent, one GPU's share, numpy with the bench's seed scheme) that the row's chip contains
and that the join pairs with it -- pairs the reference would lose (a kept row it drops) or
add (a dropped row it keeps).  Both the count on the sample and the expectation from the
chip's area.  Host only (oracle.pip_join over the undecided rows' chips).
    python3 tools/dp_rows_impact.py > profiles/r6/c3_undecided_rows_impact.json
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import bench_workloads as W  # noqa: E402
import mosaic_amd as M  # noqa: E402
import oracle as O  # noqa: E402
import jts_overlay as JO  # noqa: E402
from geom_util import wkb_area  # noqa: E402


def main(n_points=125_000_000, chunk=10_000_000):
    t0 = time.time()
    P = W.tract_polygons()
    T = M.tessellate(P, M.H3IndexSystem(), 10)
    U = T.undecided
    t_tess = time.time() - t0
    n = len(U)
    boxes = []
    for i in range(n):
        pts = [p for pc in JO.wkb_rings(U.row(i)[2]) for r in pc for p in r]
        xs, ys = [p[0] for p in pts], [p[1] for p in pts]
        boxes.append((min(xs), min(ys), max(xs), max(ys)))
    x0, y0, x1, y1 = W.TRACT_EXTENT
    rng = np.random.default_rng(0x20250314)
    cx, cy = [], []
    for s in range(0, n_points, chunk):
        m = min(chunk, n_points - s)
        x, y = rng.uniform(x0, x1, m), rng.uniform(y0, y1, m)
        sel = np.zeros(m, bool)
        for b in boxes:
            sel |= (x >= b[0]) & (x <= b[2]) & (y >= b[1]) & (y <= b[3])
        cx.append(x[sel])
        cy.append(y[sel])
    x, y = np.concatenate(cx), np.concatenate(cy)
    pts, polys = O.pip_join(0, 10, x, y, U.cell, U.polygon_id, np.zeros(n, np.uint8), U.wkb_offsets, U.wkb)
    key = {(int(U.cell[i]), int(U.polygon_id[i])): i for i in range(n)}
    cells = O.h3_points_to_cells(x[pts], y[pts], 10) if len(pts) else np.zeros(0, np.int64)
    per = np.zeros(n, np.int64)
    for c, p in zip(cells.tolist(), polys.tolist()):
        per[key[(c, p)]] += 1
    ext = (x1 - x0) * (y1 - y0)
    rows = [{"cell": int(U.cell[i]), "polygon": int(U.polygon_id[i]), "kind": ["", "dp_sensitive", "unresolved"][U.kind[i]],
             "kept": bool(U.kept[i]), "core": bool(U.is_core[i]), "chip_area_deg2": wkb_area(U.row(i)[2]),
             "pairs_at_stake": int(per[i]), "expected_pairs": wkb_area(U.row(i)[2]) / ext * n_points}
            for i in range(n)]
    out = {"what": "C3 (74,000 tract-like polygons, H3 r10): rows left undecided by mosaicFill's rule and the "
                   "pairs at stake among %d uniform points (one GPU's share of C3)" % n_points,
           "rows_total": len(T), "undecided_rows": n, "core_stats": T.core_stats,
           "pairs_at_stake_total": int(per.sum()), "expected_pairs_total": float(sum(r["expected_pairs"] for r in rows)),
           "fraction_of_points": float(per.sum()) / n_points, "tessellate_s": round(t_tess, 2),
           "seconds": round(time.time() - t0, 1), "rows": rows}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
