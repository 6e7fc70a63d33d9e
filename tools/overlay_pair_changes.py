"""Pairs that change between round 5's border chips (the Sutherland-Hodgman clip) and round
6's (JTS OverlayNG's cut, mosaic_amd/csrc/jts_overlay.h), on adversarial points a few ulps
from every polygon-edge x cell-edge crossing (tests/geom_util.crossing_adversaries): NYC r9
and the C4 London-like districts at BNG res 3 / 4 (plus 0.01-m points on the square lines
near each crossing), and on 2M uniform points (NYC bbox).  Both tables are joined by the
ORACLE (oracle.pip_join: the reference's join + JTS PointLocator); host only.
    python3 tools/overlay_pair_changes.py > profiles/r6/overlay_pair_changes.json
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
from geom_util import crossing_adversaries  # noqa: E402
from test_tessellate_host import _bng_cell_rings, _h3_cell_rings  # noqa: E402
import jts_overlay as JO  # noqa: E402


def pairs(t, code, res, x, y):
    p, q = O.pip_join(code, res, x, y, t.cell, t.polygon_id, t.is_core, t.wkb_offsets, t.wkb)
    return set(zip(p.tolist(), q.tolist()))


def compare(name, P, isys, res, cell_rings_of, grid_step=None, uniform=None):
    t0 = time.time()
    old = M.tessellate(P, isys, res, chip_geometry="sutherland_hodgman")
    new = M.tessellate(P, isys, res)
    x, y = crossing_adversaries(P, new, cell_rings_of, grid_step=grid_step)
    po, pn = pairs(old, isys.code, res, x, y), pairs(new, isys.code, res, x, y)
    d = po ^ pn

    def doubled(ps):  # points matched by two polygons (the districts / zones tile the plane)
        from collections import Counter
        return sum(1 for v in Counter(i for i, _ in ps).values() if v > 1)
    out = {"workload": name, "rows_round5": len(old), "rows_round6": len(new), "adversarial_points": int(len(x)),
           "pairs_round5": len(po), "pairs_round6": len(pn), "pairs_only_round5": len(po - pn),
           "pairs_only_round6": len(pn - po), "points_changed": len({i for i, _ in d}),
           "points_in_two_polygons_round5": doubled(po), "points_in_two_polygons_round6": doubled(pn),
           "chip_stats": {k: v for k, v in new.core_stats.items() if k in
                          ("overlay_chips", "multi_piece", "coerced", "coerce_nodes", "lower_dim")}}
    if uniform is not None:
        ux, uy = uniform
        uo, un = pairs(old, isys.code, res, ux, uy), pairs(new, isys.code, res, ux, uy)
        out.update({"uniform_points": int(len(ux)), "uniform_pairs_changed": len(uo ^ un)})
    out["seconds"] = round(time.time() - t0, 1)
    print(json.dumps(out), file=sys.stderr)
    return out


def main():
    res = []
    P = W.nyc_zones()
    rng = np.random.default_rng(0x20250314)
    x0, y0, x1, y1 = P.bounds()
    uni = (rng.uniform(x0, x1, 2_000_000), rng.uniform(y0, y1, 2_000_000))
    res.append(compare("NYC 263 zones, H3 r9", P, M.H3IndexSystem(), 9, lambda c, w: _h3_cell_rings(c), uniform=uni))
    L = W.london_districts()
    for r in (3, 4):
        edge = 10.0 ** (6 - r)
        res.append(compare("C4 London-like districts, BNG r%d" % r, L, M.BNGIndexSystem(), r,
                           lambda c, w, e=edge: _bng_cell_rings([q for pc in JO.wkb_rings(w) for q in pc], e),
                           grid_step=0.01))
    print(json.dumps({"what": __doc__.split("\n")[0:6], "results": res}, indent=1))


if __name__ == "__main__":
    main()
