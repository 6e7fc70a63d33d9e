#!/usr/bin/env python3
"""Re-derive H3's faceNeighbors table (mosaic_amd/csrc/h3_boundary.h kFaceNeighbors) from
the icosahedron geometry: for each face and each of its three edge quadrants, the
neighbour face, ccw 60-degree rotation and translation that carry lattice points just
beyond the edge onto the neighbour's lattice with the smallest displacement on the
sphere (both faces' gnomonic projections agree on the shared edge).  Every entry of the
table must be the unique best candidate.  Run: python tools/check_h3_face_neighbors.py"""
import itertools
import math
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_h3_tables as G  # noqa: E402
from gen_h3_edge_fixture import hex2d_to_geo  # noqa: E402


def table():
    src = open(os.path.join(HERE, "..", "mosaic_amd", "csrc", "h3_boundary.h")).read()
    body = src[src.index("kFaceNeighbors[20][4] = {"):]
    rows = re.findall(r"\{\{(\d+), 0, 0, 0, 0\}, \{([\d, ]+)\}, \{([\d, ]+)\}, \{([\d, ]+)\}\}", body)[:20]
    return {int(r[0]): {q + 1: tuple(int(v) for v in r[q + 1].split(",")) for q in range(3)} for r in rows}


def rot_ccw(c):
    i, j, k = c
    return G.norm_ijk(i + k, i + j, j + k)


def hex2d(c):
    i, j = c[0] - c[2], c[1] - c[2]
    return i - 0.5 * j, j * G.M_SQRT3_2


def dist(a, b):
    return math.acos(max(-1.0, min(1.0, math.sin(a[0]) * math.sin(b[0]) +
                                    math.cos(a[0]) * math.cos(b[0]) * math.cos(a[1] - b[1]))))


def main():
    res, max_dim, unit = 2, 14, 7
    T = table()
    assert len(T) == 20
    trans = set(itertools.permutations((2, 0, 2))) | set(itertools.permutations((2, 2, 0)))
    bad = 0
    for f in range(20):
        for q in (1, 2, 3):
            pts = sorted({G.norm_ijk(i, j, k) for i in range(20) for j in range(20) for k in range(20)})
            pts = [c for c in pts if max_dim < sum(c) <= max_dim + 2 and
                   ((3 if c[1] > 0 else 2) if c[2] > 0 else 1) == q][:30]
            best = None
            for g in range(20):
                if g == f:
                    continue
                for r in range(6):
                    for t in trans:
                        err = 0.0
                        for c in pts:
                            d = c
                            for _ in range(r):
                                d = rot_ccw(d)
                            d = G.norm_ijk(d[0] + t[0] * unit, d[1] + t[1] * unit, d[2] + t[2] * unit)
                            err = max(err, dist(hex2d_to_geo(*hex2d(c), f, res), hex2d_to_geo(*hex2d(d), g, res)))
                        if best is None or err < best[0]:
                            best = (err, (g, *G.norm_ijk(*t), r))
            ok = best[1] == T[f][q]
            bad += not ok
            print("face %2d quadrant %d: derived %s table %s %s" % (f, q, best[1], T[f][q], "ok" if ok else "MISMATCH"))
    print("all 60 entries derived" if not bad else "%d mismatches" % bad)
    return bad


if __name__ == "__main__":
    sys.exit(1 if main() else 0)
