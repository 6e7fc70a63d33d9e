#!/usr/bin/env python3
"""tests/golden/h3_edge_points.npz: points on and within 1e-14 deg of H3 cell corners and
edges, with the oracle's cells -- the adversarial fixture of the exact H3 route.

For random points on the sphere at resolution `res` the oracle's geoToHex2d gives
(face, hex2d); the nearest lattice centre's six corners (distance 1/sqrt3 at 30 + 60k
degrees) and points along its six edges are mapped back to (lon, lat) by H3's
_hex2dToGeo, then perturbed by at most 1e-14 degrees.  Expected cells come from the
oracle twice: with glibc's libm (the reference's) and with correctly rounded libm
(libquadmath) -- they differ only where glibc misrounds an argument that decides the
cell, and the device route (correctly rounded by construction) must equal the latter
everywhere.  Run: python tools/gen_h3_edge_fixture.py (a few seconds).
"""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import oracle as O  # noqa: E402
import gen_h3_tables as G  # noqa: E402

SQRT7 = 2.6457513110645905905016157536392604257102
AP7_ROT = 0.333473172251832115336090755351601070065900389
SIN60 = 0.8660254037844386467637231707529361834714


def hex2d_to_geo(x, y, face, res):
    """H3 _hex2dToGeo (substrate 0), in radians."""
    r = math.hypot(x, y)
    lat0, lon0 = G.FACE_CENTER_GEO[face]
    if r < 1e-16:
        return lat0, lon0
    theta = math.atan2(y, x)
    for _ in range(res):
        r /= SQRT7
    r = math.atan(r * G.RES0_U_GNOMONIC)
    if res % 2:
        theta = G.pos_angle(theta + AP7_ROT)
    theta = G.pos_angle(G.FACE_AXES_AZ_CII[face][0] - theta)
    return G.az_distance(lat0, lon0, theta, r)


def nearest_centre(x, y):
    j0 = round(y / SIN60)
    best = None
    for j in (j0 - 1, j0, j0 + 1):
        i = round(x + 0.5 * j)
        for ii in (i - 1, i, i + 1):
            cx, cy = ii - 0.5 * j, j * SIN60
            d = (cx - x) ** 2 + (cy - y) ** 2
            if best is None or d < best[0]:
                best = (d, cx, cy)
    return best[1], best[2]


def main():
    rng = np.random.default_rng(20261017)
    plan = {0: 600, 1: 600, 2: 600, 5: 1200, 9: 4000, 10: 4000, 15: 4000}  # seed points per resolution
    lon, lat, res_col = [], [], []
    for res, n_seed in plan.items():
        u = rng.uniform(-1.0, 1.0, n_seed)
        slon = rng.uniform(-math.pi, math.pi, n_seed)
        slat = np.arcsin(u)
        for k in range(n_seed):
            face, vx, vy = O.h3_geo_to_hex2d(float(slat[k]), float(slon[k]), res)
            cx, cy = nearest_centre(vx, vy)
            pts = []
            for c in range(6):  # corners
                a = math.radians(30 + 60 * c)
                pts.append((cx + math.cos(a) / math.sqrt(3), cy + math.sin(a) / math.sqrt(3), 0.0))
            for c in range(6):  # a random point on each edge, perturbed
                a0, a1 = math.radians(30 + 60 * c), math.radians(90 + 60 * c)
                t = rng.uniform()
                ex = cx + ((1 - t) * math.cos(a0) + t * math.cos(a1)) / math.sqrt(3)
                ey = cy + ((1 - t) * math.sin(a0) + t * math.sin(a1)) / math.sqrt(3)
                pts.append((ex, ey, 1e-14))
            for (px, py, eps) in pts:
                la, lo = hex2d_to_geo(px, py, face, res)
                lo_d, la_d = math.degrees(lo), math.degrees(la)
                if eps:
                    lo_d += rng.uniform(-eps, eps)
                    la_d += rng.uniform(-eps, eps)
                lon.append(lo_d)
                lat.append(la_d)
                res_col.append(res)
    lon = np.array(lon)
    lat = np.array(lat)
    res_col = np.array(res_col, dtype=np.int8)
    cell_glibc = np.empty(len(lon), np.int64)
    cell_cr = np.empty(len(lon), np.int64)
    for res in plan:
        m = res_col == res
        cell_glibc[m] = O.h3_points_to_cells(lon[m], lat[m], res)
        with O.h3_libm("cr"):
            cell_cr[m] = O.h3_points_to_cells(lon[m], lat[m], res)
    out = os.path.join(ROOT, "tests", "golden", "h3_edge_points.npz")
    np.savez_compressed(out, lon=lon, lat=lat, res=res_col, cell_glibc=cell_glibc, cell_cr=cell_cr)
    d = np.count_nonzero(cell_glibc != cell_cr)
    print("%d points, %d cells where glibc's libm and correct rounding disagree -> %s" % (len(lon), d, out))


if __name__ == "__main__":
    main()
