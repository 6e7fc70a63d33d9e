"""Exactness of the join's st_contains path, on the CPU (no GPU needed).

The device chip table answers st_contains(chip, point) by an envelope test, a
per-chip 16x16 classification grid (a cell whose widened rectangle meets no edge
takes the PointLocator verdict of its centre) and, for mixed cells, a ray crossing
over the edges of the point's y-strip (mosaic_amd/csrc/pip_core.h,
chip_table.h).  `mgpu_test_chip_contains_host` builds that same table on the host
and evaluates both that path and the sequential JTS PointLocator
(RayCrossingCounter + CGAlgorithmsDD, the reference's MosaicGeometryJTS.contains ->
JTS Geometry.contains, MosaicGeometryJTS.scala:197); they must agree on every
point, adversarial ones included: exact vertices, points on edges, points on and
one ulp either side of grid-cell and strip boundaries, envelope corners.  A sample is
also checked against the oracle's own WKB-parsing st_contains.
"""
import ctypes
import struct
import sys
import os

import numpy as np
import pytest

import mosaic_amd as M
from mosaic_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402  (test infrastructure: the checker)


def rings_of(blob):
    """Rings of a Polygon / MultiPolygon WKB (either byte order) as (k, 2) arrays."""
    out = []

    def rd(off):
        e = ">" if blob[off] == 0 else "<"
        t = struct.unpack_from(e + "I", blob, off + 1)[0] & 0xFFFF
        off += 5
        if t % 1000 == 3:
            nr = struct.unpack_from(e + "I", blob, off)[0]
            off += 4
            for _ in range(nr):
                n = struct.unpack_from(e + "I", blob, off)[0]
                off += 4
                out.append(np.frombuffer(blob, dtype=e + "f8", count=2 * n, offset=off).reshape(n, 2).astype(float))
                off += 16 * n
        else:
            n = struct.unpack_from(e + "I", blob, off)[0]
            off += 4
            for _ in range(n):
                off = rd(off)
        return off

    rd(0)
    return out


def adversarial(rings, rng, k_rand=24):
    allv = np.concatenate(rings)
    x0, y0 = allv.min(0)
    x1, y1 = allv.max(0)
    pts = [allv, rng.uniform([x0, y0], [x1, y1], (k_rand, 2))]
    # on edges: midpoints and random fractions (rounded to doubles: on or next to the edge)
    for r in rings:
        a, b = r[:-1], r[1:]
        t = rng.uniform(0, 1, (len(a), 1))
        pts += [(a + b) / 2, a + (b - a) * t]
    # grid-cell / strip boundaries (16 cells per axis) and their ulp neighbours
    gx = x0 + (x1 - x0) * np.arange(17) / 16
    gy = y0 + (y1 - y0) * np.arange(17) / 16
    cx = rng.choice(gx, 12)
    cy = rng.uniform(y0, y1, 12)
    pts += [np.stack([cx, cy], 1), np.stack([np.nextafter(cx, -np.inf), cy], 1), np.stack([np.nextafter(cx, np.inf), cy], 1)]
    cy2 = rng.choice(gy, 12)
    cx2 = rng.uniform(x0, x1, 12)
    pts += [np.stack([cx2, cy2], 1), np.stack([cx2, np.nextafter(cy2, -np.inf)], 1), np.stack([cx2, np.nextafter(cy2, np.inf)], 1)]
    # envelope corners and vertex ulp neighbours
    pts += [np.array([[x0, y0], [x1, y1], [x0, y1], [x1, y0]])]
    v = allv[rng.integers(0, len(allv), 8)]
    pts += [np.stack([np.nextafter(v[:, 0], np.inf), v[:, 1]], 1), np.stack([v[:, 0], np.nextafter(v[:, 1], -np.inf)], 1)]
    return np.concatenate(pts)


def run(c, rows, x, y):
    n = len(rows)
    rows = np.ascontiguousarray(rows, dtype=np.int64)
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    a = np.empty(n, dtype=np.int8)
    b = np.empty(n, dtype=np.int8)
    p = lambda arr: arr.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    st = N.lib().mgpu_test_chip_contains_host(c.index_system, len(c), p(c.cell), p(c.polygon_id), p(c.is_core),
                                               p(c.wkb_offsets), p(c.wkb), n, p(rows), p(x), p(y), p(a), p(b))
    N.check(st)
    return a, b


def check_table(c, seed, max_chips=None, oracle_sample=4000):
    rng = np.random.default_rng(seed)
    border = np.nonzero(c.is_core == 0)[0]
    if max_chips is not None and len(border) > max_chips:
        border = rng.choice(border, max_chips, replace=False)
    rows, xs, ys = [], [], []
    for r in border:
        blob = bytes(c.wkb[c.wkb_offsets[r]:c.wkb_offsets[r + 1]])
        pts = adversarial(rings_of(blob), rng)
        rows.append(np.full(len(pts), r))
        xs.append(pts[:, 0])
        ys.append(pts[:, 1])
    rows, x, y = np.concatenate(rows), np.concatenate(xs), np.concatenate(ys)
    join_path, locator = run(c, rows, x, y)
    bad = np.nonzero(join_path != locator)[0]
    assert len(bad) == 0, "grid/strip path differs from the PointLocator at %d of %d points, e.g. row %d (%r, %r)" % (
        len(bad), len(rows), rows[bad[0]], x[bad[0]], y[bad[0]])
    assert locator.sum() > 0 and (locator == 0).sum() > 0
    k = rng.choice(len(rows), min(oracle_sample, len(rows)), replace=False)
    ref = np.array([O.st_contains(bytes(c.wkb[c.wkb_offsets[rows[i]]:c.wkb_offsets[rows[i] + 1]]), x[i], y[i])
                    for i in k], dtype=np.int8)
    assert np.array_equal(join_path[k], ref)
    return len(rows)


def test_nyc_r9_border_chips_exact(nyc_chips_r9):
    assert check_table(nyc_chips_r9, 1) > 300_000


def test_nyc_r8_border_chips_exact(nyc_zones):
    assert check_table(M.tessellate(nyc_zones, M.H3IndexSystem(), 8), 2) > 50_000


def test_london_bng_border_chips_exact():
    z = M.Polygons.from_npz(os.path.join(ROOT, "tests", "golden", "london_postcode_zones.npz"))
    c = M.tessellate(z, M.BNGIndexSystem(), 3)
    assert check_table(c, 3, max_chips=3000) > 30_000


def test_null_geometry_rows():
    z = M.Polygons.from_npz(os.path.join(ROOT, "tests", "golden", "nyc_taxi_zones.npz"))
    c = M.tessellate(z, M.H3IndexSystem(), 9, keep_core_geometries=False)
    core = np.nonzero(c.is_core)[0][:10]
    a, b = run(c, core, np.zeros(len(core)), np.zeros(len(core)))
    assert (a == -1).all() and (b == -1).all()
