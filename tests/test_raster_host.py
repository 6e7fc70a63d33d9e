"""The chip table's pixel index, checked against the oracle on the CPU (no GPU needed).

The streaming join kernel answers a point whose pixel is "pure" straight from the pixel
(mosaic_amd/csrc/chip_table.h "Pixel index", built by capi.cpp build_raster_*): one
certificate per pixel says that every point in it takes the same chip cell(s) and lies
in the interior / exterior of each of their chips.  `mgpu_test_raster_host` builds the
same table on the host and looks points up exactly as the kernel does
(mosaic_amd/csrc/raster.h), so every pure-pixel answer can be compared with the
oracle's join (H3 v3.7 geoToH3 / BNG pointToIndex + hash join + JTS contains, the
reference's path: H3IndexSystem.scala:168-170, BNGIndexSystem.scala:284-334,
ST_Contains.scala:21-44) -- on random points and on adversarial ones: chip vertices,
points on chip edges (core chips carry their hexagon, so hex edges too) and their ulp
neighbours.
"""
import ctypes
import os
import sys

import numpy as np
import pytest

import mosaic_amd as M
from mosaic_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle as O  # noqa: E402  (test infrastructure: the checker)
from test_pip_exact_host import adversarial, rings_of  # noqa: E402


def raster_lookup(c, res, x, y, hook="mgpu_test_raster_host"):
    n = len(x)
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    kind = np.empty(n, np.int8)
    first = np.empty(n, np.uint32)
    mask = np.empty(n, np.uint32)
    cpoly = np.empty(len(c), np.int32)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    N.check(getattr(N.lib(), hook)(c.index_system, res, len(c), p(c.cell), p(c.polygon_id), p(c.is_core),
                                   p(c.wkb_offsets), p(c.wkb), n, p(x), p(y), p(kind), p(first), p(mask), p(cpoly)))
    return kind, first, mask, cpoly


def adversarial_points(c, rng, n_chips):
    rows = rng.choice(len(c), min(n_chips, len(c)), replace=False)
    pts = []
    for r in rows:
        blob = bytes(c.wkb[c.wkb_offsets[r]:c.wkb_offsets[r + 1]])
        if blob:
            pts.append(adversarial(rings_of(blob), rng, k_rand=4))
    return np.concatenate(pts)


def check_raster(c, res, x, y, min_pure, hook="mgpu_test_raster_host"):
    kind, first, mask, cpoly = raster_lookup(c, res, x, y, hook)
    assert not (kind == 4).any(), "no pixel index was built"
    assert not (kind == 3).any()
    pure = kind <= 1
    assert pure.mean() >= min_pure, "pure fraction %.3f" % pure.mean()
    # the pixel answers as (point, polygon) pairs
    gi, gq = [], []
    for j in range(32):
        sel = np.nonzero((kind == 1) & (((mask >> j) & 1) == 1))[0]
        gi.append(sel)
        gq.append(cpoly[first[sel] + j])
    gi, gq = np.concatenate(gi), np.concatenate(gq)
    o = np.lexsort((gq, gi))
    gi, gq = gi[o], gq[o]
    op, oq = O.pip_join(c.index_system, res, x, y, c.cell, c.polygon_id, c.is_core, c.wkb_offsets, c.wkb)
    keep = pure[op]
    op, oq = op[keep], oq[keep]
    assert len(op) == len(gi) and np.array_equal(op, gi) and np.array_equal(oq, gq), \
        "pixel answers differ from the oracle (%d vs %d pairs)" % (len(gi), len(op))
    return pure.mean(), len(gi)


def test_raster_nyc_r9_uniform_and_adversarial(nyc_chips_r9):
    rng = np.random.default_rng(11)
    n = 400_000
    x = rng.uniform(-74.25559136315209, -73.7000090639354, n)
    y = rng.uniform(40.496115395170364, 40.91553277700258, n)
    frac, pairs = check_raster(nyc_chips_r9, 9, x, y, 0.85)
    assert pairs > 100_000
    a = adversarial_points(nyc_chips_r9, rng, 2500)
    check_raster(nyc_chips_r9, 9, a[:, 0], a[:, 1], 0.05)


def test_raster_nyc_r10(nyc_zones):
    c = M.tessellate(nyc_zones, M.H3IndexSystem(), 10)
    rng = np.random.default_rng(12)
    n = 200_000
    x = rng.uniform(-74.1, -73.8, n)
    y = rng.uniform(40.6, 40.85, n)
    check_raster(c, 10, x, y, 0.6)
    a = adversarial_points(c, rng, 2000)
    check_raster(c, 10, a[:, 0], a[:, 1], 0.02)


def test_raster_wrong_resolution_has_no_index(nyc_chips_r9):
    kind, _, _, _ = raster_lookup(nyc_chips_r9, 8, np.array([-73.9]), np.array([40.7]))
    assert kind[0] == 4


def test_raster_bng_london_r4():
    # (mgpu_test_raster_host builds BNG tables with their pixel index: the index is the
    # subject here; the join path builds it only with the raster_bng option)
    import bench_workloads as W
    c = M.tessellate(W.london_districts(), M.BNGIndexSystem(), 4)
    rng = np.random.default_rng(13)
    x, y = W.london_points(300_000, 14)
    check_raster(c, 4, x, y, 0.85)
    a = adversarial_points(c, rng, 3000)
    # plus whole-metre and sub-metre points on cell / pixel lines (pixels tile cells)
    e = rng.integers(503000, 561000, 20000).astype(np.float64)
    nn = rng.integers(155000, 201000, 20000).astype(np.float64)
    xs = np.concatenate([a[:, 0], e, np.nextafter(e, -np.inf), e + 0.999999])
    ys = np.concatenate([a[:, 1], nn, nn, np.nextafter(nn, np.inf)])
    check_raster(c, 4, xs, ys, 0.02)


def test_raster_bng_postcodes_r3_and_quadrant():
    z = M.Polygons.from_npz(os.path.join(ROOT, "tests", "golden", "london_postcode_zones.npz"))
    rng = np.random.default_rng(15)
    for res in (3, -4):
        c = M.tessellate(z, M.BNGIndexSystem(), res)
        kind, _, _, _ = raster_lookup(c, res, np.array([530000.0]), np.array([180000.0]))
        if kind[0] == 4:
            continue  # no dense grid at this resolution: nothing to check
        x = rng.uniform(503000, 561000, 100_000)
        y = rng.uniform(155000, 201000, 100_000)
        check_raster(c, res, x, y, 0.3)


def test_raster_skewed_fractal_polygons():
    import bench_workloads as W
    P = W.skewed_polygons()
    c = M.tessellate(P, M.H3IndexSystem(), 9)
    x, y = W.boundary_points(P, 200_000, 16, 0.003)
    check_raster(c, 9, x, y, 0.2)


def test_cell_answers_bng_london():
    # the fused join's per-cell answer grids (BNG cells with border chips): every answered
    # point's matches equal the oracle's, on random points, chip-edge adversaries and
    # whole-metre points on square lines
    import bench_workloads as W
    res = 3
    c = M.tessellate(W.london_districts(), M.BNGIndexSystem(), res)
    rng = np.random.default_rng(20)
    x, y = W.london_points(300_000, 21)
    hook = "mgpu_test_cell_answers_host"
    frac, pairs = check_raster(c, res, x, y, 0.3, hook)
    print("res %d: %.3f of the points answered, %d pairs" % (res, frac, pairs))
    assert pairs > 50_000
    a = adversarial_points(c, rng, 3000)
    e = rng.integers(503000, 561000, 20000).astype(np.float64)
    nn = rng.integers(155000, 201000, 20000).astype(np.float64)
    xs = np.concatenate([a[:, 0], e, np.nextafter(e, -np.inf), e + 0.999999])
    ys = np.concatenate([a[:, 1], nn, nn, np.nextafter(nn, np.inf)])
    check_raster(c, res, xs, ys, 0.02, hook)
    # res 4: border cells are 7.6% of the cells -- the builder leaves the grids out
    c4 = M.tessellate(W.london_districts(), M.BNGIndexSystem(), 4)
    kind, _, _, _ = raster_lookup(c4, 4, np.array([530000.0]), np.array([180000.0]), hook)
    assert kind[0] == 4


def test_cell_answers_bng_crowded_cells():
    # 40 nested squares: cells of 40 chips (no answer grid; their core masks use bit 15)
    # beside cells of 7 / 15 chips that have one -- the entries' flag must not be misread
    base, sc, res = (530000.0, 180000.0), 3000.0, 3
    sq = [(0.0, 0.0), (1.0, 0.0), (1.0, 1.0), (0.0, 1.0), (0.0, 0.0)]
    polys = [(pid, [[[(base[0] + sc * u * (1 + 0.01 * pid), base[1] + sc * v * (1 + 0.013 * pid))
                      for u, v in sq]]]) for pid in range(40, 0, -1)]
    c = M.tessellate(M.Polygons.from_lists(polys), M.BNGIndexSystem(), res)
    rng = np.random.default_rng(33)
    x = base[0] + sc * rng.uniform(-0.1, 1.6, 60_000)
    y = base[1] + sc * rng.uniform(-0.1, 1.6, 60_000)
    check_raster(c, res, x, y, 0.05, "mgpu_test_cell_answers_host")


def test_whole_cell_shortcut_nyc_r9(nyc_chips_r9):
    # H3 whole-cell chips (the reference's demoted border-set cells: one chip, the cell's
    # own hexagon) answer a point deep inside the cell without a candidate; every such
    # answer equals the oracle's JTS contains, on uniform points and chip-edge adversaries
    rng = np.random.default_rng(23)
    n = 400_000
    x = rng.uniform(-74.25559136315209, -73.7000090639354, n)
    y = rng.uniform(40.496115395170364, 40.91553277700258, n)
    hook = "mgpu_test_whole_cells_host"
    frac, pairs = check_raster(nyc_chips_r9, 9, x, y, 0.02, hook)
    print("whole-cell answers: %.3f of the points" % frac)
    a = adversarial_points(nyc_chips_r9, rng, 2500)
    check_raster(nyc_chips_r9, 9, a[:, 0], a[:, 1], 0.0, hook)


def test_whole_cell_shortcut_tracts_r10():
    # 400 tract-like polygons (the C3 generator on a small extent) at res 10
    import bench_workloads as W
    ext = (-74.3, 40.5, -73.9, 40.8)
    P = W.tract_polygons(n_cells=400, extent=ext)
    c = M.tessellate(P, M.H3IndexSystem(), 10)
    x, y = W.extent_points(ext, 300_000, 5)
    frac, _ = check_raster(c, 10, np.asarray(x), np.asarray(y), 0.01, "mgpu_test_whole_cells_host")
    print("whole-cell answers: %.3f of the points" % frac)


def _blob_hash(c):
    import ctypes
    import hashlib
    from mosaic_amd import _native as N
    out, nb = ctypes.c_void_p(), ctypes.c_int64()
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    N.check(N.lib().mgpu_chips_host_blob(0, len(c), p(c.cell), p(c.polygon_id), p(c.is_core), p(c.wkb_offsets),
                                         p(c.wkb), ctypes.byref(out), ctypes.byref(nb)))
    try:
        return nb.value, hashlib.sha256(ctypes.string_at(out.value, nb.value)).hexdigest()[:16]
    finally:
        N.lib().mgpu_host_free(out)


def test_nyc_r9_blob_bytes_pinned(nyc_zones, nyc_chips_r9):
    """The NYC r9 chip-table blob (mgpu_chips_host_blob: headers, strips, lattice grid,
    pixel index with its 16x16 sub-pixels) is byte-for-byte the one round 5's builder
    produced before its speed-ups (per-pixel edge lists, shared corner sines, row-parity
    verdicts, hashed classes): sha256 prefix of the whole blob, for round 5's chips (the
    Sutherland-Hodgman clip, kept as chip_geometry="sutherland_hodgman") and round 6's (the
    JTS overlay: one zero-area row fewer, other crossing vertices, separate pieces).  Blob
    version 13 adds the (empty) palette arrays: round 5's bytes were 86778112 /
    a145d3f4556f4f6a; the palette-compressed second level (MGPU_RASTER_PAL=1) gives
    28048896 / 9b2d36e77e294e9d and 27949568 / 615fde4ca9269ef5 -- off: slower on C2 (§4).
    The blob keeps input row ids, so the tessellator's row order is part of its bytes: since
    the tessellator emits each polygon's rows in cell order (the same rows: the order-free
    checksum in tests/test_tessellate_host.py is unchanged) the pins moved from
    22e5b22b2ea161e5 / fa0a071a53ada4f2 (the walk's interior-then-border order)."""
    import mosaic_amd as M
    sh = M.tessellate(nyc_zones, M.H3IndexSystem(), 9, chip_geometry="sutherland_hodgman")
    assert _blob_hash(sh) == (86778624, 'd985992852f4d714')
    assert _blob_hash(nyc_chips_r9) == (86478848, '7e17fca5c22213e6')
