"""grid_tessellateexplode across icosahedron faces, and H3 cell geometry (host, no GPU).

Known answers from the reference's own documentation: the MULTIPOLYGON of
docs/source/api/spatial-indexing.rst:539-552 tessellated at H3 res 0 (8 chips, all
border, one of them a MULTIPOLYGON) and its grid_polyfill (:216-219, the cells whose
centre lies in the polygon); the res-9 core chips of NYC taxi zone 1 shown in
docs/source/usage/kepler.ipynb (cell 23 output).  Invariants on multi-face polygons:
chips of one cell never repeat, chip areas add up to the polygon's area, and the join
over the chips equals containment in the original polygons.  The cell geometry
(h3_boundary.h, h3ToGeoBoundary / h3ToGeo) is checked against geoToH3: every centre
maps back to its cell, every vertex nudged towards the centre too.
"""
import ctypes

import numpy as np
import pytest

import mosaic_amd as M
from geom_util import nyc_points
import oracle as O
from mosaic_amd import _native
from geom_util import brute_force_pairs, polygons_area, wkb_area, wkt_to_parts

DOC_WKT = "MULTIPOLYGON (((30 20, 45 40, 10 40, 30 20)), ((15 5, 40 10, 10 20, 5 10, 15 5)))"
DOC_TESSELLATE_RES0 = [577481099093999615, 578044049047420927, 578782920861286399, 577023702256844799,
                       577938495931154431, 577586652210266111, 577269992861466623, 578360708396220415]
DOC_MULTIPOLYGON_CHIP = 577586652210266111  # "[01 06 00 ...": the chip meets both parts
DOC_POLYFILL_RES0 = [577586652210266111, 578360708396220415, 577269992861466623]
KEPLER_ZONE1_RES9_CORE = [
    617733150781997055, 617733150856445951, 617733150856970239, 617733150784094207, 617733150843600895,
    617733150843863039, 617733150844125183, 617733150784880639, 617733150844387327, 617733150844649471,
    617733150785404927, 617733150844911615, 617733150785667071, 617733150845173759, 617733150785929215,
    617733150786453503, 617733150846222335, 617733150847270911, 617733150847795199, 617733150848057343]


def _P(a):
    return ctypes.c_void_p(a.ctypes.data)


def cell_geometry(cells):
    cells = np.ascontiguousarray(cells, dtype=np.int64)
    n = len(cells)
    xy = np.zeros((n, 20))
    nv = np.zeros(n, np.int32)
    c = np.zeros((n, 2))
    _native.check(_native.lib().mgpu_test_h3_boundary_host(_P(cells), n, _P(xy), _P(nv), _P(c)))
    return xy.reshape(n, 10, 2), nv, c


def _wkb(c, i):
    return bytes(c.wkb[c.wkb_offsets[i]:c.wkb_offsets[i + 1]])


def _check_invariants(P, c):
    for k, pid in enumerate(P.poly_id):
        rows = np.nonzero(c.polygon_id == pid)[0]
        assert len(np.unique(c.cell[rows])) == len(rows)
        area = sum(wkb_area(_wkb(c, i)) for i in rows)
        assert area == pytest.approx(polygons_area(P, k), rel=1e-9), pid


def test_doc_multipolygon_res0():
    P = M.Polygons.from_lists([(1, wkt_to_parts(DOC_WKT))])
    c = M.tessellate(P, M.H3IndexSystem(), 0)
    assert sorted(c.cell.tolist()) == sorted(DOC_TESSELLATE_RES0)
    assert not c.is_core.any()
    k = int(np.nonzero(c.cell == DOC_MULTIPOLYGON_CHIP)[0][0])
    w = _wkb(c, k)
    assert int.from_bytes(w[1:5], "little" if w[0] == 1 else "big") == 6
    _check_invariants(P, c)
    # grid_polyfill: the cells whose centre lies in the polygon
    _, _, centre = cell_geometry(c.cell)
    wkb_poly = M.Polygons.from_lists([(1, wkt_to_parts(DOC_WKT))])
    from geom_util import polygon_set_wkbs
    (_, w_all), = polygon_set_wkbs(wkb_poly)
    inside = [int(c.cell[i]) for i in range(len(c)) if O.st_contains(w_all, centre[i, 0], centre[i, 1])]
    assert sorted(inside) == sorted(DOC_POLYFILL_RES0)


@pytest.mark.parametrize("res", [1, 2, 3])
def test_doc_multipolygon_finer(res):
    P = M.Polygons.from_lists([(1, wkt_to_parts(DOC_WKT))])
    c = M.tessellate(P, M.H3IndexSystem(), res, core_rule="clip")
    _check_invariants(P, c)
    # (H3 children are not nested in their parents' boundaries, so no parent invariant)
    assert len(c) > {1: 20, 2: 100, 3: 500}[res]


def test_kepler_zone1_core_chips(nyc_zones):
    """The notebook shows the first 20 rows of zone 1's res-9 chips ("only showing top 20
    rows"), all `is_core = true` -- mosaicFill emits core chips first.  The listing comes
    from a Mosaic older than the one under /root/reference (before v0.3.11's issue-360
    change of the tessellation, CHANGELOG.md): its core rows include cells whose centre
    lies only 0.60 r from the boundary (r = 0.4.3's getBufferRadius, 0.0041 deg here), so
    0.4.3's polyfill(buffer(-r)) does not produce them; every one of them is at least 1.05
    circumradii deep, i.e. wholly inside -- the clip rule's core set holds them all.  The
    listing pins no border row either way (test_mosaicfill_rule_*)."""
    k = int(np.nonzero(nyc_zones.poly_id == 1)[0][0])
    P = nyc_zones.select([k])
    clip = M.tessellate(P, M.H3IndexSystem(), 9, core_rule="clip")
    assert set(KEPLER_ZONE1_RES9_CORE) <= set(clip.cell[clip.is_core.astype(bool)].tolist())
    mf = M.tessellate(P, M.H3IndexSystem(), 9)
    assert sorted(mf.cell.tolist()) == sorted(clip.cell.tolist())
    missing = set(KEPLER_ZONE1_RES9_CORE) - set(mf.cell[mf.is_core.astype(bool)].tolist())
    assert len(missing) == 7  # the listing's cells 0.60-0.94 r deep (an older radius)


def _star(cx, cy, r0, r1, k, seed):
    rng = np.random.default_rng(seed)
    ang = np.sort(rng.uniform(0, 2 * np.pi, k))[::1]
    rad = rng.uniform(r0, r1, k)
    shell = [(cx + r * np.cos(a), cy + r * np.sin(a)) for a, r in zip(ang, rad)]
    shell.append(shell[0])
    hole = [(cx + 0.1 * r0 * np.cos(a), cy + 0.1 * r0 * np.sin(a)) for a in np.linspace(2 * np.pi, 0, 9)]
    return [[shell, hole]]


def test_multi_face_polygons_join_equals_brute_force():
    """Polygons across the face 4 / face 9 edge, around an icosahedron vertex (pentagon
    base cells) and across several faces: invariants at res 2-5, and the join over the
    chips at res 5 equals containment in the original polygons."""
    _, _, pent = cell_geometry([(1 << 59) | (bc << 45) | 0x1FFFFFFFFFFF for bc in (14, 24, 38)])
    P = M.Polygons.from_lists([
        (1, _star(15.0, 5.0, 2.0, 4.0, 40, 1)),               # across the face 4 / 9 edge
        (2, _star(pent[0, 0], pent[0, 1], 1.0, 3.0, 30, 2)),  # around a pentagon
        (3, _star(pent[1, 0], pent[1, 1], 0.5, 2.0, 25, 3)),
        (4, _star(-40.0, -30.0, 6.0, 12.0, 50, 4)),           # large, several faces
    ])
    # (geometric invariants of the clip: chips tile the polygon.  mosaicFill's rule at
    # these coarse resolutions promotes / drops cells whose size differs from the
    # centroid cell's -- test_mosaicfill_rule_coarse_cells)
    for res in (2, 3, 4, 5):
        c = M.tessellate(P, M.H3IndexSystem(), res, core_rule="clip")
        _check_invariants(P, c)
    rng = np.random.default_rng(5)
    xs, ys = [], []
    for (cx, cy, r) in [(15.0, 5.0, 4.0), (pent[0, 0], pent[0, 1], 3.0), (pent[1, 0], pent[1, 1], 2.0),
                        (-40.0, -30.0, 12.0)]:
        xs.append(rng.uniform(cx - r, cx + r, 4000))
        ys.append(rng.uniform(cy - r, cy + r, 4000))
    x, y = np.concatenate(xs), np.concatenate(ys)
    pts, polys = O.pip_join(0, 5, x, y, c.cell, c.polygon_id, c.is_core, c.wkb_offsets, c.wkb)
    got = set(zip(pts.tolist(), polys.tolist()))
    want = brute_force_pairs(P, x, y, O)
    # chips are cell polygons with straight lon/lat edges; a point between such an edge
    # and the true (gnomonic) cell border is indexed to the neighbour: vanishingly rare
    assert len(got ^ want) <= len(want) // 2000, (len(got ^ want), len(want))


@pytest.mark.parametrize("res", [0, 1, 2, 3, 5, 8, 11, 15])
def test_cell_geometry_consistent_with_geo_to_h3(res):
    rng = np.random.default_rng(40 + res)
    n = 4000
    lon = rng.uniform(-180, 180, n)
    lat = np.degrees(np.arcsin(rng.uniform(-1, 1, n)))
    cells = np.unique(O.h3_points_to_cells(lon, lat, res))
    if res <= 1:  # every base cell / all res-1 cells, pentagons included
        cells = np.unique(np.concatenate([cells, O.h3_points_to_cells(*_sphere_grid(), res)]))
    xy, nv, centre = cell_geometry(cells)
    assert np.array_equal(O.h3_points_to_cells(centre[:, 0], centre[:, 1], res), cells)
    pent = np.array([((int(h) >> 45) & 127) in (4, 14, 24, 38, 49, 58, 63, 72, 83, 97, 107, 117) and
                     (int(h) & ((1 << (3 * 15)) - 1)) >> (3 * (15 - res)) == 0 for h in cells])
    if res % 2 == 0:  # Class II: 6 vertices, 5 for pentagons
        assert np.array_equal(nv, np.where(pent, 5, 6))
    else:  # Class III: distortion vertices where an edge crosses an icosahedron edge
        assert (nv[~pent] >= 6).all() and (nv[~pent] <= 8).all() and (nv[pent] == 10).all()
    bad = tot = 0
    for k in range(10):
        m = nv > k
        v, cc = xy[m, k], centre[m]
        d = cc - v
        ok = np.abs(d[:, 0]) < 180  # (antimeridian cells)
        p = v + 1e-3 * d
        got = O.h3_points_to_cells(p[:, 0], p[:, 1], res)
        bad += int(((got != cells[m]) & ok).sum())
        tot += int(m.sum())
    # H3's boundary joins its vertices by geodesic-free straight lon/lat edges: near the
    # poles and for the largest cells a vertex nudged inwards can leave the true region
    assert bad <= (tot // 200 if res <= 3 else 0), (bad, tot)


def _sphere_grid():
    lon, lat = np.meshgrid(np.linspace(-179.5, 179.5, 360), np.linspace(-89.5, 89.5, 180))
    return lon.ravel(), lat.ravel()



# ---------------------------------------------------------------- mosaicFill's cell selection
# The reference picks cells by Mosaic.mosaicFill (core/Mosaic.scala:61-99): radius r =
# H3IndexSystem.getBufferRadius (:79-90, the largest distance from the polygon's centroid
# to a vertex of the centroid's cell, planar degrees); core = polyfill(buffer(-r)) (cells
# whose centre lies in the carved polygon); border = polyfill(boundary.buffer(1.01 r)
# .simplify(0.01 r)) minus core, each clipped (getBorderChips, IndexSystem.scala:178-195:
# is_core when the clip equals the cell, dropped when empty).  The builder here clips
# every cell that meets the polygon instead.  Both give the same chip rows exactly when
# (i) no chip cell lies outside core-set and band (a blind spot) and (ii) every core-set
# cell lies wholly inside the polygon (else the reference marks a cell core that is not).

def _parts(P, k):
    for q in range(P.poly_part_off[k], P.poly_part_off[k + 1]):
        yield [P.xy[P.ring_off[r]:P.ring_off[r + 1]] for r in range(P.part_ring_off[q], P.part_ring_off[q + 1])]


def _area_centroid(P, k):
    """JTS Centroid of a (multi)polygon: area-weighted ring centroids, holes subtracted."""
    sx = sy = sa = 0.0
    for rings in _parts(P, k):
        for j, r in enumerate(rings):
            x, y = r[:, 0], r[:, 1]
            cr = x[:-1] * y[1:] - x[1:] * y[:-1]
            a = cr.sum() / 2
            cx, cy = ((x[:-1] + x[1:]) * cr).sum() / (6 * a), ((y[:-1] + y[1:]) * cr).sum() / (6 * a)
            w = abs(a) * (1.0 if j == 0 else -1.0)
            sx, sy, sa = sx + w * cx, sy + w * cy, sa + w
    return sx / sa, sy / sa


def _signed_distance(P, k, px, py):
    """Distance from each point to the polygon's boundary, positive inside (even-odd)."""
    segs = np.concatenate([np.concatenate([r[:-1], r[1:]], 1) for rings in _parts(P, k) for r in rings])
    ax, ay, bx, by = (segs[:, i][None, :] for i in range(4))
    X, Y = px[:, None], py[:, None]
    dx, dy = bx - ax, by - ay
    t = np.clip(((X - ax) * dx + (Y - ay) * dy) / np.maximum(dx * dx + dy * dy, 1e-300), 0, 1)
    d = np.hypot(ax + t * dx - X, ay + t * dy - Y).min(1)
    cross = ((ay > Y) != (by > Y)) & (X < (bx - ax) * (Y - ay) / np.where(by != ay, by - ay, 1) + ax)
    inside = (cross.sum(1) % 2) == 1
    return np.where(inside, d, -d)


def _mosaicfill_selection(P, c, res):
    """Per chip row: (d = signed centre distance, r, R = the cell's circumradius), and
    the counts of rows where the two constructions could part."""
    xy, nv, ctr = cell_geometry(c.cell)
    R = np.array([np.hypot(*(xy[i, :nv[i]] - ctr[i]).T).max() for i in range(len(c))])
    d = np.zeros(len(c))
    r = np.zeros(len(c))
    for k, pid in enumerate(P.poly_id):
        rows = np.nonzero(c.polygon_id == pid)[0]
        if not len(rows):
            continue
        gx, gy = _area_centroid(P, k)
        cell0 = O.h3_points_to_cells(np.array([gx]), np.array([gy]), res)
        vxy, vn, _ = cell_geometry(cell0)
        r[rows] = np.hypot(vxy[0, :vn[0], 0] - gx, vxy[0, :vn[0], 1] - gy).max()
        d[rows] = _signed_distance(P, k, ctr[rows, 0], ctr[rows, 1])
    core = c.is_core.astype(bool)
    core_set = d >= r  # polyfill(buffer(-r)): centre in the carved polygon
    # polyfill(boundary.buffer(1.01 r).simplify(0.01 r)): the simplification moves the
    # band's edge by at most 0.01 r, so |d| <= r is inside it for certain
    band = np.abs(d) <= r
    return {
        "rows": len(c), "core": int(core.sum()),
        "core_set": int(core_set.sum()), "band": int((band & ~core_set).sum()),
        # (i) a chip the reference never visits
        "blind": int((~core_set & ~band).sum()),
        # (ii) the reference marks the cell core, the clip does not
        "core_mismatch": int((core_set & ~core).sum()),
        # JTS approximates buffer(-r)'s arcs by chords (8 per quadrant: <= 1.93% of r):
        # rows within that of the carved edge whose flag the approximation could flip
        "buffer_sensitive": int(((d >= 0.98 * r) & (d < r) & ~core).sum()),
        "min_r_minus_R": float((r - R).min()), "max_R_over_r": float((R / r).max()),
        "_d": d, "_r": r,
    }


def _jts_sets(P, c, d, r):
    """The reference's sets near the thresholds from the independent numpy restatement of
    JTS's buffers (oracle/jts_buffer.py): per row, in carved (core), in the band, and
    DP-sensitive (band membership within the band simplification's 0.01 r); rows far from
    both thresholds by the exact distance."""
    from jts_buffer import MosaicFillSets
    xy, nv, ctr = cell_geometry(c.cell)
    core = d >= r
    band = np.ones(len(c), bool)
    dp = np.zeros(len(c), bool)
    near_core = (d >= 0.97 * r) & (d < 1.05 * r)
    near_band = np.abs(d) >= 0.95 * r
    for k, pid in enumerate(P.poly_id):
        rows = np.nonzero((c.polygon_id == pid) & (near_core | near_band))[0]
        if not len(rows):
            continue
        sets = MosaicFillSets([[np.asarray(ring) for ring in rings] for rings in _parts(P, k)], r[rows[0]])
        nc = rows[near_core[rows]]
        if len(nc):
            core[nc] = sets.core(ctr[nc, 0], ctr[nc, 1])
        nb = rows[near_band[rows] & ~core[rows]]
        if len(nb):
            band[nb] = sets.in_band(ctr[nb, 0], ctr[nb, 1])
            dp[nb] = [sets.dp_sensitive((ctr[i, 0], ctr[i, 1])) for i in nb]
    return core, band, dp


def _assert_rule(P, res, expect=None):
    """The default (mosaicFill) table against an independent restatement of its sets: the
    same rows as the clip; core exactly where the numpy restatement of JTS's buffer(-r)
    holds the centre (exact distances away from r); the clip's whole cells outside that set
    are the demoted rows; no row undecided (ambiguous), none outside the band."""
    clip = M.tessellate(P, M.H3IndexSystem(), res, core_rule="clip")
    mf = M.tessellate(P, M.H3IndexSystem(), res)
    assert np.array_equal(clip.cell, mf.cell) and np.array_equal(clip.polygon_id, mf.polygon_id)
    s = _mosaicfill_selection(P, clip, res)
    d, r = s.pop("_d"), s.pop("_r")
    core_set, band, dp = _jts_sets(P, clip, d, r)
    assert np.array_equal(mf.is_core.astype(bool), core_set)
    assert band[~core_set].all()
    assert s["blind"] == 0 and s["core_mismatch"] == 0, s
    whole = clip.is_core.astype(bool)
    st = mf.core_stats
    assert st["demoted"] == int((whole & ~mf.is_core.astype(bool)).sum()) and st["promoted"] == st["dropped"] == 0
    assert st["unresolved"] == 0 and st["band_dropped"] == 0, st
    assert st["ambiguous"] == st["dp_sensitive"] == int(dp.sum()), (st, int(dp.sum()))
    assert st["core_below_r"] == int((core_set & (d < r)).sum())
    assert st["border_above_r"] == int((~core_set & (d >= r)).sum())
    for i in np.nonzero(whole & ~mf.is_core.astype(bool))[0][:50]:
        # a demoted row's chip is the whole cell, written clockwise (JTS overlay's shell)
        w = _wkb(mf, i)
        assert w and wkb_area(w) == pytest.approx(wkb_area(_wkb(clip, i)), rel=1e-12)
    print("res %d:" % res, st, s)
    if expect:
        assert (st["rows"], st["core"], st["demoted"], st["ambiguous"]) == expect, st
    return clip, mf


# (rows: round 5's Sutherland-Hodgman clip gave 2795 / 11890 / 64041 -- 2 / 1 / 17 rows whose
# polygon only touches the cell (exact intersection area 0: the overlay gives no chip, as
# MosaicChip.isEmpty drops the reference's), and at r10 it missed 4 real chips (exact areas
# 7.8e-16 .. 5.4e-13 deg^2) whose shoelace cancelled to <= 0: test_overlay_rows_vs_clip)
@pytest.mark.parametrize("res,expect", [(8, (2793, 29, 125, 0)), (9, (11889, 2229, 1713, 0)),
                                        (10, (64028, 34257, 7469, 0))])
def test_mosaicfill_rule_nyc(nyc_zones, res, expect):
    """NYC taxi zones: mosaicFill's flags (core set = polyfill(buffer(-r)), JTS's chorded
    buffer) vs the clip's (every wholly covered cell): the same rows; at res 9, 1,713 of
    3,942 whole cells are border chips under the reference's rule; 2 rows (r10: 6) whose
    centre is < r deep are core because they lie inside a fillet's chords; no row is left
    undecided."""
    _assert_rule(nyc_zones, res, expect)


def test_mosaicfill_rule_tracts():
    """The C3 tract-like polygons at res 10 (a 400-tract sample): the same checks.  One
    row of 41,147 stays DP-sensitive: its centre is 0.9962 r from a reflex vertex, 0.00998 r
    inside the band's fillet chord around it -- whether the band's Douglas-Peucker pass
    cuts that chord depends on the ring's start vertex in JTS's buffer output."""
    import bench_workloads as W
    T = W.tract_polygons(n_cells=2000, extent=(-74.5, 40.5, -74.0, 41.0), seed=3)
    _, mf = _assert_rule(T.select(range(0, len(T), 5)), 10)
    assert mf.core_stats["ambiguous"] == 1


def test_mosaicfill_rule_pairs_on_adversarial_points(nyc_zones):
    """How much the rule changes the join (the oracle, same inputs): on the NYC r9
    adversarial fixture -- points on chip vertices and edge midpoints -- the clip table's
    pairs are a superset of mosaicFill's; every extra pair is a point on the boundary of
    a whole cell the reference keeps as a border chip (st_contains is false on it).  On
    uniform points the two tables give the same pairs."""
    import struct
    from test_gpu_parity import adversarial_points
    clip = M.tessellate(nyc_zones, M.H3IndexSystem(), 9, core_rule="clip")
    mf = M.tessellate(nyc_zones, M.H3IndexSystem(), 9)
    x, y = adversarial_points(clip)
    a = set(zip(*[v.tolist() for v in O.pip_join(0, 9, x, y, clip.cell, clip.polygon_id, clip.is_core,
                                                   clip.wkb_offsets, clip.wkb)]))
    b = set(zip(*[v.tolist() for v in O.pip_join(0, 9, x, y, mf.cell, mf.polygon_id, mf.is_core,
                                                   mf.wkb_offsets, mf.wkb)]))
    extra = a - b
    print("adversarial points %d: clip %d pairs, mosaicFill %d, clip-only %d, mosaicFill-only %d"
          % (len(x), len(a), len(b), len(extra), len(b - a)))
    assert b <= a and len(extra) > 0
    demoted = {(int(c), int(p)) for c, p, w, m in zip(clip.cell, clip.polygon_id, clip.is_core, mf.is_core) if w and not m}
    cells = O.h3_points_to_cells(x, y, 9)
    assert all((int(cells[i]), pid) in demoted for i, pid in extra)
    u, v = nyc_points(300_000, 12)
    pa = O.pip_join(0, 9, u, v, clip.cell, clip.polygon_id, clip.is_core, clip.wkb_offsets, clip.wkb)
    pb = O.pip_join(0, 9, u, v, mf.cell, mf.polygon_id, mf.is_core, mf.wkb_offsets, mf.wkb)
    assert all(np.array_equal(p, q) for p, q in zip(pa, pb))


def test_mosaicfill_rule_coarse_cells():
    """Where chip cells differ in size from the polygon's centroid cell (coarse
    resolutions, multi-face polygons) mosaicFill's sets cover the polygon imperfectly:
    a cell whose centre is >= r deep is core although it sticks out (promoted), one
    beyond the border band is never visited (dropped).  The join over such a table
    differs from true containment only inside those cells."""
    _, _, pent = cell_geometry([(1 << 59) | (bc << 45) | 0x1FFFFFFFFFFF for bc in (14,)])
    P = M.Polygons.from_lists([(2, _star(pent[0, 0], pent[0, 1], 1.0, 3.0, 30, 2)),
                               (4, _star(-40.0, -30.0, 6.0, 12.0, 50, 4))])
    # (res 3: at res 4 the dropped rows of round 5 were the clip's zero-area slivers of cells
    # the polygon only touches -- no chip under the overlay, test_overlay_rows_vs_clip)
    res = 3
    clip = M.tessellate(P, M.H3IndexSystem(), res, core_rule="clip")
    mf = M.tessellate(P, M.H3IndexSystem(), res)
    st = mf.core_stats
    print(st)
    assert st["promoted"] + st["dropped"] > 0
    changed = set(zip(clip.cell.tolist(), clip.polygon_id.tolist())) ^ set(zip(mf.cell.tolist(), mf.polygon_id.tolist()))
    rng = np.random.default_rng(9)
    x = np.concatenate([rng.uniform(-52, -28, 8000), rng.uniform(pent[0, 0] - 3, pent[0, 0] + 3, 4000)])
    y = np.concatenate([rng.uniform(-42, -18, 8000), rng.uniform(pent[0, 1] - 3, pent[0, 1] + 3, 4000)])
    got = set(zip(*[v.tolist() for v in O.pip_join(0, res, x, y, mf.cell, mf.polygon_id, mf.is_core, mf.wkb_offsets,
                                                   mf.wkb)]))
    want = set(zip(*[v.tolist() for v in O.pip_join(0, res, x, y, clip.cell, clip.polygon_id, clip.is_core,
                                                      clip.wkb_offsets, clip.wkb)]))
    cells = O.h3_points_to_cells(x, y, res)
    clip_core = {(int(c), int(p)) for c, p, k in zip(clip.cell, clip.polygon_id, clip.is_core) if k}
    mf_core = {(int(c), int(p)) for c, p, k in zip(mf.cell, mf.polygon_id, mf.is_core) if k}
    moved = (clip_core ^ mf_core) | changed
    assert all((int(cells[i]), pid) in moved for i, pid in got ^ want)


# ---------------------------------------------------------------- antimeridian and poles
def _wkb_parts_x(w):
    """The x ranges of the parts of a Polygon / MultiPolygon WKB (little or big endian)."""
    import struct
    bo = "<" if w[0] == 1 else ">"
    typ = struct.unpack(bo + "I", w[1:5])[0]
    def poly(pos):
        nr = struct.unpack(bo + "I", w[pos:pos + 4])[0]
        pos += 4
        xs = []
        for _ in range(nr):
            npt = struct.unpack(bo + "I", w[pos:pos + 4])[0]
            pos += 4
            pts = np.frombuffer(w[pos:pos + 16 * npt], dtype=bo + "f8").reshape(-1, 2)
            xs.append(pts[:, 0])
            pos += 16 * npt
        allx = np.concatenate(xs)
        return (allx.min(), allx.max()), pos
    if typ == 3:
        return [poly(5)[0]]
    n = struct.unpack(bo + "I", w[5:9])[0]
    pos, out = 9, []
    for _ in range(n):
        r, pos = poly(pos + 5)
        out.append(r)
    return out


@pytest.mark.parametrize("res", [2, 3, 4])
def test_antimeridian_cells(res):
    """A Fiji-like MULTIPOLYGON on both sides of the antimeridian: cells across it are
    cut into western and eastern parts (makeSafeGeometry, H3IndexSystem.scala:386-410),
    so a chip there is a MULTIPOLYGON with one part each side; chips of a cell never
    repeat, chip areas add up to the polygon's, and the join over the chips finds only
    true containments (the rest: chips' straight lon/lat edges against the true cells)."""
    P = M.Polygons.from_lists([(7, [
        [[(177.5, -18.5), (180.0, -18.5), (180.0, -15.5), (177.5, -15.5), (177.5, -18.5)]],
        [[(-180.0, -18.5), (-178.0, -18.5), (-178.0, -15.5), (-180.0, -15.5), (-180.0, -18.5)]]])])
    c = M.tessellate(P, M.H3IndexSystem(), res, core_rule="clip")
    _check_invariants(P, c)
    split = 0
    for i in range(len(c)):
        w = _wkb(c, i)
        if not w:
            continue
        parts = _wkb_parts_x(w)
        assert all(lo >= -180.0 and hi <= 180.0 for lo, hi in parts)
        if len(parts) == 2 and min(p[0] for p in parts) < 0 < max(p[1] for p in parts):
            split += 1
    assert split >= 1  # cells straddle the antimeridian at these resolutions
    rng = np.random.default_rng(60 + res)
    x = np.concatenate([rng.uniform(177.0, 180.0, 3000), rng.uniform(-180.0, -177.5, 3000)])
    y = rng.uniform(-19.0, -15.0, 6000)
    pts, polys = O.pip_join(0, res, x, y, c.cell, c.polygon_id, c.is_core, c.wkb_offsets, c.wkb)
    got = set(zip(pts.tolist(), polys.tolist()))
    want = brute_force_pairs(P, x, y, O)
    assert got <= want and len(got) > 0.97 * len(want)


@pytest.mark.parametrize("res", [1, 2, 3])
def test_polar_cap_cells(res):
    """A polar cap (lat >= 84, every longitude): the cell holding the pole is the cap
    between its boundary and the pole (makePoleGeometry, H3IndexSystem.scala:361-384), the
    cells across the antimeridian are cut; chip areas add up to the cap's area in lon/lat,
    the pole's cell is a chip, and the join over the chips finds only true containments.
    Near a pole a cell's straight lon/lat edges stray far from its true (geodesic)
    border, so geoToH3 sends some points to a cell whose chip does not hold them -- as in
    the reference, whose chips are the same lon/lat polygons; the share shrinks with the
    cell size (measured: 86% of the cap's points matched at res 1, 98% at 2, 99% at 3)."""
    for north in (True, False):
        s = 1 if north else -1
        lat0 = 84.0 * s
        ring = [(-180.0, lat0), (180.0, lat0), (180.0, 90.0 * s), (-180.0, 90.0 * s), (-180.0, lat0)]
        if not north:
            ring = ring[::-1]
        P = M.Polygons.from_lists([(3, [[ring]])])
        c = M.tessellate(P, M.H3IndexSystem(), res, core_rule="clip")
        _check_invariants(P, c)
        pole = int(O.h3_points_to_cells(np.array([0.0]), np.array([90.0 * s]), res)[0])
        assert pole in set(c.cell.tolist())
        rng = np.random.default_rng(70 + res)
        x = rng.uniform(-180, 180, 5000)
        y = s * rng.uniform(84.0, 90.0, 5000)
        pts, polys = O.pip_join(0, res, x, y, c.cell, c.polygon_id, c.is_core, c.wkb_offsets, c.wkb)
        got = set(zip(pts.tolist(), polys.tolist()))
        want = brute_force_pairs(P, x, y, O)
        assert got <= want and len(got) > {1: 0.8, 2: 0.95, 3: 0.98}[res] * len(want), (north, len(got), len(want))


def _jts_intersection(p1, p2, q1, q2):
    """JTS 1.20 Intersection.intersection (what RobustLineIntersector computes for a
    proper crossing), in the same operation order (Python floats are IEEE doubles)."""
    midx = (max(min(p1[0], p2[0]), min(q1[0], q2[0])) + min(max(p1[0], p2[0]), max(q1[0], q2[0]))) / 2.0
    midy = (max(min(p1[1], p2[1]), min(q1[1], q2[1])) + min(max(p1[1], p2[1]), max(q1[1], q2[1]))) / 2.0
    p1x, p1y, p2x, p2y = p1[0] - midx, p1[1] - midy, p2[0] - midx, p2[1] - midy
    q1x, q1y, q2x, q2y = q1[0] - midx, q1[1] - midy, q2[0] - midx, q2[1] - midy
    px, py, pw = p1y - p2y, p2x - p1x, p1x * p2y - p2x * p1y
    qx, qy, qw = q1y - q2y, q2x - q1x, q1x * q2y - q2x * q1y
    x, y, w = py * qw - qy * pw, qx * pw - px * qw, px * qy - qx * py
    return (x / w + midx, y / w + midy)


def _make_pole_geometry(boundary, north):
    """makePoleGeometry (H3IndexSystem.scala:361-380) restated: shiftEast, sort by
    longitude, the line's part in [0, 180] up to its crossing with x = 180, the pole edge
    (180, pole) -> (-180, pole), the part beyond 180 shifted west, closed at the start."""
    pl = 90.0 if north else -90.0
    v = sorted(((x + 360.0 if x < 0 else x, y) for x, y in boundary), key=lambda p: p[0])
    k = next(i for i, p in enumerate(v) if p[0] > 180.0)
    cut = _jts_intersection(v[k - 1], v[k], (180.0, 90.0), (180.0, -90.0))
    west = v[:k] + [cut]
    east = [(cut[0] - 360.0, cut[1])] + [(x - 360.0, y) for x, y in v[k:]]
    return west + [(180.0, pl), (-180.0, pl)] + east + [west[0]]


@pytest.mark.parametrize("res", [0, 1, 2, 3, 5, 9])
def test_pole_cell_geometry_matches_make_pole_geometry(res):
    """an H3 pole cell's geometry (as a core chip of it carries it) is the
    reference's ring byte for byte -- vertex order, start, orientation (the south cap
    clockwise) and the JTS crossing with x = 180."""
    import struct
    for north in (True, False):
        s = 1 if north else -1
        pole = int(O.h3_points_to_cells(np.array([0.0]), np.array([90.0 * s]), res)[0])
        buf = np.zeros(4096, np.uint8)
        ln = ctypes.c_int64()
        _native.check(_native.lib().mgpu_test_h3_cell_wkb_host(pole, _P(buf), len(buf), ctypes.byref(ln)))
        w = bytes(buf[:ln.value])
        xy, nv, _ = cell_geometry(np.array([pole]))
        want = _make_pole_geometry([tuple(p) for p in xy[0, :nv[0]]], north)
        bo = "<" if w[0] == 1 else ">"  # (JTS's WKBWriter default: big endian)
        assert struct.unpack(bo + "I", w[1:5])[0] == 3 and struct.unpack(bo + "I", w[5:9])[0] == 1
        npt = struct.unpack(bo + "I", w[9:13])[0]
        got = np.frombuffer(w[13:13 + 16 * npt], dtype=bo + "f8").reshape(-1, 2)
        assert np.array_equal(got, np.array(want)), (north, got.tolist(), want)
        signed = 0.5 * sum(got[t, 0] * got[t + 1, 1] - got[t + 1, 0] * got[t, 1] for t in range(npt - 1))
        assert (signed > 0) == north  # the south cap is clockwise, as the reference's
        assert got[0, 0] >= 0 and got[0, 0] == min(p[0] for p in got if p[0] >= 0)


@pytest.mark.parametrize("res", [9, 10])
def test_jts_buffer_flags_pair_impact(nyc_zones, res):
    """What deciding the threshold rows by JTS's chorded buffer (instead of exact distance,
    round 4's MGPU_CORE_DISTANCE) changes: NYC r9 2 rows (r10 6) turn core -- centres
    0.99 r..r deep inside a fillet's chords; each row's cell is checked for sticking out of
    its polygon (the clip's chip is then not the whole cell) and the join over the two
    tables is compared on 1e6 uniform points (the oracle, both tables)."""
    old = M.tessellate(nyc_zones, M.H3IndexSystem(), res, core_rule="distance")
    new = M.tessellate(nyc_zones, M.H3IndexSystem(), res)
    clip = M.tessellate(nyc_zones, M.H3IndexSystem(), res, core_rule="clip")
    assert np.array_equal(old.cell, new.cell) and np.array_equal(old.polygon_id, new.polygon_id)
    changed = np.nonzero(old.is_core != new.is_core)[0]
    assert len(changed) == new.core_stats["core_below_r"] + new.core_stats["border_above_r"]
    assert len(changed) == {9: 2, 10: 6}[res] and (new.is_core[changed] == 1).all()
    # a changed row sticks out iff the polygon does not hold its whole cell (the clip rule's
    # flag is 0: the cell's chip is partial)
    sticks_out = int((clip.is_core[changed] == 0).sum())
    u, v = nyc_points(1_000_000, 77)
    pa = O.pip_join(0, res, u, v, old.cell, old.polygon_id, old.is_core, old.wkb_offsets, old.wkb)
    pb = O.pip_join(0, res, u, v, new.cell, new.polygon_id, new.is_core, new.wkb_offsets, new.wkb)
    a, b = set(zip(*[x.tolist() for x in pa])), set(zip(*[x.tolist() for x in pb]))
    print("res %d: %d rows flip to core, %d stick out; pairs %d -> %d, +%d -%d"
          % (res, len(changed), sticks_out, len(a), len(b), len(b - a), len(a - b)))
    assert not (a - b)  # core only adds matches (points of the cell outside the polygon)
    if sticks_out == 0:
        assert a == b


# ---------------------------------------------------------------- border chips as JTS cuts them
# (round 6) mosaic_amd/csrc/jts_overlay.h restates `polygon INTERSECTION cell` as OverlayNG
# computes it (IndexSystem.scala:184-188, MosaicGeometryJTS.scala:139-152) and
# coerceChipGeometry's re-noding (IndexSystem.scala:293-303); oracle/jts_overlay.py restates
# the node arithmetic independently (exact orientation, Intersection.intersection in IEEE
# doubles).  Parity with JTS itself is unpinned beyond the published algorithm.
import jts_overlay as JO  # noqa: E402  (oracle/, test infrastructure)


def _h3_cell_rings(cell):
    buf = (ctypes.c_uint8 * 8192)()
    n = ctypes.c_int64()
    _native.check(_native.lib().mgpu_test_h3_cell_wkb_host(ctypes.c_int64(int(cell)), buf, 8192, ctypes.byref(n)))
    return [r for pc in JO.wkb_rings(bytes(buf[:n.value])) for r in pc]


def _bng_cell_rings(chip_rings, edge):
    xs = [p[0] for r in chip_rings for p in r]
    ys = [p[1] for r in chip_rings for p in r]
    i, j = float(np.floor((min(xs) + max(xs)) / 2 / edge)), float(np.floor((min(ys) + max(ys)) / 2 / edge))
    x, y = i * edge, j * edge
    return [[(x, y), (x + edge, y), (x + edge, y + edge), (x, y + edge), (x, y)]]


def _poly_rings(P, k):
    return [[tuple(map(float, v)) for v in P.xy[P.ring_off[r]:P.ring_off[r + 1]]]
            for q in range(P.poly_part_off[k], P.poly_part_off[k + 1])
            for r in range(P.part_ring_off[q], P.part_ring_off[q + 1])]


def _check_overlay_chips(P, c, cell_rings_of, is_multi, limit=None):
    """every border chip of c against oracle/jts_overlay.check_chip -> (chips, crossings, coerce nodes)"""
    idx = {int(p): i for i, p in enumerate(P.poly_id)}
    cache = {}
    n = cross = coerce = 0
    rows = np.nonzero(~c.is_core.astype(bool))[0]
    if limit is not None:
        rows = rows[:: max(1, len(rows) // limit)]
    for i in rows:
        k = idx[int(c.polygon_id[i])]
        if k not in cache:
            cache[k] = _poly_rings(P, k)
        w = _wkb(c, i)
        a, b = JO.check_chip(w, cache[k], cell_rings_of(c.cell[i], w), is_multi(k))
        n, cross, coerce = n + 1, cross + a, coerce + b
    return n, cross, coerce


def test_overlay_chip_vertices_nyc_r9(nyc_zones, nyc_chips_r9):
    """Every NYC r9 border chip (9,660; the zones are MULTIPOLYGONs): its vertices are polygon
    vertices, cell vertices, RobustLineIntersector's nodes of the two ORIGINAL segments (the
    independent restatement's, bit for bit), or coerceChipGeometry's re-noding nodes -- only
    in the one-piece chips, whose type differs from the zone's; every proper crossing node
    is a vertex."""
    P, c = nyc_zones, nyc_chips_r9
    assert P.poly_type is not None and (P.poly_type == 6).all()
    n, cross, coerce = _check_overlay_chips(P, c, lambda cell, w: _h3_cell_rings(cell), lambda k: True)
    st = c.core_stats
    print("chips", n, "crossing vertices", cross, "coerce vertices", coerce, st)
    assert n == st["overlay_chips"] + st["demoted"] and cross > 15000
    assert coerce == st["coerce_nodes"] > 0 and st["coerced"] == st["overlay_chips"] - st["multi_piece"]


def test_overlay_chip_vertices_bng_and_tracts():
    """The same on BNG squares (London-like districts, POLYGONs, edges along the extent's km
    lines: collinear overlaps) at res 3 and 4, and on tract-like POLYGONs at H3 r10 (a sample):
    no re-noding unless a chip falls apart into pieces."""
    import bench_workloads as W
    L = W.london_districts(n_cells=40)
    for res in (3, 4):
        edge = 10.0 ** (6 - res)
        c = M.tessellate(L, M.BNGIndexSystem(), res)
        n, cross, coerce = _check_overlay_chips(
            L, c, lambda cell, w: _bng_cell_rings([r for pc in JO.wkb_rings(w) for r in pc], edge), lambda k: False)
        st = c.core_stats
        assert n > 100 and cross > 100 and coerce == st["coerce_nodes"], (res, n, cross, coerce, st)
        assert st["coerced"] == st["multi_piece"] + st["lower_dim"]
    T = W.tract_polygons(n_cells=60)
    c = M.tessellate(T, M.H3IndexSystem(), 10)
    n, cross, coerce = _check_overlay_chips(T, c, lambda cell, w: _h3_cell_rings(cell), lambda k: False, limit=3000)
    assert n > 1000 and cross > 1000 and coerce == 0 or c.core_stats["multi_piece"] > 0


def test_overlay_separate_pieces_and_holes():
    """A U-shaped polygon whose two arms cross one cell: OverlayNG's result is a MULTIPOLYGON
    of two separate pieces (round 5's clip bridged them into one ring along the cell
    boundary); a polygon with a hole inside the cell keeps it as the chip's hole.  Points
    between the arms and in the hole: no pair, by either table."""
    res = 4
    edge = 100.0
    x0, y0 = 530000.0, 180000.0
    # arms 20 m wide, 40 m apart, crossing the square [x0, x0 + 100] x [y0, y0 + 100]
    u = [(x0 + 10, y0 - 50), (x0 + 90, y0 - 50), (x0 + 90, y0 + 150), (x0 + 70, y0 + 150), (x0 + 70, y0 - 30),
         (x0 + 30, y0 - 30), (x0 + 30, y0 + 150), (x0 + 10, y0 + 150), (x0 + 10, y0 - 50)]
    h_shell = [(x0 - 150, y0 + 150 + 200), (x0 - 150, y0 + 150 + 50), (x0 + 250, y0 + 150 + 50),
               (x0 + 250, y0 + 150 + 200), (x0 - 150, y0 + 150 + 200)]
    hole = [(x0 + 40, y0 + 230), (x0 + 60, y0 + 230), (x0 + 60, y0 + 270), (x0 + 40, y0 + 270), (x0 + 40, y0 + 230)]
    P = M.Polygons.from_lists([(1, [[u[::-1]]]), (2, [[h_shell[::-1], hole]])], poly_type=np.array([3, 3]))
    new = M.tessellate(P, M.BNGIndexSystem(), res)
    old = M.tessellate(P, M.BNGIndexSystem(), res, chip_geometry="sutherland_hodgman")
    ucell = O.bng_point_to_index(x0 + 50, y0 + 50, res)
    hcell = O.bng_point_to_index(x0 + 50, y0 + 250, res)
    i = [k for k in range(len(new)) if new.cell[k] == ucell and new.polygon_id[k] == 1][0]
    pieces = JO.wkb_rings(_wkb(new, i))
    assert len(pieces) == 2 and all(len(pc) == 1 for pc in pieces)
    assert _wkb(new, i)[1:5] == b"\x00\x00\x00\x06"  # big-endian MULTIPOLYGON
    for pc in pieces:  # shells clockwise (OverlayNG)
        assert JO.orient(pc[0][0], pc[0][1], pc[0][2]) <= 0 or len(pc[0]) > 4
    j = [k for k in range(len(old)) if old.cell[k] == ucell and old.polygon_id[k] == 1][0]
    assert len(JO.wkb_rings(_wkb(old, j))) == 1  # round 5: one bridged ring
    i = [k for k in range(len(new)) if new.cell[k] == hcell and new.polygon_id[k] == 2][0]
    pieces = JO.wkb_rings(_wkb(new, i))
    assert len(pieces) == 1 and len(pieces[0]) == 2  # shell + the hole
    # containment over the chips equals containment in the polygons
    rng = np.random.default_rng(6)
    px = np.concatenate([x0 + rng.uniform(0, 100, 4000), x0 + rng.uniform(0, 100, 4000)])
    py = np.concatenate([y0 + rng.uniform(0, 100, 4000), y0 + 200 + rng.uniform(0, 100, 4000)])
    want = brute_force_pairs(P, px, py, O)
    assert len(want) > 1000
    for t in (new, old):
        pts, polys = O.pip_join(1, res, px, py, t.cell, t.polygon_id, t.is_core, t.wkb_offsets, t.wkb)
        assert set(zip(pts.tolist(), polys.tolist())) == want


def test_overlay_rows_vs_clip(nyc_zones):
    """Rows round 5's Sutherland-Hodgman clip and the overlay disagree on (NYC r10): the
    clip's extra rows have an exact (rational) intersection area of 0 -- the polygon only
    touches the cell, OverlayNG gives lines / points, which coerceChipGeometry and
    MosaicChip.isEmpty drop; the overlay's extra rows are real chips (exact area > 0) whose
    shoelace in absolute coordinates had cancelled to <= 0 in the clip."""
    from fractions import Fraction as F

    def area(r):
        x0, y0 = r[0]
        return sum((r[q][0] - x0) * (r[q + 1][1] - y0) - (r[q + 1][0] - x0) * (r[q][1] - y0)
                   for q in range(len(r) - 1)) / 2

    def clip_exact(ring, cell):  # exact rational clip against the convex ccw cell: the area
        pts = [(F(x), F(y)) for x, y in ring[:-1]]
        c = [(F(x), F(y)) for x, y in cell]
        for e in range(len(c) - 1):
            a, b = c[e], c[e + 1]
            side = lambda p: (b[0] - a[0]) * (p[1] - a[1]) - (b[1] - a[1]) * (p[0] - a[0])  # noqa: E731
            out = []
            if not pts:
                break
            prev = pts[-1]
            sp = side(prev)
            for cur in pts:
                sc = side(cur)
                if (sc >= 0) != (sp >= 0):
                    t = sp / (sp - sc)
                    out.append((prev[0] + t * (cur[0] - prev[0]), prev[1] + t * (cur[1] - prev[1])))
                if sc >= 0:
                    out.append(cur)
                prev, sp = cur, sc
            pts = out
        return abs(area(pts + [pts[0]])) if len(pts) >= 3 else F(0)

    P = nyc_zones
    old = M.tessellate(P, M.H3IndexSystem(), 10, chip_geometry="sutherland_hodgman")
    new = M.tessellate(P, M.H3IndexSystem(), 10)
    ko = {(int(old.polygon_id[i]), int(old.cell[i])) for i in range(len(old))}
    kn = {(int(new.polygon_id[i]), int(new.cell[i])) for i in range(len(new))}
    idx = {int(p): i for i, p in enumerate(P.poly_id)}

    def exact(pid, cell):
        k, tot = idx[pid], F(0)
        cr = _h3_cell_rings(cell)
        assert len(cr) == 1
        for q in range(P.poly_part_off[k], P.poly_part_off[k + 1]):
            for j, r in enumerate(range(P.part_ring_off[q], P.part_ring_off[q + 1])):
                ring = [tuple(map(float, v)) for v in P.xy[P.ring_off[r]:P.ring_off[r + 1]]]
                tot += clip_exact(ring, cr[0]) * (1 if j == 0 else -1)
        return tot

    assert (len(ko - kn), len(kn - ko)) == (17, 4)
    assert all(exact(*k) == 0 for k in ko - kn)
    assert all(exact(*k) > 0 for k in kn - ko)


def test_rows_in_cell_order_and_order_free_checksum(nyc_zones, nyc_chips_r9):
    """Each polygon's rows come out in cell order, whichever cells the builder's lattice
    walk classified as interior or border (round 6 coarsened that walk's sampling from
    res 5 and moved far border cells to the scanline's row crossings); the rows themselves
    -- cells, polygons, flags and chip WKB, compared with the order taken out -- are the
    ones the previous walk produced (sha256 prefix of the rows sorted by (cell, polygon); the
    previous builder's rows gave the same bytes -- checked on NYC r7/r9/r10, C3, C4 r3/r4
    and C5 when the walk changed)."""
    import hashlib
    c = nyc_chips_r9
    pid = c.polygon_id
    starts = np.flatnonzero(np.r_[True, pid[1:] != pid[:-1]])
    assert len(starts) == len(np.unique(pid))  # each polygon's rows together, in input order
    for a, b in zip(starts, np.r_[starts[1:], len(c)]):
        assert np.all(np.diff(c.cell[a:b]) > 0)
    h = hashlib.sha256()
    for i in np.lexsort((c.polygon_id, c.cell)):
        h.update(np.int64(c.cell[i]).tobytes() + np.int32(pid[i]).tobytes() + np.uint8(c.is_core[i]).tobytes())
        h.update(c.wkb[c.wkb_offsets[i]:c.wkb_offsets[i + 1]].tobytes())
    assert (len(c), h.hexdigest()[:16]) == (11889, "9fe363c45cbaf510")


@pytest.mark.parametrize("case", ["nyc_r9", "nyc_r10", "bng_r4"])
def test_overlay_chain_shortcut_equals_general_graph(nyc_zones, case):
    """The overlay's one-crossing-chain shortcut (jts_overlay.h Clipper::one_crossing_chain:
    most border cells) writes the chip the general noded graph would: with the test hook on,
    every cell it answers is cut again by the graph and compared vertex for vertex."""
    import bench_workloads as W
    L = _native.lib()
    cnt = np.zeros(2, np.int64)
    _native.check(L.mgpu_test_overlay_verify(1, cnt.ctypes.data))
    try:
        if case == "bng_r4":
            M.tessellate(W.london_districts(), M.BNGIndexSystem(), 4)
        else:
            M.tessellate(nyc_zones, M.H3IndexSystem(), 9 if case == "nyc_r9" else 10)
    finally:
        _native.check(L.mgpu_test_overlay_verify(0, cnt.ctypes.data))
    assert cnt[0] > 1000 and cnt[1] == 0, cnt
