"""Host-side product logic (no GPU): the C-ABI library loads and exports what the
header declares, BNG StringType ids, resolution validation, and the chip-table
builder (grid_tessellateexplode) checked against the reference's invariants and
against brute-force JTS-semantics containment on the original polygons."""
import json
import os
import re

import numpy as np
import pytest

import mosaic_amd as M
import oracle as O
from geom_util import brute_force_pairs, polygons_area, wkb_area, nyc_points

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def test_library_exports_every_header_symbol():
    from mosaic_amd import _native as N
    hdr = "".join(open(os.path.join(ROOT, "include", h)).read() for h in ("mosaic_gpu.h", "mosaic_arrow.h"))
    declared = set(re.findall(r"\b(mgpu_[a-z0-9_]+)\s*\(", hdr))
    assert declared == set(N.EXPORTS)
    L = N.lib()
    for s in declared:
        assert hasattr(L, s), s
    assert b"gfx950" in L.mgpu_version()


def test_resolution_validation():
    h3, bng = M.H3IndexSystem(), M.BNGIndexSystem()
    assert h3.get_resolution(9) == 9 and h3.get_resolution("10") == 10
    with pytest.raises(M.IllegalStateException):
        h3.get_resolution(16)
    with pytest.raises(M.IllegalArgumentException):
        h3.get_resolution(1.5)
    assert bng.get_resolution("500m") == -4 and bng.get_resolution(4) == 4
    with pytest.raises(M.IllegalStateException):
        bng.get_resolution(0)
    with pytest.raises(M.IllegalStateException):
        bng.get_resolution(True)
    from mosaic_amd import _native as N
    assert N.lib().mgpu_check_resolution(0, 15) == 0 and N.lib().mgpu_check_resolution(1, -6) == 0
    assert N.lib().mgpu_check_resolution(1, 7) == N.MGPU_E_RESOLUTION
    assert M.get_index_system("bng").name == "BNG"
    with pytest.raises(M.IllegalArgumentException):
        M.get_index_system("CUSTOM(0,1,0,1,2,1,1)")


def test_bng_format_parse_kats():
    d = json.load(open(os.path.join(GOLDEN, "bng_kats.json")))
    bng = M.BNGIndexSystem()
    for k in d["point_to_index"]:
        cell = O.bng_point_to_index(k["e"], k["n"], k["res"])
        if k["cell"] is not None:
            assert cell == k["cell"]
        assert bng.format(cell) == k["str"], k
    for p in d["parse"]:
        assert bng.parse(p["str"]) == p["cell"]
    # TestBNGIndexSystem.scala:84 parse("NW") == encode(1, 5, 0, 0, 0, 1, -2)
    assert bng.parse("NW") == 100000 + 1 * 1000 + 5 * 10
    # transform_join_bng.ipynb cell 51: the joined point lies in chip TQ3586NW
    j = d["join"]
    assert bng.format(O.bng_point_to_index(j["e"], j["n"], -4)) == j["index_id"]
    with pytest.raises(M.IllegalArgumentException):
        bng.format(-5)


def test_bng_format_round_trip_random():
    rng = np.random.default_rng(3)
    bng = M.BNGIndexSystem()
    e = rng.uniform(0, 700000, 2000)
    n = rng.uniform(0, 1300000, 2000)
    for res in (1, 2, 3, 4, 5, 6, -2, -3, -4, -5, -6):
        cells = O.bng_points_to_cells(e, n, res)
        strs = bng.format_many(cells)
        assert np.array_equal(bng.parse_many(strs), cells), res


def test_tessellation_covers_each_zone_exactly(nyc_zones, nyc_chips_r9):
    """MosaicExplodeBehaviors.scala:415-457 (issue 382): the chips of a polygon
    add up to the polygon's area; chips never overlap (one chip per cell)."""
    c = nyc_chips_r9
    assert len(c) > 10000 and c.is_core.sum() > 2000
    for pid in (1, 2, 43, 132, 138, 161, 230, 263):
        k = int(np.nonzero(nyc_zones.poly_id == pid)[0][0])
        rows = np.nonzero(c.polygon_id == pid)[0]
        assert len(np.unique(c.cell[rows])) == len(rows)
        area = sum(wkb_area(bytes(c.wkb[c.wkb_offsets[i]:c.wkb_offsets[i + 1]])) for i in rows)
        assert area == pytest.approx(polygons_area(nyc_zones, k), rel=1e-8), pid


def test_tessellation_join_equals_brute_force(nyc_zones, nyc_chips_r9):
    """is_core OR st_contains over the chips == contains over the original zones."""
    x, y = nyc_points(20000, 11)
    c = nyc_chips_r9
    pts, polys = O.pip_join(0, 9, x, y, c.cell, c.polygon_id, c.is_core, c.wkb_offsets, c.wkb)
    assert set(zip(pts.tolist(), polys.tolist())) == brute_force_pairs(nyc_zones, x, y, O)
    # chip cells are exactly the cells the points are indexed to
    cells = set(c.cell.tolist())
    got = O.h3_points_to_cells(x[pts], y[pts], 9)
    assert set(got.tolist()) <= cells


def test_tessellation_no_core_geometry(nyc_zones):
    c = M.tessellate(nyc_zones.select(range(10)), M.H3IndexSystem(), 9, keep_core_geometries=False)
    core = c.is_core.astype(bool)
    lens = np.diff(c.wkb_offsets)
    assert (lens[core] == 0).all() and (lens[~core] > 0).all()


def _bng_synthetic(seed=5, n=12):
    """UK-style polygons in eastings/northings: jittered star polygons with holes."""
    rng = np.random.default_rng(seed)
    polys = []
    for p in range(n):
        cx, cy = rng.uniform(510000, 555000), rng.uniform(160000, 195000)
        k = int(rng.integers(8, 40))
        ang = np.sort(rng.uniform(0, 2 * np.pi, k))
        rad = rng.uniform(800, 3000, k)
        shell = [(cx + r * np.cos(a), cy + r * np.sin(a)) for a, r in zip(ang, rad)]
        shell.append(shell[0])
        hole = [(cx + 200 * np.cos(a), cy + 200 * np.sin(a)) for a in np.linspace(2 * np.pi, 0, 9)]
        polys.append((p + 1, [[shell, hole]]))
    return M.Polygons.from_lists(polys)


@pytest.mark.parametrize("res", [3, 4, -3, -4])
def test_bng_tessellation_join_equals_brute_force(res):
    P = _bng_synthetic()
    c = M.tessellate(P, M.BNGIndexSystem(), res)
    assert len(c) > 0
    rng = np.random.default_rng(7)
    x = rng.uniform(505000, 560000, 20000)
    y = rng.uniform(155000, 200000, 20000)
    pts, polys = O.pip_join(1, res, x, y, c.cell, c.polygon_id, c.is_core, c.wkb_offsets, c.wkb)
    assert set(zip(pts.tolist(), polys.tolist())) == brute_force_pairs(P, x, y, O)


def test_tessellation_rejects_unsupported():
    P = _bng_synthetic(n=2)
    with pytest.raises(M.MosaicGpuError):
        M.tessellate(P, M.BNGIndexSystem(), -1)
    with pytest.raises(M.IllegalStateException):
        M.tessellate(P, M.H3IndexSystem(), 16)


# BNGIndexSystem.format restated line by line from BNGIndexSystem.scala:119-134
# (letterMap :88-104, quadrants :40, indexDigits = Long.toString :440-442); None where
# the Scala code throws (a lookup out of bounds, "".toInt)
_BNG_LETTERS = [["SV", "SW", "SX", "SY", "SZ", "TV", "TW", "TX"], ["SQ", "SR", "SS", "ST", "SU", "TQ", "TR", "TS"],
                ["SL", "SM", "SN", "SO", "SP", "TL", "TM", "TN"], ["SF", "SG", "SH", "SJ", "SK", "TF", "TG", "TH"],
                ["SA", "SB", "SC", "SD", "SE", "TA", "TB", "TC"], ["NV", "NW", "NX", "NY", "NZ", "OV", "OW", "OX"],
                ["NQ", "NR", "NS", "NT", "NU", "OQ", "OR", "OS"], ["NL", "NM", "NN", "NO", "NP", "OL", "OM", "ON"],
                ["NF", "NG", "NH", "NJ", "NK", "OF", "OG", "OH"], ["NA", "NB", "NC", "ND", "NE", "OA", "OB", "OC"],
                ["HV", "HW", "HX", "HY", "HZ", "JV", "JW", "JX"], ["HQ", "HR", "HS", "HT", "HU", "JQ", "JR", "JS"],
                ["HL", "HM", "HN", "HO", "HP", "JL", "JM", "JN"], ["HF", "HG", "HH", "HJ", "HK", "JF", "JG", "JH"]]
_BNG_QUADRANTS = ["", "SW", "NW", "NE", "SE"]


def _scala_bng_format(i):
    d = str(i)
    try:
        if len(d) < 6:
            return _BNG_LETTERS[int(d[3:5])][int(d[1:3])][0]
        p = _BNG_LETTERS[int(d[3:5])][int(d[1:3])]
        c = d[5:-1]
        k = len(c) // 2
        return p + c[:k] + c[k:2 * k] + _BNG_QUADRANTS[int(d[-1])]
    except (ValueError, IndexError):
        return None


def test_bng_format_matches_scala_restatement():
    """The shared (host + device) formatter, bng_core.h format_cell, against the Scala
    code restated above: random ids over the whole positive int64 range (incl. beyond
    2^53, where the formatter switches from double to integer digit arithmetic)."""
    rng = np.random.default_rng(9)
    ids = np.concatenate([rng.integers(1, 10 ** 16, 20_000), rng.integers(10 ** 16, 2 ** 63 - 1, 5_000, dtype=np.int64),
                          np.arange(1, 20_000), [2 ** 53 - 1, 2 ** 53, 2 ** 53 + 1, 2 ** 63 - 1]]).astype(np.int64)
    bng = M.BNGIndexSystem()
    ok = np.array([_scala_bng_format(int(i)) is not None for i in ids])
    got = bng.format_many(ids[ok])
    assert got == [_scala_bng_format(int(i)) for i in ids[ok]]
    for i in ids[~ok][:200]:
        with pytest.raises(M.IllegalArgumentException):
            bng.format(int(i))
