"""The oracle (CPU restatement, test infrastructure) pinned against the reference's
own known answers (tests/golden/*, mined by tools/extract_kats.py):

* 176 H3 (lon, lat, res) -> cell ids from the reference's docs and notebook outputs
* BNG ids at all 12 resolutions (TestBNGIndexSystem.scala:12-75) and the
  transform_join_bng.ipynb cell-38 points (as strings)
* ST_ContainsBehaviors.scala:22-36 (polygon with two holes)
* 59 end-to-end point -> taxi-zone results of the reference's
  `is_core OR st_contains` join (Quickstart notebooks, python / sql / scala)
"""
import base64
import json
import os

import numpy as np
import pytest

import oracle as O
from geom_util import wkt_to_wkb

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    return json.load(open(os.path.join(GOLDEN, name)))


def test_h3_kats_all_match():
    kats = load("h3_kats.json")["kats"]
    assert len(kats) >= 170
    bad = [k for k in kats if O.h3_point_to_index(k["lon"], k["lat"], k["res"]) != k["cell"]]
    assert not bad, bad[:5]


def test_h3_kats_batch_equals_scalar():
    kats = load("h3_kats.json")["kats"]
    for res in (9, 10):
        ks = [k for k in kats if k["res"] == res]
        got = O.h3_points_to_cells([k["lon"] for k in ks], [k["lat"] for k in ks], res)
        assert [int(v) for v in got] == [k["cell"] for k in ks]


def test_h3_invalid_inputs():
    assert O.h3_point_to_index(float("nan"), 10.0, 9) == 0
    assert O.h3_point_to_index(10.0, float("inf"), 9) == 0
    assert O.lib().orc_h3_geo_to_h3(0.1, 0.1, 16) == 0


def test_bng_kats_numeric():
    kats = [k for k in load("bng_kats.json")["point_to_index"] if k["cell"] is not None]
    assert len(kats) == 12
    for k in kats:
        assert O.bng_point_to_index(k["e"], k["n"], k["res"]) == k["cell"], k


def test_bng_nan_raises():
    with pytest.raises(ValueError):
        O.bng_point_to_index(float("nan"), 100.0, 5)
    with pytest.raises(ValueError):
        O.bng_point_to_index(100.0, float("nan"), 5)


def test_st_contains_two_holes():
    d = load("st_contains_kats.json")
    w = wkt_to_wkb(d["polygon_wkt"])
    for c in d["cases"]:
        assert O.st_contains(w, c["x"], c["y"]) == c["expected"]
    # both byte orders, and boundary / hole-boundary points are not contained
    wl = wkt_to_wkb(d["polygon_wkt"], little_endian=True)
    for x, y, loc in [(35, 25, O.LOC_INTERIOR), (25, 25, O.LOC_EXTERIOR), (10, 50, O.LOC_BOUNDARY),
                      (20, 25, O.LOC_BOUNDARY), (5, 5, O.LOC_EXTERIOR), (110, 110, O.LOC_BOUNDARY)]:
        assert O.wkb_locate(w, x, y) == loc
        assert O.wkb_locate(wl, x, y) == loc


def test_bng_notebook_chip_wkb():
    """transform_join_bng.ipynb cell 45: a JTS big-endian chip (500 m BNG cell with a
    duplicated closing vertex)."""
    chip = load("bng_kats.json")["chip"]
    w = base64.b64decode(chip["wkb_b64"])
    assert w[0] == 0  # big-endian, as JTS WKBWriter writes
    import struct
    (t,) = struct.unpack(">I", w[1:5])
    assert t == 3
    # the chip is the 500 m cell TQ3482NW = [534000, 534500] x [182500, 183000]
    assert O.wkb_locate(w, 534250.0, 182750.0) == O.LOC_INTERIOR
    assert O.wkb_locate(w, 534000.0, 182750.0) == O.LOC_BOUNDARY
    assert O.wkb_locate(w, 533999.0, 182750.0) == O.LOC_EXTERIOR


def test_pip_end_to_end_kats(nyc_chips_r9):
    """Every notebook (point -> zone) result is reproduced by the oracle join on our chips."""
    kats = load("pip_kats.json")["kats"]
    assert len(kats) >= 55
    c = nyc_chips_r9
    x = np.array([k["lon"] for k in kats])
    y = np.array([k["lat"] for k in kats])
    pts, polys = O.pip_join(0, 9, x, y, c.cell, c.polygon_id, c.is_core, c.wkb_offsets, c.wkb)
    got = {}
    for p, q in zip(pts, polys):
        got.setdefault(int(p), []).append(int(q))
    for i, k in enumerate(kats):
        assert got.get(i), ("no zone for", k)
        assert set(got[i]) <= set(k["objectids"]) and len(got[i]) == 1, (k, got.get(i))
        if k["cell_r9"] is not None:
            assert O.h3_point_to_index(k["lon"], k["lat"], 9) == k["cell_r9"]


def test_bng_kring_restatement_known_answers():
    """The oracle's kRing / kLoop restatement on hand-checked cases: a 1 km cell in the
    middle of TQ has 8 neighbours in its first loop and 16 in the second, all valid;
    the SV square's south-west corner cell loses the candidates west / south of the grid."""
    c = O.bng_point_to_index(530500.0, 180500.0, 3)
    l1, l2 = O.bng_k_loop(c, 1), O.bng_k_loop(c, 2)
    assert len(l1) == 8 and len(l2) == 16 and len(set(l1 + l2)) == 24 and c not in l1 + l2
    assert O.bng_k_ring(c, 2) == [c] + l1 + l2
    # the first loop starts at the south-west corner neighbour and runs east along the bottom
    assert l1[0] == O.bng_point_to_index(529500.0, 179500.0, 3)
    assert l1[1] == O.bng_point_to_index(530500.0, 179500.0, 3)
    # at the grid's south-west corner some candidates are dropped; the reference's
    # truncating arithmetic folds others (negative eastings) onto in-grid ids, kept
    corner = O.bng_point_to_index(0.5, 0.5, 3)
    lc = O.bng_k_loop(corner, 1)
    assert len(lc) < 8
    assert {O.bng_point_to_index(1000.0, 0.0, 3), O.bng_point_to_index(1000.0, 1000.0, 3),
            O.bng_point_to_index(0.0, 1000.0, 3)} <= set(lc)


def test_h3_kring_restatement_doc_known_answer():
    """The oracle's H3 kRing (H3IndexSystem.scala:182-184 -> H3 v3.7 kRing) against the
    reference's documented output (docs/source/api/spatial-indexing.rst:776-784):
    grid_cellkringexplode(613177664827555839, 2) starts with these four ids."""
    r = O.h3_k_ring(613177664827555839, 2)
    assert len(r) == 19 and len(set(r)) == 19
    assert r[:4] == [613177664827555839, 613177664825458687, 613177664831750143, 613177664884178943]


def test_h3_neighbor_tables_consistent_away_from_pentagons():
    """Derived base-cell neighbour tables (tools/gen_h3_neighbors.py): at every
    resolution, cells whose 2-neighbourhood stays among hexagon base cells have 19
    distinct kRing(2) ids, mutual kRing(1) adjacency, and hexRing(2) == kRing(2)'s
    outer 12 (same cyclic order, started at the cell two steps in I).  (Pentagon neighbourhoods,
    which the device path walks as H3 does, are checked against the oracle by
    test_gpu_parity.py's pentagon kRing tests and as geometric balls by
    test_h3_kring_geometry_host.py.)"""
    pent = {4, 14, 24, 38, 49, 58, 63, 72, 83, 97, 107, 117}
    rng = np.random.default_rng(7)
    tested = 0
    for res in range(1, 16):
        lon = rng.uniform(-180, 180, 60)
        lat = np.degrees(np.arcsin(rng.uniform(-1, 1, 60)))
        for c in O.h3_points_to_cells(lon, lat, res):
            c = int(c)
            if any(((x >> 45) & 127) in pent for x in O.h3_k_ring(c, 3)):
                continue
            tested += 1
            r1, r2 = O.h3_k_ring(c, 1), O.h3_k_ring(c, 2)
            assert len(r2) == 19 and len(set(r2)) == 19 and r2[:7] == r1
            for nb in r1[1:]:
                assert c in O.h3_k_ring(nb, 1)
            assert O.h3_k_loop(c, 2) == [r2[-1]] + r2[7:-1]  # hexRing starts at the I-I cell
    assert tested > 600
