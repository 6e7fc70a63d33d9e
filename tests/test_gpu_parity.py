"""Parity of the HIP path (through the C ABI) with the oracle, on the same seeded inputs.

Bit-exact is the bar: identical cell ids, identical (point_id, polygon_id) pair
sequences, identical st_contains results.  Sizes are what the oracle finishes in
seconds; the full-size case checks size-independent properties plus a sampled
slice against the oracle.
"""
import json
import os

import numpy as np
import pytest
import torch

import mosaic_amd as M
import oracle as O
from geom_util import NYC_BBOX, nyc_points, wkt_to_wkb

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def T(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(dev)


def gpu_cells(x, y, res, dev, isys=None):
    out, st = (isys or M.H3IndexSystem()).points_to_index(T(x, dev), T(y, dev), res, stats=True)
    return out.cpu().numpy(), st


def assert_h3_exact(got, lon, lat, res):
    """H3 cells bit for bit equal to the reference's: the oracle with glibc's libm and
    x87 long double, as H3-Java's JNI library computes them on this host.  Returns the
    number of these points where a correctly rounded libm would have given another cell
    (the cells the device's near-tie pass took from the reference's libm)."""
    gl = O.h3_points_to_cells(lon, lat, res)
    bad = np.nonzero(got != gl)[0]
    assert bad.size == 0, ("%d cells differ from the reference (glibc) oracle; first: %s" %
                           (bad.size, [(lon[i], lat[i], got[i], gl[i]) for i in bad[:3]]))
    with O.h3_libm("cr"):
        cr = O.h3_points_to_cells(lon, lat, res)
    return int(np.count_nonzero(gl != cr))


# ---------------------------------------------------------------- cell ids

def test_h3_kats_on_gpu(gpu):
    kats = json.load(open(os.path.join(GOLDEN, "h3_kats.json")))["kats"]
    for res in (9, 10):
        ks = [k for k in kats if k["res"] == res]
        got, _ = gpu_cells([k["lon"] for k in ks], [k["lat"] for k in ks], res, gpu)
        assert got.tolist() == [k["cell"] for k in ks]


@pytest.mark.parametrize("res", [0, 1, 5, 8, 9, 10, 11, 13, 15])
def test_h3_cells_global_equal_oracle(gpu, res):
    """Points uniform on the sphere: every icosahedron face, pentagons, overage."""
    rng = np.random.default_rng(100 + res)
    n = 400_000
    lon = rng.uniform(-180, 180, n)
    lat = np.degrees(np.arcsin(rng.uniform(-1, 1, n)))
    got, st = gpu_cells(lon, lat, res, gpu)
    assert_h3_exact(got, lon, lat, res)


def test_h3_edge_fixture_on_gpu(gpu):
    """180k points on / within 1e-14 deg of H3 cell corners and edges at res 0-15
    (tests/golden/h3_edge_points.npz, tools/gen_h3_edge_fixture.py): every cell equals
    the fixture's reference column (glibc libm, x87 -- H3-Java's arithmetic), 0 mismatches,
    including the 139 points where glibc misrounds a deciding argument; and the live
    oracle on this host agrees.  With the h3_libm option set to correctly rounded, the
    fixture's correctly rounded column instead."""
    f = np.load(os.path.join(GOLDEN, "h3_edge_points.npz"))
    lon, lat, res = f["lon"], f["lat"], f["res"]
    fixed = 0
    for r in np.unique(res):
        m = res == r
        got, st = gpu_cells(lon[m], lat[m], int(r), gpu)
        bad = np.nonzero(got != f["cell_glibc"][m])[0]
        assert bad.size == 0, (int(r), bad.size)
        assert np.array_equal(got, O.h3_points_to_cells(lon[m], lat[m], int(r)))
        fixed += st["libm_overrides"]
    assert fixed == int(np.count_nonzero(f["cell_glibc"] != f["cell_cr"]))
    with M.default_context(gpu).options(h3_libm=1):
        for r in np.unique(res):
            m = res == r
            got, st = gpu_cells(lon[m], lat[m], int(r), gpu)
            assert np.array_equal(got, f["cell_cr"][m]), int(r)
            assert st["libm_overrides"] == 0


def test_h3_cells_nyc_equal_oracle(gpu):
    x, y = nyc_points(2_000_000, 1)
    got, st = gpu_cells(x, y, 9, gpu)
    assert np.array_equal(got, O.h3_points_to_cells(x, y, 9))


def test_h3_invalid_coordinates_raise(gpu):
    with pytest.raises(M.IllegalArgumentException):
        gpu_cells([1.0, float("nan")], [1.0, 2.0], 9, gpu)
    with pytest.raises(M.IllegalStateException):
        gpu_cells([1.0], [1.0], 16, gpu)


@pytest.mark.parametrize("res", [1, 2, 3, 4, 5, 6, -1, -2, -3, -4, -5, -6])
def test_bng_cells_equal_oracle(gpu, res):
    rng = np.random.default_rng(200 + abs(res))
    n = 300_000
    e = rng.uniform(-50_000, 750_000, n)
    nn = rng.uniform(-50_000, 1_350_000, n)
    e[:5] = [3e9, -3e9, 538825.0, 0.0, -0.5]   # d2i saturation, exact KAT point, zero, -0 truncation
    nn[:5] = [1e3, 5e12, 179111.0, 0.0, 99999.99]
    got, _ = gpu_cells(e, nn, res, gpu, M.BNGIndexSystem())
    ref = O.bng_points_to_cells(e, nn, res)
    assert np.array_equal(got, ref)


def test_bng_format_device_equals_host(gpu):
    """BNG StringType ids formatted by the HIP kernel == the host formatter == the
    reference's known answers (TestBNGIndexSystem.scala), at all 12 resolutions."""
    bng = M.BNGIndexSystem()
    rng = np.random.default_rng(17)
    e = rng.uniform(0, 700_000, 100_000)
    nn = rng.uniform(0, 1_300_000, 100_000)
    for res in (1, 2, 3, 4, 5, 6, -1, -2, -3, -4, -5, -6):
        cells = O.bng_points_to_cells(e, nn, res)
        chars, off = bng.format_device(torch.from_numpy(cells).to(gpu))
        raw, o = chars.cpu().numpy().tobytes(), off.cpu().numpy()
        got = [raw[o[i]:o[i + 1]].decode() for i in range(len(cells))]
        assert got == bng.format_many(cells), res
    d = json.load(open(os.path.join(GOLDEN, "bng_kats.json")))
    cells = np.array([O.bng_point_to_index(k["e"], k["n"], k["res"]) for k in d["point_to_index"]], np.int64)
    chars, off = bng.format_device(torch.from_numpy(cells).to(gpu))
    raw, o = chars.cpu().numpy().tobytes(), off.cpu().numpy()
    assert [raw[o[i]:o[i + 1]].decode() for i in range(len(cells))] == [k["str"] for k in d["point_to_index"]]
    with pytest.raises(M.IllegalArgumentException):
        bng.format_device(torch.tensor([1051000, -5], dtype=torch.int64, device=gpu))
    chars, off = bng.format_device(torch.zeros(0, dtype=torch.int64, device=gpu))
    assert off.cpu().tolist() == [0] and chars.numel() == 0


def test_h3_string_ids_on_gpu(gpu):
    """grid_longlatascellid with StringType ids: the device H3 formatter == h3ToString
    (lowercase hex) of the oracle's cells, at res 0, 9 and 15."""
    rng = np.random.default_rng(31)
    x, y = rng.uniform(-180, 180, 50_000), rng.uniform(-90, 90, 50_000)
    for res in (0, 9, 15):
        chars, off = M.grid_longlatascellid(T(x, gpu), T(y, gpu), res, cell_id_type="string")
        raw, o = chars.cpu().numpy().tobytes(), off.cpu().numpy()
        got = [raw[o[i]:o[i + 1]].decode() for i in range(len(x))]
        assert got == ["%x" % c for c in O.h3_points_to_cells(x, y, res)], res
    e, nn = rng.uniform(0, 700_000, 1000), rng.uniform(0, 1_300_000, 1000)
    chars, off = M.grid_longlatascellid(T(e, gpu), T(nn, gpu), 3, index_system=M.BNGIndexSystem(),
                                        cell_id_type="string")
    raw, o = chars.cpu().numpy().tobytes(), off.cpu().numpy()
    assert [raw[o[i]:o[i + 1]].decode() for i in range(1000)] == \
        M.BNGIndexSystem().format_many(O.bng_points_to_cells(e, nn, 3))


@pytest.mark.parametrize("res", [1, 2, 3, 4, 5, 6, -1, -2, -3, -4, -5, -6])
def test_bng_kring_kloop_equal_oracle(gpu, res):
    """grid_cellkring / grid_cellkloop on the GPU == the oracle's restatement of
    BNGIndexSystem.kRing / kLoop (BNGIndexSystem.scala:221-252), lists in order, for
    cells all over the grid (the edges of the 700 km x 1300 km extent included, where
    isValid drops candidates)."""
    rng = np.random.default_rng(400 + abs(res) + (res < 0))
    e = np.concatenate([rng.uniform(0, 700_000, 300), [0.5, 699_999.0, 350_000.0, 1.0]])
    nn = np.concatenate([rng.uniform(0, 1_300_000, 300), [0.5, 1_299_999.0, 0.5, 1_299_999.0]])
    cells = O.bng_points_to_cells(e, nn, res)
    I = M.BNGIndexSystem()
    for k in (0, 1, 2, 3):
        for loop in (False, True):
            refs, ok = [], []
            for c in cells:
                try:
                    refs.append(O.bng_k_loop(int(c), k) if loop else O.bng_k_ring(int(c), k))
                    ok.append(True)
                except ValueError:  # the reference throws (NumberFormatException)
                    ok.append(False)
            ok = np.array(ok)
            good = cells[ok]
            ids, off = M.grid_cellkring(torch.from_numpy(good).to(gpu), k, I, loop_only=loop)
            ids, off = ids.cpu().numpy(), off.cpu().numpy()
            for i, c in enumerate(good):
                assert list(ids[off[i]:off[i + 1]]) == refs[i], (res, k, loop, int(c))
            if (~ok).any():
                with pytest.raises(M.IllegalArgumentException):
                    M.grid_cellkring(torch.from_numpy(cells[~ok]).to(gpu), k, I, loop_only=loop)


H3_PENTAGON_BASE_CELLS = {4, 14, 24, 38, 49, 58, 63, 72, 83, 97, 107, 117}


def h3_pentagon_cells(res):
    """The 12 pentagons of a resolution: a pentagon base cell with every digit 0."""
    unused = sum(7 << (3 * (15 - r)) for r in range(res + 1, 16))
    return [(1 << 59) | (res << 52) | (b << 45) | unused for b in sorted(H3_PENTAGON_BASE_CELLS)]


def assert_h3_rings_equal_oracle(gpu, cells, ks=(0, 1, 2, 4), tag=""):
    I = M.H3IndexSystem()
    cells = np.asarray(cells, dtype=np.int64)
    for k in ks:
        for loop in (False, True):
            refs = [O.h3_k_loop(int(c), k) if loop else O.h3_k_ring(int(c), k) for c in cells]
            ids, off = M.grid_cellkring(torch.from_numpy(cells).to(gpu), k, I, loop_only=loop)
            ids, off = ids.cpu().numpy(), off.cpu().numpy()
            for i, c in enumerate(cells):
                assert [int(v) for v in ids[off[i]:off[i + 1]]] == refs[i], (tag, k, loop, hex(int(c)))


@pytest.mark.parametrize("res", [1, 2, 3, 5, 7, 9, 11, 13, 15])
def test_h3_kring_kloop_equal_oracle(gpu, res):
    """grid_cellkring / grid_cellkloop for H3 on the GPU == the oracle's restatement of
    H3IndexSystem.kRing / kLoop (H3IndexSystem.scala:182-205 -> H3 v3.7 kRing spiral /
    hexRing), lists in order, on global cells -- base-cell crossings and pentagon
    neighbourhoods included (the walks that meet a pentagon take H3's _kRingInternal
    hash-set order, and kLoop Mosaic's kRing(k) diff kRing(k - 1) in Scala HashSet
    order); ids that are no H3 cell raise IllegalArgumentException."""
    rng = np.random.default_rng(900 + res)
    lon = rng.uniform(-180, 180, 600)
    lat = np.degrees(np.arcsin(rng.uniform(-1, 1, 600)))
    cells = O.h3_points_to_cells(lon, lat, res).astype(np.int64)
    assert_h3_rings_equal_oracle(gpu, cells, tag="global r%d" % res)
    with pytest.raises(M.IllegalArgumentException):
        M.grid_cellkring(torch.tensor([1051200030000], dtype=torch.int64, device=gpu), 1, M.H3IndexSystem())


@pytest.mark.parametrize("res", [0, 1, 2, 4, 6, 9, 12, 15])
def test_h3_kring_kloop_pentagons_equal_oracle(gpu, res):
    """The 12 pentagons of a resolution and the cells of their 2-rings (polar pentagons
    4 and 117 included): device == oracle for k = 0..4, ring and loop."""
    pents = h3_pentagon_cells(res)
    near = sorted({c for p in pents for c in O.h3_k_ring(p, 2)})
    assert_h3_rings_equal_oracle(gpu, pents + near, ks=(0, 1, 2, 3, 4), tag="pentagons r%d" % res)


def test_h3_kring_kloop_pentagons_large_k(gpu):
    """k beyond 64 near pentagons (the walk's stack lives in scratch, any k the entry
    accepts): four res-5 pentagons (polar 4 and 117 among them) and a neighbour, k = 65
    and 80, ring and loop, == the oracle.  (A walk is one lane's depth-first search: k =
    100 over 14 cells took ~2.5 min.)"""
    pents = h3_pentagon_cells(5)
    pick = [p for p in pents if ((p >> 45) & 127) in (4, 117)] + [p for p in pents if ((p >> 45) & 127) not in (4, 117)][:2]
    near = [O.h3_k_ring(pick[0], 1)[1]]
    assert_h3_rings_equal_oracle(gpu, pick + near, ks=(65, 80), tag="pentagons large k")


def test_index_system_scalar_k_ring_k_loop(gpu):
    """IndexSystem.kRing / kLoop (scalar surface of the mirror) == the oracle, H3 and BNG."""
    import numpy as np
    h = 613177664827555839
    assert M.H3IndexSystem().k_ring(h, 2) == O.h3_k_ring(h, 2)
    assert M.H3IndexSystem().k_loop(h, 3) == O.h3_k_loop(h, 3)
    b = int(O.bng_points_to_cells(np.array([530_123.0]), np.array([180_456.0]), 3)[0])
    assert M.BNGIndexSystem().k_ring(b, 2) == O.bng_k_ring(b, 2)
    assert M.BNGIndexSystem().k_loop(b, 2) == O.bng_k_loop(b, 2)


def test_h3_kring_doc_known_answer(gpu):
    """docs/source/api/spatial-indexing.rst:776-784 (grid_cellkringexplode of
    613177664827555839, k = 2): the first four ids of the reference's output."""
    ids, off = M.grid_cellkring(torch.tensor([613177664827555839], dtype=torch.int64, device=gpu), 2,
                                M.H3IndexSystem())
    got = [int(v) for v in ids.cpu().numpy()]
    assert len(got) == 19 and len(set(got)) == 19
    assert got[:4] == [613177664827555839, 613177664825458687, 613177664831750143, 613177664884178943]


def test_bng_nan_raises(gpu):
    with pytest.raises(M.IllegalStateException):
        gpu_cells([float("nan")], [100.0], 5, gpu, M.BNGIndexSystem())


def test_empty_inputs(gpu, nyc_chips_r9):
    e = torch.empty(0, dtype=torch.float64, device=gpu)
    assert M.grid_longlatascellid(e, e, 9).numel() == 0
    r = M.pip_join(e, e, nyc_chips_r9, 9)
    assert len(r) == 0


# ---------------------------------------------------------------- st_contains

def test_st_contains_two_holes_on_gpu(gpu):
    d = json.load(open(os.path.join(GOLDEN, "st_contains_kats.json")))
    for le in (False, True):
        w = wkt_to_wkb(d["polygon_wkt"], little_endian=le)
        ct = M.ChipTable.from_rows([(False, 1, w, 7)])
        pts = [(c["x"], c["y"]) for c in d["cases"]] + [(10, 50), (20, 25), (5, 5)]
        out = M.st_contains(ct, torch.zeros(len(pts), dtype=torch.int64), T([p[0] for p in pts], gpu),
                            T([p[1] for p in pts], gpu))
        assert out.cpu().tolist() == [1, 0, 0, 0, 0]


def test_st_contains_random_pairs_equal_oracle(gpu, nyc_chips_r9):
    c = nyc_chips_r9
    rng = np.random.default_rng(9)
    n = 200_000
    rows = rng.integers(0, len(c), n)
    # points near each chosen chip: jitter around one of its vertices, plus exact vertices
    x = np.empty(n)
    y = np.empty(n)
    import struct
    for k, r in enumerate(rows):
        b = c.wkb_offsets[r]
        e = c.wkb_offsets[r + 1]
        blob = bytes(c.wkb[b:e])
        # first coordinate pair of the first ring: header(5) + nrings(4) + npts(4) for a Polygon,
        # + 9 more bytes for a MultiPolygon's first part
        off = 13 if blob[4] == 3 else 22
        vx, vy = struct.unpack(">dd", blob[off:off + 16])
        if k % 4 == 0:
            x[k], y[k] = vx, vy
        else:
            x[k] = vx + rng.normal(0, 0.002)
            y[k] = vy + rng.normal(0, 0.002)
    out = M.st_contains(c, torch.from_numpy(rows), T(x, gpu), T(y, gpu)).cpu().numpy()
    ref = np.array([O.st_contains(bytes(c.wkb[c.wkb_offsets[r]:c.wkb_offsets[r + 1]]), x[k], y[k])
                    for k, r in enumerate(rows)], dtype=np.int8)
    assert np.array_equal(out, ref)
    assert ref.sum() > 0 and (ref == 0).sum() > 0


# ---------------------------------------------------------------- the join

def oracle_join(c, x, y, res=9, isys=0):
    return O.pip_join(isys, res, x, y, c.cell, c.polygon_id, c.is_core, c.wkb_offsets, c.wkb)


def test_pip_join_nyc_equals_oracle(gpu, nyc_chips_r9):
    x, y = nyc_points(3_000_000, 2)
    r = M.pip_join(T(x, gpu), T(y, gpu), nyc_chips_r9, 9)
    gp, gq = r.numpy()
    op, oq = oracle_join(nyc_chips_r9, x, y)
    assert len(gp) == len(op) and np.array_equal(gp, op) and np.array_equal(gq, oq)
    assert r.stats["n_pairs"] == len(op) and r.stats["n_candidates"] > 0
    assert np.all(np.diff(gp) >= 0)


def test_pip_join_explicit_point_ids_and_base(gpu, nyc_chips_r9):
    x, y = nyc_points(300_000, 3)
    ids = np.arange(300_000, dtype=np.int64) * 7 + 11
    r = M.pip_join(T(x, gpu), T(y, gpu), nyc_chips_r9, 9, point_id=torch.from_numpy(ids).to(gpu))
    op, oq = oracle_join(nyc_chips_r9, x, y)
    gp, gq = r.numpy()
    assert np.array_equal(gp, ids[op]) and np.array_equal(gq, oq)
    r2 = M.pip_join(T(x, gpu), T(y, gpu), nyc_chips_r9, 9, point_id_base=10 ** 12)
    assert np.array_equal(r2.numpy()[0], op + 10 ** 12)


def test_pip_join_capacity(gpu, nyc_chips_r9):
    x, y = nyc_points(100_000, 4)
    op, oq = oracle_join(nyc_chips_r9, x, y)
    with pytest.raises(M.CapacityError) as ei:
        M.pip_join(T(x, gpu), T(y, gpu), nyc_chips_r9, 9, capacity=10)
    assert ei.value.required == len(op)
    # undersized preallocated output: without a capacity the pairs go to exact-size
    # arrays (mgpu_pip_join_fetch); with one, the bound holds
    small = (torch.empty(10, dtype=torch.int64, device=gpu), torch.empty(10, dtype=torch.int32, device=gpu))
    gp, gq = M.pip_join(T(x, gpu), T(y, gpu), nyc_chips_r9, 9, out=small).numpy()
    assert np.array_equal(gp, op) and np.array_equal(gq, oq)
    with pytest.raises(M.CapacityError):
        M.pip_join(T(x, gpu), T(y, gpu), nyc_chips_r9, 9, out=small, capacity=10)


def test_pip_join_default_capacity_grows(gpu):
    """Overlapping polygons: every point matches 5 zones (> the 2 kept in registers, and
    more pairs than the default capacity), forcing both slow paths."""
    sq = [(0.0, 0.0), (1.0, 0.0), (1.0, 1.0), (0.0, 1.0), (0.0, 0.0)]
    polys = [(pid, [[[(x * (1 + 0.01 * pid), y * (1 + 0.01 * pid)) for x, y in sq]]]) for pid in (5, 3, 9, 1, 7)]
    P = M.Polygons.from_lists(polys)
    c = M.tessellate(P, M.H3IndexSystem(), 5)
    rng = np.random.default_rng(8)
    x = rng.uniform(0.05, 0.95, 50_000)
    y = rng.uniform(0.05, 0.95, 50_000)
    r = M.pip_join(T(x, gpu), T(y, gpu), c, 5)
    op, oq = oracle_join(c, x, y, res=5)
    gp, gq = r.numpy()
    assert len(op) > 4 * len(x)
    assert np.array_equal(gp, op) and np.array_equal(gq, oq)


def adversarial_points(c):
    """Points exactly on chip vertices and edge midpoints (most chip vertices are H3
    cell vertices, i.e. within a few ulps of three cells' common corner)."""
    import struct
    xs, ys = [], []
    for r in range(0, len(c), 3):
        blob = bytes(c.wkb[c.wkb_offsets[r]:c.wkb_offsets[r + 1]])
        if not blob or blob[4] != 3:
            continue
        (npts,) = struct.unpack(">I", blob[9:13])
        pts = [struct.unpack(">dd", blob[13 + 16 * i:29 + 16 * i]) for i in range(npts)]
        for i in range(npts - 1):
            xs += [pts[i][0], 0.5 * (pts[i][0] + pts[i + 1][0])]
            ys += [pts[i][1], 0.5 * (pts[i][1] + pts[i + 1][1])]
    return np.array(xs), np.array(ys)


def test_pip_join_adversarial_points(gpu, nyc_chips_r9):
    """Points on chip vertices and edge midpoints, i.e. on H3 cell corners, where a
    last-bit difference in libm moves the cell: cells and every pair equal the oracle
    with correctly rounded libm, no point excluded.  Against the oracle with glibc's
    libm (the reference's) the cells differ at exactly the points where glibc's
    misrounding moves the cell (diagnosed by the oracle's two modes); the kernel flagged
    each of them as a near-tie."""
    c = nyc_chips_r9
    x, y = adversarial_points(c)
    cells, st = gpu_cells(x, y, 9, gpu)
    n_cr = assert_h3_exact(cells, x, y, 9)
    assert st["libm_overrides"] == n_cr <= st["n_near_ties"]
    r = M.pip_join(T(x, gpu), T(y, gpu), c, 9)
    op, oq = oracle_join(c, x, y)
    gp, gq = r.numpy()
    assert np.array_equal(gp, op) and np.array_equal(gq, oq)


@pytest.mark.parametrize("pipeline", [0, 1, 2])
def test_pip_join_adversarial_override_pass(gpu, nyc_chips_r9, pipeline):
    """The override pass after the host's libm moved some cells reruns only the tiles
    (fused) / chunks (split) holding those points -- the binned pipeline whole -- and the
    pairs still equal the reference (glibc) oracle's, with the adversarial points spread
    through a larger batch of uniform points (so most tiles are clean)."""
    c = nyc_chips_r9
    ax, ay = adversarial_points(c)
    rng = np.random.default_rng(91)
    n = 600_000
    x = rng.uniform(-74.25, -73.70, n)
    y = rng.uniform(40.50, 40.91, n)
    at = np.sort(rng.choice(n, len(ax), replace=False))
    x[at], y[at] = ax, ay
    op, oq = oracle_join(c, x, y)
    ctx = M.default_context(gpu)
    with ctx.options(pipeline=pipeline):
        r = M.pip_join(T(x, gpu), T(y, gpu), c, 9)
    assert r.stats["pipeline"] == pipeline
    assert r.stats["libm_overrides"] > 0
    gp, gq = r.numpy()
    assert np.array_equal(gp, op) and np.array_equal(gq, oq)


@pytest.mark.parametrize("pipeline", [0, 1, 2])
def test_pip_join_negative_polygon_ids(gpu, nyc_chips_r9, pipeline):
    """Polygon ids are caller-supplied int32: negative ids (and INT32_MIN) must come out
    as given in every pipeline -- the split emit's one-match LDS shortcut must not use the
    id's sign as a flag (advisor finding, round 4)."""
    c0 = nyc_chips_r9
    pid = -c0.polygon_id.astype(np.int64) * 1000
    pid[c0.polygon_id == c0.polygon_id.max()] = -2 ** 31
    c = M.ChipTable(c0.cell, pid.astype(np.int32), c0.is_core, c0.wkb_offsets, c0.wkb)
    x, y = nyc_points(400_000, 17)
    op, oq = oracle_join(c, x, y)
    assert (oq < 0).all() and (oq == -2 ** 31).any()
    ctx = M.default_context(gpu)
    with ctx.options(pipeline=pipeline):
        r = M.pip_join(T(x, gpu), T(y, gpu), c, 9)
    assert r.stats["pipeline"] == pipeline
    gp, gq = r.numpy()
    assert np.array_equal(gp, op) and np.array_equal(gq, oq)


def test_pip_join_async_adversarial_points(gpu, nyc_chips_r9):
    """mgpu_pip_join_async + mgpu_pip_join_finish on the adversarial points: the pairs
    equal the reference (glibc) oracle's -- which differ from the correctly rounded
    oracle's on this set (21 cells move) -- and the synchronous join's, in both libm
    modes; finish without a pending join, or after another call ended it, raises."""
    c = nyc_chips_r9
    x, y = adversarial_points(c)
    op, oq = oracle_join(c, x, y)
    with O.h3_libm("cr"):
        cp, cq = oracle_join(c, x, y)
    assert not (len(op) == len(cp) and np.array_equal(op, cp) and np.array_equal(oq, cq))
    xt, yt = T(x, gpu), T(y, gpu)
    sync = M.pip_join(xt, yt, c, 9)
    aj = M.pip_join_async(xt, yt, c, 9)
    r = aj.finish()
    gp, gq = r.numpy()
    assert np.array_equal(gp, op) and np.array_equal(gq, oq)
    assert int(aj.count.item()) == len(op)
    assert r.stats["n_near_ties"] == sync.stats["n_near_ties"] > 0
    assert r.stats["libm_overrides"] == sync.stats["libm_overrides"]
    ctx = M.default_context(gpu)
    with ctx.options(h3_libm=1):  # MGPU_LIBM_CORRECTLY_ROUNDED
        gp2, gq2 = M.pip_join_async(xt, yt, c, 9).finish().numpy()
    assert np.array_equal(gp2, cp) and np.array_equal(gq2, cq)
    with pytest.raises(M.IllegalArgumentException):
        aj2 = M.pip_join_async(xt, yt, c, 9)
        M.pip_join(xt, yt, c, 9)  # another call on the context ends the pending join
        aj2.finish()
    with pytest.raises(M.IllegalArgumentException):
        M.AsyncJoin(ctx, None, None, None, None).finish()


def test_pip_join_bng_equals_oracle(gpu):
    from test_host import _bng_synthetic
    P = _bng_synthetic(seed=21, n=40)
    for res in (3, 4, -4, -2, -3, -5):
        c = M.tessellate(P, M.BNGIndexSystem(), res)
        rng = np.random.default_rng(res + 50)
        x = np.round(rng.uniform(505000, 560000, 1_000_000), 2)  # 0.01 m granularity like UPRNs
        y = np.round(rng.uniform(155000, 200000, 1_000_000), 2)
        r = M.pip_join(T(x, gpu), T(y, gpu), c, res, index_system=M.BNGIndexSystem())
        op, oq = oracle_join(c, x, y, res=res, isys=1)
        gp, gq = r.numpy()
        assert np.array_equal(gp, op) and np.array_equal(gq, oq), res


def test_pip_join_kats_on_gpu(gpu, nyc_chips_r9):
    kats = json.load(open(os.path.join(GOLDEN, "pip_kats.json")))["kats"]
    r = M.pip_join(T([k["lon"] for k in kats], gpu), T([k["lat"] for k in kats], gpu), nyc_chips_r9, 9)
    gp, gq = r.numpy()
    assert list(gp) == list(range(len(kats)))
    for k, q in zip(kats, gq):
        assert int(q) in k["objectids"]


def assert_device_blob_is_host_blob(d, c):
    """The upload (blob pieces staged straight to the device through pinned buffers) left
    exactly the bytes mgpu_chips_host_blob assembles on the host, padding included."""
    import ctypes
    from mosaic_amd import _native as N
    ptr, nbytes = d.device_blob()
    out, nb = ctypes.c_void_p(), ctypes.c_int64()
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    N.check(N.lib().mgpu_chips_host_blob(c.index_system, len(c), p(c.cell), p(c.polygon_id), p(c.is_core),
                                         p(c.wkb_offsets), p(c.wkb if c.wkb.size else np.zeros(1, np.uint8)),
                                         ctypes.byref(out), ctypes.byref(nb)))
    try:
        assert nb.value == nbytes
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        piece = 256 << 20
        buf = np.empty(min(piece, nbytes), np.uint8)
        for off in range(0, nbytes, piece):
            n = min(piece, nbytes - off)
            assert hip.hipMemcpy(buf.ctypes.data, ptr + off, n, 2) == 0  # device to host
            host = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(out.value + off))
            assert np.array_equal(buf[:n], host), "device blob differs in [%d, %d)" % (off, off + n)
    finally:
        N.lib().mgpu_host_free(out)


def test_chip_blob_roundtrip(gpu, nyc_chips_r9):
    """The replicated chip table (what RCCL broadcast carries) joins identically."""
    d = nyc_chips_r9.upload()
    assert_device_blob_is_host_blob(d, nyc_chips_r9)
    ptr, nbytes = d.device_blob()
    buf = torch.empty(nbytes, dtype=torch.uint8, device=gpu)
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    assert hip.hipMemcpy(buf.data_ptr(), ptr, nbytes, 3) == 0  # device to device
    d2 = M.DeviceChips.from_device_blob(d.ctx, buf.data_ptr(), nbytes)
    del buf
    x, y = nyc_points(200_000, 5)
    a = M.pip_join(T(x, gpu), T(y, gpu), d, 9).numpy()
    b = M.pip_join(T(x, gpu), T(y, gpu), d2, 9).numpy()
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert d2.info()["chips"] == len(nyc_chips_r9)


def test_pip_join_full_size_properties(gpu, nyc_chips_r9):
    """BASELINE C2 size (1e8 points): pairs ascend by point, every polygon id is a
    real zone, and a 1e6-point strided slice equals the oracle on those points."""
    n = 100_000_000
    g = torch.Generator(device=gpu)
    g.manual_seed(77)
    x = torch.rand(n, dtype=torch.float64, device=gpu, generator=g) * (NYC_BBOX[2] - NYC_BBOX[0]) + NYC_BBOX[0]
    y = torch.rand(n, dtype=torch.float64, device=gpu, generator=g) * (NYC_BBOX[3] - NYC_BBOX[1]) + NYC_BBOX[1]
    r = M.pip_join(x, y, nyc_chips_r9, 9)
    p = r.point_id
    assert bool((p[1:] >= p[:-1]).all())
    frac = len(r) / n
    assert 0.30 < frac < 0.42, frac
    idx = torch.arange(0, n, 100, device=gpu)
    xs, ys = x[idx].cpu().numpy(), y[idx].cpu().numpy()
    op, oq = oracle_join(nyc_chips_r9, xs, ys)
    mask = (p % 100) == 0
    gp = (p[mask] // 100).cpu().numpy()
    gq = r.polygon_id[mask].cpu().numpy()
    assert np.array_equal(gp, op) and np.array_equal(gq, oq)
    # near-tie audit: the points whose cell an ulp of libm could move, all of them,
    # recomputed by the oracle (glibc, as H3-Java) -- cells and pairs
    ties = M.default_context(gpu).last_near_ties()
    assert len(ties) == r.stats["n_near_ties"]
    if len(ties) == 0:
        return
    ti = torch.from_numpy(ties).to(gpu)
    xt, yt = x[ti].cpu().numpy(), y[ti].cpu().numpy()
    assert_h3_exact(gpu_cells(xt, yt, 9, gpu)[0], xt, yt, 9)
    op, oq = oracle_join(nyc_chips_r9, xt, yt)
    sel = torch.isin(p, ti)
    pos = {int(v): k for k, v in enumerate(ties)}
    gp = np.array([pos[int(v)] for v in p[sel].cpu().numpy()], dtype=np.int64)
    gq = r.polygon_id[sel].cpu().numpy()
    assert np.array_equal(gp, op) and np.array_equal(gq, oq)


def test_cells_full_size_near_tie_audit(gpu):
    """3e7 global points at res 9 and 15: every point the route resolved inside its tie
    band (the mgpu_last_near_ties list, uncapped) has the reference's (glibc) cell, and so
    does a strided 1e6-point sample."""
    n = 30_000_000
    g = torch.Generator(device=gpu)
    g.manual_seed(78)
    x = torch.rand(n, dtype=torch.float64, device=gpu, generator=g) * 360.0 - 180.0
    y = torch.rand(n, dtype=torch.float64, device=gpu, generator=g) * 180.0 - 90.0
    for res in (9, 15):
        cells, st = M.grid_longlatascellid(x, y, res, stats=True)
        ties = M.default_context(gpu).last_near_ties()
        assert len(ties) == st["n_near_ties"]
        idx = np.unique(np.concatenate([ties, np.arange(0, n, 30)]))
        ti = torch.from_numpy(idx).to(gpu)
        xt, yt = x[ti].cpu().numpy(), y[ti].cpu().numpy()
        assert_h3_exact(cells[ti].cpu().numpy(), xt, yt, res)


# ---------------------------------------------------------------- BASELINE configs C4 / C5

def test_pip_join_c4_london_districts_bng(gpu):
    """C4 (BNG): UPRN-like points x Voronoi districts covering the London extent."""
    import bench_workloads as W
    P = W.london_districts()
    for res in (3, 4):
        c = M.tessellate(P, M.BNGIndexSystem(), res)
        x, y = W.london_points(1_000_000, 40 + res)
        r = M.pip_join(T(x, gpu), T(y, gpu), c, res, index_system=M.BNGIndexSystem())
        op, oq = oracle_join(c, x, y, res=res, isys=1)
        gp, gq = r.numpy()
        assert np.array_equal(gp, op) and np.array_equal(gq, oq), res
        assert len(gp) > 0.95 * len(x)  # the districts tile the extent


@pytest.mark.parametrize("res", [3, 4])
def test_pip_join_bng_split_grid_codes(gpu, res):
    """BNG through the split pipeline with the dense grid entry as the code (option
    bng_split, round 6): a cell of core chips answers its points, an answer-grid square
    (res 3) answers its points, the rest are mixed -- pairs equal the oracle's and the
    fused pipeline's (bng_split = 0), on uniform points plus chip vertices / edge points and
    whole-metre points on square lines."""
    import bench_workloads as W
    from test_raster_host import adversarial_points as chip_adversaries
    P = W.london_districts()
    c = M.tessellate(P, M.BNGIndexSystem(), res)
    rng = np.random.default_rng(71 + res)
    a = chip_adversaries(c, rng, 1500)
    x0, y0 = W.london_points(400_000, 17 + res)
    sq = rng.integers(50300, 56100, 20000).astype(np.float64) * 10.0
    nn = rng.integers(155000, 201000, 20000).astype(np.float64)
    x = np.concatenate([x0, a[:, 0], sq, np.nextafter(sq, -np.inf)])
    y = np.concatenate([y0, a[:, 1], nn, nn])
    op, oq = oracle_join(c, x, y, res=res, isys=1)
    ctx = M.default_context(gpu)
    d = c.upload(ctx)
    for split in (1, 0):
        with ctx.options(bng_split=split):
            r = M.pip_join(T(x, gpu), T(y, gpu), d, res, index_system=M.BNGIndexSystem())
        assert r.stats["pipeline"] == (1 if split else 0), (split, r.stats["pipeline"])
        gp, gq = r.numpy()
        assert np.array_equal(gp, op) and np.array_equal(gq, oq), (res, split)


def test_pip_join_c4_answer_grid_edges(gpu):
    """C4 res 3 joins through the cells' answer grids (10 m squares): chip vertices and
    edge points (and their ulp neighbours), whole-metre points on square lines and just
    below them -- every pair equals the oracle's."""
    import bench_workloads as W
    from test_raster_host import adversarial_points as chip_adversaries
    P = W.london_districts()
    c = M.tessellate(P, M.BNGIndexSystem(), 3)
    rng = np.random.default_rng(58)
    a = chip_adversaries(c, rng, 2500)
    sq = rng.integers(50300, 56100, 60000).astype(np.float64) * 10.0  # square lines (10 m)
    nn = rng.integers(155000, 201000, 60000).astype(np.float64)
    x = np.concatenate([a[:, 0], sq, np.nextafter(sq, -np.inf), sq + 9.999999, nn * 0 + 530000.5])
    y = np.concatenate([a[:, 1], nn, nn, np.nextafter(nn * 1.0, np.inf), nn])
    r = M.pip_join(T(x, gpu), T(y, gpu), c, 3, index_system=M.BNGIndexSystem())
    op, oq = oracle_join(c, x, y, res=3, isys=1)
    gp, gq = r.numpy()
    assert np.array_equal(gp, op) and np.array_equal(gq, oq)


@pytest.mark.parametrize("pipeline", [0, 1, 2])
def test_pip_join_overlay_crossing_adversaries(gpu, nyc_zones, nyc_chips_r9, pipeline):
    """Round 6's border chips (JTS OverlayNG's cut, jts_overlay.h) through every pipeline on
    points a few ulps from the polygon-edge x cell-edge crossings (their chip vertices are
    RobustLineIntersector's nodes): NYC r9 (a 1,500-chip sample) and the London-like
    districts at BNG r4 with 0.01-m points on the square lines -- every pair equals the
    oracle's over the same table."""
    import bench_workloads as W
    from geom_util import crossing_adversaries
    from test_tessellate_host import _bng_cell_rings, _h3_cell_rings
    import jts_overlay as JO
    c = nyc_chips_r9
    x, y = crossing_adversaries(nyc_zones, c, lambda cell, w: _h3_cell_rings(cell), max_chips=1500)
    ctx = M.default_context(gpu)
    with ctx.options(pipeline=pipeline):
        r = M.pip_join(T(x, gpu), T(y, gpu), c, 9)
    op, oq = oracle_join(c, x, y)
    gp, gq = r.numpy()
    assert len(op) > 1000 and np.array_equal(gp, op) and np.array_equal(gq, oq)
    L = W.london_districts()
    cb = M.tessellate(L, M.BNGIndexSystem(), 4)
    x, y = crossing_adversaries(L, cb, lambda cell, w: _bng_cell_rings([q for pc in JO.wkb_rings(w) for q in pc], 100.0),
                                max_chips=3000, grid_step=0.01)
    with ctx.options(pipeline=pipeline):
        r = M.pip_join(T(x, gpu), T(y, gpu), cb, 4, index_system=M.BNGIndexSystem())
    op, oq = oracle_join(cb, x, y, res=4, isys=1)
    gp, gq = r.numpy()
    assert len(op) > 1000 and np.array_equal(gp, op) and np.array_equal(gq, oq)


def test_pip_join_c5_skewed_fractal(gpu):
    """C5: points concentrated on the boundaries of 49k-vertex fractal polygons."""
    import bench_workloads as W
    P = W.skewed_polygons()
    c = M.tessellate(P, M.H3IndexSystem(), 9)
    x, y = W.boundary_points(P, 400_000, 11, 0.003)
    r = M.pip_join(T(x, gpu), T(y, gpu), c, 9)
    op, oq = oracle_join(c, x, y)
    gp, gq = r.numpy()
    assert np.array_equal(gp, op) and np.array_equal(gq, oq)
    assert 0.2 * len(x) < len(gp) < 0.9 * len(x)


def test_pip_join_c3_tracts_res10(gpu):
    """C3's polygons (tract-like Voronoi partition, jittered shared edges) at res 10,
    on a 3,000-tract block the oracle finishes in seconds: every point in one tract."""
    import bench_workloads as W
    E = (-75.0, 40.0, -74.5, 40.4)
    P = W.tract_polygons(n_cells=3000, extent=E, seed=21)
    c = M.tessellate(P, M.H3IndexSystem(), 10, keep_core_geometries=False)
    x, y = W.extent_points(E, 400_000, 12)
    r = M.pip_join(T(x, gpu), T(y, gpu), c, 10)
    op, oq = oracle_join(c, x, y, res=10)
    gp, gq = r.numpy()
    assert np.array_equal(gp, op) and np.array_equal(gq, oq)
    assert len(np.unique(gp)) == len(gp) and len(gp) > 0.99 * len(x)


def test_pip_join_c3_full_table(gpu):
    """BASELINE config C3 as the bench builds it: all 74,000 tract-like polygons at H3
    res 10 (9.4M chips, 5.5M of them core, keepCoreGeometries=false -- far beyond the
    caches), 1.2M points uniform over the whole extent, pair-for-pair against the oracle
    (exactly one tract per point)."""
    import bench_workloads as W
    P = W.tract_polygons()
    c = M.tessellate(P, M.H3IndexSystem(), 10, keep_core_geometries=False)
    assert len(c) > 9_000_000 and len(np.unique(c.polygon_id)) == W.N_TRACTS
    d = c.upload()
    assert_device_blob_is_host_blob(d, c)
    x, y = W.extent_points(W.TRACT_EXTENT, 1_200_000, 31)
    r = M.pip_join(T(x, gpu), T(y, gpu), d, 10)
    gp, gq = r.numpy()
    op, oq = O.pip_join(0, 10, x, y, c.cell, c.polygon_id, c.is_core, c.wkb_offsets, c.wkb)
    assert np.array_equal(gp, op) and np.array_equal(gq, oq)
    assert len(np.unique(gp)) == len(gp) and len(gp) > 0.99 * len(x)


@pytest.mark.parametrize("isys", ["h3", "bng"])
def test_pip_join_more_than_32_chips_per_cell(gpu, isys):
    """40 nested, overlapping polygons: every cell holds 40 chips, past the 32 the
    streaming kernel keeps in a lane mask, so every tile goes through pip_fix_kernel."""
    if isys == "h3":
        base, sc, res, I = (-74.0, 40.7), 0.02, 7, M.H3IndexSystem()
    else:
        base, sc, res, I = (530000.0, 180000.0), 3000.0, 3, M.BNGIndexSystem()
    sq = [(0.0, 0.0), (1.0, 0.0), (1.0, 1.0), (0.0, 1.0), (0.0, 0.0)]
    polys = [(pid, [[[(base[0] + sc * u * (1 + 0.01 * pid), base[1] + sc * v * (1 + 0.013 * pid))
                      for u, v in sq]]]) for pid in range(40, 0, -1)]
    c = M.tessellate(M.Polygons.from_lists(polys), I, res)
    rng = np.random.default_rng(33)
    x = base[0] + sc * rng.uniform(-0.1, 1.6, 60_000)
    y = base[1] + sc * rng.uniform(-0.1, 1.6, 60_000)
    r = M.pip_join(T(x, gpu), T(y, gpu), c, res, index_system=I)
    op, oq = oracle_join(c, x, y, res=res, isys=0 if isys == "h3" else 1)
    gp, gq = r.numpy()
    assert len(op) > 10 * len(x)
    assert np.array_equal(gp, op) and np.array_equal(gq, oq)


def test_pip_join_bng_near_origin(gpu):
    """Chips and points around the BNG origin: negative eastings / northings give cell
    ids outside the (column, row) bijection (the reference's truncating arithmetic), so
    the dense grid must step aside for them -- chips there disable it, points there
    take the id + hash route."""
    I = M.BNGIndexSystem()
    rng = np.random.default_rng(77)
    x = np.round(rng.uniform(-3000, 3000, 400_000), 2)
    y = np.round(rng.uniform(-3000, 3000, 400_000), 2)
    sq = lambda a, b, c, d: [[[(a, b), (c, b), (c, d), (a, d), (a, b)]]]
    for polys in ([(1, sq(-1500, -700, 1300, 2100)), (2, sq(-2900, -2900, 2950, 2950))],   # chips at negative cells
                  [(1, sq(10, 20, 1990, 2500)), (2, sq(300, 300, 2900, 2900))]):         # chips positive only
        for res in (4, -4, 3):
            c = M.tessellate(M.Polygons.from_lists(polys), I, res)
            r = M.pip_join(T(x, gpu), T(y, gpu), c, res, index_system=I)
            op, oq = oracle_join(c, x, y, res=res, isys=1)
            gp, gq = r.numpy()
            assert np.array_equal(gp, op) and np.array_equal(gq, oq), res
            # a join at another resolution than the chips': no dense grid either
            r2 = M.pip_join(T(x, gpu), T(y, gpu), c, 5, index_system=I)
            op2, oq2 = oracle_join(c, x, y, res=5, isys=1)
            assert np.array_equal(r2.numpy()[0], op2) and np.array_equal(r2.numpy()[1], oq2)


# ---------------------------------------------------------------- round 2 additions

def test_pip_join_strided_point_ids(gpu, nyc_chips_r9):
    """A non-contiguous point_id column (a strided view) joins like its contiguous copy."""
    x, y = nyc_points(200_000, 31)
    ids_all = torch.arange(400_000, dtype=torch.int64, device=gpu) * 3 + 5
    ids = ids_all[::2]
    assert not ids.is_contiguous()
    r = M.pip_join(T(x, gpu), T(y, gpu), nyc_chips_r9, 9, point_id=ids)
    op, oq = oracle_join(nyc_chips_r9, x, y)
    gp, gq = r.numpy()
    assert np.array_equal(gp, ids.cpu().numpy()[op]) and np.array_equal(gq, oq)


def test_st_contains_bad_row_raises(gpu, nyc_chips_r9):
    d = nyc_chips_r9.upload()
    rows = torch.tensor([0, len(nyc_chips_r9), 1], dtype=torch.int64, device=gpu)
    with pytest.raises(M.IllegalArgumentException):
        M.st_contains(d, rows, T([-73.9, -73.9, -73.9], gpu), T([40.7, 40.7, 40.7], gpu))


def test_join_rejects_chips_of_another_index_system(gpu, nyc_chips_r9):
    d = nyc_chips_r9.upload()  # H3 chips
    x, y = nyc_points(1000, 32)
    with pytest.raises(M.IllegalArgumentException):
        M.pip_join(T(x, gpu), T(y, gpu), d, 4, index_system=M.BNGIndexSystem())


def test_pixel_index_on_off_identical(gpu, nyc_chips_r9):
    """The join answers identically with and without the chip table's pixel index
    (context option raster = 0 at upload builds the table without it), on uniform and
    adversarial points, H3 (NYC r9) and BNG (London districts r4)."""
    import bench_workloads as W
    cases = [(nyc_chips_r9, 9, M.H3IndexSystem(), nyc_points(2_000_000, 33))]
    ax, ay = adversarial_points(nyc_chips_r9)
    cases.append((nyc_chips_r9, 9, M.H3IndexSystem(), (ax, ay)))
    cb = M.tessellate(W.london_districts(), M.BNGIndexSystem(), 4)
    cases.append((cb, 4, M.BNGIndexSystem(), W.london_points(2_000_000, 34)))
    ctx = M.default_context(gpu)
    for c, res, isys, (x, y) in cases:
        with ctx.options(raster=0):
            d0 = c.upload()
        with ctx.options(raster_bng=1):
            d1 = c.upload()
        a = M.pip_join(T(x, gpu), T(y, gpu), d0, res, index_system=isys).numpy()
        rb = M.pip_join(T(x, gpu), T(y, gpu), d1, res, index_system=isys)
        b = rb.numpy()
        assert rb.stats["pipeline"] == 1  # the split pipeline (classify / mixed / emit)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
        with ctx.options(pipeline=0):  # the fused kernel's own pixel-index pass
            rf = M.pip_join(T(x, gpu), T(y, gpu), d1, res, index_system=isys)
        assert rf.stats["pipeline"] == 0
        f = rf.numpy()
        assert np.array_equal(a[0], f[0]) and np.array_equal(a[1], f[1])
    # and the oracle on a uniform slice (the adversarial set's near-ties are
    # test_pip_join_adversarial_points' subject)
    x, y = nyc_points(300_000, 35)
    b = M.pip_join(T(x, gpu), T(y, gpu), nyc_chips_r9.upload(), 9).numpy()
    op, oq = oracle_join(nyc_chips_r9, x, y)
    assert np.array_equal(b[0], op) and np.array_equal(b[1], oq)


def test_comm_single_rank(gpu, nyc_chips_r9):
    """The C ABI's RCCL path on a one-rank communicator: broadcast from the root keeps the
    table, the all-gathered offsets are (0, total)."""
    import ctypes
    from mosaic_amd import _native as N
    from mosaic_amd import dist as D
    ctx = M.GpuContext(gpu)
    uid = (ctypes.c_uint8 * N.MGPU_COMM_ID_BYTES)()
    N.check(N.lib().mgpu_comm_unique_id(uid))
    N.check(N.lib().mgpu_comm_init(ctx.handle, uid, 0, 1))
    assert D.comm_info(ctx) == (0, 1)
    # a root without a table: every rank (here the one) agrees on the failure after the
    # header broadcast and skips the bulk broadcast -- an error, not a hang
    outp = ctypes.c_void_p()
    s = torch.cuda.current_stream(gpu).cuda_stream
    with pytest.raises(M.IllegalArgumentException):
        N.check(N.lib().mgpu_chips_broadcast(ctx.handle, None, 0, ctypes.byref(outp), s))
    d = nyc_chips_r9.upload(ctx)
    d2 = D.broadcast_chips(d, ctx)
    assert d2 is d
    off, tot, counts = D.global_offsets(12345, ctx)
    assert (off, tot, list(counts)) == (0, 12345, [12345])
    # a host blob shipped by the host and uploaded joins like the table itself
    b = D.upload_host_blob(D.host_blob(nyc_chips_r9), ctx)
    x, y = nyc_points(100_000, 36)
    r1 = M.pip_join(T(x, gpu), T(y, gpu), d, 9).numpy()
    r2 = M.pip_join(T(x, gpu), T(y, gpu), b, 9).numpy()
    assert np.array_equal(r1[0], r2[0]) and np.array_equal(r1[1], r2[1])
    ctx.close()


def test_broadcast_receiver_path(gpu, nyc_chips_r9):
    """The receiving rank's side of mgpu_chips_broadcast (mgpu_test_receive_blob: the same
    header check, allocation and adoption, the bulk copy done locally): a valid blob joins
    like the original; a corrupt header and a failed allocation return errors at once."""
    import ctypes
    from mosaic_amd import _native as N
    from mosaic_amd import dist as D
    ctx = M.default_context(gpu)
    d = nyc_chips_r9.upload(ctx)
    blob = torch.from_numpy(np.frombuffer(D.host_blob(nyc_chips_r9), np.uint8).copy()).to(gpu)
    out = ctypes.c_void_p()
    N.check(N.lib().mgpu_test_receive_blob(ctx.handle, blob.data_ptr(), 0, ctypes.byref(out)))
    got = M.DeviceChips(None, ctx, handle=out)
    x, y = nyc_points(50_000, 37)
    r1 = M.pip_join(T(x, gpu), T(y, gpu), d, 9).numpy()
    r2 = M.pip_join(T(x, gpu), T(y, gpu), got, 9).numpy()
    assert np.array_equal(r1[0], r2[0]) and np.array_equal(r1[1], r2[1])
    bad = blob.clone()
    bad[:8] = 0  # no magic: "the root sent no chip-table blob"
    st = N.lib().mgpu_test_receive_blob(ctx.handle, bad.data_ptr(), 0, ctypes.byref(out))
    assert st == N.MGPU_E_INVALID_ARG and "no chip-table blob" in N.last_error()
    st = N.lib().mgpu_test_receive_blob(ctx.handle, blob.data_ptr(), 1, ctypes.byref(out))
    assert st == N.MGPU_E_DEVICE and "hipMalloc" in N.last_error()


# ---------------------------------------------------------------- SpatialKNN's ring join

@pytest.mark.parametrize("isys_name,res,k,loop_only,keep,maxd", [
    ("H3", 9, 1, False, 0, -1.0), ("H3", 9, 2, True, 5, -1.0), ("H3", 8, 1, False, 3, 0.004),
    ("BNG", 3, 1, False, 0, -1.0), ("BNG", 3, 2, True, 4, 2500.0), ("H3", 2, 1, False, 0, -1.0)])
def test_ring_join_equals_oracle(gpu, isys_name, res, k, loop_only, keep, maxd):
    """grid_ring_join (GridRingNeighbours.transform + resultTransform, one iteration, point
    landmarks x point candidates) == the oracle's restatement, pairs and distances bit for
    bit: kRing (iteration 1) and kLoop (iteration k) cells, self matches dropped (some
    candidates are copies of landmarks), the distance threshold, the per-landmark cut; H3
    res 2 around a pentagon (the kRing walks' pentagon fallback)."""
    rng = np.random.default_rng(300 + res + 10 * k)
    if isys_name == "BNG":
        isys, code = M.BNGIndexSystem(), 1
        lx, ly = rng.uniform(520_000, 540_000, 1000), rng.uniform(170_000, 190_000, 1000)
        rx, ry = rng.uniform(518_000, 542_000, 8000), rng.uniform(168_000, 192_000, 8000)
    elif res == 2:
        isys, code = M.H3IndexSystem(), 0
        import ctypes
        from mosaic_amd import _native as N
        xy, nv, ctr = np.zeros(20), np.zeros(1, np.int32), np.zeros(2)  # base cell 14's centre (a pentagon)
        N.check(N.lib().mgpu_test_h3_boundary_host(np.array([(1 << 59) | (14 << 45) | 0x1FFFFFFFFFFF], np.int64).ctypes.data,
                                                     1, xy.ctypes.data, nv.ctypes.data, ctr.ctypes.data))
        lx, ly = rng.uniform(ctr[0] - 8, ctr[0] + 8, 600), rng.uniform(ctr[1] - 6, ctr[1] + 6, 600)
        rx, ry = rng.uniform(ctr[0] - 12, ctr[0] + 12, 2500), rng.uniform(ctr[1] - 9, ctr[1] + 9, 2500)
    else:
        isys, code = M.H3IndexSystem(), 0
        lx, ly = nyc_points(3000, 40 + k)
        rx, ry = nyc_points(30000, 50 + k)
    rx[:500], ry[:500] = lx[:500], ly[:500]  # self matches
    got = M.grid_ring_join(T(lx, gpu), T(ly, gpu), T(rx, gpu), T(ry, gpu), res, k, index_system=isys,
                           loop_only=loop_only, max_per_left=keep, max_distance=maxd, left_id_base=7)
    gl, gr, gd = (v.cpu().numpy() for v in got)
    ol, orr, od = O.ring_join(code, res, k, lx, ly, rx, ry, loop_only=loop_only, max_per_left=keep,
                              max_distance=maxd, left_id_base=7)
    assert len(ol) > len(lx) // 2
    assert np.array_equal(gl, ol) and np.array_equal(gr, orr)
    assert np.array_equal(gd.view(np.int64), od.view(np.int64))


@pytest.mark.parametrize("isys_name,res,keep", [("H3", 9, 0), ("H3", 9, 3), ("BNG", 3, 0)])
def test_ring_join_left_outer_equals_oracle(gpu, isys_name, res, keep):
    """left_outer = True: the left_outer join's null row (right -1, distance NaN) first for
    every landmark with a ring cell that holds no candidate (GridRingNeighbours.scala:128,
    151), sparse candidates so many cells are empty; otherwise the pairs of left_outer =
    False."""
    rng = np.random.default_rng(77 + res)
    if isys_name == "BNG":
        isys, code = M.BNGIndexSystem(), 1
        lx, ly = rng.uniform(520_000, 540_000, 700), rng.uniform(170_000, 190_000, 700)
        rx, ry = rng.uniform(518_000, 542_000, 300), rng.uniform(168_000, 192_000, 300)
    else:
        isys, code = M.H3IndexSystem(), 0
        lx, ly = nyc_points(2000, 61)
        rx, ry = nyc_points(3000, 62)
    got = M.grid_ring_join(T(lx, gpu), T(ly, gpu), T(rx, gpu), T(ry, gpu), res, 1, index_system=isys,
                           max_per_left=keep, left_outer=True)
    gl, gr, gd = (v.cpu().numpy() for v in got)
    ol, orr, od = O.ring_join(code, res, 1, lx, ly, rx, ry, max_per_left=keep, left_outer=True)
    assert (orr == -1).sum() > 100 and (orr >= 0).sum() > 100
    assert np.array_equal(gl, ol) and np.array_equal(gr, orr)
    assert np.array_equal(gd.view(np.int64), od.view(np.int64))  # (NaN rows: the same quiet NaN)
    plain = [v.cpu().numpy() for v in M.grid_ring_join(T(lx, gpu), T(ly, gpu), T(rx, gpu), T(ry, gpu), res, 1,
                                                       index_system=isys, max_per_left=keep)]
    assert np.array_equal(plain[1], gr[gr >= 0]) and np.array_equal(plain[0], gl[gr >= 0])


@pytest.mark.parametrize("isys_name,res", [("H3", 9), ("BNG", 3)])
def test_ring_join_final_equals_oracle(gpu, isys_name, res):
    """SpatialKNN's exactness iteration (mgpu_ring_join_final, GridRingNeighbours.scala:82-90):
    per landmark the cells of grid_tessellate(st_buffer(landmark, radius)) minus its iterated
    kRing, joined with the candidates.  The oracle takes the circles' chip tables from the
    tessellator (as every chip table input) and restates the rest: the 32-gon circle, the
    kRing difference, the join, distances, order, the left_outer null rows.  Landmarks with
    radius NaN / 0 have no cells."""
    rng = np.random.default_rng(91 + res)
    if isys_name == "BNG":
        isys, code = M.BNGIndexSystem(), 1
        lx, ly = rng.uniform(520_000, 540_000, 300), rng.uniform(170_000, 190_000, 300)
        rx, ry = rng.uniform(518_000, 542_000, 20000), rng.uniform(168_000, 192_000, 20000)
        radius = rng.uniform(500, 4000, len(lx))
    else:
        isys, code = M.H3IndexSystem(), 0
        lx, ly = nyc_points(400, 63)
        rx, ry = nyc_points(60000, 64)
        radius = rng.uniform(0.001, 0.008, len(lx))
    radius[:5] = [np.nan, 0.0, -1.0, radius[3], radius[4]]
    kit = rng.integers(1, 4, len(lx)).astype(np.int32)
    got = M.grid_ring_join_final(T(lx, gpu), T(ly, gpu), radius, kit, T(rx, gpu), T(ry, gpu), res, index_system=isys,
                                 left_outer=True, left_id_base=3)
    gl, gr, gd = (v.cpu().numpy() for v in got)
    # the circles' cells from the tessellator
    ok = np.nonzero((radius > 0) & np.isfinite(radius))[0]
    P = M.Polygons.from_lists([(int(i), [[O.jts_circle(lx[i], ly[i], radius[i])]]) for i in ok])
    chips = M.tessellate(P, isys, res, keep_core_geometries=False)
    buf = [[] for _ in lx]
    for c, p in zip(chips.cell.tolist(), chips.polygon_id.tolist()):
        buf[p].append(c)
    cells = O.ring_join_final_cells(code, res, lx, ly, radius, kit, buf)
    assert sum(len(c) for c in cells) > 2 * len(lx)
    ol, orr, od = O.ring_join(code, res, 0, lx, ly, rx, ry, left_id_base=3, left_outer=True, cells=cells)
    assert (orr >= 0).sum() > len(lx)
    assert np.array_equal(gl, ol) and np.array_equal(gr, orr)
    assert np.array_equal(gd.view(np.int64), od.view(np.int64))
    assert not np.isin(np.arange(3, 6), gl).any()  # the NaN / 0 / negative radius landmarks 0-2


def test_ring_join_batched_equals_oracle(gpu):
    """Landmarks processed in batches of bounded candidate pairs (option ring_batch, here
    500 pairs: dozens of batches, some landmarks alone in theirs) give the same rows as
    the oracle, with the cut, the threshold and the left_outer null rows."""
    lx, ly = nyc_points(3000, 71)
    rx, ry = nyc_points(40000, 72)
    rx[:300], ry[:300] = lx[:300], ly[:300]
    with M.default_context(gpu).options(ring_batch=500):
        got = M.grid_ring_join(T(lx, gpu), T(ly, gpu), T(rx, gpu), T(ry, gpu), 9, 1, max_per_left=4,
                               max_distance=0.004, left_outer=True)
    gl, gr, gd = (v.cpu().numpy() for v in got)
    ol, orr, od = O.ring_join(0, 9, 1, lx, ly, rx, ry, max_per_left=4, max_distance=0.004, left_outer=True)
    assert len(ol) > 3000
    assert np.array_equal(gl, ol) and np.array_equal(gr, orr)
    assert np.array_equal(gd.view(np.int64), od.view(np.int64))
