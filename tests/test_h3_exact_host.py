"""The exact H3 route (mosaic_amd/csrc/h3_exact.h) on the host, against the oracle.

The reference's geoToH3 runs H3 v3.7 C on x86-64: five expressions on long-double
constants evaluated by the x87 unit, and glibc's sin/cos/tan/acos/atan2.  The product's
route emulates the x87 expressions bit for bit and uses correctly rounded libm
(double-double, rounded once).  Checked here:
  * each emulated x87 expression == the compiler's real `long double` expression;
  * each correctly rounded function == libquadmath's 113-bit function rounded once;
  * the whole route == the oracle with correctly rounded libm, bit for bit, on random
    points and on the corner/edge fixture (tests/golden/h3_edge_points.npz);
  * against the oracle with glibc's libm (the reference's) the route differs only where
    glibc misrounds: every disagreement is a point where the oracle's two libm modes
    disagree too, and there are none on uniformly random points.
Same header on the device: tests/test_gpu_parity.py repeats the fixture and corner checks
on the MI355X.
"""
import ctypes
import os

import numpy as np
import pytest

import oracle as O
from mosaic_amd import _native

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
X87_OPS = {5: "x + M_2PI", 6: "x - M_2PI", 7: "x * M_SQRT7", 8: "x / M_SIN60", 9: "x - M_AP7_ROT_RADS",
           10: "x / M_SQRT7", 11: "x + M_AP7_ROT_RADS", 12: "x < EPSILON", 13: "x >= M_2PI"}


def _P(a):
    return ctypes.c_void_p(a.ctypes.data)


def elementary(fn, a, b=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    out = np.empty_like(a)
    bb = None if b is None else np.ascontiguousarray(b, dtype=np.float64)
    _native.check(_native.lib().mgpu_test_h3_elementary_host(fn, _P(a), None if bb is None else _P(bb), len(a), _P(out)))
    return out


def route(lon, lat, res):
    lon = np.ascontiguousarray(lon, dtype=np.float64)
    lat = np.ascontiguousarray(lat, dtype=np.float64)
    out = np.empty(len(lon), np.int64)
    _native.check(_native.lib().mgpu_test_h3_route_host(_P(lon), _P(lat), len(lon), int(res), _P(out)))
    return out


def _x87_args(fn, rng, n):
    if fn in (5,):
        a = rng.uniform(-6.3, 0.0, n)
    elif fn in (6, 13):
        a = rng.uniform(6.2, 6.4, n)
    elif fn in (9, 11):
        a = rng.uniform(0.0, 6.3, n)
    elif fn == 12:
        a = np.concatenate([rng.uniform(0, 3e-16, n // 2), 1e-16 * (1 + rng.integers(-4, 5, n - n // 2) * 2.0 ** -52)])
    else:
        a = np.ldexp(rng.uniform(0.5, 1.0, n), rng.integers(-30, 40, n))
    # edge values: exact ties of the double rounding are most likely on short significands
    a[:1000] = np.round(a[:1000] * 2 ** 20) / 2 ** 20
    return a


@pytest.mark.parametrize("fn", sorted(X87_OPS))
def test_x87_emulation_equals_long_double(fn):
    rng = np.random.default_rng(100 + fn)
    a = _x87_args(fn, rng, 400_000)
    got = elementary(fn, a)
    ref = O.h3_elementary(fn, a)
    bad = np.nonzero(got.view(np.int64) != ref.view(np.int64))[0]
    assert bad.size == 0, (X87_OPS[fn], [(a[i], got[i], ref[i]) for i in bad[:3]])


CR_ARGS = {
    0: lambda r, n: r.uniform(-7.0, 7.0, n),      # sin: lat, lon, lon - face lon, theta
    1: lambda r, n: r.uniform(-7.0, 7.0, n),
    2: lambda r, n: r.uniform(0.0, 0.8, n),       # tan(r), r = angular distance to the face centre
    3: lambda r, n: np.concatenate([r.uniform(0.75, 1.0, n // 2), r.uniform(-1.0, 1.0, n - n // 2)]),
}


@pytest.mark.parametrize("fn", [0, 1, 2, 3, 4])
def test_correctly_rounded_libm(fn):
    """h3_exact.h's functions == libquadmath's, rounded once (bit for bit); and how
    often glibc's libm (the reference's) rounds the other way on the same arguments."""
    rng = np.random.default_rng(200 + fn)
    n = 300_000
    if fn == 4:
        a, b = rng.normal(size=n), rng.normal(size=n)
    else:
        a, b = CR_ARGS[fn](rng, n), None
    got = elementary(fn, a, b)
    cr = O.h3_elementary(20 + fn, a, b)
    bad = np.nonzero(got.view(np.int64) != cr.view(np.int64))[0]
    assert bad.size == 0, [(a[i], got[i], cr[i]) for i in bad[:3]]
    glibc = O.h3_elementary(fn, a, b)
    miss = np.count_nonzero(glibc != cr)
    # glibc 2.35's dbl-64 functions are accurate to < 1 ulp, not correctly rounded
    assert miss < n // 100
    print("fn %d: glibc misrounds %d of %d arguments" % (fn, miss, n))


def test_route_equals_correctly_rounded_oracle_global():
    rng = np.random.default_rng(7)
    n = 300_000
    for res in (0, 3, 7, 9, 10, 12, 15):
        lon = rng.uniform(-180.0, 180.0, n)
        lat = np.degrees(np.arcsin(rng.uniform(-1.0, 1.0, n)))
        got = route(lon, lat, res)
        with O.h3_libm("cr"):
            cr = O.h3_points_to_cells(lon, lat, res)
        assert np.array_equal(got, cr), res
        # uniformly random points never come close enough to a cell edge for glibc's
        # last-bit rounding to matter
        assert np.array_equal(got, O.h3_points_to_cells(lon, lat, res)), res


def test_route_on_edge_fixture():
    """Corners and edges of H3 cells (the fixture's generator: tools/gen_h3_edge_fixture.py)."""
    f = np.load(os.path.join(GOLDEN, "h3_edge_points.npz"))
    lon, lat, res = f["lon"], f["lat"], f["res"]
    glibc_vs_cr = np.nonzero(f["cell_glibc"] != f["cell_cr"])[0]
    assert len(lon) >= 100_000 and glibc_vs_cr.size < len(lon) // 500
    for r in np.unique(res):
        m = res == r
        got = route(lon[m], lat[m], int(r))
        assert np.array_equal(got, f["cell_cr"][m]), int(r)
        # the fixture pins the oracle in both libm modes
        assert np.array_equal(O.h3_points_to_cells(lon[m], lat[m], int(r)), f["cell_glibc"][m])
        with O.h3_libm("cr"):
            assert np.array_equal(O.h3_points_to_cells(lon[m], lat[m], int(r)), f["cell_cr"][m])


def glibc_route(lon, lat, res):
    lon = np.ascontiguousarray(lon, np.float64)
    lat = np.ascontiguousarray(lat, np.float64)
    out = np.zeros(len(lon), np.int64)
    assert _native.lib().mgpu_test_h3_glibc_host(lon.ctypes.data, lat.ctypes.data, len(lon), int(res),
                                                 out.ctypes.data) == 0
    return out


def test_near_tie_resolver_equals_reference_on_edge_fixture():
    """The library's near-tie resolver (h3_glibc.cpp: platform glibc libm, x87 long
    double, gcc without FMA contraction -- H3-Java's JNI arithmetic) equals the fixture's
    reference column on all 180k corner / edge points, 0 mismatches, including the points
    where glibc misrounds a deciding argument; and the oracle's glibc mode on this host."""
    f = np.load(os.path.join(GOLDEN, "h3_edge_points.npz"))
    lon, lat, res = f["lon"], f["lat"], f["res"]
    for r in np.unique(res):
        m = res == r
        got = glibc_route(lon[m], lat[m], int(r))
        assert np.array_equal(got, f["cell_glibc"][m]), int(r)
        assert np.array_equal(got, O.h3_points_to_cells(lon[m], lat[m], int(r))), int(r)


def test_near_tie_resolver_equals_reference_global():
    rng = np.random.default_rng(8)
    n = 200_000
    for res in (0, 1, 5, 9, 10, 15):
        lon = rng.uniform(-180.0, 180.0, n)
        lat = np.degrees(np.arcsin(rng.uniform(-1.0, 1.0, n)))
        assert np.array_equal(glibc_route(lon, lat, res), O.h3_points_to_cells(lon, lat, res)), res
    # H3-Java rejects non-finite input (geoToH3 returns H3_NULL)
    assert glibc_route([np.nan, 1.0], [1.0, np.inf], 9).tolist() == [0, 0]
