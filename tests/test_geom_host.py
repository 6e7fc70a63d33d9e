"""Geometry decoding for grid_pointascellid on a geometry column, on the CPU (no GPU).

The reference reads the point of a WKB / WKT row with JTS (GeometryAPI.scala:81-89 ->
WKBReader / WKTReader, then getCentroid in PointIndexGeom.scala:33-47).  WKT numbers go
through java.lang.Double.parseDouble, which rounds the decimal value exactly; Python's
float() rounds the same way (both are correctly rounded, round-half-even), so it is the
oracle for `mgpu::dec::parse_number` (mosaic_amd/csrc/decimal.h).  The same header code
runs inside the decode kernel, so the host entry points check the device parser.
"""
import ctypes
import struct

import numpy as np
import pytest

from mosaic_amd import _native as N


def parse(s):
    b = s.encode()
    v = ctypes.c_double()
    n = N.lib().mgpu_test_parse_number(b, len(b), ctypes.byref(v))
    return n, v.value


def decode(fmt, data):
    if isinstance(data, str):
        data = data.encode()
    buf = ctypes.create_string_buffer(data, max(len(data), 1))
    x, y = ctypes.c_double(), ctypes.c_double()
    st = N.lib().mgpu_test_decode_point(fmt, buf, len(data), ctypes.byref(x), ctypes.byref(y))
    return st, x.value, y.value


def same(a, b):
    return (a == b and np.signbit(a) == np.signbit(b)) or (a != a and b != b)


KNOWN = ["-73.956758", "40.769978", "0", "-0", ".5", "5.", "0.0000", "1e-400", "1e400", "NaN",
         "2.2250738585072011e-308", "2.2250738585072012e-308", "4.9e-324", "2.4703282292062327e-324",
         "2.4703282292062328e-324", "1.7976931348623157e308", "1.7976931348623158e308",
         "1.7976931348623159e308", "9007199254740993", "9007199254740992.5", "123456789012345678901234567890",
         "0.1", "0.30000000000000004", "1E22", "1e23", "8.98846567431158e307", "4.35623e-5",
         "+12.5", "1.00000000000000011102230246251565404236316680908203125",
         "1.00000000000000011102230246251565404236316680908203124",
         "1.00000000000000011102230246251565404236316680908203126"]


@pytest.mark.parametrize("s", KNOWN)
def test_parse_known(s):
    n, v = parse(s)
    assert n == len(s)
    assert same(v, float(s)), (s, v, float(s))


def test_parse_random_against_float():
    rng = np.random.default_rng(5)
    strs = []
    for _ in range(6000):
        nd = int(rng.integers(1, 30))
        dg = "".join(map(str, rng.integers(0, 10, nd)))
        p = int(rng.integers(0, nd + 1))
        body = dg[:p] + "." + dg[p:] if p < nd else dg
        if body.startswith("."):
            body = "0" + body
        e = int(rng.choice([0, 0, int(rng.integers(-340, 320))]))
        s = ("-" if rng.random() < 0.3 else "") + body + ("e%d" % e if e else "")
        strs.append(s)
    # shortest reprs and their half-way neighbours
    for v in rng.standard_normal(1500) * 10.0 ** rng.integers(-300, 300, 1500):
        strs.append(repr(float(v)))
        a, b = float(v), float(np.nextafter(v, np.inf))
        from decimal import Decimal
        mid = (Decimal(a) + Decimal(b)) / 2
        strs.append(format(mid, "e"))
    bad = []
    for s in strs:
        n, v = parse(s)
        if n != len(s) or not same(v, float(s)):
            bad.append((s, n, v, float(s)))
    assert not bad, bad[:10]


def test_parse_stops_at_delimiters():
    assert parse("12.5 40")[0] == 4
    assert parse("-3)")[0] == 2
    assert parse("1e")[0] == 0  # an exponent marker needs digits (Java: NumberFormatException)
    assert parse("abc")[0] == 0
    assert parse("-")[0] == 0


def wkb_point(x, y, le=True, z=None, srid=None):
    bo = "<" if le else ">"
    t = 1
    if z is not None:
        t |= 0x80000000
    if srid is not None:
        t |= 0x20000000
    b = struct.pack(bo + "BI", 1 if le else 0, t)
    if srid is not None:
        b += struct.pack(bo + "I", srid)
    b += struct.pack(bo + "dd", x, y)
    if z is not None:
        b += struct.pack(bo + "d", z)
    return b


def test_wkb_points():
    assert decode(N.MGPU_GEOM_WKB, wkb_point(-73.95, 40.77)) == (0, -73.95, 40.77)
    assert decode(N.MGPU_GEOM_WKB, wkb_point(-73.95, 40.77, le=False)) == (0, -73.95, 40.77)
    assert decode(N.MGPU_GEOM_WKB, wkb_point(1.5, 2.5, z=9.0, srid=4326)) == (0, 1.5, 2.5)
    iso_z = struct.pack("<BIddd", 1, 1001, 3.0, 4.0, 5.0)
    assert decode(N.MGPU_GEOM_WKB, iso_z) == (0, 3.0, 4.0)
    assert decode(N.MGPU_GEOM_WKB, wkb_point(float("nan"), float("nan")))[0] == 3  # POINT EMPTY
    assert decode(N.MGPU_GEOM_WKB, wkb_point(1.0, 2.0)[:-1])[0] == 1  # truncated
    assert decode(N.MGPU_GEOM_WKB, b"")[0] == 1
    assert decode(N.MGPU_GEOM_WKB, struct.pack("<BII", 1, 3, 0))[0] == 2  # polygon: unsupported
    pts = [(1.0, 2.0), (3.0, 5.0), (-4.0, 0.5)]
    mp = struct.pack("<BII", 1, 4, len(pts)) + b"".join(wkb_point(*p) for p in pts)
    st, x, y = decode(N.MGPU_GEOM_WKB, mp)
    assert st == 0 and x == (1.0 + 3.0 - 4.0) / 3 and y == (2.0 + 5.0 + 0.5) / 3


def test_wkt_points():
    W = N.MGPU_GEOM_WKT
    assert decode(W, "POINT (-73.956758 40.769978)") == (0, -73.956758, 40.769978)
    assert decode(W, "  point(1 2)") == (0, 1.0, 2.0)
    assert decode(W, "POINT Z (1 2 3)") == (0, 1.0, 2.0)
    assert decode(W, "POINT ZM (1 2 3 4)") == (0, 1.0, 2.0)
    assert decode(W, "POINT (1e2 -2.5E-1)") == (0, 100.0, -0.25)
    assert decode(W, "POINT EMPTY")[0] == 3
    assert decode(W, "POINT (1)")[0] == 1
    assert decode(W, "POINT (1 2")[0] == 1
    assert decode(W, "LINESTRING (1 2, 3 4)")[0] == 2
    st, x, y = decode(W, "MULTIPOINT ((1 2), (3 5))")
    assert st == 0 and (x, y) == (2.0, 3.5)
    st, x, y = decode(W, "MULTIPOINT (1 2, 3 5, 5 8)")
    assert st == 0 and (x, y) == (3.0, 5.0)
    assert decode(W, "MULTIPOINT EMPTY")[0] == 3
