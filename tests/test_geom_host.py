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
    assert decode(N.MGPU_GEOM_WKB, struct.pack("<BII", 1, 3, 0))[0] == 3  # POLYGON EMPTY
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
    assert decode(W, "LINESTRING (1 2, 3 4)") == (0, 2.0, 3.0)
    assert decode(W, "CIRCULARSTRING (1 2, 3 4, 5 6)")[0] == 2  # (no JTS WKT type)
    st, x, y = decode(W, "MULTIPOINT ((1 2), (3 5))")
    assert st == 0 and (x, y) == (2.0, 3.5)
    st, x, y = decode(W, "MULTIPOINT (1 2, 3 5, 5 8)")
    assert st == 0 and (x, y) == (3.0, 5.0)
    assert decode(W, "MULTIPOINT EMPTY")[0] == 3


# ---------------------------------------------------------------- centroids of any geometry
# The reference takes JTS's Centroid of whatever the row holds (PointIndexGeom.scala:
# 33-47); the oracle is oracle/jts_centroid.py's restatement of JTS 1.20 Centroid.
import sys  # noqa: E402
import os  # noqa: E402
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import jts_centroid as JC  # noqa: E402


def _w_seq(bo, pts, z):
    b = struct.pack(bo + "I", len(pts))
    for p in pts:
        b += struct.pack(bo + "dd", *p) + (struct.pack(bo + "d", 7.0) if z else b"")
    return b


def w_geom(kind, data, le=True, z=False):
    """WKB of ('point', p) / ('line', pts) / ('poly', rings) / ('multi...', [parts]) /
    ('collection', [(kind, data), ...])."""
    bo = "<" if le else ">"
    codes = {"point": 1, "line": 2, "poly": 3, "mpoint": 4, "mline": 5, "mpoly": 6, "collection": 7}
    t = codes[kind] + (1000 if z else 0)
    b = struct.pack(bo + "BI", 1 if le else 0, t)
    if kind == "point":
        return b + struct.pack(bo + "dd", *data) + (struct.pack(bo + "d", 7.0) if z else b"")
    if kind == "line":
        return b + _w_seq(bo, data, z)
    if kind == "poly":
        return b + struct.pack(bo + "I", len(data)) + b"".join(_w_seq(bo, r, z) for r in data)
    sub = {"mpoint": "point", "mline": "line", "mpoly": "poly"}.get(kind)
    parts = [(sub, d) for d in data] if sub else data
    return b + struct.pack(bo + "I", len(parts)) + b"".join(w_geom(k, d, not le if kind == "collection" else le, z)
                                                           for k, d in parts)


def _star(rng, cx, cy, r, k, ccw=True):
    ang = np.sort(rng.uniform(0, 2 * np.pi, k))
    rad = rng.uniform(0.4 * r, r, k)
    pts = [(float(cx + q * np.cos(a)), float(cy + q * np.sin(a))) for a, q in zip(ang, rad)]
    pts.append(pts[0])
    return pts if ccw else pts[::-1]


def _random_geoms(seed, n):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        cx, cy = rng.uniform(-170, 170), rng.uniform(-80, 80)
        kind = ["poly", "mpoly", "line", "mline", "mpoint", "collection", "point"][i % 7]
        shell = _star(rng, cx, cy, rng.uniform(0.01, 2.0), int(rng.integers(3, 40)), bool(rng.random() < 0.5))
        hole = _star(rng, cx, cy, 0.2 * abs(shell[0][0] - cx) + 1e-4, 6, bool(rng.random() < 0.5))
        if kind == "poly":
            out.append((kind, [shell, hole] if rng.random() < 0.5 else [shell]))
        elif kind == "mpoly":
            other = _star(rng, cx + 5, cy, 1.0, 9, bool(rng.random() < 0.5))
            out.append((kind, [[shell, hole], [other]]))
        elif kind == "line":
            out.append((kind, shell[:-1]))
        elif kind == "mline":
            out.append((kind, [shell[:5], hole[:4]]))
        elif kind == "mpoint":
            out.append((kind, shell[:7]))
        elif kind == "collection":
            out.append((kind, [("point", shell[0]), ("line", hole[:4]), ("poly", [shell]),
                               ("collection", [("mpoint", hole[:3])])]))
        else:
            out.append((kind, shell[0]))
    return out


def test_centroid_any_wkb_equals_jts_restatement():
    """WKB of every type (both byte orders, ISO Z, nested collections) and the same rows
    as hex text (upper / lower case): the decoder's centroid equals the JTS Centroid
    restatement bit for bit."""
    for le in (True, False):
        for g in _random_geoms(11 if le else 12, 140):
            w = w_geom(*g, le=le, z=(g[0] == "poly" and le))
            want = JC.centroid_wkb(w)
            st, x, y = decode(N.MGPU_GEOM_WKB, w)
            assert st == 0 and (x, y) == want, (g[0], (x, y), want)
            for hx in (w.hex(), w.hex().upper()):
                assert decode(N.MGPU_GEOM_HEX, hx) == (0, x, y)


def test_centroid_special_cases():
    """Flat / degenerate rings, zero-length lines (their first point), empty members,
    rings and lines the non-strict WKBReader repairs, and hex text."""
    sq = [(0.0, 0.0), (2.0, 0.0), (2.0, 2.0), (0.0, 2.0), (0.0, 0.0)]
    flat = [(0.0, 1.0), (3.0, 1.0), (1.0, 1.0), (0.0, 1.0)]  # zero area: the lines decide
    for g in [("poly", [sq]), ("poly", [sq[::-1]]), ("poly", [flat]), ("line", [(1.0, 1.0), (1.0, 1.0)]),
              ("mpoly", [[sq], [[(5.0, 5.0), (6.0, 5.0), (6.0, 6.0), (5.0, 5.0)]]]),
              ("collection", [("poly", []), ("point", (3.0, 4.0))]),
              ("mline", [[(0.0, 0.0), (3.0, 4.0)], [(1.0, 1.0), (1.0, 1.0)]])]:
        w = w_geom(*g)
        assert decode(N.MGPU_GEOM_WKB, w)[1:] == JC.centroid_wkb(w), g
    assert decode(N.MGPU_GEOM_WKB, w_geom("poly", [sq]))[1:] == (1.0, 1.0)
    assert decode(N.MGPU_GEOM_WKB, w_geom("collection", []))[0] == 3  # empty
    # JTS 1.20's WKBReader is not strict by default: it repairs a one-point line (extended
    # to two) and rings that are not rings (ensureValidRing: closed, padded to 4 points);
    # the oracle restates the same repair
    for g in [("line", [(1.0, 1.0)]), ("poly", [sq[:-1]]), ("poly", [sq[:2] + sq[:1]]), ("poly", [sq[:3]]),
              ("poly", [sq, [(0.5, 0.5), (1.0, 0.5), (1.0, 1.0)]]), ("mline", [[(2.0, 3.0)], [(0.0, 0.0), (3.0, 4.0)]])]:
        w = w_geom(*g)
        st, x, y = decode(N.MGPU_GEOM_WKB, w)
        assert st == 0 and (x, y) == JC.centroid_wkb(w), (g, (x, y), JC.centroid_wkb(w))
    assert decode(N.MGPU_GEOM_WKB, w_geom("line", [(1.0, 1.0)]))[1:] == (1.0, 1.0)
    assert decode(N.MGPU_GEOM_WKB, w_geom("poly", [sq[:-1]]))[1:] == (1.0, 1.0)  # closed: the square
    assert decode(N.MGPU_GEOM_HEX, w_geom("point", (1.0, 2.0)).hex() + "0")[0] == 0  # odd last char ignored
    assert decode(N.MGPU_GEOM_HEX, "01zz")[0] == 1


def test_hypot_port():
    """StrictMath.hypot (fdlibm) as the decoder ports it: equal to the oracle's port, and
    within an ulp of the exact value."""
    from decimal import Decimal, getcontext
    getcontext().prec = 60
    rng = np.random.default_rng(3)
    for a, b in zip(rng.standard_normal(400) * 10.0 ** rng.integers(-300, 300, 400), rng.standard_normal(400)):
        h = JC.hypot(float(a), float(b))
        exact = (Decimal(float(a)) ** 2 + Decimal(float(b)) ** 2).sqrt()
        assert abs(Decimal(h) - exact) <= Decimal(np.spacing(h))


def test_geojson_points():
    J = N.MGPU_GEOM_GEOJSON
    assert decode(J, '{"type": "Point", "coordinates": [-73.956758, 40.769978]}') == (0, -73.956758, 40.769978)
    assert decode(J, '{"coordinates":[1,2,3],"type":"Point","crs":{"type":"name","properties":{"name":"x"}}}') == (0, 1.0, 2.0)
    st, x, y = decode(J, '{"type":"MultiPoint","coordinates":[[1,2],[3,5],[5,8]]}')
    assert st == 0 and (x, y) == (3.0, 5.0)
    assert decode(J, '{"type":"Point","coordinates":[]}')[0] == 3
    assert decode(J, '{"type":"MultiPoint","coordinates":[]}')[0] == 3
    st, x, y = decode(J, '{"type":"Polygon","coordinates":[[[0,0],[3,0],[0,3],[0,0]]]}')
    assert st == 0 and (x, y) == (1.0, 1.0)
    assert decode(J, '{"type":"Point","coordinates":[1]}')[0] == 1
    assert decode(J, '{"type":"Blob"}')[0] == 1


def _internal_rows(geoms):
    """InternalGeometryType rows (type id, boundaries + holes) of the WKB test shapes."""
    rows = []
    for kind, d in geoms:
        if kind == "point":
            rows.append((1, [[[d]]]))
        elif kind == "mpoint":
            rows.append((2, [[list(d)]]))
        elif kind == "line":
            rows.append((3, [[list(d)]]))
        elif kind == "mline":
            rows.append((4, [[list(l)] for l in d]))
        elif kind == "poly":
            rows.append((5, [list(d)]))
        elif kind == "mpoly":
            rows.append((6, [list(p) for p in d]))
    return rows


def test_internal_geometry_centroids_equal_wkb():
    """The InternalGeometryType layout gives the same centroid as the WKB of the same shape."""
    geoms = [g for g in _random_geoms(13, 120) if g[0] != "collection"]
    rows = _internal_rows(geoms)
    tid, rp, pr, ro, xy = [], [0], [0], [0], []
    for t, parts in rows:
        tid.append(t)
        for part in parts:
            for ring in part:
                xy.extend(ring)
                ro.append(len(xy))
            pr.append(len(ro) - 1)
        rp.append(len(pr) - 1)
    A = lambda a, dt: np.ascontiguousarray(a, dtype=dt)
    tid, rp, pr, ro, xy = A(tid, np.int32), A(rp, np.int64), A(pr, np.int64), A(ro, np.int64), A(xy, np.float64)
    n = len(tid)
    x, y, st = np.zeros(n), np.zeros(n), np.zeros(n, np.int32)
    P = lambda a: ctypes.c_void_p(a.ctypes.data)
    N.check(N.lib().mgpu_test_internal_centroid(n, P(tid), P(rp), P(pr), P(ro), P(xy), P(x), P(y), P(st)))
    for i, g in enumerate(geoms):
        assert st[i] == 0 and (x[i], y[i]) == JC.centroid_wkb(w_geom(*g)), (i, g[0])


# ---------------------------------------------------------------- WKT / GeoJSON of every type
def _wkt(kind, d, z=False):
    """WKT text of the _random_geoms shapes (repr: the shortest round-tripping decimals)."""
    zs = " Z" if z else ""
    c = lambda p: "%r %r" % p + (" 7.0" if z else "")  # noqa: E731
    seq = lambda pts: "(" + ", ".join(c(p) for p in pts) + ")"  # noqa: E731
    poly = lambda rings: "(" + ", ".join(seq(r) for r in rings) + ")"  # noqa: E731
    if kind == "point":
        return "POINT%s (%s)" % (zs, c(d))
    if kind == "line":
        return "LINESTRING%s %s" % (zs, seq(d))
    if kind == "poly":
        return "POLYGON%s %s" % (zs, poly(d))
    if kind == "mpoint":
        return "MULTIPOINT%s (%s)" % (zs, ", ".join("(%s)" % c(p) for p in d))
    if kind == "mline":
        return "MULTILINESTRING%s (%s)" % (zs, ", ".join(seq(l) for l in d))
    if kind == "mpoly":
        return "MULTIPOLYGON%s (%s)" % (zs, ", ".join(poly(q) for q in d))
    return "GEOMETRYCOLLECTION%s (%s)" % (zs, ", ".join(_wkt(k, v, z) for k, v in d))


def _json(kind, d):
    pos = lambda p: "[%r, %r]" % p  # noqa: E731
    seq = lambda pts: "[" + ", ".join(pos(p) for p in pts) + "]"  # noqa: E731
    poly = lambda rings: "[" + ", ".join(seq(r) for r in rings) + "]"  # noqa: E731
    names = {"point": "Point", "line": "LineString", "poly": "Polygon", "mpoint": "MultiPoint",
             "mline": "MultiLineString", "mpoly": "MultiPolygon"}
    if kind == "collection":
        return '{"geometries": [%s], "type": "GeometryCollection"}' % ", ".join(_json(k, v) for k, v in d)
    coords = {"point": lambda: pos(d), "line": lambda: seq(d), "poly": lambda: poly(d), "mpoint": lambda: seq(d),
              "mline": lambda: "[" + ", ".join(seq(l) for l in d) + "]",
              "mpoly": lambda: "[" + ", ".join(poly(q) for q in d) + "]"}[kind]()
    return '{"type": "%s", "coordinates": %s}' % (names[kind], coords)


def test_centroid_any_wkt_geojson_equals_jts_restatement():
    """grid_pointascellid on WKT (StringType) and GeoJSON (JSONType) rows of every geometry
    type -- GeometryAPI.geometry (GeometryAPI.scala:81-89) reads them with JTS's WKTReader /
    GeoJsonReader, PointIndexGeom takes getCentroid -- equals the JTS Centroid restatement of
    the same geometry (as WKB) bit for bit; Z coordinates are ignored."""
    for seed in (21, 22):
        for g in _random_geoms(seed, 140):
            want = JC.centroid_wkb(w_geom(*g))
            assert decode(N.MGPU_GEOM_WKT, _wkt(*g))[1:] == want, (g[0], _wkt(*g)[:80])
            assert decode(N.MGPU_GEOM_WKT, _wkt(*g, z=True))[1:] == want
            assert decode(N.MGPU_GEOM_GEOJSON, _json(*g))[1:] == want, (g[0], _json(*g)[:80])


def test_text_geometry_special_cases():
    """EMPTY members, strict rings (WKTReader / GeoJsonReader throw where WKBReader
    repairs), nesting."""
    W, J = N.MGPU_GEOM_WKT, N.MGPU_GEOM_GEOJSON
    assert decode(W, "POLYGON EMPTY")[0] == 3
    assert decode(W, "GEOMETRYCOLLECTION EMPTY")[0] == 3
    assert decode(W, "GEOMETRYCOLLECTION (POINT EMPTY, LINESTRING EMPTY)")[0] == 3
    assert decode(W, "GEOMETRYCOLLECTION (POINT (1 2), GEOMETRYCOLLECTION (POINT (3 4)))") == (0, 2.0, 3.0)
    assert decode(W, "MULTIPOLYGON (EMPTY, ((0 0, 3 0, 0 3, 0 0)))") == (0, 1.0, 1.0)
    assert decode(W, "POLYGON ((0 0, 3 0, 0 3))")[0] == 1        # not closed
    assert decode(W, "POLYGON ((0 0, 3 0, 0 0))")[0] == 1        # fewer than 4 points
    assert decode(W, "LINESTRING (1 2)")[0] == 1                 # one point
    assert decode(W, "LINEARRING (0 0, 3 0, 0 3, 0 0)")[0] == 0
    assert decode(W, "POLYGON ((0 0, 3 0, 0 3, 0 0)")[0] == 1    # truncated
    assert decode(W, "GEOMETRYCOLLECTION (POINT (1 2)")[0] == 1
    assert decode(J, '{"type":"Polygon","coordinates":[[[0,0],[1,0],[1,1]]]}')[0] == 1
    assert decode(J, '{"type":"LineString","coordinates":[[0,0]]}')[0] == 1
    assert decode(J, '{"type":"GeometryCollection","geometries":[]}')[0] == 3
    assert decode(J, '{"type":"GeometryCollection","geometries":[{"type":"Point","coordinates":[1,2]},'
                     '{"type":"GeometryCollection","geometries":[{"type":"Point","coordinates":[3,4]}]}]}') == (0, 2.0, 3.0)
    assert decode(J, '{"type":"Polygon","coordinates":[]}')[0] == 3
