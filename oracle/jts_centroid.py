"""ORACLE -- TEST INFRASTRUCTURE ONLY.

A pure-Python restatement of what the reference computes for grid_pointascellid on a
non-point geometry row: PointIndexGeom.nullSafeEval (expressions/index/
PointIndexGeom.scala:33-47) -> GeometryAPI.geometry (core/geometry/api/
GeometryAPI.scala:81-89: JTS WKBReader, WKBReader.hexToBytes for HexType) ->
getCentroid = org.locationtech.jts.algorithm.Centroid (JTS 1.20, a dependency absent
from /root/reference: pom.xml:98-107), restated from its published algorithm:

  * one accumulator over the geometry's components in order; polygons: a triangle fan
    from the FIRST shell's first point (areaBasePt), each triangle (base, p_i, p_i+1)
    adding sign * area2 * (base + p_i + p_i+1) to cg3 and sign * area2 to areasum2, the
    sign + for a shell that is not CCW and for a hole that is (Orientation.isCCW);
    lines (and every ring): segment length (Coordinate.distance = Math.hypot) times the
    segment midpoint; points: their sum;
  * result: cg3 / 3 / areasum2 if areasum2 != 0, else lineCentSum / totalLength if the
    length is > 0, else ptCentSum / ptCount, else empty.

Orientation.isCCW follows JTS 1.20 (highest point reached by a rising segment, the next
lower point, pointed cap -> orientation index, flat cap -> direction of the top); the
orientation index is computed exactly (fractions) -- JTS's CGAlgorithmsDD gives the
exact sign.  Math.hypot is StrictMath.hypot (fdlibm e_hypot.c, JDK 8), ported below.
Only tests/ import this module.  No JTS exists in this image: the centroid values are
"parity unpinned" beyond this restatement (no reference fixture holds one).
"""
import math
import struct
from fractions import Fraction


def _hi(v):
    return struct.unpack("<q", struct.pack("<d", v))[0] >> 32


def _lo(v):
    return struct.unpack("<Q", struct.pack("<d", v))[0] & 0xFFFFFFFF


def _with_hi(v, h):
    u = struct.unpack("<Q", struct.pack("<d", v))[0]
    u = ((h & 0xFFFFFFFF) << 32) | (u & 0xFFFFFFFF)
    return struct.unpack("<d", struct.pack("<Q", u))[0]


def hypot(x, y):
    """fdlibm __ieee754_hypot (e_hypot.c) -- java.lang.StrictMath.hypot."""
    ha, hb, k = _hi(x) & 0x7fffffff, _hi(y) & 0x7fffffff, 0
    if hb > ha:
        a, b = y, x
        ha, hb = hb, ha
    else:
        a, b = x, y
    a, b = _with_hi(a, ha), _with_hi(b, hb)
    if ha - hb > 0x3c00000:
        return a + b
    if ha > 0x5f300000:
        if ha >= 0x7ff00000:
            w = a + b
            if ((ha & 0xfffff) | _lo(a)) == 0:
                w = a
            if ((hb ^ 0x7ff00000) | _lo(b)) == 0:
                w = b
            return w
        ha -= 0x25800000
        hb -= 0x25800000
        k += 600
        a, b = _with_hi(a, ha), _with_hi(b, hb)
    if hb < 0x20b00000:
        if hb <= 0x000fffff:
            if (hb | _lo(b)) == 0:
                return a
            t1 = _with_hi(0.0, 0x7fd00000)
            b *= t1
            a *= t1
            k -= 1022
        else:
            ha += 0x25800000
            hb += 0x25800000
            k -= 600
            a, b = _with_hi(a, ha), _with_hi(b, hb)
    w = a - b
    if w > b:
        t1 = _with_hi(0.0, ha)
        t2 = a - t1
        w = math.sqrt(t1 * t1 - (b * (-b) - t2 * (a + t1)))
    else:
        a = a + a
        y1 = _with_hi(0.0, hb)
        y2 = b - y1
        t1 = _with_hi(0.0, ha + 0x00100000)
        t2 = a - t1
        w = math.sqrt(t1 * y1 - (w * (-w) - (t1 * y2 + t2 * b)))
    if k != 0:
        return _with_hi(1.0, _hi(1.0) + (k << 20)) * w
    return w


def orientation_index(p, q, r):
    """The exact sign of the turn p -> q -> r (1: counter-clockwise)."""
    d = (Fraction(q[0]) - Fraction(p[0])) * (Fraction(r[1]) - Fraction(q[1])) - \
        (Fraction(q[1]) - Fraction(p[1])) * (Fraction(r[0]) - Fraction(q[0]))
    return (d > 0) - (d < 0)


def is_ccw(ring):
    """org.locationtech.jts.algorithm.Orientation.isCCW (JTS 1.20)."""
    n = len(ring) - 1
    if n < 3:
        return False
    up_hi, prev_y, up_low, i_up_hi = ring[0], ring[0][1], None, 0
    for i in range(1, n + 1):
        py = ring[i][1]
        if py > prev_y and py >= up_hi[1]:
            up_hi, i_up_hi, up_low = ring[i], i, ring[i - 1]
        prev_y = py
    if i_up_hi == 0:
        return False
    i_down_low = i_up_hi
    while True:
        i_down_low = (i_down_low + 1) % n
        if not (i_down_low != i_up_hi and ring[i_down_low][1] == up_hi[1]):
            break
    down_low = ring[i_down_low]
    down_hi = ring[i_down_low - 1 if i_down_low > 0 else n - 1]
    if up_hi == down_hi:
        if up_low == up_hi or down_low == up_hi or up_low == down_low:
            return False
        return orientation_index(up_low, up_hi, down_low) == 1
    return down_hi[0] - up_hi[0] < 0


class Centroid:
    def __init__(self):
        self.base = None
        self.cg3 = [0.0, 0.0]
        self.areasum2 = 0.0
        self.line = [0.0, 0.0]
        self.length = 0.0
        self.pt = [0.0, 0.0]
        self.count = 0

    def point(self, p):
        self.count += 1
        self.pt[0] += p[0]
        self.pt[1] += p[1]

    def segments(self, pts):
        ln = 0.0
        for a, b in zip(pts[:-1], pts[1:]):
            s = hypot(a[0] - b[0], a[1] - b[1])
            if s == 0.0:
                continue
            ln += s
            self.line[0] += s * ((a[0] + b[0]) / 2)
            self.line[1] += s * ((a[1] + b[1]) / 2)
        self.length += ln
        if ln == 0.0 and pts:
            self.point(pts[0])

    def ring(self, pts, shell):
        if shell and pts and self.base is None:
            self.base = pts[0]
        sign = 1.0 if (not is_ccw(pts) if shell else is_ccw(pts)) else -1.0
        b = self.base
        for p1, p2 in zip(pts[:-1], pts[1:]):
            tx, ty = b[0] + p1[0] + p2[0], b[1] + p1[1] + p2[1]
            a2 = (p1[0] - b[0]) * (p2[1] - b[1]) - (p2[0] - b[0]) * (p1[1] - b[1])
            self.cg3[0] += sign * a2 * tx
            self.cg3[1] += sign * a2 * ty
            self.areasum2 += sign * a2
        self.segments(pts)

    def result(self):
        if abs(self.areasum2) > 0.0:
            return self.cg3[0] / 3 / self.areasum2, self.cg3[1] / 3 / self.areasum2
        if self.length > 0.0:
            return self.line[0] / self.length, self.line[1] / self.length
        if self.count > 0:
            return self.pt[0] / self.count, self.pt[1] / self.count
        return None


def _ensure_valid_ring(pts):
    """JTS WKBReader, not strict (its default): CoordinateSequences.ensureValidRing --
    fewer than 4 points padded to 4 with the first, an open ring closed with it."""
    n = len(pts)
    if n == 0:
        return pts
    if n <= 3:
        return list(pts) + [pts[0]] * (4 - n)
    if pts[0][0] == pts[-1][0] and pts[0][1] == pts[-1][1]:
        return pts
    return list(pts) + [pts[0]]


def _read(b, o, c):
    """One WKB geometry at o into the accumulator; returns the next offset."""
    le = b[o] == 1
    bo = "<" if le else ">"
    t = struct.unpack_from(bo + "I", b, o + 1)[0]
    o += 5
    d = 2
    if t & 0x20000000:
        o += 4
    if t & 0x80000000:
        d += 1
    if t & 0x40000000:
        d += 1
    t &= 0x0FFFFFFF
    if 1000 <= t < 4000:
        d += 2 if t // 1000 == 3 else 1
        t %= 1000

    def seq(o):
        n = struct.unpack_from(bo + "I", b, o)[0]
        o += 4
        pts = [struct.unpack_from(bo + "dd", b, o + 8 * d * i) for i in range(n)]
        return pts, o + 8 * d * n

    if t == 1:
        p = struct.unpack_from(bo + "dd", b, o)
        if not (math.isnan(p[0]) and math.isnan(p[1])):
            c.point(p)
        return o + 8 * d
    if t == 2:
        pts, o = seq(o)
        if len(pts) == 1:  # non-strict WKBReader: CoordinateSequences.extend to 2 points
            pts = pts * 2
        if pts:
            c.segments(pts)
        return o
    if t == 3:
        nr = struct.unpack_from(bo + "I", b, o)[0]
        o += 4
        rings = []
        for _ in range(nr):
            pts, o = seq(o)
            rings.append(_ensure_valid_ring(pts))
        if rings and rings[0]:
            for k, r in enumerate(rings):
                if r:
                    c.ring(r, k == 0)
        return o
    n = struct.unpack_from(bo + "I", b, o)[0]
    o += 4
    for _ in range(n):
        o = _read(b, o, c)
    return o


def centroid_wkb(b):
    """JTS Centroid of a WKB geometry: (x, y), or None when empty."""
    c = Centroid()
    _read(bytes(b), 0, c)
    return c.result()
