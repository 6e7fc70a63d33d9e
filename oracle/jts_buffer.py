"""TEST INFRASTRUCTURE ONLY (the checker; never imported by the product path).

An independent numpy restatement of the JTS 1.20 buffer pieces that decide mosaicFill's
chip flags (core/Mosaic.scala:69-93):

    carved = geometry.buffer(-r)                                      Mosaic.scala:71
    band   = geometry.boundary.buffer(1.01 r).simplify(0.01 r)        Mosaic.scala:75-84
             (geometry.buffer(1.01 r).simplify(0.01 r) when carved is empty)
    core   = polyfill(carved), border = polyfill(band) diff core      Mosaic.scala:92-93

`MosaicGeometryJTS.buffer` (core/geometry/MosaicGeometryJTS.scala:86-115) is a default
`BufferOp` (round joins, 8 quadrant segments).  JTS is a Maven dependency of the
reference (pom.xml:98-102), not in /root/reference and not in this image: this file
restates its published algorithm --
  * OffsetCurveSetBuilder: removeRepeatedPoints, isErodedCompletely (shells of a negative
    buffer, holes of a positive one), ring side / labels from Orientation.isCCW
    (addRingSide), addRingBothSides for closed lines, isRingCurveInverted;
  * OffsetCurveBuilder: BufferInputLineSimplifier (tolerance 0.01 * distance, the sign
    selecting the side), OffsetSegmentGenerator (fillets of nSegs = round(angle / (pi/16))
    chords with vertices on the circle, inside turns by the offsets' intersection or
    closing segments at 1/81 of the way to the vertex, points closer than 1e-6 * distance
    dropped);
  * BufferBuilder: the result is the set of faces whose depth (the labels crossed from
    outside) is >= 1 -- here the signed winding number of the raw curves;
  * DouglasPeuckerSimplifier(0.01 r) of the band moves its outline by <= 0.01 r: a centre
    within that distance of the band's outline is reported as DP-sensitive.
The C++ tessellator (mosaic_amd/csrc/jts_buffer.h) restates the same algorithm; this
file is written separately (exact rational orientation fallback, JTS's highest-point
isCCW, vectorised winding numbers) so the host tests compare two restatements.  Parity
with JTS itself is unpinned: no JTS build exists here and no reference fixture lists a
buffer's vertices.
"""
import math
from fractions import Fraction

import numpy as np

CW, COLLINEAR, CCW = -1, 0, 1
LEFT, RIGHT = 1, 2
INTERIOR, EXTERIOR = 0, 2


def orientation_index(p1, p2, q):
    """CGAlgorithmsDD.orientationIndex: the filtered determinant, exact fallback."""
    detleft = (p1[0] - q[0]) * (p2[1] - q[1])
    detright = (p1[1] - q[1]) * (p2[0] - q[0])
    det = detleft - detright
    if detleft > 0.0:
        if detright <= 0.0:
            return int(det > 0) - int(det < 0)
        detsum = detleft + detright
    elif detleft < 0.0:
        if detright >= 0.0:
            return int(det > 0) - int(det < 0)
        detsum = -detleft - detright
    else:
        return int(det > 0) - int(det < 0)
    if abs(det) >= 1e-15 * detsum:
        return int(det > 0) - int(det < 0)
    F = Fraction
    e = (F(p2[0]) - F(p1[0])) * (F(q[1]) - F(p2[1])) - (F(p2[1]) - F(p1[1])) * (F(q[0]) - F(p2[0]))
    return int(e > 0) - int(e < 0)


def seg_distance(p, a, b):
    """Distance.pointToSegment."""
    if a[0] == b[0] and a[1] == b[1]:
        return math.sqrt((p[0] - a[0]) ** 2 + (p[1] - a[1]) ** 2)
    len2 = (b[0] - a[0]) ** 2 + (b[1] - a[1]) ** 2
    r = ((p[0] - a[0]) * (b[0] - a[0]) + (p[1] - a[1]) * (b[1] - a[1])) / len2
    if r <= 0.0:
        return math.sqrt((p[0] - a[0]) ** 2 + (p[1] - a[1]) ** 2)
    if r >= 1.0:
        return math.sqrt((p[0] - b[0]) ** 2 + (p[1] - b[1]) ** 2)
    s = ((a[1] - p[1]) * (b[0] - a[0]) - (a[0] - p[0]) * (b[1] - a[1])) / len2
    return abs(s) * math.sqrt(len2)


def remove_repeated(pts):
    out = []
    for p in pts:
        p = (float(p[0]), float(p[1]))
        if not out or out[-1] != p:
            out.append(p)
    return out


def is_ccw(ring):
    """Orientation.isCCW (JTS 1.20): the orientation of the cap at the highest point."""
    n = len(ring) - 1
    if n < 3:
        return False
    up_hi, prev_y, up_lo, i_up_hi = ring[0], ring[0][1], None, 0
    for i in range(1, n + 1):
        py = ring[i][1]
        if py > prev_y and py >= up_hi[1]:
            up_hi, i_up_hi, up_lo = ring[i], i, ring[i - 1]
        prev_y = py
    if i_up_hi == 0:
        return False
    i_down_lo = i_up_hi
    while True:
        i_down_lo = (i_down_lo + 1) % n
        if not (i_down_lo != i_up_hi and ring[i_down_lo][1] == up_hi[1]):
            break
    down_lo = ring[i_down_lo]
    down_hi = ring[i_down_lo - 1 if i_down_lo > 0 else n - 1]
    if up_hi == down_hi:
        if up_lo == up_hi or down_lo == up_hi or up_lo == down_lo:
            return False
        return orientation_index(up_lo, up_hi, down_lo) == CCW
    return down_hi[0] - up_hi[0] < 0


def simplify_input(line, signed_tol):
    """BufferInputLineSimplifier.simplify: repeated passes deleting shallow concavities
    on the side selected by the tolerance's sign (isShallowSampled as JTS calls it: with
    the middle vertex in the parameter named for the section's end)."""
    tol = abs(signed_tol)
    turn = CW if signed_tol < 0 else CCW
    n = len(line)
    deleted = [False] * n

    def nxt(i):
        i += 1
        while i < n and deleted[i]:
            i += 1
        return i

    def shallow(p0, p1, p2):
        return seg_distance(p1, p0, p2) < tol

    def deletable(i0, i1, i2):
        p0, p1, p2 = line[i0], line[i1], line[i2]
        if orientation_index(p0, p1, p2) != turn or not shallow(p0, p1, p2):
            return False
        step = max(1, (i2 - i0) // 10)
        return all(shallow(p0, p1, line[i]) for i in range(i0, i2, step))

    while True:
        changed = False
        i = 1
        mid = nxt(i)
        last = nxt(mid)
        while last < n:
            if deletable(i, mid, last):
                deleted[mid] = True
                changed = True
                i = last
            else:
                i = mid
            mid = nxt(i)
            last = nxt(mid)
        if not changed:
            break
    return [p for p, d in zip(line, deleted) if not d]


def _offset(a, b, side, dist):
    sign = 1.0 if side == LEFT else -1.0
    dx, dy = b[0] - a[0], b[1] - a[1]
    ln = math.sqrt(dx * dx + dy * dy)
    ux, uy = sign * dist * dx / ln, sign * dist * dy / ln
    return (a[0] - uy, a[1] + ux), (b[0] - uy, b[1] + ux)


def _seg_intersection(p1, p2, q1, q2):
    o1, o2 = orientation_index(p1, p2, q1), orientation_index(p1, p2, q2)
    o3, o4 = orientation_index(q1, q2, p1), orientation_index(q1, q2, p2)
    if o1 * o2 > 0 or o3 * o4 > 0 or (o1 == o2 == o3 == o4 == 0):
        return None
    for o, pt in ((o1, q1), (o2, q2), (o3, p1), (o4, p2)):
        if o == 0:
            return pt
    dxp, dyp, dxq, dyq = p2[0] - p1[0], p2[1] - p1[1], q2[0] - q1[0], q2[1] - q1[1]
    t = ((q1[0] - p1[0]) * dyq - (q1[1] - p1[1]) * dxq) / (dxp * dyq - dyp * dxq)
    return (p1[0] + t * dxp, p1[1] + t * dyp)


def ring_curve(ring, side, dist, simplify=True):
    """OffsetCurveBuilder.getRingCurve of a closed ring (>= 4 points), distance > 0."""
    pts = simplify_input(ring, -0.01 * dist if side == RIGHT else 0.01 * dist) if simplify else list(ring)
    out = []
    min_vd = dist * 1e-6
    quantum = math.pi / 2.0 / 8

    def add(p):
        if out and math.hypot(p[0] - out[-1][0], p[1] - out[-1][1]) < min_vd:
            return
        out.append((p[0], p[1]))

    def fillet(c, p0, p1, direction):
        a0 = math.atan2(p0[1] - c[1], p0[0] - c[0])
        a1 = math.atan2(p1[1] - c[1], p1[0] - c[0])
        if direction == CW and a0 <= a1:
            a0 += 2 * math.pi
        elif direction != CW and a0 >= a1:
            a0 -= 2 * math.pi
        add(p0)
        total = abs(a0 - a1)
        k = int(total / quantum + 0.5)
        if k >= 1:
            inc = total / k
            f = -1.0 if direction == CW else 1.0
            for i in range(k):
                a = a0 + f * i * inc
                add((c[0] + dist * math.cos(a), c[1] + dist * math.sin(a)))
        add(p1)

    n = len(pts) - 1
    if n < 1:
        return []
    s1, s2 = pts[n - 1], pts[0]
    for i in range(1, n + 1):
        s0, s1, s2 = s1, s2, pts[i]
        o0a, o0b = _offset(s0, s1, side, dist)
        o1a, o1b = _offset(s1, s2, side, dist)
        if s1 == s2:
            continue
        o = orientation_index(s0, s1, s2)
        if o == COLLINEAR:
            if (s2[0] - s1[0]) * (s1[0] - s0[0]) + (s2[1] - s1[1]) * (s1[1] - s0[1]) < 0:
                fillet(s1, o0b, o1a, CW)
        elif (o == CW and side == LEFT) or (o == CCW and side == RIGHT):  # outside turn
            if math.hypot(o0b[0] - o1a[0], o0b[1] - o1a[1]) < dist * 1e-3:
                add(o0b)
                continue
            if i != 1:
                add(o0b)
            fillet(s1, o0b, o1a, o)
            add(o1a)
        else:  # inside turn
            ip = _seg_intersection(o0a, o0b, o1a, o1b)
            if ip is not None:
                add(ip)
            elif math.hypot(o0b[0] - o1a[0], o0b[1] - o1a[1]) < dist * 1e-3:
                add(o0b)
            else:
                add(o0b)
                add(((80 * o0b[0] + s1[0]) / 81, (80 * o0b[1] + s1[1]) / 81))
                add(((80 * o1a[0] + s1[0]) / 81, (80 * o1a[1] + s1[1]) / 81))
                add(o1a)
    if out and out[0] != out[-1]:
        out.append(out[0])
    return out


def _eroded_completely(ring, buffer_distance):
    if len(ring) < 4:
        return buffer_distance < 0
    if len(ring) == 4:
        a, b, c = ring[0], ring[1], ring[2]
        la, lb, lc = math.dist(b, c), math.dist(a, c), math.dist(a, b)
        s = la + lb + lc
        inc = ((la * a[0] + lb * b[0] + lc * c[0]) / s, (la * a[1] + lb * b[1] + lc * c[1]) / s)
        return seg_distance(inc, a, b) < abs(buffer_distance)
    xs = [p[0] for p in ring]
    ys = [p[1] for p in ring]
    return buffer_distance < 0 and 2 * abs(buffer_distance) > min(max(ys) - min(ys), max(xs) - min(xs))


def _inverted(ring, dist, curve):
    if dist == 0 or len(ring) <= 3 or len(ring) >= 9 or len(curve) > 4 * len(ring):
        return False
    tol = 0.99 * abs(dist)

    def far(p):
        return min(seg_distance(p, ring[i], ring[i + 1]) for i in range(len(ring) - 1)) > tol

    for i in range(len(curve) - 1):
        if far(curve[i]) or far(((curve[i][0] + curve[i + 1][0]) / 2, (curve[i][1] + curve[i + 1][1]) / 2)):
            return False
    return True


class Curves:
    """Raw offset curves with their depth signs; depth(p) = sum sign * winding."""

    def __init__(self):
        self.a = []
        self.b = []
        self.s = []

    def add_ring_side(self, coord, dist, side, cw_left, cw_right):
        left = cw_left
        if len(coord) >= 4 and is_ccw(coord):
            left = cw_right
            side = RIGHT if side == LEFT else LEFT
        c = ring_curve(coord, side, dist)
        if len(c) < 2 or _inverted(coord, dist, c):
            return
        sign = 1 if left == INTERIOR else -1
        c = np.asarray(c)
        keep = np.any(c[:-1] != c[1:], axis=1)
        self.a.append(c[:-1][keep])
        self.b.append(c[1:][keep])
        self.s.append(np.full(int(keep.sum()), sign, np.int64))

    def finish(self):
        if self.a:
            self.A, self.B, self.S = np.concatenate(self.a), np.concatenate(self.b), np.concatenate(self.s)
        else:
            self.A = self.B = np.zeros((0, 2))
            self.S = np.zeros(0, np.int64)
        return self

    def depth(self, px, py):
        """Signed crossings of the rightward ray (half-open in y), per query point."""
        px, py = np.atleast_1d(px), np.atleast_1d(py)
        out = np.zeros(len(px), np.int64)
        ax, ay, bx, by = self.A[:, 0], self.A[:, 1], self.B[:, 0], self.B[:, 1]
        for k in range(0, len(px), 64):
            X, Y = px[k:k + 64, None], py[k:k + 64, None]
            up = (ay <= Y) & (by > Y)
            down = (by <= Y) & (ay > Y)
            with np.errstate(divide="ignore", invalid="ignore"):
                xi = (bx - ax) * (Y - ay) / (by - ay) + ax
            right = X < xi
            out[k:k + 64] = ((up & right) * self.S - (down & right) * self.S).sum(1)
        return out

    def outline_distance(self, p, q, eps):
        """Distance from p to the result's outline (pieces with depth >= 1 on one side
        only), or inf beyond q."""
        A, B = self.A, self.B
        if not len(A):
            return math.inf
        d = np.array([seg_distance(p, A[k], B[k]) for k in range(len(A))])
        best = math.inf
        for k in np.nonzero(d <= q)[0]:
            a, b = A[k], B[k]
            dx, dy = b[0] - a[0], b[1] - a[1]
            ex, ey = B[:, 0] - A[:, 0], B[:, 1] - A[:, 1]
            den = dx * ey - dy * ex
            with np.errstate(divide="ignore", invalid="ignore"):
                t = ((A[:, 0] - a[0]) * ey - (A[:, 1] - a[1]) * ex) / den
                u = ((A[:, 0] - a[0]) * dy - (A[:, 1] - a[1]) * dx) / den
            ok = (den != 0) & (t > 0) & (t < 1) & (u >= 0) & (u <= 1)
            ok[k] = False
            ts = np.unique(np.concatenate([[0.0, 1.0], t[ok]]))
            ln = math.hypot(dx, dy)
            nx, ny = -dy / ln * eps, dx / ln * eps
            for t0, t1 in zip(ts[:-1], ts[1:]):
                pa = (a[0] + t0 * dx, a[1] + t0 * dy)
                pb = (a[0] + t1 * dx, a[1] + t1 * dy)
                dd = seg_distance(p, pa, pb)
                if dd >= best or dd > q:
                    continue
                m = ((pa[0] + pb[0]) / 2, (pa[1] + pb[1]) / 2)
                dl, dr = self.depth(np.array([m[0] + nx, m[0] - nx]), np.array([m[1] + ny, m[1] - ny]))
                if (dl >= 1) != (dr >= 1):
                    best = dd
        return best

    def any_positive(self, eps):
        A, B = self.A, self.B
        if not len(A):
            return False
        dx, dy = B[:, 0] - A[:, 0], B[:, 1] - A[:, 1]
        ln = np.hypot(dx, dy)
        nx, ny = -dy / ln * eps, dx / ln * eps
        for t in (0.5, 0.25, 0.75):
            mx, my = A[:, 0] + t * dx, A[:, 1] + t * dy
            if (self.depth(np.concatenate([mx + nx, mx - nx]), np.concatenate([my + ny, my - ny])) >= 1).any():
                return True
        return False


def carved_curves(parts, r):
    """geometry.buffer(-r): OffsetCurveSetBuilder.addPolygon with a negative distance."""
    c = Curves()
    for rings in parts:
        shell = [tuple(map(float, p)) for p in rings[0]]
        if _eroded_completely(shell, -r):
            continue
        sh = remove_repeated(shell)
        if len(sh) < 3:
            continue
        c.add_ring_side(sh, r, RIGHT, EXTERIOR, INTERIOR)
        for h in rings[1:]:
            c.add_ring_side(remove_repeated(h), r, LEFT, INTERIOR, EXTERIOR)
    return c.finish()


def band_curves(parts, d, whole):
    """geometry.boundary.buffer(d) (closed lines: addRingBothSides), or geometry.buffer(d)."""
    c = Curves()
    for rings in parts:
        for k, ring in enumerate(rings):
            rr = remove_repeated(ring)
            if len(rr) < 4 or rr[0] != rr[-1]:
                continue
            if not whole:
                c.add_ring_side(rr, d, LEFT, EXTERIOR, INTERIOR)
                c.add_ring_side(rr, d, RIGHT, INTERIOR, EXTERIOR)
            elif k == 0:
                c.add_ring_side(rr, d, LEFT, EXTERIOR, INTERIOR)
            elif not _eroded_completely([tuple(map(float, p)) for p in ring], -d):
                c.add_ring_side(rr, d, RIGHT, INTERIOR, EXTERIOR)
    return c.finish()


class MosaicFillSets:
    """mosaicFill's core and band sets of one polygon (parts: lists of closed rings)."""

    def __init__(self, parts, r):
        self.parts, self.r = parts, r
        self.carved = carved_curves(parts, r)
        self.carved_empty = not self.carved.any_positive(1e-7 * r)
        self._band = None

    @property
    def band(self):
        if self._band is None:
            self._band = band_curves(self.parts, 1.01 * self.r, self.carved_empty)
        return self._band

    def core(self, px, py):
        if self.carved_empty:
            return np.zeros(len(np.atleast_1d(px)), bool)
        return self.carved.depth(px, py) >= 1

    def in_band(self, px, py):
        return self.band.depth(px, py) >= 1

    def dp_sensitive(self, p):
        return self.band.outline_distance(p, 0.01 * self.r * (1 + 1e-6), 1e-7 * self.r) < math.inf
