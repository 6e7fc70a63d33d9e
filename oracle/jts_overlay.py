"""TEST INFRASTRUCTURE ONLY (an oracle; never imported by the product path).

An independent restatement of the arithmetic JTS 1.20's OverlayNG uses for the nodes of
`polygon INTERSECTION cell` (JTS is a Maven dependency of the reference, pom.xml:98-102,
absent here; called by IndexSystem.getBorderChips, core/index/IndexSystem.scala:184-188 ->
MosaicGeometryJTS.intersection, core/geometry/MosaicGeometryJTS.scala:139-152, and
coerceChipGeometry, IndexSystem.scala:293-303):

* ``line_intersection``: RobustLineIntersector.computeIntersect -- the envelope test, the
  four orientation indices (here EXACT, by rational arithmetic: JTS's CGAlgorithmsDD sign
  agrees with the exact sign except for determinants below ~2^-100 relative, which no
  fixture here reaches), the collinear case (computeCollinearIntersection), the endpoint
  cases, and for a proper crossing Intersection.intersection (homogeneous coordinates about
  the midpoint of the envelopes' overlap -- IEEE doubles, every product rounded on its own,
  as Python's floats do) with isInSegmentEnvelopes / nearestEndpoint;
* ``chip_nodes``: the nodes the noding of a polygon against a cell produces;
* ``check_chip``: what a chip's WKB may hold -- every vertex is a polygon vertex, a cell
  vertex, one of those nodes, or (coerceChipGeometry's difference with the cell boundary)
  the node of its two ring neighbours' edge with a cell segment; every proper crossing node
  is a vertex.

The product's restatement (mosaic_amd/csrc/jts_overlay.h) is written separately (C++,
CGAlgorithmsDD's filtered double-double orientation, its own ring building).
Parity with JTS itself is unpinned beyond the published algorithm: no JTS is in this image
and no reference fixture lists an overlay's vertices.
"""
import math
import struct
from fractions import Fraction


def orient(p, q, r):
    """sign of the exact cross product (q - p) x (r - p) (a float filter with a generous
    error bound, then rationals)"""
    l = (q[0] - p[0]) * (r[1] - p[1])
    rr = (q[1] - p[1]) * (r[0] - p[0])
    det = l - rr
    if abs(det) > 1e-14 * (abs(l) + abs(rr)):
        return int(det > 0) - int(det < 0)
    d = (Fraction(q[0]) - Fraction(p[0])) * (Fraction(r[1]) - Fraction(p[1])) - \
        (Fraction(q[1]) - Fraction(p[1])) * (Fraction(r[0]) - Fraction(p[0]))
    return (d > 0) - (d < 0)


def env_has(p1, p2, q):
    return min(p1[0], p2[0]) <= q[0] <= max(p1[0], p2[0]) and min(p1[1], p2[1]) <= q[1] <= max(p1[1], p2[1])


def env_meet(p1, p2, q1, q2):
    return not (min(p1[0], p2[0]) > max(q1[0], q2[0]) or max(p1[0], p2[0]) < min(q1[0], q2[0]) or
                min(p1[1], p2[1]) > max(q1[1], q2[1]) or max(p1[1], p2[1]) < min(q1[1], q2[1]))


def hom_intersection(p1, p2, q1, q2):
    """Intersection.intersection (JTS 1.20 algorithm/Intersection.java) or None"""
    int_min_x = max(min(p1[0], p2[0]), min(q1[0], q2[0]))
    int_max_x = min(max(p1[0], p2[0]), max(q1[0], q2[0]))
    int_min_y = max(min(p1[1], p2[1]), min(q1[1], q2[1]))
    int_max_y = min(max(p1[1], p2[1]), max(q1[1], q2[1]))
    midx = (int_min_x + int_max_x) / 2.0
    midy = (int_min_y + int_max_y) / 2.0
    p1x, p1y, p2x, p2y = p1[0] - midx, p1[1] - midy, p2[0] - midx, p2[1] - midy
    q1x, q1y, q2x, q2y = q1[0] - midx, q1[1] - midy, q2[0] - midx, q2[1] - midy
    px, py = p1y - p2y, p2x - p1x
    pw = p1x * p2y - p2x * p1y
    qx, qy = q1y - q2y, q2x - q1x
    qw = q1x * q2y - q2x * q1y
    x = py * qw - qy * pw
    y = qx * pw - px * qw
    w = px * qy - qx * py
    try:
        xi, yi = x / w, y / w
    except ZeroDivisionError:  # (Java: NaN / infinity)
        return None
    if not (math.isfinite(xi) and math.isfinite(yi)):
        return None
    return (xi + midx, yi + midy)


def _seg_dist(p, a, b):
    """Distance.pointToSegment"""
    if a == b:
        return math.hypot(p[0] - a[0], p[1] - a[1])
    len2 = (b[0] - a[0]) * (b[0] - a[0]) + (b[1] - a[1]) * (b[1] - a[1])
    r = ((p[0] - a[0]) * (b[0] - a[0]) + (p[1] - a[1]) * (b[1] - a[1])) / len2
    if r <= 0.0:
        return math.hypot(p[0] - a[0], p[1] - a[1])
    if r >= 1.0:
        return math.hypot(p[0] - b[0], p[1] - b[1])
    s = ((a[1] - p[1]) * (b[0] - a[0]) - (a[0] - p[0]) * (b[1] - a[1])) / len2
    return abs(s) * math.sqrt(len2)


def _nearest_endpoint(p1, p2, q1, q2):
    best, m = p1, _seg_dist(p1, q1, q2)
    for pt, a, b in ((p2, q1, q2), (q1, p1, p2), (q2, p1, p2)):
        d = _seg_dist(pt, a, b)
        if d < m:
            best, m = pt, d
    return best


def line_intersection(p1, p2, q1, q2):
    """RobustLineIntersector.computeIntersect -> (points, proper)"""
    if not env_meet(p1, p2, q1, q2):
        return [], False
    pq1, pq2 = orient(p1, p2, q1), orient(p1, p2, q2)
    if pq1 * pq2 > 0:
        return [], False
    qp1, qp2 = orient(q1, q2, p1), orient(q1, q2, p2)
    if qp1 * qp2 > 0:
        return [], False
    if pq1 == pq2 == qp1 == qp2 == 0:
        q1p, q2p, p1q, p2q = env_has(p1, p2, q1), env_has(p1, p2, q2), env_has(q1, q2, p1), env_has(q1, q2, p2)
        for c, a, b in ((q1p and q2p, q1, q2), (p1q and p2q, p1, p2), (q1p and p1q, q1, p1), (q1p and p2q, q1, p2),
                        (q2p and p1q, q2, p1), (q2p and p2q, q2, p2)):
            if c:
                return ([a] if a == b else [a, b]), False
        return [], False
    if 0 in (pq1, pq2, qp1, qp2):
        if p1 in (q1, q2):
            return [p1], False
        if p2 in (q1, q2):
            return [p2], False
        return [q1 if pq1 == 0 else q2 if pq2 == 0 else p1 if qp1 == 0 else p2], False
    ip = hom_intersection(p1, p2, q1, q2)
    if ip is None:
        ip = _nearest_endpoint(p1, p2, q1, q2)
    if not (env_has(p1, p2, ip) and env_has(q1, q2, ip)):
        ip = _nearest_endpoint(p1, p2, q1, q2)
    return [ip], True


def _segments(rings):
    for r in rings:
        for k in range(len(r) - 1):
            if r[k] != r[k + 1]:
                yield r[k], r[k + 1]


def chip_nodes(poly_rings, cell_rings):
    """(all nodes, proper crossing nodes) of the polygon's segments against the cell's"""
    xs = [p[0] for r in cell_rings for p in r]
    ys = [p[1] for r in cell_rings for p in r]
    x0, x1, y0, y1 = min(xs), max(xs), min(ys), max(ys)
    cell_segs = list(_segments(cell_rings))
    nodes, proper = set(), set()
    for a, b in _segments(poly_rings):
        if max(a[0], b[0]) < x0 or min(a[0], b[0]) > x1 or max(a[1], b[1]) < y0 or min(a[1], b[1]) > y1:
            continue
        for c, d in cell_segs:
            pts, pr = line_intersection(a, b, c, d)
            nodes.update(pts)
            if pr:
                proper.update(pts)
    return nodes, proper


def wkb_rings(w):
    """-> list of pieces, each a list of rings (list of (x, y)); BE/LE POLYGON / MULTIPOLYGON"""
    out = []

    def geom(o):
        e = "<" if w[o] == 1 else ">"
        t = struct.unpack_from(e + "I", w, o + 1)[0] & 0xFFFF
        o += 5
        if t == 3:
            n = struct.unpack_from(e + "I", w, o)[0]
            o += 4
            piece = []
            for _ in range(n):
                m = struct.unpack_from(e + "I", w, o)[0]
                o += 4
                piece.append([struct.unpack_from(e + "dd", w, o + 16 * k) for k in range(m)])
                o += 16 * m
            out.append(piece)
        elif t in (6, 7):
            n = struct.unpack_from(e + "I", w, o)[0]
            o += 4
            for _ in range(n):
                o = geom(o)
        else:
            raise ValueError("unexpected WKB type %d" % t)
        return o

    geom(0)
    return out


def check_chip(chip_wkb, poly_rings, cell_rings, poly_is_multi):
    """Assert a border chip's vertices are what the overlay's arithmetic allows (module doc).
    Returns (n crossing vertices, n coerce vertices)."""
    pieces = wkb_rings(chip_wkb)
    nodes, proper = chip_nodes(poly_rings, cell_rings)
    pverts = {p for r in poly_rings for p in r}
    cverts = {p for r in cell_rings for p in r}
    verts = set()
    n_coerce = 0
    coerced = bool(poly_is_multi) != (len(pieces) > 1)
    cell_segs = list(_segments(cell_rings))
    for piece in pieces:
        for ring in piece:
            assert ring[0] == ring[-1] and len(ring) >= 4, "ring not closed"
            m = len(ring) - 1
            for k in range(m):
                v = ring[k]
                verts.add(v)
                if v in pverts or v in cverts or v in nodes:
                    continue
                # a node coerceChipGeometry's difference added on the edge prev -> next
                prev, nxt = ring[(k - 1) % m], ring[(k + 1) % m]
                ok = any(v in line_intersection(prev, nxt, c, d)[0] for c, d in cell_segs)
                assert ok, "chip vertex %r is neither an input vertex nor a node" % (v,)
                assert coerced, "a re-noded vertex %r in a chip coerceChipGeometry leaves alone" % (v,)
                n_coerce += 1
    missing = [p for p in proper if p not in verts]
    assert not missing, "crossing nodes missing from the chip: %r" % missing[:3]
    return len(proper), n_coerce
