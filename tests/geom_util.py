"""Small geometry helpers for the tests: WKT polygons -> WKB, areas, random points."""
import re
import struct

import numpy as np


def _rings(body):
    rings = []
    for r in re.findall(r"\(([^()]*)\)", body):
        pts = [tuple(float(v) for v in p.split()) for p in r.split(",")]
        rings.append(pts)
    return rings


def wkt_to_parts(wkt):
    wkt = wkt.strip()
    if wkt.upper().startswith("MULTIPOLYGON"):
        inner = wkt[wkt.index("(") + 1:wkt.rindex(")")]
        parts, depth, start = [], 0, None
        for i, ch in enumerate(inner):
            if ch == "(":
                if depth == 0:
                    start = i
                depth += 1
            elif ch == ")":
                depth -= 1
                if depth == 0:
                    parts.append(_rings(inner[start + 1:i]))
        return parts
    if wkt.upper().startswith("POLYGON"):
        return [_rings(wkt[wkt.index("(") + 1:wkt.rindex(")")])]
    raise ValueError(wkt)


def parts_to_wkb(parts, little_endian=False, force_multi=False):
    bo = "<" if little_endian else ">"
    flag = 1 if little_endian else 0

    def poly(p):
        b = struct.pack(bo + "BII", flag, 3, len(p))
        for r in p:
            b += struct.pack(bo + "I", len(r)) + b"".join(struct.pack(bo + "dd", x, y) for x, y in r)
        return b
    if len(parts) == 1 and not force_multi:
        return poly(parts[0])
    return struct.pack(bo + "BII", flag, 6, len(parts)) + b"".join(poly(p) for p in parts)


def wkt_to_wkb(wkt, **kw):
    return parts_to_wkb(wkt_to_parts(wkt), **kw)


def ring_area(r):
    a = 0.0
    for (x1, y1), (x2, y2) in zip(r[:-1], r[1:]):
        a += x1 * y2 - x2 * y1
    return 0.5 * a


def polygons_area(polys, p):
    tot = 0.0
    for q in range(polys.poly_part_off[p], polys.poly_part_off[p + 1]):
        for k, r in enumerate(range(polys.part_ring_off[q], polys.part_ring_off[q + 1])):
            ring = polys.xy[polys.ring_off[r]:polys.ring_off[r + 1]]
            a = abs(ring_area([tuple(v) for v in ring]))
            tot += a if k == 0 else -a
    return tot


def wkb_area(wkb):
    """Area of a big/little-endian Polygon/MultiPolygon WKB (2-D)."""
    pos = [0]

    def rd(fmt, n):
        v = struct.unpack_from(fmt, wkb, pos[0])
        pos[0] += n
        return v

    def geom():
        bo = "<" if wkb[pos[0]] == 1 else ">"
        pos[0] += 1
        (t,) = rd(bo + "I", 4)
        if t == 3:
            (nr,) = rd(bo + "I", 4)
            a = 0.0
            for k in range(nr):
                (np_,) = rd(bo + "I", 4)
                pts = [rd(bo + "dd", 16) for _ in range(np_)]
                ra = abs(ring_area(pts))
                a += ra if k == 0 else -ra
            return a
        (n,) = rd(bo + "I", 4)
        return sum(geom() for _ in range(n))
    return geom()


def polygon_set_wkbs(polys):
    out = []
    for p in range(len(polys)):
        parts = []
        for q in range(polys.poly_part_off[p], polys.poly_part_off[p + 1]):
            parts.append([[tuple(v) for v in polys.xy[polys.ring_off[r]:polys.ring_off[r + 1]]]
                          for r in range(polys.part_ring_off[q], polys.part_ring_off[q + 1])])
        out.append((int(polys.poly_id[p]), parts_to_wkb(parts)))
    return out


NYC_BBOX = (-74.25559136315209, 40.496115395170364, -73.7000090639354, 40.91553277700258)


def nyc_points(n, seed):
    rng = np.random.default_rng(seed)
    return rng.uniform(NYC_BBOX[0], NYC_BBOX[2], n), rng.uniform(NYC_BBOX[1], NYC_BBOX[3], n)


def brute_force_pairs(polys, x, y, oracle):
    """(point, polygon) pairs by JTS-semantics contains against the ORIGINAL polygons."""
    pairs = set()
    for k, (pid, w) in enumerate(polygon_set_wkbs(polys)):
        lo = polys.ring_off[polys.part_ring_off[polys.poly_part_off[k]]]
        hi = polys.ring_off[polys.part_ring_off[polys.poly_part_off[k + 1]]]
        xs = polys.xy[lo:hi]
        mn, mx = xs.min(0), xs.max(0)
        idx = np.nonzero((x >= mn[0]) & (x <= mx[0]) & (y >= mn[1]) & (y <= mx[1]))[0]
        for i in idx:
            if oracle.st_contains(w, x[i], y[i]):
                pairs.add((int(i), pid))
    return pairs
