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
    """shoelace about the ring's first vertex (absolute lon / lat products would cancel a
    small chip's area into rounding noise)"""
    if len(r) < 2:
        return 0.0
    x0, y0 = r[0]
    a = 0.0
    for (x1, y1), (x2, y2) in zip(r[:-1], r[1:]):
        a += (x1 - x0) * (y2 - y0) - (x2 - x0) * (y1 - y0)
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


def crossing_adversaries(P, table, cell_rings_of, ulps=3, steps=4, max_chips=None, grid_step=None):
    """Points a few ulps from every place a polygon edge crosses a cell edge (the
    reference's chip vertices there come from JTS's RobustLineIntersector: oracle/
    jts_overlay.py): points on the ORIGINAL polygon segment near the crossing (rounded
    a + t (b - a) for t around the crossing's parameter, `steps` each way, 2^-50 apart) and
    the crossing node's ulp neighbourhood (+-`ulps` in x and y).  grid_step (BNG): also the
    0.01-m points on the square line nearest the crossing, 3 each way.
    -> (x, y) float64 arrays."""
    import jts_overlay as JO
    idx = {int(p): i for i, p in enumerate(P.poly_id)}
    rows = np.nonzero(~table.is_core.astype(bool))[0]
    if max_chips is not None:
        rows = rows[:: max(1, len(rows) // max_chips)]
    xs, ys = [], []
    cache = {}
    for i in rows:
        k = idx[int(table.polygon_id[i])]
        if k not in cache:
            cache[k] = [[tuple(map(float, v)) for v in P.xy[P.ring_off[r]:P.ring_off[r + 1]]]
                        for q in range(P.poly_part_off[k], P.poly_part_off[k + 1])
                        for r in range(P.part_ring_off[q], P.part_ring_off[q + 1])]
        w = bytes(table.wkb[table.wkb_offsets[i]:table.wkb_offsets[i + 1]])
        cell = cell_rings_of(table.cell[i], w)
        cx = [p[0] for r in cell for p in r]
        cy = [p[1] for r in cell for p in r]
        x0, x1, y0, y1 = min(cx), max(cx), min(cy), max(cy)
        csegs = [(r[j], r[j + 1]) for r in cell for j in range(len(r) - 1)]
        for ring in cache[k]:
            for j in range(len(ring) - 1):
                a, b = ring[j], ring[j + 1]
                if a == b or max(a[0], b[0]) < x0 or min(a[0], b[0]) > x1 or max(a[1], b[1]) < y0 or min(a[1], b[1]) > y1:
                    continue
                for c, d in csegs:
                    pts, proper = JO.line_intersection(a, b, c, d)
                    if not proper:
                        continue
                    X = pts[0]
                    ax = 0 if abs(b[0] - a[0]) >= abs(b[1] - a[1]) else 1
                    t = (X[ax] - a[ax]) / (b[ax] - a[ax])
                    for s in range(-steps, steps + 1):
                        tt = t + s * 2.0 ** -50
                        xs.append(a[0] + tt * (b[0] - a[0]))
                        ys.append(a[1] + tt * (b[1] - a[1]))
                    for dx in range(-ulps, ulps + 1):
                        for dy in range(-ulps, ulps + 1):
                            px, py = X
                            for _ in range(abs(dx)):
                                px = np.nextafter(px, np.inf if dx > 0 else -np.inf)
                            for _ in range(abs(dy)):
                                py = np.nextafter(py, np.inf if dy > 0 else -np.inf)
                            xs.append(float(px))
                            ys.append(float(py))
                    if grid_step:
                        # the square line the crossing lies on (vertical: x fixed, else y fixed)
                        if c[0] == d[0]:
                            base = round(X[1], 2)
                            for s in range(-3, 4):
                                xs.append(c[0])
                                ys.append(round(base + s * grid_step, 2))
                        else:
                            base = round(X[0], 2)
                            for s in range(-3, 4):
                                xs.append(round(base + s * grid_step, 2))
                                ys.append(c[1])
    return np.array(xs, np.float64), np.array(ys, np.float64)
