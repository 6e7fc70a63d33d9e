"""H3 kRing / kLoop checked against cell geometry, independent of the neighbour tables.

The device kRing (h3_ring.h) and the oracle's restatement share the derived
baseCellNeighbors / rotation tables (tools/gen_h3_neighbors.py -> h3_neighbors.inc), so
their agreement (tests/test_gpu_parity.py test_h3_kring_kloop_equal_oracle) cannot catch a
wrong table entry.  This test checks the oracle's lists -- hence, through that GPU test,
the device's -- against geometry built from different tables (faceIjkBaseCells +
faceNeighbors, h3_boundary.h): two cells are neighbours when their h3ToGeoBoundary
polygons share an edge.  For every neighbourhood among hexagon base cells, base-cell
crossings included: kRing(h, k) has 1 + 3k(k+1) distinct cells, its j-th spiral ring is
exactly the cells at graph distance j from h, and kLoop(h, k) lists ring k with each
cell adjacent to the next (cyclically).  H3IndexSystem.kRing / kLoop:
H3IndexSystem.scala:182-205.
"""
import numpy as np
import pytest

import oracle as O
from test_tessellate_host import cell_geometry

H3_PENTAGON_BASE_CELLS = {4, 14, 24, 38, 49, 58, 63, 72, 83, 97, 107, 117}


def _vertex_keys(cells):
    xy, nv, _ = cell_geometry(cells)
    keys = {}
    for i, h in enumerate(cells):
        # (distortion vertices of two cells across an icosahedron edge agree to ~1e-7 deg:
        # H3 intersects in float)
        keys[int(h)] = {(round(x, 5), round(y, 5)) for x, y in xy[i, :nv[i]]}
    return keys


def _adjacent(a, b):
    return len(a & b) >= 2


@pytest.mark.parametrize("res", [1, 2, 3, 5, 8, 10])
def test_kring_rings_are_graph_distances(res):
    rng = np.random.default_rng(300 + res)
    lon = rng.uniform(-180, 180, 400)
    lat = np.degrees(np.arcsin(rng.uniform(-1, 1, 400)))
    cells = np.unique(O.h3_points_to_cells(lon, lat, res))
    checked = crossings = 0
    for c in cells:
        c = int(c)
        k = 3 if res >= 3 else 1
        ring = O.h3_k_ring(c, k)
        if any(((x >> 45) & 127) in H3_PENTAGON_BASE_CELLS for x in O.h3_k_ring(c, k + 1)):
            continue
        assert len(ring) == 1 + 3 * k * (k + 1) and len(set(ring)) == len(ring) and ring[0] == c
        crossings += len({(x >> 45) & 127 for x in ring}) > 1
        keys = _vertex_keys(np.array(ring, dtype=np.int64))
        # graph distances from c over shared-edge adjacency within the ring set
        dist = {c: 0}
        frontier = [c]
        while frontier:
            nxt = []
            for u in frontier:
                for v in ring:
                    if v not in dist and _adjacent(keys[u], keys[v]):
                        dist[v] = dist[u] + 1
                        nxt.append(v)
            frontier = nxt
        for j in range(k + 1):
            lo, hi = (0, 1) if j == 0 else (1 + 3 * j * (j - 1), 1 + 3 * j * (j + 1))
            assert all(dist.get(v) == j for v in ring[lo:hi]), (hex(c), j)
        loop = O.h3_k_loop(c, k)
        assert sorted(loop) == sorted(ring[1 + 3 * k * (k - 1):])
        assert all(_adjacent(keys[loop[i]], keys[loop[(i + 1) % len(loop)]]) for i in range(len(loop)))
        checked += 1
    assert checked > 50 and (res > 3 or crossings > 5)


def _geo_neighbours(cells, res):
    """Each cell's neighbours from geometry alone: a point just outside the midpoint of
    every boundary edge (h3ToGeoBoundary, distortion vertices included), indexed by
    geoToH3 -- faceIjkBaseCells + faceNeighbors, not the neighbour tables."""
    xy, nv, ctr = cell_geometry(np.asarray(cells, dtype=np.int64))

    def unit(lon, lat):
        lo, la = np.radians(lon), np.radians(lat)
        return np.stack([np.cos(la) * np.cos(lo), np.cos(la) * np.sin(lo), np.sin(la)], -1)

    out = {}
    for i, h in enumerate(cells):
        v = unit(xy[i, :nv[i], 0], xy[i, :nv[i], 1])
        c = unit(ctr[i, 0], ctr[i, 1])
        m = v + np.roll(v, -1, 0)
        m /= np.linalg.norm(m, axis=1)[:, None]
        p = m + 0.05 * (m - c)
        p /= np.linalg.norm(p, axis=1)[:, None]
        lon, lat = np.degrees(np.arctan2(p[:, 1], p[:, 0])), np.degrees(np.arcsin(p[:, 2]))
        nb = set(int(x) for x in O.h3_points_to_cells(lon, lat, res)) - {int(h)}
        out[int(h)] = nb
    return out


@pytest.mark.parametrize("res,kmax", [(1, 3), (2, 4), (3, 5), (5, 5), (8, 4)])
def test_pentagon_krings_are_geometric_balls(res, kmax):
    """Around pentagons -- the polar ones 4 and 117 among them -- kRing(h, k) (H3's
    _kRingInternal hash-set walk) is exactly the set of cells within k steps of h over
    geometric adjacency, and kLoop(h, k) the cells at exactly k steps; for the pentagon
    itself and for cells next to it, k = 1..kmax.  Adjacency comes from cell geometry and
    geoToH3 only (no neighbour table).  (This pins the sets; the lists' order -- the
    walk's hash-set order -- follows the derived direction tables.)"""
    unused = sum(7 << (3 * (15 - r)) for r in range(res + 1, 16))
    pents = [(1 << 59) | (res << 52) | (b << 45) | unused for b in sorted(H3_PENTAGON_BASE_CELLS)]
    nbr_cache = {}

    def neighbours(cells):
        need = [c for c in cells if c not in nbr_cache]
        if need:
            nbr_cache.update(_geo_neighbours(need, res))
        return {c: nbr_cache[c] for c in cells}

    checked = 0
    for p in pents:
        starts = [p] + sorted(neighbours([p])[p])[:2]
        for h in starts:
            dist = {h: 0}
            frontier = [h]
            for step in range(1, kmax + 1):
                nxt = []
                for u, nb in neighbours(frontier).items():
                    for v in nb:
                        if v not in dist:
                            dist[v] = step
                            nxt.append(v)
                frontier = nxt
                ball = {v for v, d in dist.items() if d <= step}
                ring = O.h3_k_ring(h, step)
                assert set(ring) == ball and len(ring) == len(ball), (hex(h), step)
                assert set(O.h3_k_loop(h, step)) == {v for v, d in dist.items() if d == step}, (hex(h), step)
                checked += 1
    assert checked == 12 * 3 * kmax
