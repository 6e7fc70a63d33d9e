"""Synthetic workloads of BASELINE.json's configs (bench.py --config, and the parity
tests at small sizes).  Everything is seeded; nothing is downloaded.

  c2  uniform points in the NYC taxi-zone bbox x the 263 NYC taxi zones (the
      reference's python/test/data/NYC_Taxi_Zones.geojson, tests/golden), H3 res 9
  c4  BNG: points uniform in the London extent [503000, 561000] x [155000, 201000]
      at 0.01 m granularity (like UPRNs, transform_join_bng.ipynb cell 21) x
      UK-style polygons: a seeded Voronoi partition of that extent into ~180
      postcode-district-like cells with wiggly (subdivided, jittered) shared edges;
      BNG res 4 (100 m) by default
  c5  skewed: points from a Gaussian mixture centred on polygon boundaries (90% within
      ~2 res-9 cells of an edge) x a few large fractal-boundary polygons (>= 10k
      vertices each), H3 res 9 -- stresses the PIP stage
"""
import os

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
NYC_BBOX = (-74.25559136315209, 40.496115395170364, -73.7000090639354, 40.91553277700258)
LONDON_BNG = (503000.0, 155000.0, 561000.0, 201000.0)


def nyc_zones():
    import mosaic_amd as M
    return M.Polygons.from_npz(os.path.join(ROOT, "tests", "golden", "nyc_taxi_zones.npz"))


def _jitter_edge(p, q, rng_key, n, amp):
    """Deterministic wiggle between p and q (the same for both neighbours of an edge)."""
    a, b = (p, q) if (p[0], p[1]) <= (q[0], q[1]) else (q, p)
    r = np.random.default_rng(abs(hash((round(a[0], 3), round(a[1], 3), round(b[0], 3), round(b[1], 3),
                                        rng_key))) % (2 ** 32))
    t = np.linspace(0, 1, n + 2)[1:-1]
    d = np.array(b) - np.array(a)
    nrm = np.array([-d[1], d[0]]) / (np.hypot(*d) + 1e-300)
    off = r.uniform(-amp, amp, n) * np.sin(np.pi * t)
    pts = np.array(a)[None, :] + t[:, None] * d[None, :] + off[:, None] * nrm[None, :]
    if (a, b) != (p, q):
        pts = pts[::-1]
    return [tuple(v) for v in pts]


def london_districts(n_cells=180, seed=4, wiggle=6):
    """Voronoi partition of LONDON_BNG with jittered shared edges (polygon ids 1..)."""
    import mosaic_amd as M
    from scipy.spatial import Voronoi
    x0, y0, x1, y1 = LONDON_BNG
    rng = np.random.default_rng(seed)
    sites = np.stack([rng.uniform(x0, x1, n_cells), rng.uniform(y0, y1, n_cells)], 1)
    # mirror the sites across the four sides so every cell is bounded by the extent
    mir = [sites, sites * [-1, 1] + [2 * x0, 0], sites * [-1, 1] + [2 * x1, 0],
           sites * [1, -1] + [0, 2 * y0], sites * [1, -1] + [0, 2 * y1]]
    vor = Voronoi(np.concatenate(mir))
    polys = []
    for i in range(n_cells):
        reg = vor.regions[vor.point_region[i]]
        if -1 in reg or not reg:
            continue
        v = vor.vertices[reg]
        c = v.mean(0)
        v = v[np.argsort(np.arctan2(v[:, 1] - c[1], v[:, 0] - c[0]))]
        v = np.clip(v, [x0, y0], [x1, y1])
        ring = []
        for k in range(len(v)):
            p, q = tuple(v[k]), tuple(v[(k + 1) % len(v)])
            ring.append(p)
            on_border = (p[0] in (x0, x1) and q[0] == p[0]) or (p[1] in (y0, y1) and q[1] == p[1])
            if not on_border:
                ring += _jitter_edge(p, q, seed, wiggle, 0.04 * np.hypot(q[0] - p[0], q[1] - p[1]))
        ring.append(ring[0])
        polys.append((i + 1, [[ring]]))
    return M.Polygons.from_lists(polys)


def _koch_ring(cx, cy, radius, depth, rng):
    """A closed fractal-boundary ring (randomised Koch-like refinement of a polygon)."""
    k = 12
    ang = np.linspace(0, 2 * np.pi, k, endpoint=False)
    pts = np.stack([cx + radius * np.cos(ang), cy + radius * np.sin(ang) * 0.8], 1)
    for _ in range(depth):
        out = []
        for a, b in zip(pts, np.roll(pts, -1, 0)):
            d = b - a
            nrm = np.array([d[1], -d[0]])  # outward for a ccw ring
            s = rng.uniform(0.15, 0.3) * (1 if rng.random() < 0.6 else -1)
            out += [a, a + d / 3, a + d / 2 + s * nrm / np.sqrt(3), a + 2 * d / 3]
        pts = np.array(out)
    ring = [tuple(p) for p in pts]
    ring.append(ring[0])
    return ring


def skewed_polygons(seed=5, depth=6):
    """Four large fractal-boundary polygons in the NYC area (12 * 4^6 = 49k vertices each)."""
    import mosaic_amd as M
    rng = np.random.default_rng(seed)
    polys = []
    for i, (cx, cy) in enumerate([(-74.05, 40.62), (-73.93, 40.72), (-73.85, 40.82), (-74.12, 40.78)]):
        polys.append((i + 1, [[_koch_ring(cx, cy, 0.05, depth, rng)]]))
    return M.Polygons.from_lists(polys)


def boundary_points(P, n, seed, sigma, dev=None):
    """90% of the points Gaussian around random boundary vertices of P, 10% uniform in
    P's bbox (numpy, or torch on `dev`)."""
    rng = np.random.default_rng(seed)
    v = np.asarray(P.xy).reshape(-1, 2)
    lo, hi = v.min(0), v.max(0)
    k = int(n * 0.9)
    idx = rng.integers(0, len(v), k)
    near = v[idx] + rng.normal(0, sigma, (k, 2))
    far = rng.uniform(lo, hi, (n - k, 2))
    pts = np.concatenate([near, far])
    rng.shuffle(pts)
    x, y = np.ascontiguousarray(pts[:, 0]), np.ascontiguousarray(pts[:, 1])
    if dev is None:
        return x, y
    import torch
    return torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev)


def london_points(n, seed, dev=None):
    """Eastings/northings uniform in LONDON_BNG at 0.01 m granularity."""
    x0, y0, x1, y1 = LONDON_BNG
    if dev is None:
        rng = np.random.default_rng(seed)
        return (np.round(rng.uniform(x0, x1, n), 2), np.round(rng.uniform(y0, y1, n), 2))
    import torch
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    x = torch.rand(n, dtype=torch.float64, device=dev, generator=g).mul_(x1 - x0).add_(x0).mul_(100).round_().div_(100)
    y = torch.rand(n, dtype=torch.float64, device=dev, generator=g).mul_(y1 - y0).add_(y0).mul_(100).round_().div_(100)
    return x, y


# C3: the 1B-point, ~74k-polygon, res-10 join.  Extent: a 4 deg x 3 deg block of the
# north-eastern US (PA / NJ / NY, one H3 icosahedron face), cut into census-tract-like
# cells of ~1.6 km^2 on average (urban-tract scale; the real CONUS tract set averages
# far larger cells, but most tract *boundaries* are urban).
TRACT_EXTENT = (-77.5, 39.5, -73.5, 42.5)
N_TRACTS = 74_000


def tract_polygons(n_cells=N_TRACTS, extent=TRACT_EXTENT, seed=3, k_lo=2, k_hi=40, amp=0.05):
    """Seeded Voronoi partition of `extent` into `n_cells` tract-like polygons (ids 1..n)
    whose shared edges are jittered polylines with k_lo..k_hi interior vertices each
    (identical in both neighbours), so a tract has ~20-400 vertices."""
    import mosaic_amd as M
    from scipy.spatial import Voronoi
    x0, y0, x1, y1 = extent
    rng = np.random.default_rng(seed)
    sites = np.stack([rng.uniform(x0, x1, n_cells), rng.uniform(y0, y1, n_cells)], 1)
    mir = [sites, sites * [-1, 1] + [2 * x0, 0], sites * [-1, 1] + [2 * x1, 0],
           sites * [1, -1] + [0, 2 * y0], sites * [1, -1] + [0, 2 * y1]]
    vor = Voronoi(np.concatenate(mir))
    V = np.clip(vor.vertices, [x0, y0], [x1, y1])
    rp = vor.ridge_points
    rv = np.array([r if len(r) == 2 else [-1, -1] for r in vor.ridge_vertices], dtype=np.int64)
    keep = ((rp[:, 0] < n_cells) | (rp[:, 1] < n_cells)) & (rv.min(1) >= 0)
    rp, rv = rp[keep], rv[keep]
    # a ridge between a site and one of its mirrors lies on the extent border: straight
    border = (rp[:, 0] % n_cells) == (rp[:, 1] % n_cells)
    lo, hi = rv.min(1), rv.max(1)
    k = rng.integers(k_lo, k_hi + 1, len(rv))
    k[border] = 0
    # interior points of ridge r, running from V[lo] to V[hi]
    start = np.zeros(len(rv) + 1, np.int64)
    start[1:] = np.cumsum(k)
    rid = np.repeat(np.arange(len(rv)), k)
    t = (np.arange(start[-1]) - start[rid] + 1) / (k[rid] + 1)
    a, b = V[lo[rid]], V[hi[rid]]
    d = b - a
    nrm = np.stack([-d[:, 1], d[:, 0]], 1)
    off = rng.uniform(-amp, amp, len(rid)) * np.sin(np.pi * t)
    P = np.clip(a + t[:, None] * d + off[:, None] * nrm, [x0, y0], [x1, y1])
    ridge_of = {(int(u), int(v)): i for i, (u, v) in enumerate(zip(lo, hi))}
    xy, ring_off = [], [0]
    ids = []
    for i in range(n_cells):
        reg = vor.regions[vor.point_region[i]]
        if -1 in reg or not reg:
            continue
        reg = np.array(reg)
        v = V[reg]
        c = v.mean(0)
        reg = reg[np.argsort(np.arctan2(v[:, 1] - c[1], v[:, 0] - c[0]))]
        pieces = []
        for j in range(len(reg)):
            p, q = int(reg[j]), int(reg[(j + 1) % len(reg)])
            pieces.append(V[p][None, :])
            r = ridge_of.get((min(p, q), max(p, q)))
            if r is not None and k[r]:
                seg = P[start[r]:start[r + 1]]
                pieces.append(seg if p < q else seg[::-1])
        pieces.append(V[int(reg[0])][None, :])
        ring = np.concatenate(pieces)
        xy.append(ring)
        ring_off.append(ring_off[-1] + len(ring))
        ids.append(i + 1)
    n = len(ids)
    return M.Polygons(ids, np.arange(n + 1), np.arange(n + 1), ring_off, np.concatenate(xy))


def extent_points(extent, n, seed, dev=None):
    """Points uniform in `extent` (numpy, or torch on `dev`)."""
    x0, y0, x1, y1 = extent
    if dev is None:
        rng = np.random.default_rng(seed)
        return rng.uniform(x0, x1, n), rng.uniform(y0, y1, n)
    import torch
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    x = torch.rand(n, dtype=torch.float64, device=dev, generator=g).mul_(x1 - x0).add_(x0)
    y = torch.rand(n, dtype=torch.float64, device=dev, generator=g).mul_(y1 - y0).add_(y0)
    return x, y
