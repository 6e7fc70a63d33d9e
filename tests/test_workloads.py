"""The synthetic workloads of BASELINE.json's configs (bench_workloads.py): shapes and
tessellation invariants on the CPU; the GPU parity of their joins is in
test_gpu_parity.py."""
import os
import sys

import numpy as np

import mosaic_amd as M

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import bench_workloads as W  # noqa: E402
import oracle as O  # noqa: E402  (test infrastructure: the checker)


def test_london_districts_partition_the_extent():
    P = W.london_districts()
    assert len(P.poly_part_off) - 1 > 150
    c = M.tessellate(P, M.BNGIndexSystem(), 3)
    x, y = W.london_points(20_000, 3)
    pts, polys = O.pip_join(1, 3, x, y, c.cell, c.polygon_id, c.is_core, c.wkb_offsets, c.wkb)
    # every point is in at most one district, and almost all in exactly one
    assert len(np.unique(pts)) == len(pts)
    assert len(pts) > 0.97 * len(x)


def test_skewed_polygons_shape():
    P = W.skewed_polygons()
    assert len(P.poly_part_off) - 1 == 4
    assert len(P.xy) > 4 * 10_000
    x, y = W.boundary_points(P, 10_000, 1, 0.003)
    assert x.shape == (10_000,) and np.isfinite(x).all() and np.isfinite(y).all()
    c = M.tessellate(P, M.H3IndexSystem(), 9)
    assert (c.is_core == 0).sum() > 100


def test_tract_polygons_partition_the_extent():
    """C3's generator: a Voronoi partition with shared jittered edges -- each point of
    the extent lies in exactly one tract (checked on a small block at res 9)."""
    E = (-75.0, 40.0, -74.8, 40.15)
    P = W.tract_polygons(n_cells=400, extent=E, seed=8)
    nv = np.diff(P.ring_off)
    assert len(P) == 400 and nv.min() >= 10 and nv.max() <= 500
    c = M.tessellate(P, M.H3IndexSystem(), 9, keep_core_geometries=False)
    x, y = W.extent_points(E, 20_000, 4)
    pts, polys = O.pip_join(0, 9, x, y, c.cell, c.polygon_id, c.is_core, c.wkb_offsets, c.wkb)
    assert len(np.unique(pts)) == len(pts)
    assert len(pts) > 0.99 * len(x)


def test_traffic_key_tracks_options_table_and_source():
    """bench.py attaches a PMC traffic profile only when its key -- context options, the
    uploaded table's size, the kernels' source hash -- equals the run's: a line run with
    --option raster_sub=8 cannot carry counters measured on the default build."""
    import bench as B
    info = {"chips": 11890, "bytes": 86787072}
    k = B.traffic_key([], info)
    assert k == B.traffic_key([], dict(info))
    assert k != B.traffic_key(["raster_sub=8"], info)
    assert k != B.traffic_key([], {"chips": 11890, "bytes": 60000000})
    assert B.traffic_key(["a=1", "b=2"], info) == B.traffic_key(["b=2", "a=1"], info)
    assert len(k["kernels_sha16"]) == 16
