"""The binned join pipeline (spatial counting sort of the points, join over
the binned points, answers gathered back into input order) against the oracle, through
the C ABI.  The context option pipeline = MGPU_PIPELINE_BINNED forces it on tables of any
size (the planner's default takes it only for tables beyond the Infinity Cache, e.g. C3)
and keeps the split pipeline of pixel-indexed tables out of the way.  Bit-exact to the
reference (the oracle with glibc's libm, as H3-Java) is the bar, as everywhere."""
import numpy as np
import pytest
import torch

import mosaic_amd as M
import oracle as O
from geom_util import nyc_points
from test_gpu_parity import T, adversarial_points, oracle_join

pytestmark = pytest.mark.gpu
BINNED = 2  # MGPU_PIPELINE_BINNED


def opts(gpu, **kw):
    """Context options of the default context (the one the tests' chip tables live on)."""
    return M.default_context(gpu).options(**kw)


def binned_join(x, y, chips, res, gpu, nb=512, xcd=1, **kw):
    with opts(gpu, pipeline=BINNED, bin_count=nb, bin_xcd=xcd):
        r = M.pip_join(T(x, gpu), T(y, gpu), chips, res, **kw)
    assert r.stats["pipeline"] == BINNED
    return r


@pytest.mark.parametrize("nb,xcd", [(1, 1), (64, 0), (200, 1), (512, 1)])
def test_binned_nyc_equals_oracle(gpu, nyc_chips_r9, nb, xcd):
    """NYC zones, H3 res 9, ragged sizes (not a multiple of any chunk or tile)."""
    d = nyc_chips_r9.upload()
    x, y = nyc_points(1_234_567, 41)
    r = binned_join(x, y, d, 9, gpu, nb=nb, xcd=xcd)
    gp, gq = r.numpy()
    op, oq = oracle_join(nyc_chips_r9, x, y)
    assert np.array_equal(gp, op) and np.array_equal(gq, oq)
    assert r.stats["n_pairs"] == len(op) and r.stats["n_candidates"] > 0


@pytest.mark.parametrize("n", [1, 7, 4095, 4097, 65537])
def test_binned_small_batches(gpu, nyc_chips_r9, n):
    d = nyc_chips_r9.upload()
    x, y = nyc_points(n, 42 + n)
    gp, gq = binned_join(x, y, d, 9, gpu).numpy()
    op, oq = oracle_join(nyc_chips_r9, x, y)
    assert np.array_equal(gp, op) and np.array_equal(gq, oq)


def test_binned_point_ids_capacity_and_fetch(gpu, nyc_chips_r9):
    """Explicit point ids, an id base, and a capacity overflow answered by
    mgpu_pip_join_fetch from the kept answers (no second join)."""
    d = nyc_chips_r9.upload()
    x, y = nyc_points(300_000, 43)
    op, oq = oracle_join(nyc_chips_r9, x, y)
    ids = np.arange(300_000, dtype=np.int64) * 5 + 3
    gp, gq = binned_join(x, y, d, 9, gpu, point_id=torch.from_numpy(ids).to(gpu)).numpy()
    assert np.array_equal(gp, ids[op]) and np.array_equal(gq, oq)
    gp, gq = binned_join(x, y, d, 9, gpu, point_id_base=10 ** 11).numpy()
    assert np.array_equal(gp, op + 10 ** 11) and np.array_equal(gq, oq)
    r = binned_join(x, y, d, 9, gpu, capacity=None)  # default capacity n + n/8 suffices here
    assert np.array_equal(r.numpy()[0], op)
    with pytest.raises(M.CapacityError) as ei:
        binned_join(x, y, d, 9, gpu, capacity=100)
    assert ei.value.required == len(op)


def test_binned_overlapping_polygons(gpu):
    """Five overlapping squares: 5 pairs per point (more than the default capacity), the
    per-point answer masks carry every match in polygon order."""
    sq = [(0.0, 0.0), (1.0, 0.0), (1.0, 1.0), (0.0, 1.0), (0.0, 0.0)]
    bx, by, sc = -74.0, 40.7, 0.05
    polys = [(pid, [[[(bx + sc * u * (1 + 0.01 * pid), by + sc * v * (1 + 0.01 * pid)) for u, v in sq]]])
             for pid in (5, 3, 9, 1, 7)]
    c = M.tessellate(M.Polygons.from_lists(polys), M.H3IndexSystem(), 8)
    rng = np.random.default_rng(44)
    x = bx + sc * rng.uniform(-0.05, 1.1, 200_000)
    y = by + sc * rng.uniform(-0.05, 1.1, 200_000)
    gp, gq = binned_join(x, y, c.upload(), 8, gpu).numpy()
    op, oq = oracle_join(c, x, y, res=8)
    assert len(op) > 3 * len(x)
    assert np.array_equal(gp, op) and np.array_equal(gq, oq)


def test_binned_adversarial_points_and_near_tie_positions(gpu, nyc_chips_r9):
    """Points on H3 cell corners: pairs equal the reference's (the oracle with glibc's
    libm), nothing excluded, in the binned and the fused pipeline.  Every point whose fast
    projection falls in its tie band is decided by the host with the reference's libm;
    mgpu_last_near_ties reports those INPUT positions.  The binned pipeline projects every
    point; the fused one answers points of certified (pure) pixels without projecting
    them -- so its list is a subset of the binned one's."""
    d = nyc_chips_r9.upload()
    x, y = adversarial_points(nyc_chips_r9)
    r = binned_join(x, y, d, 9, gpu)
    ties_b = d.ctx.last_near_ties()
    gp, gq = r.numpy()
    op, oq = oracle_join(nyc_chips_r9, x, y)
    assert np.array_equal(gp, op) and np.array_equal(gq, oq)
    with opts(gpu, pipeline=0):
        rf = M.pip_join(T(x, gpu), T(y, gpu), d, 9)
    ties_f = d.ctx.last_near_ties()
    assert rf.stats["pipeline"] == 0
    assert len(ties_b) == r.stats["n_near_ties"] > 0 and len(ties_f) == rf.stats["n_near_ties"] > 0
    assert np.array_equal(ties_b, np.unique(ties_b)) and np.array_equal(ties_f, np.unique(ties_f))
    assert set(ties_f.tolist()) <= set(ties_b.tolist())
    # ... and every position the fused list lacks lies in a certified pixel (the host's
    # replica of the pixel index, tests/test_raster_host.py), which the fused join answers
    # without projecting
    from test_raster_host import raster_lookup
    only_b = np.array(sorted(set(ties_b.tolist()) - set(ties_f.tolist())), dtype=np.int64)
    if len(only_b):
        kind, _, _, _ = raster_lookup(nyc_chips_r9, 9, x[only_b], y[only_b])
        assert (kind <= 1).all(), "%d of %d binned-only near-ties not in a certified pixel" % ((kind > 1).sum(), len(only_b))
    assert np.array_equal(rf.numpy()[0], op) and np.array_equal(rf.numpy()[1], oq)


@pytest.mark.parametrize("keys,libm", [(0, 0), (1, 0), (0, 1), (1, 1)])
def test_binned_grid_keys_adversarial(gpu, nyc_chips_r9, keys, libm):
    """The binning pass's per-slot grid keys (option bin_keys, kernels.hip bin_key_of) and
    the join's own projection give the same pairs on points at H3 cell corners, with the
    reference's libm (near-ties queued by the scatter kernel, settled on the host) and with
    the correctly rounded one (near-tie tiles sent to the fix kernel)."""
    d = nyc_chips_r9.upload()
    ax, ay = adversarial_points(nyc_chips_r9)
    rng = np.random.default_rng(5)
    x, y = nyc_points(300_000, 6)
    at = np.sort(rng.choice(len(x), len(ax), replace=False))
    x[at], y[at] = ax, ay
    if libm:
        with O.h3_libm("cr"):
            op, oq = oracle_join(nyc_chips_r9, x, y)
    else:
        op, oq = oracle_join(nyc_chips_r9, x, y)
    with opts(gpu, bin_keys=keys, h3_libm=libm):
        r = binned_join(x, y, d, 9, gpu, nb=64)
    gp, gq = r.numpy()
    assert np.array_equal(gp, op) and np.array_equal(gq, oq)
    assert r.stats["n_near_ties"] > 0


def test_binned_bng_london(gpu):
    """BNG (C4's districts, res 3 and 4): bins over the dense grid's box."""
    import bench_workloads as W
    P = W.london_districts()
    for res in (3, 4):
        c = M.tessellate(P, M.BNGIndexSystem(), res)
        x, y = W.london_points(1_000_000, 45 + res)
        r = binned_join(x, y, c.upload(), res, gpu, index_system=M.BNGIndexSystem())
        op, oq = oracle_join(c, x, y, res=res, isys=1)
        gp, gq = r.numpy()
        assert np.array_equal(gp, op) and np.array_equal(gq, oq), res


def test_binned_points_outside_and_nan(gpu, nyc_chips_r9):
    """Points far outside the chip table's extent (clamped to edge bins, matching
    nothing) mixed with inside points; a NaN coordinate still raises as in the reference."""
    d = nyc_chips_r9.upload()
    x, y = nyc_points(200_000, 46)
    x[::7] += 3.0
    y[::11] -= 2.0
    gp, gq = binned_join(x, y, d, 9, gpu).numpy()
    op, oq = oracle_join(nyc_chips_r9, x, y)
    assert np.array_equal(gp, op) and np.array_equal(gq, oq)
    x[5] = np.nan
    with opts(gpu, pipeline=BINNED):
        with pytest.raises(M.IllegalArgumentException):
            M.pip_join(T(x, gpu), T(y, gpu), d, 9)


def test_binned_c3_full_table(gpu):
    """BASELINE config C3's whole table (74,000 tract-like polygons, 9.4M chips at res
    10) -- the case the binned pipeline is for -- with 2.5M points: the planner picks it
    by itself (table beyond the Infinity Cache, batch >= 2^21 points), pairs equal the
    reference (the oracle, glibc libm) and the fused pipeline."""
    import bench_workloads as W
    P = W.tract_polygons()
    c = M.tessellate(P, M.H3IndexSystem(), 10, keep_core_geometries=False)
    d = c.upload()
    x, y = W.extent_points(W.TRACT_EXTENT, 2_500_000, 47)
    r = M.pip_join(T(x, gpu), T(y, gpu), d, 10)
    assert r.stats["pipeline"] == BINNED
    gp, gq = r.numpy()
    op, oq = O.pip_join(0, 10, x, y, c.cell, c.polygon_id, c.is_core, c.wkb_offsets, c.wkb)
    assert np.array_equal(gp, op) and np.array_equal(gq, oq)
    with opts(gpu, pipeline=0):
        rf = M.pip_join(T(x, gpu), T(y, gpu), d, 10)
    assert rf.stats["pipeline"] == 0
    fp, fq = rf.numpy()
    assert np.array_equal(fp, gp) and np.array_equal(fq, gq)
