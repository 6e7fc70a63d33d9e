"""Multi-process protocol of the sharded join on CPU (gloo, world_size 2).

The GPU path shards points by contiguous id range, replicates the chip table, and
all-gathers per-rank pair counts for the output offsets (mosaic_amd/dist.py).  Here
each rank runs the oracle on its shard; the concatenation in rank order, placed at
the all-gathered offsets, must equal the single-process join.
"""
import os
import sys

import numpy as np
import torch.multiprocessing as mp

from mosaic_amd.dist import global_offsets, shard_range

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shard_range_partition():
    for n in (0, 1, 7, 100, 1001):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            sizes = [e - b for b, e in spans]
            assert max(sizes) - min(sizes) <= 1


def _worker(rank, world, port, x, y, chips, q):
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b, e = shard_range(len(x), rank, world)
    cell, poly, core, off, wkb = chips
    pts, polys = O.pip_join(0, 9, x[b:e], y[b:e], cell, poly, core, off, wkb, threads=2)
    offset, total, counts = global_offsets(len(pts))
    q.put((rank, offset, total, pts + b, polys))
    dist.destroy_process_group()


def test_sharded_join_matches_single_process(nyc_chips_r9):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from geom_util import nyc_points
    x, y = nyc_points(60000, 17)
    c = nyc_chips_r9
    chips = (c.cell, c.polygon_id, c.is_core, c.wkb_offsets, c.wkb)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, world, port, x, y, chips, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    total = res[0][2]
    out_p = np.full(total, -1, dtype=np.int64)
    out_q = np.full(total, -1, dtype=np.int32)
    for rank, offset, tot, pts, polys in res:
        assert tot == total
        out_p[offset:offset + len(pts)] = pts
        out_q[offset:offset + len(pts)] = polys
    op, oq = O.pip_join(0, 9, x, y, *chips)
    assert np.array_equal(out_p, op) and np.array_equal(out_q, oq)
