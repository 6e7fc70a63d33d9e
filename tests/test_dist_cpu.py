"""Multi-process protocol of the sharded join on CPU (gloo, world_size 2).

The GPU path (mosaic_amd/dist.py over the C ABI's mgpu_comm_* / mgpu_chips_broadcast /
mgpu_pair_offsets, RCCL) shards points by contiguous id range, replicates the chip
table as ONE self-describing blob, and all-gathers per-rank pair counts for the output
offsets.  Here the same protocol runs on the control plane: rank 0 builds the chip
table's host blob (mgpu_chips_host_blob), it is broadcast (gloo), rank 1 checks it
(mgpu_host_blob_info) and evaluates st_contains on it (the blob is a complete chip
table), each rank joins its shard (oracle), counts are all-gathered, and the shards
placed at their offsets must equal the single-process join.
"""
import os
import sys

import numpy as np
import torch.multiprocessing as mp

from mosaic_amd.dist import (blob_contains, blob_info, broadcast_host_blob, gather_offsets_host, host_blob,
                             host_bytes, shard_range)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shard_range_partition():
    for n in (0, 1, 7, 100, 1001):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            sizes = [e - b for b, e in spans]
            assert max(sizes) - min(sizes) <= 1


def test_host_blob_roundtrip(nyc_chips_r9):
    import mosaic_amd  # noqa: F401
    b = host_blob(nyc_chips_r9)
    info = blob_info(b)
    assert info["chips"] == len(nyc_chips_r9) and info["index_system"] == 0 and info["cells"] > 1000
    bad = bytearray(b)
    bad[0] ^= 1
    import pytest
    from mosaic_amd import IllegalArgumentException
    with pytest.raises(IllegalArgumentException):
        blob_info(bytes(bad))
    with pytest.raises(IllegalArgumentException):
        blob_info(b[:-256])


def test_host_bytes_beyond_32_bit_sizes():
    """A host buffer larger than 2^32 bytes comes back whole (C3's 4.7 GB blob once came
    back mod 2^32 through ctypes.string_at's C-int size)."""
    n = (1 << 32) + 4099
    buf = np.zeros(n, dtype=np.uint8)  # calloc'd: pages appear as they are touched
    buf[-3:] = (7, 8, 9)
    buf[(1 << 32) - 1] = 5
    b = host_bytes(buf.ctypes.data, n)
    assert len(b) == n and b[-3:] == bytes((7, 8, 9)) and b[(1 << 32) - 1] == 5
    del b
    assert host_bytes(buf.ctypes.data, 0) == b""


def _worker(rank, world, port, x, y, chips, q):
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    import mosaic_amd as M
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cell, poly, core, off, wkb = chips
    blob = None
    if rank == 0:
        t = M.ChipTable(cell, poly, core, off, wkb)
        blob = host_blob(t)
    # small pieces: the chunked path (C3's 4.7 GB blob goes in 1 GiB pieces) end to end
    blob = broadcast_host_blob(blob, 0, piece=65_537)
    info = blob_info(blob)
    # the received blob answers st_contains like the oracle on its own rows
    rng = np.random.default_rng(rank)
    rows = rng.integers(0, len(cell), 400)
    px = x[rng.integers(0, len(x), 400)]
    py = y[rng.integers(0, len(y), 400)]
    got = blob_contains(blob, rows, px, py)
    ref = [O.st_contains(bytes(wkb[off[r]:off[r + 1]]), a, b) if off[r + 1] > off[r] else -1
           for r, a, b in zip(rows, px, py)]
    b, e = shard_range(len(x), rank, world)
    pts, polys = O.pip_join(0, 9, x[b:e], y[b:e], cell, poly, core, off, wkb, threads=2)
    offset, total, counts = gather_offsets_host(len(pts))
    q.put((rank, offset, total, pts + b, polys, info["chips"], bool(np.array_equal(got, np.array(ref, np.int8)))))
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
    res = sorted(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    total = res[0][2]
    out_p = np.full(total, -1, dtype=np.int64)
    out_q = np.full(total, -1, dtype=np.int32)
    for rank, offset, tot, pts, polys, nchips, contains_ok in res:
        assert tot == total and nchips == len(c) and contains_ok
        out_p[offset:offset + len(pts)] = pts
        out_q[offset:offset + len(pts)] = polys
    op, oq = O.pip_join(0, 9, x, y, *chips)
    assert np.array_equal(out_p, op) and np.array_equal(out_q, oq)
