"""Multi-GPU point-in-polygon join: points sharded, chip table replicated.

The reference scales this path with Spark data parallelism: the chip side is
broadcast to the executors (BroadcastHashJoin) or both sides shuffled, SURVEY §3.D.
On one MI355X node the MI355X-native plan, all of it behind the C ABI
(include/mosaic_gpu.h "Multi-GPU", mosaic_amd/csrc/comm.cpp):
  * points are independent -> contiguous point-id ranges per GPU, no shuffle;
  * every rank's context joins one RCCL communicator (mgpu_comm_init); the unique id
    travels through torch.distributed's control plane (any backend, gloo is enough);
  * the chip table is built once (rank 0) and replicated with mgpu_chips_broadcast:
    one RCCL broadcast of the self-describing blob straight into each receiving
    allocation (its 1 KiB header first, to size it);
  * per-GPU pair counts are combined with mgpu_pair_offsets (one RCCL all-gather) to give
    every rank its global output offset -- the only exchange step on the path.
Concatenating the shards in rank order is then globally ordered by point id.

For a host that ships chip tables itself (a JVM driver broadcasting bytes to its
executors), the same blob exists in host memory: host_blob / blob_info /
upload_host_blob (mgpu_chips_host_blob, mgpu_host_blob_info, mgpu_chips_upload_blob).
"""
import ctypes

import numpy as np

from . import _native as N
from .chips import DeviceChips


def shard_range(n_total, rank, world):
    """Contiguous [begin, end) of global point indices owned by `rank`."""
    base, extra = divmod(int(n_total), int(world))
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


# ---------------------------------------------------------------- RCCL (native)

def init_comm(ctx, group=None):
    """Join ctx to the job's RCCL communicator: rank 0 creates the unique id
    (mgpu_comm_unique_id), torch.distributed carries it to every rank, each rank calls
    mgpu_comm_init (which blocks until all ranks have joined)."""
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    uid = (ctypes.c_uint8 * N.MGPU_COMM_ID_BYTES)()
    if rank == 0:
        N.check(N.lib().mgpu_comm_unique_id(uid))
    obj = [bytes(uid)]
    dist.broadcast_object_list(obj, src=0, group=group)
    buf = (ctypes.c_uint8 * N.MGPU_COMM_ID_BYTES).from_buffer_copy(obj[0])
    N.check(N.lib().mgpu_comm_init(ctx.handle, buf, rank, world))


def comm_info(ctx):
    r, w = ctypes.c_int32(), ctypes.c_int32()
    N.check(N.lib().mgpu_comm_info(ctx.handle, ctypes.byref(r), ctypes.byref(w)))
    return r.value, w.value


def broadcast_chips(chips, ctx, root=0, stream=None):
    """Replicate rank `root`'s uploaded chip table to every rank (mgpu_chips_broadcast:
    one RCCL broadcast into the receiving allocation).  `chips` is a DeviceChips on
    `root` (ignored elsewhere); returns a DeviceChips on every rank."""
    import torch
    rank, _ = comm_info(ctx)
    s = stream if stream is not None else torch.cuda.current_stream(ctx.device).cuda_stream
    out = ctypes.c_void_p()
    src = chips.handle if (rank == root and chips is not None) else None
    N.check(N.lib().mgpu_chips_broadcast(ctx.handle, src, int(root), ctypes.byref(out), s))
    if rank == root:
        return chips
    return DeviceChips(None, ctx, handle=out)


def global_offsets(local_count, ctx, stream=None):
    """mgpu_pair_offsets (RCCL all-gather): (this rank's offset, total, per-rank counts)."""
    import torch
    _, world = comm_info(ctx)
    s = stream if stream is not None else torch.cuda.current_stream(ctx.device).cuda_stream
    off, tot = ctypes.c_int64(), ctypes.c_int64()
    counts = np.zeros(world, dtype=np.int64)
    N.check(N.lib().mgpu_pair_offsets(ctx.handle, int(local_count), ctypes.byref(off), ctypes.byref(tot),
                                      counts.ctypes.data, s))
    return off.value, tot.value, counts


# ---------------------------------------------------------------- host blobs

def host_blob(table):
    """The chip table as one self-describing host blob (bytes), no GPU needed."""
    p = ctypes.c_void_p()
    nb = ctypes.c_int64()
    wkb = table.wkb if table.wkb.size else np.zeros(1, np.uint8)
    N.check(N.lib().mgpu_chips_host_blob(table.index_system, len(table), table.cell.ctypes.data,
                                         table.polygon_id.ctypes.data, table.is_core.ctypes.data,
                                         table.wkb_offsets.ctypes.data, wkb.ctypes.data, ctypes.byref(p),
                                         ctypes.byref(nb)))
    try:
        return host_bytes(p.value, nb.value)
    finally:
        N.lib().mgpu_host_free(p)


def host_bytes(address, size):
    """`size` bytes at a host address as bytes, for any size (not ctypes.string_at: its
    size is a C int -- C3's 4.7 GB blob came back mod 2^32)."""
    if size == 0:
        return b""
    arr = np.ctypeslib.as_array(ctypes.cast(ctypes.c_void_p(address), ctypes.POINTER(ctypes.c_uint8)),
                                shape=(int(size),))
    return arr.tobytes()


def blob_info(blob):
    """Check a received blob (magic, version, size, offsets); its contents."""
    isys, a, b, c = ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    N.check(N.lib().mgpu_host_blob_info(blob, len(blob), ctypes.byref(isys), ctypes.byref(a), ctypes.byref(b),
                                        ctypes.byref(c)))
    return {"index_system": isys.value, "chips": a.value, "cells": b.value, "vertices": c.value}


def upload_host_blob(blob, ctx):
    h = ctypes.c_void_p()
    N.check(N.lib().mgpu_chips_upload_blob(ctx.handle, blob, len(blob), ctypes.byref(h)))
    return DeviceChips(None, ctx, handle=h)


def broadcast_host_blob(blob, src=0, group=None, piece=1 << 30):
    """Control-plane replication of a host blob (torch.distributed, e.g. gloo): what a
    host without RCCL (or a JVM driver) does instead of mgpu_chips_broadcast.  The blob
    travels in pieces of at most `piece` bytes (default 1 GiB: every gloo message stays
    well inside 32-bit sizes)."""
    import torch
    import torch.distributed as dist
    rank = dist.get_rank(group)
    size = torch.tensor([len(blob) if rank == src else 0], dtype=torch.int64)
    dist.broadcast(size, src, group=group)
    n = int(size.item())
    out = np.empty(n, dtype=np.uint8) if rank != src else None
    piece = int(piece)
    for off in range(0, n, piece):
        m = min(piece, n - off)
        if rank == src:
            t = torch.from_numpy(np.frombuffer(blob, dtype=np.uint8, count=m, offset=off).copy())
        else:
            t = torch.from_numpy(out[off:off + m])
        dist.broadcast(t, src, group=group)
    return blob if rank == src else out.tobytes()


def gather_offsets_host(local_count, group=None):
    """The all-gather of mgpu_pair_offsets on the control plane (CPU protocol tests)."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    mine = torch.tensor([int(local_count)], dtype=torch.int64)
    allc = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(allc, mine, group=group)
    counts = np.array([int(c.item()) for c in allc], dtype=np.int64)
    return int(counts[:rank].sum()), int(counts.sum()), counts


def blob_contains(blob, rows, x, y):
    """st_contains of (chip row, point) pairs evaluated on a host blob (test aid)."""
    rows = np.ascontiguousarray(rows, dtype=np.int64)
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    out = np.empty(len(rows), np.int8)
    N.check(N.lib().mgpu_test_blob_contains_host(blob, len(blob), len(rows), rows.ctypes.data, x.ctypes.data,
                                                  y.ctypes.data, out.ctypes.data))
    return out
