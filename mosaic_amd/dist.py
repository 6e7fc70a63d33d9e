"""Multi-GPU point-in-polygon join: points sharded, chip table replicated.

The reference scales this path with Spark data parallelism: the chip side is
broadcast (BroadcastHashJoin) or both sides shuffled (SortMergeJoin), SURVEY §3.D.
On one MI355X node the MI355X-native plan is:
  * points are independent -> contiguous point-id ranges per GPU, no shuffle;
  * the chip table is built once (rank 0) and replicated as ONE device blob with
    a single RCCL broadcast over xGMI (the blob is self-describing, see
    mosaic_amd/csrc/capi.cpp BlobHeader);
  * per-GPU pair counts are combined with one RCCL all_gather to give every rank
    its global output offset (the only exchange step on the path).
Concatenating the shards in rank order is then globally ordered by point id.
One process per GPU; the torch.distributed backend "nccl" is RCCL on ROCm.
"""
import numpy as np

from .chips import DeviceChips


def shard_range(n_total, rank, world):
    """Contiguous [begin, end) of global point indices owned by `rank`."""
    base, extra = divmod(int(n_total), int(world))
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def broadcast_chips(chips, ctx, src=0, group=None):
    """Replicate rank `src`'s uploaded chip table to every rank (one broadcast).

    `chips` is a DeviceChips on `src` (ignored elsewhere).  Returns a DeviceChips on
    every rank."""
    import torch
    import torch.distributed as dist
    rank = dist.get_rank(group)
    dev = ctx.device
    backend = dist.get_backend(group)
    size = torch.zeros(1, dtype=torch.int64, device=dev if backend == "nccl" else "cpu")
    if rank == src:
        ptr, nbytes = chips.device_blob()
        size[0] = nbytes
    dist.broadcast(size, src, group=group)
    nbytes = int(size.item())
    buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    if rank == src:
        # the broadcast's source: a tensor copy of the library-owned blob
        torch.cuda.synchronize(dev)
        _copy_device(ptr, buf.data_ptr(), nbytes)
    if backend == "nccl":
        dist.broadcast(buf, src, group=group)
    else:  # gloo: stage through host memory
        host = buf.cpu()
        dist.broadcast(host, src, group=group)
        buf.copy_(host.to(dev))
    if rank == src:
        return chips
    torch.cuda.synchronize(dev)
    return DeviceChips.from_device_blob(ctx, buf.data_ptr(), nbytes)


def _copy_device(src_ptr, dst_ptr, nbytes):
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.restype = ctypes.c_int
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    st = hip.hipMemcpy(ctypes.c_void_p(dst_ptr), ctypes.c_void_p(src_ptr), ctypes.c_size_t(nbytes), 3)
    if st != 0:
        raise RuntimeError("hipMemcpy device->device failed (%d)" % st)


def global_offsets(local_count, device=None, group=None):
    """All-gather the per-rank pair counts; return (this rank's offset, total, counts)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = device if (device is not None and dist.get_backend(group) == "nccl") else "cpu"
    mine = torch.tensor([int(local_count)], dtype=torch.int64, device=dev)
    allc = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(allc, mine, group=group)
    counts = np.array([int(c.item()) for c in allc], dtype=np.int64)
    return int(counts[:rank].sum()), int(counts.sum()), counts
