"""The IndexSystem plugin boundary, MI355X-backed.

Mirrors the reference's abstract class
  src/main/scala/com/databricks/labs/mosaic/core/index/IndexSystem.scala:15-318
and its two grid implementations used on the point-in-polygon path,
  H3IndexSystem  (H3IndexSystem.scala:24-412)  and
  BNGIndexSystem (BNGIndexSystem.scala:30-555),
selected by name like IndexSystemFactory.getIndexSystem
(IndexSystemFactory.scala:15-63).  Same method names (snake_case), same argument
meaning, same exception classes.  The per-row methods of the reference become
batch methods over device tensors; the scalar forms are kept for API parity and
run as a batch of one.
"""
import numpy as np

from . import _native as N
from ._native import IllegalArgumentException, IllegalStateException


class IndexSystem:
    """Abstract index system (IndexSystem.scala:15)."""

    code = None
    name = None
    crs_id = None
    cell_id_type = "long"  # IndexSystem(cellIdType); LongType for H3, StringType for BNG

    def __init__(self):
        self._cell_id_type = self.cell_id_type

    # -- resolution -------------------------------------------------------
    @property
    def resolutions(self):
        raise NotImplementedError

    def get_resolution(self, res):
        raise NotImplementedError

    # -- cell ids ---------------------------------------------------------
    def get_cell_id_data_type(self):
        return self._cell_id_type

    def set_cell_id_data_type(self, dt):
        """IndexSystem.setCellIdDataType (IndexSystem.scala:43-45); "long" or "string"."""
        if dt not in ("long", "string"):
            raise IllegalArgumentException(N.MGPU_E_INVALID_ARG, "Cell ID data type not supported.")
        self._cell_id_type = dt

    def format(self, cell_id):
        raise NotImplementedError

    def parse(self, cell_id):
        raise NotImplementedError

    def format_cell_id(self, cell_id, dt=None):
        """IndexSystem.formatCellId (IndexSystem.scala:48-57)."""
        dt = dt or self._cell_id_type
        if dt == "long":
            return self.parse(cell_id) if isinstance(cell_id, str) else int(cell_id)
        if dt == "string":
            return cell_id if isinstance(cell_id, str) else self.format(int(cell_id))
        raise IllegalArgumentException(N.MGPU_E_INVALID_ARG, "Cell ID data type not supported.")

    serialize_cell_id = format_cell_id  # IndexSystem.serializeCellId (IndexSystem.scala:61-70)

    # -- point -> cell ----------------------------------------------------
    def points_to_index(self, x, y, resolution, out=None, ctx=None, stream=None, stats=False):
        """Batch IndexSystem.pointToIndex over device tensors (float64 SoA).

        Returns an int64 device tensor of cell ids (and the stats dict if asked)."""
        import torch
        from .context import default_context
        res = self.get_resolution(resolution)
        ctx = ctx or default_context(x.device)
        _check_points(x, y)
        n = x.numel()
        if out is None:
            out = torch.empty(n, dtype=torch.int64, device=x.device)
        st = N.MgpuStats()
        s = stream if stream is not None else torch.cuda.current_stream(x.device).cuda_stream
        N.check(N.lib().mgpu_points_to_cells(ctx.handle, self.code, res, x.data_ptr(), y.data_ptr(), n,
                                             out.data_ptr(), s, st))
        return (out, st.as_dict()) if stats else out

    def point_to_index(self, lon, lat, resolution):
        """Scalar IndexSystem.pointToIndex(lon, lat, res) (IndexSystem.scala:237)."""
        import torch
        from .context import default_context
        ctx = default_context()
        dev = ctx.device
        x = torch.tensor([float(lon)], dtype=torch.float64, device=dev)
        y = torch.tensor([float(lat)], dtype=torch.float64, device=dev)
        return int(self.points_to_index(x, y, resolution, ctx=ctx)[0].item())

    def format_device(self, cells, ctx=None, stream=None):
        """StringType cell ids of a device int64 column (IndexSystem.serializeCellId,
        IndexSystem.scala:61-70; mgpu_format_cells_device, HIP): BNG format / H3 hex.
        Returns (chars: uint8 tensor of the concatenated ids, offsets: int64 tensor of n + 1)."""
        import ctypes
        import torch
        from .context import default_context
        if cells.dtype != torch.int64 or not cells.is_cuda:
            raise IllegalArgumentException(N.MGPU_E_INVALID_ARG, "cells must be an int64 device tensor")
        cells = cells.contiguous()
        ctx = ctx or default_context(cells.device)
        n = cells.numel()
        off = torch.empty(n + 1, dtype=torch.int64, device=cells.device)
        cap = max(16 * n, 1)  # an id is at most 16 chars
        out = torch.empty(cap, dtype=torch.uint8, device=cells.device)
        tot = ctypes.c_int64()
        s = stream if stream is not None else torch.cuda.current_stream(cells.device).cuda_stream
        st = N.lib().mgpu_format_cells_device(ctx.handle, self.code, cells.data_ptr(), n, out.data_ptr(), cap,
                                              off.data_ptr(), ctypes.byref(tot), s)
        N.check(st, "cell id has no string form")
        return out[:tot.value], off

    def k_ring(self, index, n):
        """IndexSystem.kRing(index, n) (H3IndexSystem.scala:182-184, BNGIndexSystem.scala:
        221-226): the list of ids, in the reference's order, on the device."""
        import torch
        from .context import default_context
        from .functions import grid_cellkring
        ctx = default_context()
        ids, _ = grid_cellkring(torch.tensor([int(index)], dtype=torch.int64, device=ctx.device), n, self, ctx=ctx)
        return [int(v) for v in ids.cpu().tolist()]

    def k_loop(self, index, n):
        """IndexSystem.kLoop(index, n) (H3IndexSystem.scala:194-205, BNGIndexSystem.scala:
        239-252) on the device."""
        import torch
        from .context import default_context
        from .functions import grid_cellkring
        ctx = default_context()
        ids, _ = grid_cellkring(torch.tensor([int(index)], dtype=torch.int64, device=ctx.device), n, self,
                                loop_only=True, ctx=ctx)
        return [int(v) for v in ids.cpu().tolist()]


def _check_points(x, y):
    if x.dtype != y.dtype or str(x.dtype) != "torch.float64":
        raise IllegalArgumentException(N.MGPU_E_INVALID_ARG, "coordinates must be float64 tensors")
    if x.shape != y.shape or x.dim() != 1 or not x.is_contiguous() or not y.is_contiguous():
        raise IllegalArgumentException(N.MGPU_E_INVALID_ARG, "coordinates must be 1-D contiguous tensors")
    if x.device.type != "cuda" or y.device != x.device:
        raise IllegalArgumentException(N.MGPU_E_INVALID_ARG, "coordinates must live on the context's GPU")


class H3IndexSystem(IndexSystem):
    """H3IndexSystem (H3IndexSystem.scala:24): H3 v3.7, resolutions 0..15, LongType ids."""

    code = N.MGPU_H3
    name = "H3"
    crs_id = 4326
    cell_id_type = "long"

    @property
    def resolutions(self):
        return set(range(16))

    def get_resolution(self, res):
        """H3IndexSystem.getResolution (H3IndexSystem.scala:45-60)."""
        if isinstance(res, bool):
            raise IllegalArgumentException(N.MGPU_E_INVALID_ARG, "Resolution must be an Int or String.")
        if isinstance(res, (int, np.integer)):
            r = int(res)
        elif isinstance(res, str):
            try:
                r = int(res)
            except ValueError:
                raise IllegalArgumentException(N.MGPU_E_INVALID_ARG, "Resolution must be an Int or String.")
        else:
            raise IllegalArgumentException(N.MGPU_E_INVALID_ARG, "Resolution must be an Int or String.")
        if r < 0 or r > 15:
            raise IllegalStateException(N.MGPU_E_RESOLUTION, "H3 resolution has to be between 0 and 15; found %d" % r)
        return r

    def format(self, cell_id):
        """H3 string form (the 15-hex-digit address)."""
        return "%x" % int(cell_id)

    def parse(self, cell_id):
        return int(cell_id, 16)

    def get_resolution_str(self, resolution):
        return str(resolution)


class BNGIndexSystem(IndexSystem):
    """BNGIndexSystem (BNGIndexSystem.scala:30): British National Grid, EPSG:27700, StringType ids."""

    code = N.MGPU_BNG
    name = "BNG"
    crs_id = 27700
    cell_id_type = "string"
    # BNGIndexSystem.resolutionMap (BNGIndexSystem.scala:46-60)
    resolution_map = {"500km": -1, "100km": 1, "50km": -2, "10km": 2, "5km": -3, "1km": 3, "500m": -4,
                      "100m": 4, "50m": -5, "10m": 5, "5m": -6, "1m": 6}

    @property
    def resolutions(self):
        return {1, -1, 2, -2, 3, -3, 4, -4, 5, -5, 6, -6}

    def get_resolution(self, res):
        """BNGIndexSystem.getResolution (BNGIndexSystem.scala:349-360)."""
        if isinstance(res, (int, np.integer)) and not isinstance(res, bool) and int(res) in self.resolutions:
            return int(res)
        if isinstance(res, str) and res in self.resolution_map:
            return self.resolution_map[res]
        raise IllegalStateException(N.MGPU_E_RESOLUTION, "BNG resolution not supported; found %s" % (res,))

    def get_resolution_str(self, resolution):
        for k, v in self.resolution_map.items():
            if v == resolution:
                return k
        return ""

    def format_many(self, cells):
        """BNGIndexSystem.format over an int64 array (host)."""
        c = np.ascontiguousarray(np.asarray(cells, dtype=np.int64))
        n = c.shape[0]
        buf = np.zeros(max(24 * n, 1), dtype=np.uint8)
        off = np.zeros(n + 1, dtype=np.int64)
        st = N.lib().mgpu_bng_format(c.ctypes.data, n, buf.ctypes.data, buf.shape[0], off.ctypes.data)
        N.check(st, "BNG cell id has no string form")
        raw = buf.tobytes()
        return [raw[off[i]:off[i + 1]].decode() for i in range(n)]

    def parse_many(self, ids):
        enc = [s.encode() for s in ids]
        off = np.zeros(len(enc) + 1, dtype=np.int64)
        off[1:] = np.cumsum([len(e) for e in enc])
        buf = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8).copy()
        out = np.zeros(len(enc), dtype=np.int64)
        N.check(N.lib().mgpu_bng_parse(buf.ctypes.data, off.ctypes.data, len(enc), out.ctypes.data),
                "not a BNG cell id")
        return out

    def format(self, cell_id):
        return self.format_many([cell_id])[0]

    def parse(self, cell_id):
        return int(self.parse_many([cell_id])[0])


def get_index_system(name):
    """IndexSystemFactory.getIndexSystem(name) (IndexSystemFactory.scala:31-63)."""
    n = str(name).upper()
    if n == "H3":
        return H3IndexSystem()
    if n == "BNG":
        return BNGIndexSystem()
    raise IllegalArgumentException(N.MGPU_E_INVALID_ARG,
                                   "Index system %s not supported by the MI355X path (H3, BNG)" % name)
