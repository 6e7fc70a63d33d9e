"""The columnar entry: Arrow C Device Data Interface arrays into the join (include/mosaic_arrow.h).

A Spark host with columnar batches (the reference evaluates row by row, CodegenFallback:
expressions/index/PointIndexGeom.scala:10-13) hands device columns over as
ArrowDeviceArray structs; this module builds those structs over torch device tensors so the
tests and the bench drive the same ABI a JVM / Arrow-native caller would.
"""
import ctypes

import numpy as np

from . import _native as N

ARROW_DEVICE_ROCM = 10
_release = ctypes.CFUNCTYPE(None, ctypes.c_void_p)


class ArrowSchema(ctypes.Structure):
    pass


ArrowSchema._fields_ = [("format", ctypes.c_char_p), ("name", ctypes.c_char_p), ("metadata", ctypes.c_char_p),
                        ("flags", ctypes.c_int64), ("n_children", ctypes.c_int64),
                        ("children", ctypes.c_void_p), ("dictionary", ctypes.c_void_p),
                        ("release", _release), ("private_data", ctypes.c_void_p)]


class ArrowArray(ctypes.Structure):
    _fields_ = [("length", ctypes.c_int64), ("null_count", ctypes.c_int64), ("offset", ctypes.c_int64),
                ("n_buffers", ctypes.c_int64), ("n_children", ctypes.c_int64),
                ("buffers", ctypes.POINTER(ctypes.c_void_p)), ("children", ctypes.c_void_p),
                ("dictionary", ctypes.c_void_p), ("release", _release), ("private_data", ctypes.c_void_p)]


class ArrowDeviceArray(ctypes.Structure):
    _fields_ = [("array", ArrowArray), ("device_id", ctypes.c_int64), ("device_type", ctypes.c_int32),
                ("sync_event", ctypes.c_void_p), ("reserved", ctypes.c_int64 * 3)]


class DeviceColumn:
    """An ArrowDeviceArray over device tensors (kept alive with it).  ``buffers``: the
    Arrow buffers in order (validity first, None = no bitmap)."""

    def __init__(self, length, buffers, offset=0, null_count=0, device_index=0):
        self._keep = [b for b in buffers if b is not None]
        self._ptrs = (ctypes.c_void_p * len(buffers))(*[None if b is None else b.data_ptr() for b in buffers])
        self.struct = ArrowDeviceArray()
        a = self.struct.array
        a.length, a.null_count, a.offset = int(length), int(null_count), int(offset)
        a.n_buffers, a.n_children = len(buffers), 0
        a.buffers = ctypes.cast(self._ptrs, ctypes.POINTER(ctypes.c_void_p))
        a.release = _release(0)
        self.struct.device_id = device_index
        self.struct.device_type = ARROW_DEVICE_ROCM

    @property
    def ref(self):
        return ctypes.byref(self.struct)


def bitmap(present, device):
    """numpy bool array -> Arrow validity bitmap (LSB first) on the device."""
    import torch
    return torch.from_numpy(np.packbits(np.asarray(present, bool), bitorder="little").copy()).to(device)


def float64_column(values, present=None, offset=0):
    """float64 device tensor (+ optional bool validity of the same length) -> column of
    length values.numel() - offset starting at ``offset``."""
    n = values.numel() - offset
    vb = None if present is None else bitmap(present, values.device)
    nulls = 0 if present is None else int((~np.asarray(present, bool)[offset:]).sum())
    return DeviceColumn(n, [vb, values], offset=offset, null_count=nulls, device_index=values.device.index or 0)


def pip_join_arrow(x_col, y_col, chips, resolution, index_system=None, point_id_col=None, capacity=None,
                   stream=None):
    """mgpu_pip_join_arrow: the join over Arrow columns.  Returns a JoinResult."""
    import torch
    from .functions import JoinResult, _H3
    isys = index_system or _H3
    res = isys.get_resolution(resolution)
    dev = chips.ctx.device
    n = x_col.struct.array.length
    cap = int(capacity if capacity is not None else max(16, n + n // 8))
    op = torch.empty(cap, dtype=torch.int64, device=dev)
    oq = torch.empty(cap, dtype=torch.int32, device=dev)
    cnt = ctypes.c_int64()
    st = N.MgpuStats()
    s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
    N.check(N.lib().mgpu_pip_join_arrow(chips.ctx.handle, chips.handle, isys.code, res, x_col.ref, y_col.ref,
                                        None if point_id_col is None else point_id_col.ref, cap, ctypes.byref(cnt),
                                        op.data_ptr(), oq.data_ptr(), s, st), required=cnt.value)
    m = int(cnt.value)
    return JoinResult(op[:m], oq[:m], st.as_dict())


def geometry_column(col, large=True):
    """functions.GeometryColumn -> Arrow binary / utf8 column (+ its schema format)."""
    import torch
    fmt = {(N.MGPU_GEOM_WKB, True): b"Z", (N.MGPU_GEOM_WKB, False): b"z",
           (N.MGPU_GEOM_WKT, True): b"U", (N.MGPU_GEOM_WKT, False): b"u"}[(col.format, large)]
    off = col.offsets if large else col.offsets.to(torch.int32)
    n = len(col)
    nulls = 0
    if col.valid is not None:
        bits = np.unpackbits(col.valid.cpu().numpy(), bitorder="little")[:n]
        nulls = int(n - bits.sum())
    arr = DeviceColumn(n, [col.valid, off, col.data], null_count=nulls, device_index=col.data.device.index or 0)
    schema = ArrowSchema()
    schema.format = fmt
    schema.release = _release(0)
    arr._keep.append(schema)
    return arr, schema


def grid_pointascellid_arrow(col, resolution, index_system=None, large=True, ctx=None, stream=None):
    """mgpu_geometry_to_cells_arrow over a GeometryColumn handed over as an Arrow array.
    Returns (cells int64, validity bitmap uint8)."""
    import torch
    from .context import default_context
    from .functions import _H3
    isys = index_system or _H3
    res = isys.get_resolution(resolution)
    dev = col.data.device
    ctx = ctx or default_context(dev)
    arr, schema = geometry_column(col, large)
    n = len(col)
    cells = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    valid = torch.empty((n + 7) // 8 + 1, dtype=torch.uint8, device=dev)
    s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
    N.check(N.lib().mgpu_geometry_to_cells_arrow(ctx.handle, isys.code, res, arr.ref, ctypes.byref(schema),
                                                 cells.data_ptr(), valid.data_ptr(), s))
    return cells[:n], valid[:(n + 7) // 8]
