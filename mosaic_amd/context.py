"""MosaicContext: index-system selection + the per-GPU native context.

Mirrors MosaicContext.build(indexSystem, geometryAPI)
  src/main/scala/com/databricks/labs/mosaic/functions/MosaicContext.scala:30-45, 1110-1114
and the config keys of package.scala:18-19 (index system, geometry API).  The
geometry API is fixed to JTS semantics (GeometryAPI("JTS"), api/GeometryAPI.scala:125-131):
that is what the chip predicates reproduce.
"""
import contextlib
import ctypes
import threading

from . import _native as N
from .index_system import get_index_system

_ctx_lock = threading.Lock()
_contexts = {}


class GpuContext:
    """Owns one mgpu_ctx (workspace + events) on one GPU."""

    def __init__(self, device=None):
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("mosaic_amd needs an MI355X GPU (no CPU fallback on the hot path)")
        dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        h = ctypes.c_void_p()
        N.check(N.lib().mgpu_ctx_create(dev.index, ctypes.byref(h)))
        self.handle = h

    def reserve(self, max_points):
        N.check(N.lib().mgpu_ctx_reserve(self.handle, int(max_points)))

    def set_option(self, key, value):
        """mgpu_ctx_set_option: the planner and tuning options of this context (keys in
        include/mosaic_gpu.h: h3_libm, pipeline, bin_count, bin_min_mb, bin_min_points,
        bin_xcd, spin_us, raster, raster_bng, raster_sub, raster_milli)."""
        N.check(N.lib().mgpu_ctx_set_option(self.handle, key.encode(), int(value)))

    def get_option(self, key):
        v = ctypes.c_int64()
        N.check(N.lib().mgpu_ctx_get_option(self.handle, key.encode(), ctypes.byref(v)))
        return v.value

    @contextlib.contextmanager
    def options(self, **kw):
        """Set options for the duration of a block, then restore them."""
        old = {k: self.get_option(k) for k in kw}
        try:
            for k, v in kw.items():
                self.set_option(k, v)
            yield self
        finally:
            for k, v in old.items():
                self.set_option(k, v)

    def last_near_ties(self):
        """Sorted input positions of the near-tie points of the last join / cell-id call
        on this context (mgpu_last_near_ties): the parity audit list."""
        import numpy as np
        n = ctypes.c_int64()
        cap = 1 << 12
        while True:
            buf = np.zeros(cap, np.int64)
            st = N.lib().mgpu_last_near_ties(self.handle, buf.ctypes.data, cap, ctypes.byref(n))
            if st == N.MGPU_E_CAPACITY and n.value > cap:
                cap = int(n.value)
                continue
            N.check(st)
            return buf[:n.value]

    def close(self):
        if self.handle:
            N.lib().mgpu_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def default_context(device=None):
    import torch
    if device is None:
        idx = torch.cuda.current_device()
    else:
        d = torch.device(device)
        idx = d.index if d.index is not None else torch.cuda.current_device()
    with _ctx_lock:
        c = _contexts.get(idx)
        if c is None:
            c = GpuContext(torch.device("cuda", idx))
            _contexts[idx] = c
        return c


class MosaicContext:
    """MosaicContext.build(indexSystem, geometryAPI) -> context exposing the SQL
    functions of the hot path (register() names: MosaicContext.scala:400-457)."""

    def __init__(self, index_system="H3", geometry_api="JTS"):
        if str(geometry_api).upper() != "JTS":
            raise N.IllegalArgumentException(N.MGPU_E_INVALID_ARG, "Only the JTS geometry API is supported")
        self.index_system = get_index_system(index_system) if isinstance(index_system, str) else index_system
        self.geometry_api = "JTS"

    @classmethod
    def build(cls, index_system="H3", geometry_api="JTS"):
        return cls(index_system, geometry_api)

    def get_index_system(self):
        return self.index_system

    # the function surface, bound to this context's index system
    def grid_longlatascellid(self, lon, lat, resolution, **kw):
        from . import functions
        return functions.grid_longlatascellid(lon, lat, resolution, index_system=self.index_system, **kw)

    grid_pointascellid = grid_longlatascellid

    def grid_tessellateexplode(self, polygons, resolution, keep_core_geometries=True):
        from . import functions
        return functions.grid_tessellateexplode(polygons, resolution, keep_core_geometries,
                                                index_system=self.index_system)

    def st_contains(self, chips, chip_rows, x, y):
        from . import functions
        return functions.st_contains(chips, chip_rows, x, y)

    def pip_join(self, x, y, chips, resolution, **kw):
        from . import functions
        return functions.pip_join(x, y, chips, resolution, index_system=self.index_system, **kw)
