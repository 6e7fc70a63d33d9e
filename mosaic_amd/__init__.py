"""mosaic_amd -- MI355X-native grid-indexed point-in-polygon join.

A drop-in for the hot path of Databricks Labs Mosaic 0.4.3 (tiems90/mosaic):
grid_pointascellid / grid_longlatascellid, grid_tessellateexplode chips with
is_core, st_contains on chip WKB, and their join -- behind the IndexSystem
plugin boundary (H3IndexSystem, BNGIndexSystem).  Compute runs in hand-written
gfx950 HIP kernels (mosaic_amd/csrc, C ABI in include/mosaic_gpu.h); there is
no CPU fallback on the data path.
"""
from ._native import (CapacityError, IllegalArgumentException, IllegalStateException, MosaicGpuError,
                      EXPORTS, LIB_PATH)
from .chips import ChipTable, DeviceChips, Polygons, tessellate
from .context import GpuContext, MosaicContext, default_context
from .functions import (AsyncJoin, GeometryColumn, InternalGeometryColumn, JoinResult, grid_cellkloop, grid_cellkring, grid_longlatascellid, grid_pointascellid,
                        grid_ring_join, grid_ring_join_final, grid_tessellateexplode, pip_join, pip_join_async, st_contains)
from .index_system import BNGIndexSystem, H3IndexSystem, IndexSystem, get_index_system

__version__ = "0.1.0"

__all__ = [
    "AsyncJoin", "BNGIndexSystem", "CapacityError", "ChipTable", "DeviceChips", "EXPORTS", "GeometryColumn", "GpuContext", "InternalGeometryColumn", "H3IndexSystem",
    "IllegalArgumentException", "IllegalStateException", "IndexSystem", "JoinResult", "LIB_PATH",
    "MosaicContext", "MosaicGpuError", "Polygons", "default_context", "get_index_system", "grid_cellkloop",
    "grid_cellkring", "grid_longlatascellid",
    "grid_pointascellid", "grid_ring_join", "grid_ring_join_final", "grid_tessellateexplode", "pip_join", "pip_join_async", "st_contains", "tessellate",
]
