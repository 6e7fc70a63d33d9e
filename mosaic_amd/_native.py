"""ctypes binding of ``mosaic_amd/libmosaic_gpu.so`` (the C ABI in include/mosaic_gpu.h).

There is no fallback: if the library is missing, or a compute entry point is
called without a GPU, the call raises.  Device memory is passed as raw pointers
(``torch.Tensor.data_ptr()``); torch is only the allocator / stream provider.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MOSAIC_AMD_LIB: profiling builds of the same sources (tools/variants.sh); default in-tree
LIB_PATH = os.environ.get("MOSAIC_AMD_LIB") or os.path.join(_HERE, "libmosaic_gpu.so")

MGPU_OK = 0
MGPU_E_INVALID_ARG = -1
MGPU_E_RESOLUTION = -2
MGPU_E_NAN = -3
MGPU_E_WKB = -4
MGPU_E_CAPACITY = -5
MGPU_RING_LEFT_OUTER = 1
MGPU_E_DEVICE = -6
MGPU_E_INTERNAL = -7
MGPU_E_UNSUPPORTED = -8
MGPU_E_EMPTY = -9

MGPU_H3 = 0
MGPU_BNG = 1

# every symbol include/mosaic_gpu.h declares
EXPORTS = (
    "mgpu_last_error", "mgpu_version", "mgpu_join_tile_points", "mgpu_ctx_create", "mgpu_ctx_destroy", "mgpu_check_resolution",
    "mgpu_points_to_cells", "mgpu_points_to_cells_host", "mgpu_bng_format", "mgpu_bng_parse",
    "mgpu_bng_format_device", "mgpu_format_cells_device", "mgpu_grid_kring",
    "mgpu_chips_upload", "mgpu_chips_destroy", "mgpu_chips_device_blob", "mgpu_chips_from_device_blob",
    "mgpu_chips_info", "mgpu_st_contains", "mgpu_pip_join", "mgpu_pip_join_async", "mgpu_pip_join_finish", "mgpu_ctx_reserve",
    "mgpu_last_near_ties",    "mgpu_pip_join_host", "mgpu_tessellate", "mgpu_tess_result_sizes", "mgpu_tess_result_copy", "mgpu_tessellate_ex", "mgpu_tessellate_geom", "mgpu_tess_result_undecided", "mgpu_tess_result_stats", "mgpu_tess_result_core_stats",
    "mgpu_tess_destroy", "mgpu_test_chip_contains_host", "mgpu_test_raster_host", "mgpu_test_cell_answers_host", "mgpu_test_whole_cells_host", "mgpu_pip_join_fetch",
    "mgpu_chips_host_blob", "mgpu_host_free", "mgpu_host_blob_info", "mgpu_chips_upload_blob",
    "mgpu_comm_unique_id", "mgpu_comm_init", "mgpu_comm_info", "mgpu_comm_destroy", "mgpu_chips_broadcast",
    "mgpu_pair_offsets", "mgpu_test_blob_contains_host", "mgpu_points_from_geometry", "mgpu_geometry_to_cells",
    "mgpu_geometry_to_cells_arrow", "mgpu_pip_join_arrow", "mgpu_test_parse_number", "mgpu_test_decode_point",
    "mgpu_test_h3_elementary_host", "mgpu_test_h3_route_host", "mgpu_test_h3_boundary_host", "mgpu_test_h3_cell_wkb_host",
    "mgpu_ctx_set_option", "mgpu_ctx_get_option", "mgpu_build_opts_default", "mgpu_chips_host_blob_ex",
    "mgpu_test_h3_glibc_host", "mgpu_internal_geometry_to_cells", "mgpu_test_internal_centroid", "mgpu_test_join_counters",
    "mgpu_test_receive_blob", "mgpu_ring_join", "mgpu_ring_join_ex", "mgpu_ring_join_final",
    "mgpu_test_overlay_verify",
)
MGPU_GEOM_WKB = 0
MGPU_GEOM_WKT = 1
MGPU_GEOM_HEX = 2
MGPU_GEOM_GEOJSON = 3
MGPU_COMM_ID_BYTES = 128
MGPU_PIPELINE_AUTO = -1
MGPU_PIPELINE_FUSED = 0
MGPU_PIPELINE_SPLIT = 1
MGPU_PIPELINE_BINNED = 2
MGPU_LIBM_REFERENCE = 0
MGPU_LIBM_CORRECTLY_ROUNDED = 1


class MosaicGpuError(RuntimeError):
    """A non-zero status from the C ABI; ``code`` is the MGPU_E_* class."""

    def __init__(self, code, msg):
        super().__init__("%s (status %d)" % (msg, code))
        self.code = code


class IllegalArgumentException(MosaicGpuError, ValueError):
    pass


class IllegalStateException(MosaicGpuError):
    pass


class CapacityError(MosaicGpuError):
    def __init__(self, code, msg, required):
        super().__init__(code, msg)
        self.required = required


class MgpuStats(ctypes.Structure):
    _fields_ = [("n_points", ctypes.c_int64), ("n_pairs", ctypes.c_int64), ("n_near_ties", ctypes.c_int64),
                ("n_candidates", ctypes.c_int64), ("kernel_ms", ctypes.c_float),
                ("stream_kernel_ms", ctypes.c_float), ("mixed_kernel_ms", ctypes.c_float),
                ("emit_kernel_ms", ctypes.c_float), ("pipeline", ctypes.c_int32), ("libm_overrides", ctypes.c_int32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class BuildOpts(ctypes.Structure):
    """mgpu_build_opts: the chip-table builder's pixel-index options."""
    _fields_ = [("raster", ctypes.c_int32), ("raster_bng", ctypes.c_int32), ("raster_sub", ctypes.c_int32),
                ("raster_milli", ctypes.c_int32)]


_lib = None

P = ctypes.c_void_p
I32 = ctypes.c_int32
I64 = ctypes.c_int64


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("mosaic_amd/libmosaic_gpu.so is not built: run `python -c 'import __graft_entry__ as g; "
                           "g.build()'` (the HIP path has no CPU fallback)")
    L = ctypes.CDLL(LIB_PATH)
    sig = {
        "mgpu_last_error": (ctypes.c_char_p, []),
        "mgpu_version": (ctypes.c_char_p, []),
        "mgpu_join_tile_points": (ctypes.c_int32, []),
        "mgpu_ctx_create": (I32, [I32, ctypes.POINTER(P)]),
        "mgpu_ctx_destroy": (I32, [P]),
        "mgpu_check_resolution": (I32, [I32, I32]),
        "mgpu_points_to_cells": (I32, [P, I32, I32, P, P, I64, P, P, ctypes.POINTER(MgpuStats)]),
        "mgpu_points_to_cells_host": (I32, [P, I32, I32, P, P, I64, P]),
        "mgpu_bng_format": (I32, [P, I64, P, I64, P]),
        "mgpu_bng_format_device": (I32, [P, P, I64, P, I64, P, ctypes.POINTER(I64), P]),
        "mgpu_format_cells_device": (I32, [P, I32, P, I64, P, I64, P, ctypes.POINTER(I64), P]),
        "mgpu_grid_kring": (I32, [P, I32, P, I64, I32, I32, P, I64, P, ctypes.POINTER(I64), P]),
        "mgpu_bng_parse": (I32, [P, P, I64, P]),
        "mgpu_chips_upload": (I32, [P, I32, I64, P, P, P, P, P, ctypes.POINTER(P)]),
        "mgpu_chips_destroy": (I32, [P]),
        "mgpu_chips_device_blob": (I32, [P, ctypes.POINTER(P), ctypes.POINTER(I64)]),
        "mgpu_chips_from_device_blob": (I32, [P, P, I64, ctypes.POINTER(P)]),
        "mgpu_chips_info": (I32, [P, ctypes.POINTER(I64), ctypes.POINTER(I64), ctypes.POINTER(I64)]),
        "mgpu_st_contains": (I32, [P, P, P, P, P, I64, P, P]),
        "mgpu_pip_join": (I32, [P, P, I32, I32, P, P, P, I64, I64, I64, ctypes.POINTER(I64), P, P, P,
                                ctypes.POINTER(MgpuStats)]),
        "mgpu_pip_join_async": (I32, [P, P, I32, I32, P, P, P, I64, I64, I64, P, P, P, P]),
        "mgpu_pip_join_finish": (I32, [P, ctypes.POINTER(I64), ctypes.POINTER(MgpuStats)]),
        "mgpu_ctx_reserve": (I32, [P, I64]),
        "mgpu_last_near_ties": (I32, [P, P, I64, ctypes.POINTER(I64)]),
        "mgpu_pip_join_host": (I32, [P, P, I32, I32, P, P, P, I64, I64, ctypes.POINTER(I64), P, P]),
        "mgpu_tessellate": (I32, [I32, I32, I64, P, P, P, P, P, I32, ctypes.POINTER(P)]),
        "mgpu_tessellate_ex": (I32, [I32, I32, I64, P, P, P, P, P, I32, I32, ctypes.POINTER(P)]),
        "mgpu_tessellate_geom": (I32, [I32, I32, I64, P, P, P, P, P, P, I32, I32, I32, ctypes.POINTER(P)]),
        "mgpu_tess_result_undecided": (I32, [P, P, P, P, P, P, P, P]),
        "mgpu_tess_result_stats": (I32, [P, P]),
        "mgpu_tess_result_core_stats": (I32, [P, P, I32]),
        "mgpu_tess_result_sizes": (I32, [P, ctypes.POINTER(I64), ctypes.POINTER(I64)]),
        "mgpu_tess_result_copy": (I32, [P, P, P, P, P, P]),
        "mgpu_tess_destroy": (I32, [P]),
        "mgpu_test_chip_contains_host": (I32, [I32, I64, P, P, P, P, P, I64, P, P, P, P, P]),
        "mgpu_pip_join_fetch": (I32, [P, I64, ctypes.POINTER(I64), P, P, P]),
        "mgpu_test_raster_host": (I32, [I32, I32, I64, P, P, P, P, P, I64, P, P, P, P, P, P]),
        "mgpu_test_cell_answers_host": (I32, [I32, I32, I64, P, P, P, P, P, I64, P, P, P, P, P, P]),
        "mgpu_test_whole_cells_host": (I32, [I32, I32, I64, P, P, P, P, P, I64, P, P, P, P, P, P]),
        "mgpu_chips_host_blob": (I32, [I32, I64, P, P, P, P, P, ctypes.POINTER(P), ctypes.POINTER(I64)]),
        "mgpu_host_free": (I32, [P]),
        "mgpu_host_blob_info": (I32, [P, I64, ctypes.POINTER(I32), ctypes.POINTER(I64), ctypes.POINTER(I64),
                                      ctypes.POINTER(I64)]),
        "mgpu_chips_upload_blob": (I32, [P, P, I64, ctypes.POINTER(P)]),
        "mgpu_comm_unique_id": (I32, [P]),
        "mgpu_comm_init": (I32, [P, P, I32, I32]),
        "mgpu_comm_info": (I32, [P, ctypes.POINTER(I32), ctypes.POINTER(I32)]),
        "mgpu_comm_destroy": (I32, [P]),
        "mgpu_chips_broadcast": (I32, [P, P, I32, ctypes.POINTER(P), P]),
        "mgpu_pair_offsets": (I32, [P, I64, ctypes.POINTER(I64), ctypes.POINTER(I64), P, P]),
        "mgpu_test_blob_contains_host": (I32, [P, I64, I64, P, P, P, P]),
        "mgpu_points_from_geometry": (I32, [P, I32, P, P, P, I64, I64, P, P, P]),
        "mgpu_geometry_to_cells": (I32, [P, I32, I32, I32, P, P, P, I64, I64, P, P, P, ctypes.POINTER(MgpuStats)]),
        "mgpu_geometry_to_cells_arrow": (I32, [P, I32, I32, P, P, P, P, P]),
        "mgpu_pip_join_arrow": (I32, [P, P, I32, I32, P, P, P, I64, ctypes.POINTER(I64), P, P, P,
                                      ctypes.POINTER(MgpuStats)]),
        "mgpu_test_parse_number": (I32, [ctypes.c_char_p, I32, ctypes.POINTER(ctypes.c_double)]),
        "mgpu_test_decode_point": (I32, [I32, P, I64, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
        "mgpu_test_h3_elementary_host": (I32, [I32, P, P, I64, P]),
        "mgpu_test_h3_route_host": (I32, [P, P, I64, I32, P]),
        "mgpu_test_h3_boundary_host": (I32, [P, I64, P, P, P]),
        "mgpu_test_overlay_verify": (I32, [ctypes.c_int32, P]),
        "mgpu_test_h3_cell_wkb_host": (I32, [I64, P, I64, P]),
        "mgpu_ctx_set_option": (I32, [P, ctypes.c_char_p, I64]),
        "mgpu_ctx_get_option": (I32, [P, ctypes.c_char_p, ctypes.POINTER(I64)]),
        "mgpu_build_opts_default": (None, [ctypes.POINTER(BuildOpts)]),
        "mgpu_chips_host_blob_ex": (I32, [I32, I64, P, P, P, P, P, ctypes.POINTER(BuildOpts), ctypes.POINTER(P),
                                          ctypes.POINTER(I64)]),
        "mgpu_test_h3_glibc_host": (I32, [P, P, I64, I32, P]),
        "mgpu_internal_geometry_to_cells": (I32, [P, I32, I32, I64, P, P, P, P, P, P, I64, P, P, P,
                                                  ctypes.POINTER(MgpuStats)]),
        "mgpu_test_internal_centroid": (I32, [I64, P, P, P, P, P, P, P, P]),
        "mgpu_test_join_counters": (I32, [P, P]),
        "mgpu_test_receive_blob": (I32, [P, P, I32, ctypes.POINTER(P)]),
        "mgpu_ring_join": (I32, [P, I32, I32, I32, I32, P, P, I64, P, P, I64, I64, I32, ctypes.c_double, I64,
                                 ctypes.POINTER(I64), P, P, P, P]),
        "mgpu_ring_join_ex": (I32, [P, I32, I32, I32, I32, P, P, I64, P, P, I64, I64, I32, ctypes.c_double, I32,
                                    I64, ctypes.POINTER(I64), P, P, P, P]),
        "mgpu_ring_join_final": (I32, [P, I32, I32, P, P, P, P, I64, P, P, I64, I64, I32, ctypes.c_double, I32, I64,
                                       ctypes.POINTER(I64), P, P, P, P]),
    }
    for name, (rt, args) in sig.items():
        f = getattr(L, name)
        f.restype = rt
        f.argtypes = args
    _lib = L
    return L


def last_error():
    m = lib().mgpu_last_error()
    return m.decode() if m else ""


def check(status, what="", required=None):
    """Map a status code to the reference's exception classes (IndexSystem.scala:54-58,
    BNGIndexSystem.scala:285, H3Core.geoToH3's IllegalArgumentException)."""
    if status == MGPU_OK:
        return
    msg = last_error() or what
    if status == MGPU_E_CAPACITY:
        raise CapacityError(status, msg, required)
    if status in (MGPU_E_RESOLUTION, MGPU_E_NAN, MGPU_E_INTERNAL, MGPU_E_EMPTY):
        raise IllegalStateException(status, msg)
    if status in (MGPU_E_INVALID_ARG, MGPU_E_WKB):
        raise IllegalArgumentException(status, msg)
    raise MosaicGpuError(status, msg)
