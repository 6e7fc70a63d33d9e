#!/usr/bin/env python3
"""Chip-table blob build time of a bench config (no GPU): tessellate, then
mgpu_chips_host_blob; with a -DMGPU_BLOB_TIMING library (MOSAIC_AMD_LIB) the builder
prints its phases to stderr."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import mosaic_amd as M
    import bench_workloads as W
    from mosaic_amd import _native as N
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    P, isys, res = {"c3": (W.tract_polygons, M.H3IndexSystem(), 10), "c2": (W.nyc_zones, M.H3IndexSystem(), 9)}[cfg]
    t = time.perf_counter()
    c = M.tessellate(P(), isys, res)
    t1 = time.perf_counter()
    out, nb = ctypes.c_void_p(), ctypes.c_int64()
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    N.check(N.lib().mgpu_chips_host_blob(isys.code, len(c), p(c.cell), p(c.polygon_id), p(c.is_core), p(c.wkb_offsets),
                                         p(c.wkb), ctypes.byref(out), ctypes.byref(nb)))
    t2 = time.perf_counter()
    N.lib().mgpu_host_free(out)
    print("%s: tessellate %.2f s, blob %.2f s (%.2f GB), threads %s" % (cfg, t1 - t, t2 - t1, nb.value / 1e9,
                                                                          os.environ.get("OMP_NUM_THREADS")))


if __name__ == "__main__":
    main()
