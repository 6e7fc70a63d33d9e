#!/usr/bin/env python3
"""The C3 tessellation's host time split (no GPU): mgpu_tessellate_geom itself at several
thread counts (OMP_NUM_THREADS is read per parallel loop), then the copy into numpy arrays
and the result's release.  Usage: tools/tess_time.py [CFG] [THREADS,...]"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import numpy as np
    import mosaic_amd as M
    import bench_workloads as W
    from mosaic_amd import _native as N
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    threads = [int(t) for t in (sys.argv[2] if len(sys.argv) > 2 else "16,8,4").split(",")]
    P, res = {"c3": (W.tract_polygons, 10), "c2": (W.nyc_zones, 9)}[cfg]
    P = P()
    L = N.lib()
    isys = M.H3IndexSystem()
    for T in threads:
        os.environ["OMP_NUM_THREADS"] = str(T)
        h = ctypes.c_void_p()
        t0 = time.perf_counter()
        N.check(L.mgpu_tessellate_geom(isys.code, res, len(P), P.poly_id.ctypes.data, P.poly_part_off.ctypes.data,
                                       P.part_ring_off.ctypes.data, P.ring_off.ctypes.data, P.xy.ctypes.data,
                                       None if P.poly_type is None else P.poly_type.ctypes.data, 0, 0, 0,
                                       ctypes.byref(h)))
        t1 = time.perf_counter()
        n, b = ctypes.c_int64(), ctypes.c_int64()
        N.check(L.mgpu_tess_result_sizes(h, ctypes.byref(n), ctypes.byref(b)))
        cell, pid = np.zeros(n.value, np.int64), np.zeros(n.value, np.int32)
        core, off, wkb = np.zeros(n.value, np.uint8), np.zeros(n.value + 1, np.int64), np.zeros(b.value, np.uint8)
        N.check(L.mgpu_tess_result_copy(h, cell.ctypes.data, pid.ctypes.data, core.ctypes.data, off.ctypes.data,
                                        wkb.ctypes.data))
        t2 = time.perf_counter()
        L.mgpu_tess_destroy(h)
        t3 = time.perf_counter()
        print("%s threads %2d: tessellate %.2f s, copy %.2f s, release %.2f s (%d rows)" %
              (cfg, T, t1 - t0, t2 - t1, t3 - t2, n.value), flush=True)


if __name__ == "__main__":
    main()
