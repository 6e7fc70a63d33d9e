#!/usr/bin/env python3
"""Chip-table blob build time of a bench config (no GPU): tessellate (or load the arrays
saved by --cache=FILE.npz), then
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
    if "--upload" in sys.argv:  # (the GPU first, as bench.py: torch sets the device up)
        import torch
        torch.cuda.set_device(0)
        M.default_context(torch.device("cuda", 0))
    P, isys, res = {"c3": (W.tract_polygons, M.H3IndexSystem(), 10), "c2": (W.nyc_zones, M.H3IndexSystem(), 9)}[cfg]
    t = time.perf_counter()
    cache = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--cache=")), None)
    if cache and os.path.exists(cache) and "--upload" not in sys.argv:  # (host blob only: the arrays)
        import numpy as np
        from types import SimpleNamespace
        z = np.load(cache)
        c = SimpleNamespace(**{k: z[k] for k in z.files})
        c.__len__ = None
        n_rows = len(c.cell)
    else:
        c = M.tessellate(P(), isys, res, keep_core_geometries=("--keep-core" in sys.argv))
        n_rows = len(c)
        if cache and "--upload" not in sys.argv:
            import numpy as np
            np.savez(cache, cell=c.cell, polygon_id=c.polygon_id, is_core=c.is_core, wkb_offsets=c.wkb_offsets, wkb=c.wkb)
    t1 = time.perf_counter()
    out, nb = ctypes.c_void_p(), ctypes.c_int64()
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    N.check(N.lib().mgpu_chips_host_blob(isys.code, n_rows, p(c.cell), p(c.polygon_id), p(c.is_core), p(c.wkb_offsets),
                                         p(c.wkb), ctypes.byref(out), ctypes.byref(nb)))
    t2 = time.perf_counter()
    if "--hash" in sys.argv:
        import hashlib
        print("blob sha256", hashlib.sha256(ctypes.string_at(out.value, nb.value)).hexdigest()[:16])
    N.lib().mgpu_host_free(out)
    print("%s: tessellate %.2f s, blob %.2f s (%.2f GB), threads %s" % (cfg, t1 - t, t2 - t1, nb.value / 1e9,
                                                                          os.environ.get("OMP_NUM_THREADS")))
    if "--upload" in sys.argv:  # (GPU) the whole upload: build + host-to-device copy
        import torch
        dev = torch.device("cuda", 0)
        ctx = M.default_context(dev)
        for _ in range(2):
            t3 = time.perf_counter()
            chips = c.upload(ctx)
            torch.cuda.synchronize()
            print("upload %.2f s" % (time.perf_counter() - t3))
            del chips


if __name__ == "__main__":
    main()
