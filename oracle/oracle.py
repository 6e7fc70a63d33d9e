"""ORACLE -- TEST INFRASTRUCTURE ONLY.

ctypes binding of ``oracle/liboracle.so``, the CPU restatement of the reference's
hot path (see ``oracle/oracle.h`` for the reference file:line each function
follows).  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg import this module; the product package ``mosaic_amd``
never does.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

_dp = ctypes.POINTER(ctypes.c_double)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_i64p = ctypes.POINTER(ctypes.c_int64)
_i32p = ctypes.POINTER(ctypes.c_int32)
_u8p = ctypes.POINTER(ctypes.c_uint8)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle/liboracle.so is not built (run `make -C oracle`)")
        L = ctypes.CDLL(path)
        L.orc_h3_geo_to_h3.restype = ctypes.c_uint64
        L.orc_h3_geo_to_h3.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_int]
        L.orc_h3_point_to_index.restype = ctypes.c_uint64
        L.orc_h3_point_to_index.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_int, ctypes.c_int]
        L.orc_h3_points_to_cells.restype = None
        L.orc_h3_points_to_cells.argtypes = [_dp, _dp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, _u64p, ctypes.c_int]
        L.orc_h3_set_libm.restype = None
        L.orc_h3_set_libm.argtypes = [ctypes.c_int]
        L.orc_h3_elementary.restype = None
        L.orc_h3_elementary.argtypes = [ctypes.c_int, _dp, _dp, ctypes.c_int64, _dp]
        L.orc_h3_geo_to_hex2d.restype = None
        L.orc_h3_geo_to_hex2d.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_int), _dp, _dp]
        L.orc_bng_point_to_index.restype = ctypes.c_int64
        L.orc_bng_point_to_index.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                             ctypes.POINTER(ctypes.c_int)]
        L.orc_bng_points_to_cells.restype = None
        L.orc_bng_points_to_cells.argtypes = [_dp, _dp, ctypes.c_int64, ctypes.c_int, _i64p, ctypes.c_int]
        L.orc_wkb_contains.restype = ctypes.c_int
        L.orc_wkb_contains.argtypes = [_u8p, ctypes.c_int64, ctypes.c_double, ctypes.c_double,
                                       ctypes.POINTER(ctypes.c_int)]
        L.orc_pip_join.restype = ctypes.c_int64
        L.orc_pip_join.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp, _dp, ctypes.c_int64,
                                   ctypes.c_int64, _i64p, _i32p, _u8p, _i64p, _u8p, _i64p, _i32p,
                                   ctypes.c_int64, ctypes.c_int]
        _LIB = L
    return _LIB


def _ptr(a, t):
    return a.ctypes.data_as(t)


def h3_point_to_index(lon, lat, res, jdk=8):
    return int(lib().orc_h3_point_to_index(float(lon), float(lat), int(res), int(jdk)))


def h3_points_to_cells(lon, lat, res, jdk=8, threads=None):
    lon = np.ascontiguousarray(lon, dtype=np.float64)
    lat = np.ascontiguousarray(lat, dtype=np.float64)
    out = np.empty(lon.shape[0], dtype=np.uint64)
    lib().orc_h3_points_to_cells(_ptr(lon, _dp), _ptr(lat, _dp), lon.shape[0], int(res), int(jdk),
                                 _ptr(out, _u64p), int(threads or os.cpu_count() or 1))
    return out.view(np.int64)


class h3_libm:
    """Context manager: the geoToH3 route's libm inside the block -- "glibc" (the
    reference's, the default) or "cr" (correctly rounded, libquadmath)."""

    def __init__(self, mode):
        self.cr = {"glibc": 0, "cr": 1}[mode]

    def __enter__(self):
        lib().orc_h3_set_libm(self.cr)
        return self

    def __exit__(self, *exc):
        lib().orc_h3_set_libm(0)
        return False


def h3_elementary(fn, a, b=None):
    """The H3 route's elementary operation `fn` (oracle.h orc_h3_elementary) on arrays."""
    a = np.ascontiguousarray(a, dtype=np.float64)
    bb = None if b is None else np.ascontiguousarray(b, dtype=np.float64)
    out = np.empty(a.shape[0], dtype=np.float64)
    lib().orc_h3_elementary(int(fn), _ptr(a, _dp), None if bb is None else _ptr(bb, _dp), a.shape[0], _ptr(out, _dp))
    return out


def h3_geo_to_hex2d(lat_rad, lon_rad, res):
    f = ctypes.c_int()
    x = ctypes.c_double()
    y = ctypes.c_double()
    lib().orc_h3_geo_to_hex2d(lat_rad, lon_rad, res, ctypes.byref(f), ctypes.byref(x), ctypes.byref(y))
    return f.value, x.value, y.value


def bng_point_to_index(e, n, res):
    err = ctypes.c_int()
    v = lib().orc_bng_point_to_index(float(e), float(n), int(res), ctypes.byref(err))
    if err.value:
        raise ValueError("NaN coordinates are not supported.")
    return int(v)


def bng_points_to_cells(e, n, res, threads=None):
    e = np.ascontiguousarray(e, dtype=np.float64)
    n = np.ascontiguousarray(n, dtype=np.float64)
    out = np.empty(e.shape[0], dtype=np.int64)
    lib().orc_bng_points_to_cells(_ptr(e, _dp), _ptr(n, _dp), e.shape[0], int(res), _ptr(out, _i64p),
                                  int(threads or os.cpu_count() or 1))
    return out


LOC_EXTERIOR, LOC_BOUNDARY, LOC_INTERIOR = 0, 1, 2


def wkb_locate(wkb: bytes, x, y):
    buf = np.frombuffer(wkb, dtype=np.uint8)
    err = ctypes.c_int()
    loc = lib().orc_wkb_contains(_ptr(buf, _u8p), len(wkb), float(x), float(y), ctypes.byref(err))
    if err.value:
        raise ValueError("unsupported or malformed WKB (%d)" % err.value)
    return loc


def st_contains(wkb: bytes, x, y):
    return wkb_locate(wkb, x, y) == LOC_INTERIOR


def pip_join(index_system, res, x, y, chip_cell, chip_poly, chip_core, wkb_offsets, wkb_blob,
             jdk=8, threads=None):
    """Sorted (point index, polygon id) pairs of the reference's join + filter."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    cc = np.ascontiguousarray(chip_cell, dtype=np.int64)
    cp = np.ascontiguousarray(chip_poly, dtype=np.int32)
    co = np.ascontiguousarray(chip_core, dtype=np.uint8)
    off = np.ascontiguousarray(wkb_offsets, dtype=np.int64)
    blob = np.ascontiguousarray(np.frombuffer(bytes(wkb_blob), dtype=np.uint8) if not isinstance(wkb_blob, np.ndarray)
                                else wkb_blob, dtype=np.uint8)
    if blob.size == 0:
        blob = np.zeros(1, dtype=np.uint8)
    nt = int(threads or os.cpu_count() or 1)
    L = lib()
    args = [int(index_system), int(res), int(jdk), _ptr(x, _dp), _ptr(y, _dp), x.shape[0], cc.shape[0],
            _ptr(cc, _i64p), _ptr(cp, _i32p), _ptr(co, _u8p), _ptr(off, _i64p), _ptr(blob, _u8p)]
    cnt = L.orc_pip_join(*args, None, None, 0, nt)
    if cnt < 0:
        raise ValueError("oracle join failed (NaN BNG coordinates or unsupported chip WKB)")
    pts = np.empty(max(cnt, 1), dtype=np.int64)
    polys = np.empty(max(cnt, 1), dtype=np.int32)
    cnt2 = L.orc_pip_join(*args, _ptr(pts, _i64p), _ptr(polys, _i32p), cnt, nt)
    assert cnt2 == cnt
    return pts[:cnt], polys[:cnt]


# ---------------------------------------------------------------- BNG kRing / kLoop
# Pure-Python restatement (small cases only) of BNGIndexSystem.kRing / kLoop
# (src/main/scala/com/databricks/labs/mosaic/core/index/BNGIndexSystem.scala:221-252)
# with the helpers they call: indexDigits (:440-442), getResolution(digits) (:451-464),
# getX / getY (:477-506), getEdgeSize (:163-170, sizeMap :64-79), isValid (:261-270).
# pointToIndex is the C restatement above.  Scala Int division truncates toward zero.

BNG_EDGE = {1: 100000, -1: 500000, 2: 10000, -2: 50000, 3: 1000, -3: 5000,
            4: 100, -4: 500, 5: 10, -5: 50, 6: 1, -6: 5}


def _jdiv(a, b):
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b > 0) else -q


def _digits_int(ds):
    return int("".join(str(d) for d in ds))  # "".toInt throws -> ValueError


def bng_resolution_of_digits(d):
    if len(d) < 6:
        return -1
    k = _jdiv(len(d) - 6, 2)
    return -(k + 2) if d[-1] > 0 else k + 1


def _bng_k(d):
    k = _jdiv(len(d) - 6, 2)
    return k


def bng_get_x(d, e):
    k = _bng_k(d)
    xs = d[1:3] + (d[5:5 + k] if k > 0 else [])
    q = d[-1]
    return _digits_int(xs) * (2 * e if q > 0 else e) + (e if q in (3, 4) else 0)


def bng_get_y(d, e):
    k = _bng_k(d)
    ys = d[3:5] + (d[5 + k:5 + 2 * k] if k > 0 else [])
    q = d[-1]
    return _digits_int(ys) * (2 * e if q > 0 else e) + (e if q in (2, 3) else 0)


def bng_is_valid(i):
    d = [int(c) for c in str(int(i))]
    xl, yl = _digits_int(d[3:5]), _digits_int(d[1:3])
    e = BNG_EDGE[bng_resolution_of_digits(d)]
    x, y = bng_get_x(d, e), bng_get_y(d, e)
    return 0 <= x <= 700000 and 0 <= y <= 1300000 and xl < 14 and yl < 8


def bng_k_loop(i, k):
    d = [int(c) for c in str(int(i))]
    r = bng_resolution_of_digits(d)
    e = BNG_EDGE[r]
    x, y = bng_get_x(d, e), bng_get_y(d, e)
    pts = ([(x + (c - k) * e, y - k * e) for c in range(2 * k)] + [(x + k * e, y + (c - k) * e) for c in range(2 * k)] +
           [(x + (k - c) * e, y + k * e) for c in range(2 * k)] + [(x - k * e, y + (k - c) * e) for c in range(2 * k)])
    out = [bng_point_to_index(float(px), float(py), r) for px, py in pts]
    return [c for c in out if bng_is_valid(c)]


def bng_k_ring(i, n):
    if n == 1:
        return [int(i)] + bng_k_loop(i, 1)
    return [int(i)] + [c for j in range(1, n + 1) for c in bng_k_loop(i, j)]


# ---------------------------------------------------------------- H3 kRing / kLoop
# H3IndexSystem.kRing / kLoop (src/main/scala/com/databricks/labs/mosaic/core/index/
# H3IndexSystem.scala:182-205) over H3-Java 3.7.0 (kRing = nonzero entries of the C
# array in order; hexRing throws PentagonEncounteredException on failure) and the C
# restatement of H3 v3.7 algos.c in h3_oracle.c.

class PentagonEncountered(Exception):
    pass


def _h3_kring_lib():
    L = lib()
    if not getattr(L, "_kring_bound", False):
        L.orc_h3_max_kring_size.restype = ctypes.c_int64
        L.orc_h3_max_kring_size.argtypes = [ctypes.c_int]
        L.orc_h3_kring_raw.restype = ctypes.c_int
        L.orc_h3_kring_raw.argtypes = [ctypes.c_uint64, ctypes.c_int, _u64p]
        L.orc_h3_hex_ring.restype = ctypes.c_int
        L.orc_h3_hex_ring.argtypes = [ctypes.c_uint64, ctypes.c_int, _u64p]
        L.orc_h3_neighbor_rotations.restype = ctypes.c_uint64
        L.orc_h3_neighbor_rotations.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        L._kring_bound = True
    return L


def h3_k_ring(h, k):
    """H3Core.kRing(h, k) as H3-Java returns it (H3IndexSystem.scala:182-184)."""
    L = _h3_kring_lib()
    buf = np.zeros(L.orc_h3_max_kring_size(k), dtype=np.uint64)
    L.orc_h3_kring_raw(int(h), int(k), _ptr(buf, _u64p))
    return [int(v) for v in buf if v != 0]


def h3_hex_ring(h, k):
    """H3Core.hexRing(h, k); raises PentagonEncountered where H3-Java throws."""
    L = _h3_kring_lib()
    buf = np.zeros(max(1, 6 * k), dtype=np.uint64)
    if L.orc_h3_hex_ring(int(h), int(k), _ptr(buf, _u64p)) != 0:
        raise PentagonEncountered()
    return [int(v) for v in buf if v != 0]


def _i32(v):
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v & 0x80000000 else v


def scala_hashset_key(v):
    """Iteration rank of a java.lang.Long in a Scala 2.12 immutable.HashSet (the trie is
    indexed by 5-bit chunks of improve(##), lowest chunk first).  ## of a boxed Long
    is BoxesRunTime.hashFromLong: the int value if it fits, else Long.hashCode."""
    v &= 0xFFFFFFFFFFFFFFFF
    sv = v - (1 << 64) if v >> 63 else v
    hc = sv if -(1 << 31) <= sv < (1 << 31) else _i32(v ^ (v >> 32))
    h = _i32(hc + ~_i32(hc << 9))
    h = _i32(h ^ ((h & 0xFFFFFFFF) >> 14))
    h = _i32(h + _i32(h << 4))
    h = _i32(h ^ ((h & 0xFFFFFFFF) >> 10))
    u = h & 0xFFFFFFFF
    return tuple((u >> s) & 31 for s in range(0, 32, 5))


def h3_k_loop(h, n):
    """H3IndexSystem.kLoop(h, n) (H3IndexSystem.scala:194-205): hexRing, or where it
    throws, kRing(n).toSet diff kRing(n - 1).toSet, in Scala 2.12 HashSet order."""
    if int(h) < 0:
        raise ValueError("requirement failed")
    try:
        return h3_hex_ring(h, n)
    except PentagonEncountered:
        a = h3_k_ring(h, n)
        b = set(h3_k_ring(h, n - 1))
        return sorted(set(a) - b, key=scala_hashset_key)


def ring_join(index_system, res, k, lx, ly, rx, ry, loop_only=False, max_per_left=0, max_distance=-1.0,
              left_id_base=0, left_outer=False, cells=None):
    """Test infrastructure: one iteration of GridRingNeighbours (models/knn/
    GridRingNeighbours.scala:121 transform + resultTransform) for point landmarks and
    point candidates, restated: the landmark's kRing(cell, k) (Mosaic.geometryKRing,
    core/Mosaic.scala:123-128) or kLoop(cell, k) (geometryKLoop :142-156) cells joined with
    the candidates' cells (Mosaic.pointChip :48-59), each (landmark, candidate) once,
    self matches dropped, st_distance = JTS Coordinate.distance (Math.hypot: the fdlibm
    port of jts_centroid.py), distance <= max_distance, ordered by (distance, candidate),
    the first max_per_left.  left_outer: the join is left_outer (GridRingNeighbours.scala:128)
    and resultTransform keeps the null group (:151): a landmark with a cell that holds no
    candidate gets a (left, -1, NaN) row first (Spark: nulls first in an ascending window).
    cells: explicit per-landmark cell lists instead of the kRing / kLoop (the exactness
    iteration, ring_join_final_cells).  Returns (left, right, distance) arrays."""
    import jts_centroid as JC
    lx, ly, rx, ry = (np.ascontiguousarray(v, dtype=np.float64) for v in (lx, ly, rx, ry))
    if index_system == 0:
        lc, rc = h3_points_to_cells(lx, ly, res), h3_points_to_cells(rx, ry, res)
        ring = (lambda c: h3_k_loop(int(c), k)) if loop_only else (lambda c: h3_k_ring(int(c), k))
    else:
        lc, rc = bng_points_to_cells(lx, ly, res), bng_points_to_cells(rx, ry, res)
        ring = (lambda c: bng_k_loop(int(c), k)) if loop_only else (lambda c: bng_k_ring(int(c), k))
    by_cell = {}
    for j, c in enumerate(rc.tolist()):
        by_cell.setdefault(c, []).append(j)
    L, R, D = [], [], []
    bits = lambda v: np.float64(v).view(np.int64)  # noqa: E731
    for i in range(len(lx)):
        got = []
        null_row = False
        for c in set(ring(lc[i]) if cells is None else cells[i]):
            if not by_cell.get(c):
                null_row = True
            for j in by_cell.get(c, ()):
                if bits(lx[i]) == bits(rx[j]) and bits(ly[i]) == bits(ry[j]):
                    continue
                d = JC.hypot(float(lx[i] - rx[j]), float(ly[i] - ry[j]))
                if max_distance >= 0 and not d <= max_distance:
                    continue
                got.append((d, j))
        got.sort()
        if max_per_left > 0:
            got = got[:max_per_left]
        if left_outer and null_row:
            got = [(float("nan"), -1)] + got
        for d, j in got:
            L.append(left_id_base + i)
            R.append(j)
            D.append(d)
    return np.array(L, np.int64), np.array(R, np.int64), np.array(D, np.float64)


def jts_circle(x, y, r):
    """JTS OffsetSegmentGenerator.createCircle (st_buffer of a point, 8 quadrant segments):
    (x + r, y), then 31 more vertices clockwise at 2 pi / 32 steps, closed."""
    import math
    pts = [(x + r, y)] + [(x + r * math.cos(-i * 2 * math.pi / 32), y + r * math.sin(-i * 2 * math.pi / 32))
                          for i in range(1, 32)]
    return pts + [pts[0]]


def ring_join_final_cells(index_system, res, lx, ly, radius, k_iterated, buffer_cells):
    """The exactness iteration's landmark cells (GridRingNeighbours.leftTransform with
    iterationID -1, GridRingNeighbours.scala:82-90): array_except(the cells of
    grid_tessellate(st_buffer(landmark, radius)) -- `buffer_cells[i]`, the chip table of the
    landmark's circle, an input as every chip table is -- , kRing(cell(landmark), k)),
    distinct, in the tessellation's order."""
    lx, ly = (np.ascontiguousarray(v, dtype=np.float64) for v in (lx, ly))
    lc = h3_points_to_cells(lx, ly, res) if index_system == 0 else bng_points_to_cells(lx, ly, res)
    out = []
    for i in range(len(lx)):
        if not (radius[i] > 0) or not np.isfinite(radius[i]):
            out.append([])
            continue
        it = set(h3_k_ring(int(lc[i]), int(k_iterated[i])) if index_system == 0
                 else bng_k_ring(int(lc[i]), int(k_iterated[i])))
        seen = []
        for c in buffer_cells[i]:
            if c not in it and c not in seen:
                seen.append(c)
        out.append(seen)
    return out
