"""The hot-path function surface, as the reference registers it.

  grid_longlatascellid(lon, lat, res)   MosaicContext.scala:429-432 -> PointIndexLonLat.scala:44-51
  grid_pointascellid(point, res)        MosaicContext.scala:453-457 -> PointIndexGeom.scala:33-47
  grid_tessellateexplode(geom, res)     MosaicContext.scala:400-408 -> MosaicExplode.scala:70-79
  st_contains(chip.wkb, point)          MosaicContext.scala:166     -> ST_Contains.scala:21-44
  pip_join(points, chips, res)          the user-level join of the Quickstart notebooks
                                        (QuickstartNotebook.ipynb:1835): cell == index_id
                                        AND (is_core OR st_contains(wkb, point))

Column arguments are float64 device tensors (structure of arrays); results stay in HBM.
"""
import numpy as np

from . import _native as N
from .chips import ChipTable, DeviceChips, tessellate
from .index_system import H3IndexSystem, _check_points

_H3 = H3IndexSystem()


def grid_longlatascellid(lon, lat, resolution, index_system=None, ctx=None, stream=None, stats=False,
                         cell_id_type="long"):
    """Cell id of every (lon, lat) -- (eastings, northings) for BNG.

    cell_id_type "long": an int64 tensor (LongType).  "string": the StringType ids
    (IndexSystem.serializeCellId -- BNG's default cell id type, BNGIndexSystem.scala:30),
    formatted on the device: (chars uint8 tensor, offsets int64 tensor of n + 1)."""
    isys = index_system or _H3
    out = isys.points_to_index(lon, lat, resolution, ctx=ctx, stream=stream, stats=stats)
    if cell_id_type == "long":
        return out
    if cell_id_type != "string":
        raise N.IllegalArgumentException(N.MGPU_E_INVALID_ARG, "cell_id_type must be 'long' or 'string'")
    cells, st = out if stats else (out, None)
    strs = isys.format_device(cells, ctx=ctx, stream=stream)
    return (strs, st) if stats else strs


class GeometryColumn:
    """A geometry column in device memory as Arrow lays out binary / utf8: one byte buffer,
    int64 offsets (n + 1), optional validity bitmap (LSB first, 1 = present).  Format:
    MGPU_GEOM_WKB (BinaryType), _WKT (StringType), _HEX (HexType: hex WKB text) or
    _GEOJSON (JSONType), GeometryAPI.geometry's input types (GeometryAPI.scala:81-89)."""

    FORMATS = {"wkb": N.MGPU_GEOM_WKB, "wkt": N.MGPU_GEOM_WKT, "hex": N.MGPU_GEOM_HEX, "geojson": N.MGPU_GEOM_GEOJSON}

    def __init__(self, fmt, data, offsets, valid=None):
        self.format, self.data, self.offsets, self.valid = fmt, data, offsets, valid

    def __len__(self):
        return self.offsets.numel() - 1

    @staticmethod
    def from_rows(rows, device="cuda", fmt=None):
        """Python rows (bytes: WKB, str: WKT unless `fmt` says "hex" / "geojson", None:
        null) -> device column."""
        import torch
        kinds = {type(r) for r in rows if r is not None}
        if len(kinds) > 1:
            raise N.IllegalArgumentException(N.MGPU_E_INVALID_ARG, "mixed binary and text rows")
        code = GeometryColumn.FORMATS[fmt] if fmt else (N.MGPU_GEOM_WKT if kinds == {str} else N.MGPU_GEOM_WKB)
        bs = [b"" if r is None else (r.encode() if isinstance(r, str) else bytes(r)) for r in rows]
        off = np.zeros(len(bs) + 1, np.int64)
        off[1:] = np.cumsum([len(b) for b in bs])
        data = np.frombuffer(b"".join(bs) or b"\0", np.uint8)
        valid = None
        if any(r is None for r in rows):
            valid = np.packbits(np.array([r is not None for r in rows], bool), bitorder="little")
            valid = torch.from_numpy(valid).to(device)
        return GeometryColumn(code, torch.from_numpy(data.copy()).to(device), torch.from_numpy(off).to(device), valid)


class InternalGeometryColumn:
    """Mosaic's InternalGeometryType column (InternalGeometry.scala: typeId, boundaries,
    holes) flattened as nested lists in device memory (mgpu_internal_geometry_to_cells):
    type_id[n]; row_part[n + 1]; part_ring[P + 1] (each part's boundary, then its holes);
    ring_off[R + 1]; xy[2 V]."""

    def __init__(self, type_id, row_part, part_ring, ring_off, xy):
        self.type_id, self.row_part, self.part_ring, self.ring_off, self.xy = type_id, row_part, part_ring, ring_off, xy

    def __len__(self):
        return self.type_id.numel()

    @staticmethod
    def from_rows(rows, device="cuda"):
        """rows: (type_id, parts), parts = [[ring, ring, ...], ...] (boundary first), a
        ring a list of (x, y)."""
        import torch
        tid, rp, pr, ro, xy = [], [0], [0], [0], []
        for t, parts in rows:
            tid.append(t)
            for part in parts:
                for ring in part:
                    xy.extend(ring)
                    ro.append(len(xy))
                pr.append(len(ro) - 1)
            rp.append(len(pr) - 1)
        T = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(device)
        return InternalGeometryColumn(T(tid, np.int32), T(rp, np.int64), T(pr, np.int64), T(ro, np.int64),
                                      T(np.array(xy, np.float64).reshape(-1, 2) if xy else np.zeros((1, 2)), np.float64))


def grid_pointascellid(points, resolution, index_system=None, ctx=None, stream=None, stats=False):
    """grid_pointascellid (PointIndexGeom.scala:33-47): the cell of each row's centroid.

    ``points``: a GeometryColumn (WKB / HEX rows of any type, WKT / GeoJSON POINT or
    MULTIPOINT rows, decoded on the GPU and reduced to JTS's centroid; null rows give
    cell 0 -- returned with the validity bitmap as (cells, valid)), an
    InternalGeometryColumn, an (n, 2) float64 tensor, or an (x, y) pair (a point's
    centroid is the point itself, MosaicGeometryJTS.scala:60-64).  Types a format does
    not build raise MGPU_E_UNSUPPORTED, an empty geometry IllegalStateException (JTS getX
    on an empty point)."""
    if isinstance(points, InternalGeometryColumn):
        import ctypes
        import torch
        from .context import default_context
        isys = index_system or _H3
        res = isys.get_resolution(resolution)
        dev = points.type_id.device
        ctx = ctx or default_context(dev)
        n = len(points)
        cells = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        st = N.MgpuStats()
        s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
        N.check(N.lib().mgpu_internal_geometry_to_cells(ctx.handle, isys.code, res, n, points.type_id.data_ptr(),
                                                        points.row_part.data_ptr(), points.part_ring.data_ptr(),
                                                        points.ring_off.data_ptr(), points.xy.data_ptr(), None, 0,
                                                        cells.data_ptr(), None, s, ctypes.byref(st)))
        return (cells[:n], st.as_dict()) if stats else cells[:n]
    if isinstance(points, GeometryColumn):
        import ctypes
        import torch
        from .context import default_context
        isys = index_system or _H3
        res = isys.get_resolution(resolution)
        dev = points.offsets.device
        ctx = ctx or default_context(dev)
        n = len(points)
        cells = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        valid = torch.empty((n + 7) // 8 + 1, dtype=torch.uint8, device=dev) if points.valid is not None else None
        st = N.MgpuStats()
        s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
        N.check(N.lib().mgpu_geometry_to_cells(ctx.handle, isys.code, res, points.format, points.data.data_ptr(),
                                               points.offsets.data_ptr(),
                                               None if points.valid is None else points.valid.data_ptr(), 0, n,
                                               cells.data_ptr(), None if valid is None else valid.data_ptr(), s,
                                               ctypes.byref(st)))
        out = cells[:n] if valid is None else (cells[:n], valid[:(n + 7) // 8])
        return (out, st.as_dict()) if stats else out
    if isinstance(points, (tuple, list)):
        x, y = points
    else:
        x, y = points[:, 0].contiguous(), points[:, 1].contiguous()
    return grid_longlatascellid(x, y, resolution, index_system=index_system, ctx=ctx, stream=stream, stats=stats)


def grid_cellkring(cells, k, index_system, loop_only=False, ctx=None, stream=None):
    """grid_cellkring / grid_cellkloop (CellKRing.scala:68, CellKLoop.scala:63 ->
    IndexSystem.kRing / kLoop) over a device int64 column, on the GPU (BNG and H3; H3
    pentagon neighbourhoods in the reference's fallback order, for k <= 64, else
    MosaicGpuError MGPU_E_UNSUPPORTED).  Returns
    (ids int64 tensor, offsets int64 tensor of n + 1): cell i's list is
    ids[offsets[i]:offsets[i + 1]], in the reference's order."""
    import ctypes
    import torch
    from .context import default_context
    if cells.dtype != torch.int64 or not cells.is_cuda:
        raise N.IllegalArgumentException(N.MGPU_E_INVALID_ARG, "cells must be an int64 device tensor")
    cells = cells.contiguous()
    ctx = ctx or default_context(cells.device)
    n = cells.numel()
    k = int(k)
    per = max(8 * k, 1) if loop_only else 1 + 4 * k * (k + 1)  # H3 hexRing(0) = [cell]
    cap = max(n * per, 1)
    out = torch.empty(cap, dtype=torch.int64, device=cells.device)
    off = torch.empty(n + 1, dtype=torch.int64, device=cells.device)
    tot = ctypes.c_int64()
    s = stream if stream is not None else torch.cuda.current_stream(cells.device).cuda_stream
    N.check(N.lib().mgpu_grid_kring(ctx.handle, index_system.code, cells.data_ptr(), n, k, 1 if loop_only else 0,
                                    out.data_ptr(), cap, off.data_ptr(), ctypes.byref(tot), s),
            required=tot.value)
    return out[:tot.value], off


def grid_cellkloop(cells, k, index_system, ctx=None, stream=None):
    """grid_cellkloop (CellKLoop.scala:63 -> IndexSystem.kLoop) on the GPU (BNG, H3)."""
    return grid_cellkring(cells, k, index_system, loop_only=True, ctx=ctx, stream=stream)


def grid_tessellateexplode(polygons, resolution, keep_core_geometries=True, index_system=None):
    """Chip rows (is_core, index_id, wkb) of every polygon -> ChipTable (host columns)."""
    return tessellate(polygons, index_system or _H3, resolution, keep_core_geometries)


def st_contains(chips, chip_rows, x, y, stream=None):
    """st_contains(chip.wkb, point) for explicit pairs: int8 tensor of 1 / 0, -1 where the
    chip geometry is NULL (SQL null)."""
    import torch
    if isinstance(chips, ChipTable):
        chips = chips.upload()
    _check_points(x, y)
    rows = chip_rows.to(device=x.device, dtype=torch.int64).contiguous()
    if rows.numel() != x.numel():
        raise N.IllegalArgumentException(N.MGPU_E_INVALID_ARG, "chip_rows and points differ in length")
    out = torch.empty(x.numel(), dtype=torch.int8, device=x.device)
    s = stream if stream is not None else torch.cuda.current_stream(x.device).cuda_stream
    N.check(N.lib().mgpu_st_contains(chips.ctx.handle, chips.handle, rows.data_ptr(), x.data_ptr(), y.data_ptr(),
                                     x.numel(), out.data_ptr(), s))
    return out


class JoinResult:
    def __init__(self, point_id, polygon_id, stats):
        self.point_id = point_id
        self.polygon_id = polygon_id
        self.stats = stats

    def __len__(self):
        return self.point_id.numel()

    def numpy(self):
        return self.point_id.cpu().numpy(), self.polygon_id.cpu().numpy()


def pip_join(x, y, chips, resolution, index_system=None, point_id=None, point_id_base=0, capacity=None,
             out=None, stream=None):
    """The grid-indexed point-in-polygon join (fused, one kernel).

    Returns a JoinResult with int64 point ids and int32 polygon ids ordered by input
    position then polygon id.  ``capacity`` bounds the output (default: n + 1/8 n
    headroom; when the pairs do not fit, arrays of the exact count are allocated and
    filled from the join's kept records by mgpu_pip_join_fetch -- the join is not redone).
    ``out`` = (point ids, polygon ids) preallocated: with ``capacity`` None, pairs that do
    not fit them go to fresh arrays of the exact count the same way; an explicit
    ``capacity`` is a hard bound (CapacityError, with the count)."""
    import torch
    isys = index_system or _H3
    res = isys.get_resolution(resolution)
    if isinstance(chips, ChipTable):
        if chips.index_system != isys.code:
            raise N.IllegalArgumentException(N.MGPU_E_INVALID_ARG, "chip table built for another index system")
        chips = chips.upload()
    _check_points(x, y)
    n = x.numel()
    if chips.ctx.device != x.device:
        raise N.IllegalArgumentException(N.MGPU_E_INVALID_ARG, "chip table on %s, points on %s" % (chips.ctx.device, x.device))
    pid_ptr = None
    if point_id is not None:
        if point_id.dtype != torch.int64 or point_id.numel() != n or point_id.device != x.device:
            raise N.IllegalArgumentException(N.MGPU_E_INVALID_ARG, "point_id must be int64 on the points' device")
        point_id = point_id.contiguous()  # kept alive (bound here) until the call returns
        pid_ptr = point_id.data_ptr()
    s = stream if stream is not None else torch.cuda.current_stream(x.device).cuda_stream
    import ctypes
    if out is not None:
        op, oq = out
        cap = min(op.numel(), oq.numel())
    else:
        cap = int(capacity if capacity is not None else max(16, n + n // 8))
        op = torch.empty(cap, dtype=torch.int64, device=x.device)
        oq = torch.empty(cap, dtype=torch.int32, device=x.device)
    cnt = ctypes.c_int64()
    st = N.MgpuStats()
    status = N.lib().mgpu_pip_join(chips.ctx.handle, chips.handle, isys.code, res, x.data_ptr(), y.data_ptr(),
                                   pid_ptr, int(point_id_base), n, cap, ctypes.byref(cnt), op.data_ptr(),
                                   oq.data_ptr(), s, st)
    if status == N.MGPU_E_CAPACITY and capacity is None:
        # the join's records are kept: write them into arrays of the exact size
        cap = int(cnt.value)
        op = torch.empty(cap, dtype=torch.int64, device=x.device)
        oq = torch.empty(cap, dtype=torch.int32, device=x.device)
        status = N.lib().mgpu_pip_join_fetch(chips.ctx.handle, cap, ctypes.byref(cnt), op.data_ptr(), oq.data_ptr(), s)
    N.check(status, required=cnt.value)
    m = int(cnt.value)
    return JoinResult(op[:m], oq[:m], st.as_dict())


class AsyncJoin:
    """A join enqueued by pip_join_async: ``finish()`` settles it (mgpu_pip_join_finish:
    the stream's wait, the H3 near-ties recomputed with the reference's libm, a rerun only
    when a cell moves) and returns the JoinResult.  ``count`` is the device-side pair
    count (one int64 tensor) the enqueued work leaves before finish."""

    def __init__(self, ctx, op, oq, count, keep):
        self._ctx, self._op, self._oq, self.count, self._keep = ctx, op, oq, count, keep
        self._done = None

    def finish(self):
        import ctypes
        if self._done is not None:
            return self._done
        cnt = ctypes.c_int64()
        st = N.MgpuStats()
        status = N.lib().mgpu_pip_join_finish(self._ctx.handle, ctypes.byref(cnt), st)
        N.check(status, required=cnt.value)
        m = int(cnt.value)
        self._done = JoinResult(self._op[:m], self._oq[:m], st.as_dict())
        return self._done


def pip_join_async(x, y, chips, resolution, index_system=None, point_id=None, point_id_base=0, capacity=None,
                   stream=None):
    """mgpu_pip_join_async: enqueue the join on the stream (nothing waits); the pairs
    equal pip_join's after ``finish()`` (include/mosaic_gpu.h).  ``capacity`` is a hard
    bound here (CapacityError from finish, with the count)."""
    import torch
    isys = index_system or _H3
    res = isys.get_resolution(resolution)
    if isinstance(chips, ChipTable):
        chips = chips.upload()
    _check_points(x, y)
    n = x.numel()
    pid_ptr = None
    if point_id is not None:
        point_id = point_id.contiguous()
        pid_ptr = point_id.data_ptr()
    s = stream if stream is not None else torch.cuda.current_stream(x.device).cuda_stream
    cap = int(capacity if capacity is not None else max(16, n + n // 8))
    op = torch.empty(cap, dtype=torch.int64, device=x.device)
    oq = torch.empty(cap, dtype=torch.int32, device=x.device)
    count = torch.zeros(1, dtype=torch.int64, device=x.device)
    N.check(N.lib().mgpu_pip_join_async(chips.ctx.handle, chips.handle, isys.code, res, x.data_ptr(), y.data_ptr(),
                                        pid_ptr, int(point_id_base), n, cap, count.data_ptr(), op.data_ptr(),
                                        oq.data_ptr(), s))
    return AsyncJoin(chips.ctx, op, oq, count, (x, y, point_id, chips))


def _ring_call(call, left_x, max_per_left):
    """Run a ring-join entry with an output sized up front, once more at the reported size."""
    import ctypes
    import torch
    n = ctypes.c_int64()
    cap = max(16, left_x.numel() * (max_per_left + 1 if max_per_left > 0 else 8))
    for _ in range(2):
        ol = torch.empty(cap, dtype=torch.int64, device=left_x.device)
        orr = torch.empty(cap, dtype=torch.int64, device=left_x.device)
        od = torch.empty(cap, dtype=torch.float64, device=left_x.device)
        st = call(cap, ctypes.byref(n), ol.data_ptr(), orr.data_ptr(), od.data_ptr())
        if st == N.MGPU_E_CAPACITY:
            cap = int(n.value)
            continue
        N.check(st)
        m = int(n.value)
        return ol[:m], orr[:m], od[:m]
    N.check(st, required=n.value)


def grid_ring_join(left_x, left_y, right_x, right_y, resolution, k=1, index_system=None, loop_only=False,
                   max_per_left=0, max_distance=-1.0, left_id_base=0, left_outer=False, stream=None):
    """One iteration of SpatialKNN's grid-ring neighbour join for point landmarks (left) and
    point candidates (right) -- GridRingNeighbours.transform (models/knn/
    GridRingNeighbours.scala:121) with its resultTransform (mgpu_ring_join_ex): the pairs whose
    cells meet in kRing(cell(landmark), k) (``loop_only``: kLoop, iterations > 1), self
    matches dropped, ``distance <= max_distance`` (< 0: none), per landmark by (distance,
    candidate index), at most ``max_per_left`` (0: all).  ``left_outer``: the left_outer
    join's null row (right -1, distance NaN) first for a landmark with a cell holding no
    candidate.  Returns (left ids, right indices, distances) on the points' device."""
    import torch
    from .context import default_context
    isys = index_system or _H3
    res = isys.get_resolution(resolution)
    _check_points(left_x, left_y)
    _check_points(right_x, right_y)
    ctx = default_context(left_x.device)
    s = stream if stream is not None else torch.cuda.current_stream(left_x.device).cuda_stream
    flags = N.MGPU_RING_LEFT_OUTER if left_outer else 0
    return _ring_call(lambda cap, n, ol, orr, od: N.lib().mgpu_ring_join_ex(
        ctx.handle, isys.code, res, int(k), 1 if loop_only else 0, left_x.data_ptr(), left_y.data_ptr(),
        left_x.numel(), right_x.data_ptr(), right_y.data_ptr(), right_x.numel(), int(left_id_base),
        int(max_per_left), float(max_distance), flags, cap, n, ol, orr, od, s), left_x, max_per_left)


def grid_ring_join_final(left_x, left_y, radius, k_iterated, right_x, right_y, resolution, index_system=None,
                         max_per_left=0, max_distance=-1.0, left_id_base=0, left_outer=False, stream=None):
    """SpatialKNN's exactness iteration (GridRingNeighbours.leftTransform with iterationID
    -1, GridRingNeighbours.scala:82-90; mgpu_ring_join_final): per landmark, the cells of
    grid_tessellate(st_buffer(landmark, radius[i])) not in kRing(cell, k_iterated[i]),
    joined with the candidates as grid_ring_join does.  ``radius`` / ``k_iterated``: host
    arrays (the landmarks' k-th match distance and their last iteration)."""
    import numpy as np
    import torch
    from .context import default_context
    isys = index_system or _H3
    res = isys.get_resolution(resolution)
    _check_points(left_x, left_y)
    _check_points(right_x, right_y)
    rad = np.ascontiguousarray(radius, dtype=np.float64)
    kit = np.ascontiguousarray(k_iterated, dtype=np.int32)
    assert rad.shape == kit.shape == (left_x.numel(),)
    ctx = default_context(left_x.device)
    s = stream if stream is not None else torch.cuda.current_stream(left_x.device).cuda_stream
    flags = N.MGPU_RING_LEFT_OUTER if left_outer else 0
    return _ring_call(lambda cap, n, ol, orr, od: N.lib().mgpu_ring_join_final(
        ctx.handle, isys.code, res, left_x.data_ptr(), left_y.data_ptr(), rad.ctypes.data, kit.ctypes.data,
        left_x.numel(), right_x.data_ptr(), right_y.data_ptr(), right_x.numel(), int(left_id_base),
        int(max_per_left), float(max_distance), flags, cap, n, ol, orr, od, s), left_x, max_per_left)
