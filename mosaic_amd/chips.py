"""Chip tables: the rows of grid_tessellateexplode and their device form.

A chip row is ChipType (core/types/ChipType.scala:17-29): `is_core`, `index_id`
and `wkb` (JTS WKBWriter, big-endian), plus the id of the polygon it came from
(the join's output key).  ``ChipTable`` holds them in host columns; ``DeviceChips``
is the uploaded, parsed, hashed form (one device allocation, see
mosaic_amd/csrc/chip_table.h).
"""
import ctypes

import numpy as np

from . import _native as N


class ChipTable:
    """Host columns of chip rows (one row per (polygon, cell) chip)."""

    def __init__(self, cell, polygon_id, is_core, wkb_offsets, wkb, index_system=N.MGPU_H3):
        self.cell = np.ascontiguousarray(cell, dtype=np.int64)
        self.polygon_id = np.ascontiguousarray(polygon_id, dtype=np.int32)
        self.is_core = np.ascontiguousarray(is_core, dtype=np.uint8)
        self.wkb_offsets = np.ascontiguousarray(wkb_offsets, dtype=np.int64)
        self.wkb = np.ascontiguousarray(np.frombuffer(wkb, dtype=np.uint8) if isinstance(wkb, (bytes, bytearray))
                                        else wkb, dtype=np.uint8)
        self.index_system = int(index_system)
        n = self.cell.shape[0]
        assert self.polygon_id.shape[0] == n and self.is_core.shape[0] == n and self.wkb_offsets.shape[0] == n + 1

    def __len__(self):
        return self.cell.shape[0]

    def row(self, i):
        """(is_core, index_id, wkb bytes or None, polygon_id) -- MosaicChip.serialize order."""
        b, e = self.wkb_offsets[i], self.wkb_offsets[i + 1]
        return (bool(self.is_core[i]), int(self.cell[i]), bytes(self.wkb[b:e]) if e > b else None,
                int(self.polygon_id[i]))

    @classmethod
    def from_rows(cls, rows, index_system=N.MGPU_H3):
        """rows: iterable of (is_core, index_id, wkb|None, polygon_id)."""
        rows = list(rows)
        blobs = [r[2] or b"" for r in rows]
        off = np.zeros(len(rows) + 1, dtype=np.int64)
        off[1:] = np.cumsum([len(b) for b in blobs])
        return cls([r[1] for r in rows], [r[3] for r in rows], [1 if r[0] else 0 for r in rows], off,
                   np.frombuffer(b"".join(blobs) or b"", dtype=np.uint8), index_system)

    def upload(self, ctx=None):
        from .context import default_context
        return DeviceChips(self, ctx or default_context())

    def stats(self):
        return {"chips": len(self), "core": int(self.is_core.sum()), "cells": int(np.unique(self.cell).shape[0]),
                "wkb_bytes": int(self.wkb_offsets[-1])}


class DeviceChips:
    """Uploaded chip table (mgpu_chips): parsed geometry + cell hash in HBM."""

    def __init__(self, table, ctx, handle=None):
        self.ctx = ctx
        self.table = table
        if handle is None:
            h = ctypes.c_void_p()
            wkb = table.wkb if table.wkb.size else np.zeros(1, np.uint8)
            N.check(N.lib().mgpu_chips_upload(ctx.handle, table.index_system, len(table), table.cell.ctypes.data,
                                              table.polygon_id.ctypes.data, table.is_core.ctypes.data,
                                              table.wkb_offsets.ctypes.data, wkb.ctypes.data, ctypes.byref(h)))
            handle = h
        self.handle = handle

    @classmethod
    def from_device_blob(cls, ctx, ptr, nbytes, table=None):
        h = ctypes.c_void_p()
        N.check(N.lib().mgpu_chips_from_device_blob(ctx.handle, ptr, int(nbytes), ctypes.byref(h)))
        return cls(table, ctx, handle=h)

    def device_blob(self):
        p = ctypes.c_void_p()
        b = ctypes.c_int64()
        N.check(N.lib().mgpu_chips_device_blob(self.handle, ctypes.byref(p), ctypes.byref(b)))
        return p.value, b.value

    def info(self):
        a, b, c = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        N.check(N.lib().mgpu_chips_info(self.handle, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        p, n = self.device_blob()
        return {"chips": a.value, "cells": b.value, "vertices": c.value, "bytes": n}

    def close(self):
        if self.handle:
            N.lib().mgpu_chips_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Polygons:
    """A polygon set as flat rings (the input of grid_tessellateexplode).

    polygon p -> parts [poly_part_off[p], poly_part_off[p+1]);
    part q -> rings [part_ring_off[q], part_ring_off[q+1]) (first ring = shell);
    ring r -> vertices xy[ring_off[r]:ring_off[r+1]] (x = lon/easting, y = lat/northing);
    poly_type[p] (optional): the geometry's WKB type, 3 = POLYGON, 6 = MULTIPOLYGON (None:
    MULTIPOLYGON iff several parts) -- coerceChipGeometry depends on it."""

    def __init__(self, poly_id, poly_part_off, part_ring_off, ring_off, xy, poly_type=None):
        self.poly_id = np.ascontiguousarray(poly_id, dtype=np.int32)
        self.poly_part_off = np.ascontiguousarray(poly_part_off, dtype=np.int64)
        self.part_ring_off = np.ascontiguousarray(part_ring_off, dtype=np.int64)
        self.ring_off = np.ascontiguousarray(ring_off, dtype=np.int64)
        self.xy = np.ascontiguousarray(xy, dtype=np.float64).reshape(-1, 2)
        self.poly_type = None if poly_type is None else np.ascontiguousarray(poly_type, dtype=np.uint8)
        assert self.poly_type is None or self.poly_type.shape[0] == self.poly_id.shape[0]

    def __len__(self):
        return self.poly_id.shape[0]

    @classmethod
    def from_npz(cls, path):
        z = np.load(path, allow_pickle=False)
        return cls(z["poly_id"], z["poly_part_off"], z["part_ring_off"], z["ring_off"], z["xy"],
                   z["poly_type"] if "poly_type" in z.files else None)

    @classmethod
    def from_lists(cls, polys, poly_type=None):
        """polys: list of (id, [part: [ring: [(x, y), ...]]])."""
        ids, pp, pr, ro, xy = [], [0], [0], [0], []
        for pid, parts in polys:
            ids.append(pid)
            for part in parts:
                for ring in part:
                    xy.extend(ring)
                    ro.append(len(xy))
                pr.append(len(ro) - 1)
            pp.append(len(pr) - 1)
        return cls(ids, pp, pr, ro, np.array(xy, dtype=np.float64).reshape(-1, 2), poly_type)

    def select(self, idx):
        out = []
        for p in idx:
            parts = []
            for q in range(self.poly_part_off[p], self.poly_part_off[p + 1]):
                rings = []
                for r in range(self.part_ring_off[q], self.part_ring_off[q + 1]):
                    rings.append([tuple(v) for v in self.xy[self.ring_off[r]:self.ring_off[r + 1]]])
                parts.append(rings)
            out.append((int(self.poly_id[p]), parts))
        return Polygons.from_lists(out, None if self.poly_type is None else self.poly_type[list(idx)])

    def bounds(self):
        return self.xy[:, 0].min(), self.xy[:, 1].min(), self.xy[:, 0].max(), self.xy[:, 1].max()


CORE_RULES = {"mosaicfill": 0, "clip": 1, "distance": 2}
CORE_STATS = ("rows", "core", "demoted", "promoted", "dropped", "ambiguous", "carved_tests", "band_tests",
              "core_below_r", "border_above_r", "band_dropped", "dp_sensitive", "unresolved", "carved_empty",
              "overlay_chips", "multi_piece", "coerced", "coerce_nodes", "lower_dim")
CHIP_GEOMETRY = {"overlay": 0, "sutherland_hodgman": 1}


def tessellate(polygons, index_system, resolution, keep_core_geometries=True, core_rule="mosaicfill",
               chip_geometry="overlay"):
    """grid_tessellateexplode over a polygon set -> ChipTable (host C++ builder).

    ``core_rule``: "mosaicfill" (default, the reference's: core iff the cell is in
    polyfill(buffer(-r)); a border-set cell the polygon holds whole is a border chip of the
    whole cell; near r the sets follow JTS's chorded buffers), "clip" (every wholly covered
    cell is core) or "distance" (round 4's form of the reference's rule: exact distances) --
    include/mosaic_gpu.h MGPU_CORE_*.  ``chip_geometry``: "overlay" (default: border chips
    as JTS OverlayNG cuts them, mosaic_amd/csrc/jts_overlay.h) or "sutherland_hodgman" (the
    ring clip of rounds 1-5).  The table's ``core_stats``: CORE_STATS
    (mgpu_tess_result_core_stats)."""
    res = index_system.get_resolution(resolution)
    L = N.lib()
    h = ctypes.c_void_p()
    p = polygons
    st = L.mgpu_tessellate_geom(index_system.code, res, len(p), p.poly_id.ctypes.data, p.poly_part_off.ctypes.data,
                                p.part_ring_off.ctypes.data, p.ring_off.ctypes.data, p.xy.ctypes.data,
                                None if p.poly_type is None else p.poly_type.ctypes.data,
                                1 if keep_core_geometries else 0, CORE_RULES[core_rule],
                                CHIP_GEOMETRY[chip_geometry], ctypes.byref(h))
    N.check(st, "tessellation failed")
    try:
        stats = np.zeros(len(CORE_STATS), np.int64)
        N.check(L.mgpu_tess_result_core_stats(h, stats.ctypes.data, len(CORE_STATS)))
        n, b = ctypes.c_int64(), ctypes.c_int64()
        N.check(L.mgpu_tess_result_sizes(h, ctypes.byref(n), ctypes.byref(b)))
        cell = np.zeros(n.value, np.int64)
        pid = np.zeros(n.value, np.int32)
        core = np.zeros(n.value, np.uint8)
        off = np.zeros(n.value + 1, np.int64)
        wkb = np.zeros(max(b.value, 1), np.uint8)
        N.check(L.mgpu_tess_result_copy(h, cell.ctypes.data, pid.ctypes.data, core.ctypes.data, off.ctypes.data,
                                        wkb.ctypes.data))
        nu, ub = ctypes.c_int64(), ctypes.c_int64()
        N.check(L.mgpu_tess_result_undecided(h, ctypes.byref(nu), ctypes.byref(ub), None, None, None, None, None))
        ucell, upoly = np.zeros(nu.value, np.int64), np.zeros(nu.value, np.int32)
        ukkc, uoff, uwkb = np.zeros((nu.value, 3), np.uint8), np.zeros(nu.value + 1, np.int64), np.zeros(max(ub.value, 1), np.uint8)
        N.check(L.mgpu_tess_result_undecided(h, ctypes.byref(nu), ctypes.byref(ub), ucell.ctypes.data, upoly.ctypes.data,
                                             ukkc.ctypes.data, uoff.ctypes.data, uwkb.ctypes.data))
    finally:
        L.mgpu_tess_destroy(h)
    t = ChipTable(cell, pid, core, off, wkb[:b.value], index_system.code)
    t.core_stats = dict(zip(CORE_STATS, stats.tolist()))
    # the rows the core rule left undecided: kind (1 DP-sensitive, 2 on a buffer curve), kept,
    # core, and the chip the row carries (or would carry, when dropped)
    t.undecided = ChipTable(ucell, upoly, ukkc[:, 2], uoff, uwkb[:ub.value], index_system.code)
    t.undecided.kind, t.undecided.kept = ukkc[:, 0].copy(), ukkc[:, 1].copy()
    return t
