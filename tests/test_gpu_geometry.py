"""grid_pointascellid on WKB / WKT geometry columns and the Arrow columnar entry, on the GPU.

Reference: PointIndexGeom.nullSafeEval (expressions/index/PointIndexGeom.scala:33-47)
decodes each row with JTS (GeometryAPI.scala:81-89), takes the centroid and indexes it;
its test (PointIndexBehaviors.scala:25-50) checks point_index_geom(centroid) against
point_index_lonlat(st_x(centroid), st_y(centroid)), and that a POLYGON EMPTY row throws
(PointIndexBehaviors.scala:134-137).  Here the cells of decoded rows must equal the
oracle's cells of the same doubles (Python's float() reads WKT text exactly as
Double.parseDouble), null rows give a 0 validity bit.
"""
import struct

import numpy as np
import pytest
import torch

import mosaic_amd as M
import oracle as O
from mosaic_amd import arrow as A
from geom_util import nyc_points

pytestmark = pytest.mark.gpu


def T(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(dev)


def wkb_point(x, y, le=True):
    bo = "<" if le else ">"
    return struct.pack(bo + "BIdd", 1 if le else 0, 1, x, y)


def test_wkt_points_h3_equal_oracle(gpu):
    x, y = nyc_points(50_000, 31)
    rows = []
    for i, (a, b) in enumerate(zip(x, y)):
        fmt = ["POINT (%r %r)", "POINT(%.6f %.6f)", "point z (%.15g %.17g 7)", "POINT (%.3e %.9e)"][i % 4]
        rows.append(fmt % (float(a), float(b)))
    xs = np.array([float(r.split("(")[1].split()[0]) for r in rows])
    ys = np.array([float(r.split("(")[1].split()[1].rstrip(")")) for r in rows])
    col = M.GeometryColumn.from_rows(rows, gpu)
    got = M.grid_pointascellid(col, 9).cpu().numpy()
    assert np.array_equal(got, O.h3_points_to_cells(xs, ys, 9))
    # the same column through the Arrow entry, int32 and int64 offsets
    for large in (False, True):
        c2, v2 = A.grid_pointascellid_arrow(col, 9, large=large)
        assert np.array_equal(c2.cpu().numpy(), got)
        assert np.all(np.unpackbits(v2.cpu().numpy(), bitorder="little")[:len(rows)] == 1)


def test_wkb_points_and_multipoints_bng(gpu):
    rng = np.random.default_rng(32)
    n = 20_000
    e = rng.uniform(503000, 561000, n)
    nn = rng.uniform(155000, 201000, n)
    rows, ex, ey = [], [], []
    for i in range(n):
        if i % 5 == 0:  # a 3-point MULTIPOINT: its centroid (JTS Centroid: sum / count)
            pts = [(e[i], nn[i]), (e[i] + 10.5, nn[i] - 3.25), (e[i] - 7.0, nn[i] + 1.0)]
            rows.append(struct.pack("<BII", 1, 4, 3) + b"".join(wkb_point(*p, le=(k % 2 == 0))
                                                                for k, p in enumerate(pts)))
            ex.append((pts[0][0] + pts[1][0] + pts[2][0]) / 3)
            ey.append((pts[0][1] + pts[1][1] + pts[2][1]) / 3)
        else:
            rows.append(wkb_point(e[i], nn[i], le=i % 3 != 0))
            ex.append(e[i])
            ey.append(nn[i])
    col = M.GeometryColumn.from_rows(rows, gpu)
    for res in (3, -4):
        got = M.grid_pointascellid(col, res, index_system=M.BNGIndexSystem()).cpu().numpy()
        assert np.array_equal(got, O.bng_points_to_cells(np.array(ex), np.array(ey), res))


def test_null_rows_and_errors(gpu):
    rows = ["POINT (-73.95 40.77)", None, "POINT (-73.90 40.70)", None]
    c, v = M.grid_pointascellid(M.GeometryColumn.from_rows(rows, gpu), 9)
    c = c.cpu().numpy()
    assert np.unpackbits(v.cpu().numpy(), bitorder="little")[:4].tolist() == [1, 0, 1, 0]
    assert c[1] == 0 and c[3] == 0
    assert c[0] == O.h3_points_to_cells(np.array([-73.95]), np.array([40.77]), 9)[0]
    with pytest.raises(M.MosaicGpuError):  # PointIndexBehaviors.scala:134-137
        M.grid_pointascellid(M.GeometryColumn.from_rows(["POLYGON EMPTY"], gpu), 5)
    with pytest.raises(M.IllegalStateException):
        M.grid_pointascellid(M.GeometryColumn.from_rows(["POINT EMPTY"], gpu), 5)
    with pytest.raises(M.MosaicGpuError):
        M.grid_pointascellid(M.GeometryColumn.from_rows(["POINT (1 2"], gpu), 5)
    with pytest.raises(M.IllegalArgumentException):  # H3 geoToH3 on a NaN coordinate
        M.grid_pointascellid(M.GeometryColumn.from_rows(["POINT (NaN 5)"], gpu), 5)


def test_pip_join_arrow_nulls_offsets_and_ids(gpu, nyc_chips_r9):
    x, y = nyc_points(200_000, 33)
    rng = np.random.default_rng(34)
    present = rng.random(len(x)) > 0.1
    off = 123
    d = nyc_chips_r9.upload()
    xc = A.float64_column(T(x, gpu), present, offset=off)
    yc = A.float64_column(T(y, gpu), offset=off)
    r = A.pip_join_arrow(xc, yc, d, 9)
    gp, gq = r.numpy()
    sel = np.nonzero(present[off:])[0]
    op, oq = O.pip_join(0, 9, x[off:][sel], y[off:][sel], nyc_chips_r9.cell, nyc_chips_r9.polygon_id,
                        nyc_chips_r9.is_core, nyc_chips_r9.wkb_offsets, nyc_chips_r9.wkb)
    # default ids: array offset + row index
    assert np.array_equal(gp, sel[op] + off) and np.array_equal(gq, oq)
    # explicit point ids
    ids = np.arange(len(x), dtype=np.int64) * 3 + 5
    pc = A.DeviceColumn(len(x) - off, [None, torch.from_numpy(ids).to(gpu)], offset=off)
    r2 = A.pip_join_arrow(xc, yc, d, 9, point_id_col=pc)
    assert np.array_equal(r2.numpy()[0], ids[off:][sel[op]])
    # the plain entry on the same points agrees
    r3 = M.pip_join(T(x[off:][sel], gpu), T(y[off:][sel], gpu), d, 9)
    assert np.array_equal(r3.numpy()[1], gq)


def test_pip_join_arrow_rejects_host_arrays(gpu, nyc_chips_r9):
    x, y = nyc_points(100, 35)
    d = nyc_chips_r9.upload()
    xc = A.float64_column(T(x, gpu))
    yc = A.float64_column(T(y, gpu))
    yc.struct.device_type = 1  # ARROW_DEVICE_CPU
    with pytest.raises(M.IllegalArgumentException):
        A.pip_join_arrow(xc, yc, d, 9)


def test_centroids_of_any_geometry_on_gpu(gpu):
    """Polygons (holes, both orientations), multipolygons, lines, collections as WKB, the
    same rows as hex text, as Mosaic's InternalGeometryType layout, as WKT and as GeoJSON:
    the device cells equal the oracle's cells of the JTS Centroid restatement
    (oracle/jts_centroid.py); a POLYGON EMPTY row raises as getX on the empty centroid
    (PointIndexBehaviors.scala:134-137)."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import jts_centroid as JC
    from test_geom_host import _internal_rows, _random_geoms, w_geom
    geoms = _random_geoms(21, 3000)
    wkbs = [w_geom(*g, le=(i % 2 == 0)) for i, g in enumerate(geoms)]
    cx, cy = np.array([JC.centroid_wkb(w) for w in wkbs]).T
    for res in (5, 9, 12):
        want = O.h3_points_to_cells(cx, cy, res)
        got = M.grid_pointascellid(M.GeometryColumn.from_rows(wkbs, gpu), res).cpu().numpy()
        assert np.array_equal(got, want), res
        hexes = [w.hex() if i % 3 else w.hex().upper() for i, w in enumerate(wkbs)]
        got = M.grid_pointascellid(M.GeometryColumn.from_rows(hexes, gpu, fmt="hex"), res).cpu().numpy()
        assert np.array_equal(got, want), res
    sel = [i for i, g in enumerate(geoms) if g[0] != "collection"]
    col = M.InternalGeometryColumn.from_rows(_internal_rows([geoms[i] for i in sel]), gpu)
    got = M.grid_pointascellid(col, 9).cpu().numpy()
    assert np.array_equal(got, O.h3_points_to_cells(cx[sel], cy[sel], 9))
    js = ['{"type": "Point", "coordinates": [%r, %r]}' % (float(a), float(b)) for a, b in zip(cx[:500], cy[:500])]
    got = M.grid_pointascellid(M.GeometryColumn.from_rows(js, gpu, fmt="geojson"), 9).cpu().numpy()
    assert np.array_equal(got, O.h3_points_to_cells(cx[:500], cy[:500], 9))
    # every type as WKT (StringType) and GeoJSON (JSONType) text: the device's text readers
    from test_geom_host import _json, _wkt
    want = O.h3_points_to_cells(cx, cy, 9)
    for fmt, rows in (("wkt", [_wkt(*g, z=(i % 5 == 0)) for i, g in enumerate(geoms)]),
                      ("geojson", [_json(*g) for g in geoms])):
        got = M.grid_pointascellid(M.GeometryColumn.from_rows(rows, gpu, fmt=fmt), 9).cpu().numpy()
        assert np.array_equal(got, want), fmt
    with pytest.raises(M.IllegalStateException):
        M.grid_pointascellid(M.GeometryColumn.from_rows([struct.pack("<BII", 1, 3, 0)], gpu), 5)
