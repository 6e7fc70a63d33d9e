#!/usr/bin/env python3
"""Mine known-answer vectors from the reference's tests, docs and notebook outputs.

Runs in the development container only (it reads /root/reference AS TEXT; nothing
of the reference is imported or executed).  Writes small JSON / NPZ fixtures to
tests/golden/ which travel with the repo.  Sources:

* H3 (lon, lat) -> cell: every notebook / doc table that shows a point next to a
  `grid_pointascellid` / `grid_longlatascellid` column (resolution is read from
  the H3 id's own resolution bits), plus docs/source/api/spatial-indexing.rst.
* end-to-end PIP: tables showing a point next to the zone name the reference's
  `is_core OR st_contains` join assigned (Quickstart notebooks, python/sql/scala).
* BNG: src/test/.../TestBNGIndexSystem.scala and transform_join_bng.ipynb.
* ST_Contains: src/test/.../ST_ContainsBehaviors.scala.
* polygons: python/test/data/NYC_Taxi_Zones.geojson (263 zones) and
  notebooks/data/London_Postcode_Zones.geojson, converted to flat ring arrays.
"""
import base64
import glob
import html
import json
import os
import re
import sys

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


def notebook_tables(path):
    """Yield (cell_index, header, rows) for every result table in a notebook."""
    nb = json.load(open(path))
    for ci, cell in enumerate(nb.get("cells", [])):
        for o in cell.get("outputs", []):
            d = o.get("data", {})
            texts = []
            for k in ("text/html", "text/plain"):
                if k in d:
                    texts.append("".join(d[k]))
            if "text" in o:
                texts.append("".join(o["text"]))
            for t in texts:
                # HTML result tables
                for tab in re.findall(r"<table class='table-result'>(.*?)</table>", t, flags=re.S):
                    hdr = [html.unescape(x) for x in re.findall(r"<th>(.*?)</th>", tab, flags=re.S)]
                    rows = []
                    for tr in re.findall(r"<tr>(.*?)</tr>", tab.split("</thead>")[-1], flags=re.S):
                        rows.append([html.unescape(x) for x in re.findall(r"<td>(.*?)</td>", tr, flags=re.S)])
                    if hdr:
                        yield ci, hdr, rows
                # Spark .show() text tables
                lines = t.splitlines()
                i = 0
                while i < len(lines):
                    if re.match(r"^\s*\+[-+]+\+?\s*$", lines[i].replace('<div class="ansiout">', "")) and i + 2 < len(lines):
                        hdr = [h.strip() for h in lines[i + 1].strip().strip("|").split("|")]
                        rows = []
                        j = i + 3
                        while j < len(lines) and not re.match(r"^\s*\+[-+]+", lines[j]):
                            if "|" in lines[j]:
                                rows.append([c.strip() for c in lines[j].strip().strip("|").split("|")])
                            j += 1
                        if len(hdr) > 1:
                            yield ci, hdr, rows
                        i = j + 1
                    else:
                        i += 1


POINT_RE = re.compile(r"^POINT \(([-0-9.eE]+) ([-0-9.eE]+)\)$")


def is_h3(v):
    try:
        x = int(v)
    except ValueError:
        return False
    return x > 0 and (x >> 59) & 15 == 1 and (x >> 63) == 0


def point_sources(hdr, row):
    """Map prefix -> (lon, lat) from numeric lon/lat columns or WKT POINT columns."""
    src = {}
    col = {h: i for i, h in enumerate(hdr)}
    for h, i in col.items():
        if i >= len(row):
            continue
        m = POINT_RE.match(row[i])
        if m:
            pre = h.split("_")[0].lower()
            src[pre] = (float(m.group(1)), float(m.group(2)))
    for h in hdr:
        hl = h.lower()
        if hl.endswith("longitude") or hl == "lon":
            pre = hl[: -len("longitude")].rstrip("_") if hl.endswith("longitude") else ""
            lat_name = [x for x in hdr if x.lower() in (pre + "_latitude", pre + "latitude", "lat")]
            if lat_name:
                try:
                    src[pre or "pt"] = (float(row[col[h]]), float(row[col[lat_name[0]]]))
                except (ValueError, IndexError):
                    pass
    return src


def mine_h3():
    kats = {}
    files = glob.glob(REF + "/notebooks/**/*.ipynb", recursive=True) + glob.glob(REF + "/docs/**/*.ipynb", recursive=True)
    for path in sorted(files):
        rel = os.path.relpath(path, REF)
        for ci, hdr, rows in notebook_tables(path):
            cell_cols = [h for h in hdr if h.lower().endswith("_h3") or h.lower() == "ix"]
            if not cell_cols:
                continue
            for row in rows:
                src = point_sources(hdr, row)
                for cc in cell_cols:
                    i = hdr.index(cc)
                    if i >= len(row) or not is_h3(row[i]):
                        continue
                    pre = cc.lower()[:-3] if cc.lower().endswith("_h3") else None
                    pt = src.get(pre) if pre else (src.get("pt") or (list(src.values())[0] if len(src) == 1 else None))
                    if pt is None:
                        continue
                    cell = int(row[i])
                    res = (cell >> 52) & 15
                    key = (pt[0], pt[1], res)
                    if key in kats and kats[key]["cell"] != cell:
                        raise SystemExit("conflicting KAT %r" % (key,))
                    kats.setdefault(key, {"lon": pt[0], "lat": pt[1], "res": res, "cell": cell,
                                          "source": "%s cell %d" % (rel, ci)})
    # docs/source/api/spatial-indexing.rst:54-59 (grid_longlatascellid(30, 10, 10))
    rst = open(REF + "/docs/source/api/spatial-indexing.rst").read()
    assert "623385352048508927" in rst
    kats[(30.0, 10.0, 10)] = {"lon": 30.0, "lat": 10.0, "res": 10, "cell": 623385352048508927,
                              "source": "docs/source/api/spatial-indexing.rst:54-59"}
    return sorted(kats.values(), key=lambda k: (k["source"], k["lon"], k["lat"], k["res"]))


def load_zones():
    feats = [json.loads(l) for l in open(REF + "/python/test/data/NYC_Taxi_Zones.geojson") if l.strip()]
    return feats


def mine_pip(zones):
    name_to_ids = {}
    for f in zones:
        name_to_ids.setdefault(f["properties"]["zone"], []).append(int(f["properties"]["objectid"]))
    kats = {}
    files = sorted(glob.glob(REF + "/notebooks/examples/*/Quickstart*/*.ipynb") +
                   glob.glob(REF + "/notebooks/examples/*/QuickstartNotebook.ipynb"))
    for path in files:
        rel = os.path.relpath(path, REF)
        for ci, hdr, rows in notebook_tables(path):
            zcols = [h for h in hdr if h.endswith("_zone")]
            for row in rows:
                src = point_sources(hdr, row)
                for zc in zcols:
                    pre = zc[: -len("_zone")]
                    i = hdr.index(zc)
                    if pre not in src or i >= len(row) or row[i] not in name_to_ids:
                        continue
                    lon, lat = src[pre]
                    h3col = pre + "_h3"
                    cell = int(row[hdr.index(h3col)]) if h3col in hdr and is_h3(row[hdr.index(h3col)]) else None
                    kats[(lon, lat)] = {"lon": lon, "lat": lat, "zone": row[i], "objectids": name_to_ids[row[i]],
                                        "cell_r9": cell, "source": "%s cell %d" % (rel, ci)}
    return sorted(kats.values(), key=lambda k: (k["source"], k["lon"], k["lat"]))


def mine_bng():
    kats = []
    t = open(REF + "/src/test/scala/com/databricks/labs/mosaic/core/index/TestBNGIndexSystem.scala").read()
    for m in re.finditer(r"val (indexResN?\d) = BNGIndexSystem\.pointToIndex\((\d+), (\d+), (-?\d)\)", t):
        var, e, n, r = m.groups()
        exp = re.search(r"%s shouldBe (\d+)L?" % var, t).group(1)
        fmt = re.search(r"BNGIndexSystem\.format\(%s\) shouldBe \"(\w+)\"" % var, t).group(1)
        kats.append({"e": float(e), "n": float(n), "res": int(r), "cell": int(exp), "str": fmt,
                     "source": "src/test/scala/com/databricks/labs/mosaic/core/index/TestBNGIndexSystem.scala"})
    parse = []
    for m in re.finditer(r'BNGIndexSystem\.parse\("(\w+)"\) shouldBe (\d+)L?', t):
        parse.append({"str": m.group(1), "cell": int(m.group(2))})
    # transform_join_bng.ipynb cell 38: res -4 (500m) and 4 (100m) strings
    nbp = REF + "/notebooks/examples/python/TransformBNG/transform_join_bng.ipynb"
    for ci, hdr, rows in notebook_tables(nbp):
        if "uprn_bng_500m" in hdr and "uprn_bng_100m_str" in hdr:
            for row in rows:
                e = float(row[hdr.index("X_COORDINATE")])
                n = float(row[hdr.index("Y_COORDINATE")])
                kats.append({"e": e, "n": n, "res": -4, "cell": None, "str": row[hdr.index("uprn_bng_500m")],
                             "source": "notebooks/examples/python/TransformBNG/transform_join_bng.ipynb cell %d" % ci})
                kats.append({"e": e, "n": n, "res": 4, "cell": None, "str": row[hdr.index("uprn_bng_100m_str")],
                             "source": "notebooks/examples/python/TransformBNG/transform_join_bng.ipynb cell %d" % ci})
    chip = None
    e2e = None
    for ci, hdr, rows in notebook_tables(nbp):
        if "chips" in hdr:
            v = rows[0][hdr.index("chips")]
            m = re.match(r"List\((true|false), (\w+), ([A-Za-z0-9+/=]+)\)", v)
            chip = {"is_core": m.group(1) == "true", "index_id": m.group(2), "wkb_b64": m.group(3),
                    "source": "notebooks/examples/python/TransformBNG/transform_join_bng.ipynb cell %d" % ci}
        if "index_geometry" in hdr and "uprn_point" in hdr:
            row = rows[0]
            m = POINT_RE.match(row[hdr.index("uprn_point")])
            e2e = {"e": float(m.group(1)), "n": float(m.group(2)), "index_id": row[hdr.index("index_id")],
                   "postcode": row[hdr.index("Name")], "index_geometry_wkt": row[hdr.index("index_geometry")],
                   "source": "notebooks/examples/python/TransformBNG/transform_join_bng.ipynb cell %d" % ci}
    return {"point_to_index": kats, "parse": parse, "chip": chip, "join": e2e}


def mine_contains():
    t = open(REF + "/src/test/scala/com/databricks/labs/mosaic/expressions/geometry/ST_ContainsBehaviors.scala").read()
    m = re.search(r'val poly = """(.*?)"""', t, flags=re.S)
    poly = "".join(ch for ch in m.group(1).replace("|", "") if ch >= " ")
    poly = re.sub(r"\s+", " ", poly).replace("( ", "(")
    rows = re.findall(r'\(poly, "POINT \((\S+) (\S+)\)", (true|false)\)', t)
    return {"polygon_wkt": poly, "cases": [{"x": float(x), "y": float(y), "expected": e == "true"} for x, y, e in rows],
            "source": "src/test/scala/com/databricks/labs/mosaic/expressions/geometry/ST_ContainsBehaviors.scala:22-36"}


def zones_to_arrays(polys):
    """polys: list of (id, [ [ring, ring...] per part ]) -> flat arrays."""
    ids, part_off, ring_off, xy = [], [0], [0], []
    poly_part_off = [0]
    for pid, parts in polys:
        ids.append(pid)
        for part in parts:
            for ring in part:
                xy.extend(ring)
                ring_off.append(len(xy))
            part_off.append(len(ring_off) - 1)
        poly_part_off.append(len(part_off) - 1)
    return dict(poly_id=np.array(ids, np.int32), poly_part_off=np.array(poly_part_off, np.int64),
                part_ring_off=np.array(part_off, np.int64), ring_off=np.array(ring_off, np.int64),
                xy=np.array(xy, np.float64).reshape(-1, 2))


def main():
    os.makedirs(OUT, exist_ok=True)
    zones = load_zones()
    h3 = mine_h3()
    pip = mine_pip(zones)
    bng = mine_bng()
    con = mine_contains()
    json.dump({"jdk_to_radians": 8, "kats": h3}, open(os.path.join(OUT, "h3_kats.json"), "w"), indent=0)
    json.dump({"kats": pip}, open(os.path.join(OUT, "pip_kats.json"), "w"), indent=0)
    json.dump(bng, open(os.path.join(OUT, "bng_kats.json"), "w"), indent=0)
    json.dump(con, open(os.path.join(OUT, "st_contains_kats.json"), "w"), indent=0)
    polys = []
    for f in zones:
        g = f["geometry"]
        parts = g["coordinates"] if g["type"] == "MultiPolygon" else [g["coordinates"]]
        polys.append((int(f["properties"]["objectid"]), [[[(float(x), float(y)) for x, y, *_ in ring] for ring in p] for p in parts]))
    arr = zones_to_arrays(polys)
    arr["zone_name"] = np.array([f["properties"]["zone"] for f in zones])
    # the geometry's WKB type (3 POLYGON, 6 MULTIPOLYGON): coerceChipGeometry depends on it
    arr["poly_type"] = np.array([6 if f["geometry"]["type"] == "MultiPolygon" else 3 for f in zones], np.uint8)
    np.savez_compressed(os.path.join(OUT, "nyc_taxi_zones.npz"), **arr)
    lon_fc = json.load(open(REF + "/notebooks/data/London_Postcode_Zones.geojson"))
    lpolys = []
    for k, f in enumerate(lon_fc["features"]):
        g = f["geometry"]
        parts = g["coordinates"] if g["type"] == "MultiPolygon" else [g["coordinates"]]
        lpolys.append((k + 1, [[[(float(x), float(y)) for x, y, *_ in ring] for ring in p] for p in parts]))
    larr = zones_to_arrays(lpolys)
    larr["poly_type"] = np.array([6 if f["geometry"]["type"] == "MultiPolygon" else 3 for f in lon_fc["features"]], np.uint8)
    larr["name"] = np.array([str(f["properties"].get("Name", f["properties"].get("name", k))) for k, f in enumerate(lon_fc["features"])])
    np.savez_compressed(os.path.join(OUT, "london_postcode_zones.npz"), **larr)
    print("h3 kats:", len(h3), "pip kats:", len(pip), "bng kats:", len(bng["point_to_index"]),
          "zones:", len(polys), "vertices:", arr["xy"].shape[0], "london:", len(lpolys))


if __name__ == "__main__":
    main()
