// WKB codec for chip geometries (host side).
//
// Reader: replaces the per-candidate `new WKBReader().read(bytes)` of
//   codegen/format/MosaicGeometryIOCodeGenJTS.scala:23-29 (and
//   MosaicGeometryJTS.fromWKB, core/geometry/MosaicGeometryJTS.scala:335)
// with a one-off flattening into the device chip table.  Accepts both byte orders
// (JTS WKBWriter emits big-endian; older engines little-endian),
// ISO (1000/2000/3000) and EWKB (Z/M/SRID flag) type codes; Z and M ordinates are
// dropped (JTS contains is 2-D).  Polygon, MultiPolygon and GeometryCollections
// of those are supported -- the chip types coerceChipGeometry produces
// (IndexSystem.scala:293-303).
// Writer: JTS WKBWriter layout, big-endian, 2-D, no SRID
//   (MosaicGeometryJTS.toWKB, core/geometry/MosaicGeometryJTS.scala:253).
#pragma once
#include <stdint.h>
#include <string.h>

#include <cmath>
#include <string>
#include <vector>

#include "huge_alloc.h"

namespace mgpu {
namespace wkb {

// Flattened polygons: part -> rings [part_ring[p], part_ring[p+1]),
// ring -> vertices [ring_vtx[r], ring_vtx[r+1]) in vtx (x, y pairs).
struct Flat {
  template <class T>
  using Vec = std::vector<T, HugeAlloc<T>>;  // (multi-GB for large tables: huge_alloc.h)
  Vec<uint32_t> part_ring{0};
  Vec<uint32_t> ring_vtx{0};
  Vec<double> ring_env;  // minx, miny, maxx, maxy per ring
  Vec<double> vtx;
};

struct GeomInfo {
  bool multi = false;      // not a top-level Polygon: PointLocator Mod-2 path
  bool rectangle = false;  // Polygon.isRectangle()
  int64_t n_points = 0;
  double env[4] = {INFINITY, INFINITY, -INFINITY, -INFINITY};
};

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  bool ok = true;
  uint32_t u32(bool le) {
    if (end - p < 4) {
      ok = false;
      return 0;
    }
    uint32_t v = le ? (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24)
                    : (uint32_t)p[3] | ((uint32_t)p[2] << 8) | ((uint32_t)p[1] << 16) | ((uint32_t)p[0] << 24);
    p += 4;
    return v;
  }
  double f64(bool le) {
    if (end - p < 8) {
      ok = false;
      return 0;
    }
    uint64_t v;
    memcpy(&v, p, 8);
    if (!le) v = __builtin_bswap64(v);  // (a little-endian host)
    p += 8;
    double d;
    memcpy(&d, &v, 8);
    return d;
  }
};

inline bool header(Reader& r, bool& le, uint32_t& type, int& dims, std::string& msg) {
  if (r.end - r.p < 1) {
    msg = "truncated WKB";
    return false;
  }
  uint8_t bo = *r.p++;
  if (bo > 1) {
    msg = "bad byte-order byte";
    return false;
  }
  le = bo == 1;
  uint32_t t = r.u32(le);
  bool z = (t & 0x80000000u) != 0, m = (t & 0x40000000u) != 0, srid = (t & 0x20000000u) != 0;
  t &= 0x0fffffffu;
  uint32_t iso = t / 1000;
  t %= 1000;
  if (iso == 1 || iso == 3) z = true;
  if (iso == 2 || iso == 3) m = true;
  if (srid) r.u32(le);
  type = t;
  dims = 2 + (z ? 1 : 0) + (m ? 1 : 0);
  if (!r.ok) msg = "truncated WKB";
  return r.ok;
}

inline bool read_polygon(Reader& r, bool le, int dims, Flat& f, GeomInfo& gi, std::string& msg) {
  uint32_t nr = r.u32(le);
  if (!r.ok) {
    msg = "truncated WKB";
    return false;
  }
  for (uint32_t k = 0; k < nr; k++) {
    uint32_t n = r.u32(le);
    if (!r.ok || (uint64_t)(r.end - r.p) < (uint64_t)n * 8 * dims) {
      msg = "truncated WKB ring";
      return false;
    }
    double e[4] = {INFINITY, INFINITY, -INFINITY, -INFINITY};
    const size_t v0 = f.vtx.size();
    f.vtx.resize(v0 + 2 * (size_t)n);
    double* out = f.vtx.data() + v0;
    for (uint32_t i = 0; i < n; i++) {
      double x = r.f64(le), y = r.f64(le);
      for (int d = 2; d < dims; d++) r.f64(le);
      out[2 * i] = x;
      out[2 * i + 1] = y;
      e[0] = std::fmin(e[0], x);
      e[1] = std::fmin(e[1], y);
      e[2] = std::fmax(e[2], x);
      e[3] = std::fmax(e[3], y);
    }
    gi.n_points += n;
    for (int q = 0; q < 2; q++) gi.env[q] = std::fmin(gi.env[q], e[q]);
    for (int q = 2; q < 4; q++) gi.env[q] = std::fmax(gi.env[q], e[q]);
    f.ring_env.insert(f.ring_env.end(), e, e + 4);
    f.ring_vtx.push_back((uint32_t)(f.vtx.size() / 2));
  }
  f.part_ring.push_back((uint32_t)(f.ring_vtx.size() - 1));
  return true;
}

inline bool read_any(Reader& r, Flat& f, GeomInfo& gi, std::string& msg, int depth) {
  bool le;
  uint32_t type;
  int dims;
  if (depth > 32) {
    msg = "geometry nesting too deep";
    return false;
  }
  if (!header(r, le, type, dims, msg)) return false;
  if (type == 3) return read_polygon(r, le, dims, f, gi, msg);
  if (type == 6 || type == 7) {
    uint32_t n = r.u32(le);
    if (!r.ok) {
      msg = "truncated WKB";
      return false;
    }
    for (uint32_t i = 0; i < n; i++)
      if (!read_any(r, f, gi, msg, depth + 1)) return false;
    return true;
  }
  msg = "unsupported chip geometry type " + std::to_string(type) + " (Polygon/MultiPolygon/GeometryCollection expected)";
  return false;
}

// Parse one chip; appends its parts to `f`.
inline bool parse(const uint8_t* data, size_t len, Flat& f, GeomInfo& gi, std::string& msg) {
  Reader r{data, data + len};
  bool le;
  uint32_t type;
  int dims;
  Reader peek = r;
  if (!header(peek, le, type, dims, msg)) return false;
  gi.multi = type != 3;
  if (type == 3) {
    Reader body = peek;
    size_t parts_before = f.part_ring.size();
    if (!read_polygon(body, le, dims, f, gi, msg)) return false;
    // Polygon.isRectangle(): no holes, 5-point shell on the envelope, axis-parallel edges
    uint32_t pr = (uint32_t)parts_before - 1;
    uint32_t nrings = f.part_ring[pr + 1] - f.part_ring[pr];
    const uint32_t sr = f.part_ring[pr];  // the shell ring
    const double* shell = f.vtx.data() + 2 * (size_t)f.ring_vtx[sr];
    if (nrings == 1 && f.ring_vtx[sr + 1] - f.ring_vtx[sr] == 5) {
      bool ok = true;
      for (int i = 0; i < 5 && ok; i++) {
        double x = shell[2 * i], y = shell[2 * i + 1];
        if (!(x == gi.env[0] || x == gi.env[2])) ok = false;
        if (!(y == gi.env[1] || y == gi.env[3])) ok = false;
      }
      for (int i = 1; i <= 4 && ok; i++) {
        bool xc = shell[2 * i] != shell[2 * i - 2], yc = shell[2 * i + 1] != shell[2 * i - 1];
        if (xc == yc) ok = false;
      }
      gi.rectangle = ok;
    }
    return true;
  }
  return read_any(r, f, gi, msg, 0);
}

// ---------------------------------------------------------------- writer

struct Writer {
  std::vector<uint8_t>& out;
  void u8(uint8_t v) { out.push_back(v); }
  void u32(uint32_t v) {
    for (int i = 3; i >= 0; i--) out.push_back((uint8_t)(v >> (8 * i)));
  }
  void f64(double d) {
    uint64_t v;
    memcpy(&v, &d, 8);
    for (int i = 7; i >= 0; i--) out.push_back((uint8_t)(v >> (8 * i)));
  }
};

// polygon = list of rings, ring = flat x,y list (closed)
using Ring = std::vector<double>;
using Polygon = std::vector<Ring>;

inline void write_polygon_body(Writer& w, const Polygon& p) {
  w.u32((uint32_t)p.size());
  for (const Ring& r : p) {
    w.u32((uint32_t)(r.size() / 2));
    for (double v : r) w.f64(v);
  }
}

// Polygon when one part, MultiPolygon otherwise (big-endian, 2-D)
inline void write_polygons(std::vector<uint8_t>& out, const std::vector<Polygon>& parts) {
  size_t n = parts.size() == 1 ? 5 : 9 + 5 * parts.size();
  for (const Polygon& p : parts) {
    n += 4;
    for (const Ring& r : p) n += 4 + 8 * r.size();
  }
  out.reserve(out.size() + n);
  Writer w{out};
  if (parts.size() == 1) {
    w.u8(0);
    w.u32(3);
    write_polygon_body(w, parts[0]);
    return;
  }
  w.u8(0);
  w.u32(6);
  w.u32((uint32_t)parts.size());
  for (const Polygon& p : parts) {
    w.u8(0);
    w.u32(3);
    write_polygon_body(w, p);
  }
}

// write_polygons from point rings (q.x, q.y; closed) without the flat copies: parts[k]
// a polygon's rings, or, with RingParts, every ring a polygon of its own; each ring
// reversed when `rev`.  One resize to the exact size.
template <bool RingParts, class Parts>
inline void write_polygons_pts(std::vector<uint8_t>& out, const Parts& parts, bool rev) {
  const size_t np = parts.size();
  size_t n = np == 1 ? 5 : 9 + 5 * np;
  for (const auto& p : parts) {
    if constexpr (RingParts) {
      n += 8 + 16 * p.size();
    } else {
      n += 4;
      for (const auto& r : p) n += 4 + 16 * r.size();
    }
  }
  const size_t o0 = out.size();
  out.resize(o0 + n);
  uint8_t* w = out.data() + o0;
  auto u8 = [&](uint8_t v) { *w++ = v; };
  auto u32 = [&](uint32_t v) {
    for (int i = 3; i >= 0; i--) *w++ = (uint8_t)(v >> (8 * i));
  };
  auto f64 = [&](double d) {
    uint64_t v;
    memcpy(&v, &d, 8);
    for (int i = 7; i >= 0; i--) *w++ = (uint8_t)(v >> (8 * i));
  };
  auto ring = [&](const auto& r) {
    u32((uint32_t)r.size());
    if (!rev)
      for (const auto& q : r) f64(q.x), f64(q.y);
    else
      for (size_t k = r.size(); k-- > 0;) f64(r[k].x), f64(r[k].y);
  };
  auto polygon = [&](const auto& p) {
    if constexpr (RingParts) {
      u32(1);
      ring(p);
    } else {
      u32((uint32_t)p.size());
      for (const auto& r : p) ring(r);
    }
  };
  u8(0);
  if (np == 1) {
    u32(3);
    polygon(parts[0]);
    return;
  }
  u32(6);
  u32((uint32_t)np);
  for (const auto& p : parts) {
    u8(0);
    u32(3);
    polygon(p);
  }
}

}  // namespace wkb
}  // namespace mgpu
