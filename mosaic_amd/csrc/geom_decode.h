// The centroid of a geometry column's row, host and device: what grid_pointascellid
// reads before pointToIndex.
//
// Reference: PointIndexGeom.nullSafeEval (expressions/index/PointIndexGeom.scala:33-47)
// decodes the row with GeometryAPI.geometry (core/geometry/api/GeometryAPI.scala:81-89:
// BinaryType -> JTS WKBReader, StringType -> JTS WKTReader, HexType -> WKBReader of
// WKBReader.hexToBytes, JSONType -> GeoJsonReader) and takes getCentroid -- JTS 1.20
// org.locationtech.jts.algorithm.Centroid (restated below: area-weighted triangle fans
// from the first shell point for polygons, length-weighted segment midpoints for lines,
// the mean of the points otherwise; one accumulator over all components in order).
// Every geometry type in all four encodings (WKB / HEX with the non-strict WKBReader's
// ring repairs; WKT and GeoJSON with their readers' strict rings).  An empty geometry has
// no centroid (JTS: empty point, getX throws) and is reported as such.
#pragma once
#include <stdint.h>

#include "decimal.h"
#include "pip_core.h"

namespace mgpu {
namespace geom {

enum DecodeStatus { kDecOk = 0, kDecMalformed = 1, kDecUnsupported = 2, kDecEmpty = 3 };

// WKB bytes: raw, or the hex text of WKBReader.hexToBytes (byteLen = length / 2 -- an
// odd last character is ignored -- each a pair of hex digits of either case)
struct BinBytes {
  const uint8_t* p;
  MGPU_DEC uint8_t at(int64_t i) const { return p[i]; }
};
MGPU_DEC int hex_nibble(char c) {
  return c >= '0' && c <= '9' ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10 : (c >= 'A' && c <= 'F') ? c - 'A' + 10 : -1;
}
struct HexBytes {
  const char* s;
  MGPU_DEC uint8_t at(int64_t i) const { return (uint8_t)((hex_nibble(s[2 * i]) << 4) | hex_nibble(s[2 * i + 1])); }
};
MGPU_DEC bool hex_valid(const char* s, int64_t chars) {
  for (int64_t i = 0; i < (chars / 2) * 2; i++)
    if (hex_nibble(s[i]) < 0) return false;
  return true;
}

template <class B>
MGPU_DEC uint32_t rd_u32(const B& b, int64_t o, bool le) {
  uint32_t v = 0;
  for (int i = 0; i < 4; i++) v |= (uint32_t)b.at(o + (le ? i : 3 - i)) << (8 * i);
  return v;
}
template <class B>
MGPU_DEC double rd_f64(const B& b, int64_t o, bool le) {
  uint64_t v = 0;
  for (int i = 0; i < 8; i++) v |= (uint64_t)b.at(o + (le ? i : 7 - i)) << (8 * i);
  union {
    uint64_t u;
    double d;
  } c;
  c.u = v;
  return c.d;
}

// one WKB geometry header at o: byte order, base type, coordinate dimension; advances *o
template <class B>
MGPU_DEC int wkb_header(const B& p, int64_t len, int64_t* o, bool* le, uint32_t* base, int* dims) {
  if (*o + 5 > len) return kDecMalformed;
  const uint8_t bo = p.at(*o);
  if (bo > 1) return kDecMalformed;
  *le = bo == 1;
  uint32_t t = rd_u32(p, *o + 1, *le);
  *o += 5;
  int d = 2;
  if (t & 0x20000000u) {  // EWKB SRID
    if (*o + 4 > len) return kDecMalformed;
    *o += 4;
  }
  if (t & 0x80000000u) d++;  // EWKB Z
  if (t & 0x40000000u) d++;  // EWKB M
  t &= 0x0FFFFFFFu;
  if (t >= 1000 && t < 4000) {  // ISO Z / M / ZM
    d += (t / 1000 == 3) ? 2 : 1;
    t %= 1000;
  }
  *base = t;
  *dims = d;
  return kDecOk;
}

// A coordinate sequence inside the WKB (n points of `dims` doubles from byte o)
template <class B>
struct WkbSeq {
  const B* b;
  int64_t o;
  uint32_t n;
  int dims;
  bool le;
  MGPU_DEC double x(int64_t i) const { return rd_f64(*b, o + 8 * dims * i, le); }
  MGPU_DEC double y(int64_t i) const { return rd_f64(*b, o + 8 * dims * i + 8, le); }
};

// A coordinate sequence as JTS's non-strict WKBReader repairs it: n points, those past the
// read ones copies of the first (rings: createClosedRing) or of the last (a one-point
// LineString: extend -- the same point)
template <class S>
struct Repaired {
  S s;
  uint32_t n;
  MGPU_DEC double x(int64_t i) const { return s.x(i < (int64_t)s.n ? i : 0); }
  MGPU_DEC double y(int64_t i) const { return s.y(i < (int64_t)s.n ? i : 0); }
};

// Orientation.isCCW(CoordinateSequence) of JTS 1.20: the first highest point reached by
// a rising segment, the next lower point after it; a pointed cap by its orientation
// index, a flat cap by the direction of its top; flat or degenerate rings are not CCW
template <class S>
MGPU_DEC bool is_ccw(const S& r) {
  const int64_t n = (int64_t)r.n - 1;
  if (n < 3) return false;
  double hx = r.x(0), hy = r.y(0), prev = hy, lx = 0, ly = 0;
  int64_t hi = 0;
  for (int64_t i = 1; i <= n; i++) {
    const double py = r.y(i);
    if (py > prev && py >= hy) {
      hx = r.x(i), hy = py, hi = i;
      lx = r.x(i - 1), ly = r.y(i - 1);
    }
    prev = py;
  }
  if (hi == 0) return false;
  int64_t dl = hi;
  do {
    dl = (dl + 1) % n;
  } while (dl != hi && r.y(dl) == hy);
  const double dlx = r.x(dl), dly = r.y(dl);
  const int64_t dh = dl > 0 ? dl - 1 : n - 1;
  const double dhx = r.x(dh), dhy = r.y(dh);
  if (hx == dhx && hy == dhy) {
    if ((lx == hx && ly == hy) || (dlx == hx && dly == hy) || (lx == dlx && ly == dly)) return false;
    return pip::orientation(lx, ly, hx, hy, dlx, dly) == 1;
  }
  return dhx - hx < 0;
}

// java.lang.Math.hypot (StrictMath.hypot: fdlibm's e_hypot.c, as JDK 8 runs it), which
// JTS's Coordinate.distance calls; sqrt is correctly rounded on both sides
MGPU_DEC double jhypot(double x, double y) {
  auto hi = [](double v) { union { double d; uint64_t u; } c; c.d = v; return (int32_t)(c.u >> 32); };
  auto lo = [](double v) { union { double d; uint64_t u; } c; c.d = v; return (uint32_t)c.u; };
  auto with_hi = [](double v, int32_t h) {
    union { double d; uint64_t u; } c;
    c.d = v;
    c.u = ((uint64_t)(uint32_t)h << 32) | (c.u & 0xFFFFFFFFull);
    return c.d;
  };
  double a, b, t1, t2, y1, y2, w;
  int32_t ha = hi(x) & 0x7fffffff, hb = hi(y) & 0x7fffffff, k = 0;
  if (hb > ha) {
    a = y, b = x;
    const int32_t j = ha;
    ha = hb, hb = j;
  } else {
    a = x, b = y;
  }
  a = with_hi(a, ha);
  b = with_hi(b, hb);
  if ((ha - hb) > 0x3c00000) return a + b;
  if (ha > 0x5f300000) {
    if (ha >= 0x7ff00000) {
      w = a + b;
      if (((ha & 0xfffff) | lo(a)) == 0) w = a;
      if (((hb ^ 0x7ff00000) | lo(b)) == 0) w = b;
      return w;
    }
    ha -= 0x25800000, hb -= 0x25800000, k += 600;
    a = with_hi(a, ha);
    b = with_hi(b, hb);
  }
  if (hb < 0x20b00000) {
    if (hb <= 0x000fffff) {
      if ((hb | lo(b)) == 0) return a;
      t1 = with_hi(0.0, 0x7fd00000);
      b *= t1;
      a *= t1;
      k -= 1022;
    } else {
      ha += 0x25800000, hb += 0x25800000, k -= 600;
      a = with_hi(a, ha);
      b = with_hi(b, hb);
    }
  }
  w = a - b;
  if (w > b) {
    t1 = with_hi(0.0, ha);
    t2 = a - t1;
    w = sqrt(t1 * t1 - (b * (-b) - t2 * (a + t1)));
  } else {
    a = a + a;
    y1 = with_hi(0.0, hb);
    y2 = b - y1;
    t1 = with_hi(0.0, ha + 0x00100000);
    t2 = a - t1;
    w = sqrt(t1 * y1 - (w * (-w) - (t1 * y2 + t2 * b)));
  }
  if (k != 0) {
    t1 = with_hi(1.0, hi(1.0) + (k << 20));
    return t1 * w;
  }
  return w;
}

// org.locationtech.jts.algorithm.Centroid (JTS 1.20), accumulated component by component
struct Centroid {
  bool has_base = false;
  double bx = 0, by = 0;
  double cgx = 0, cgy = 0, area2 = 0;   // cg3, areasum2
  double lcx = 0, lcy = 0, length = 0;  // lineCentSum, totalLength
  double pcx = 0, pcy = 0;              // ptCentSum
  int64_t points = 0;
  MGPU_DEC void add_point(double x, double y) {
    points += 1;
    pcx += x;
    pcy += y;
  }
  template <class S>
  MGPU_DEC void add_line(const S& r) {
    double len = 0.0;
    for (int64_t i = 0; i + 1 < (int64_t)r.n; i++) {
      const double x0 = r.x(i), y0 = r.y(i), x1 = r.x(i + 1), y1 = r.y(i + 1);
      const double seg = jhypot(x0 - x1, y0 - y1);  // Coordinate.distance
      if (seg == 0.0) continue;
      len += seg;
      const double mx = (x0 + x1) / 2;
      lcx += seg * mx;
      const double my = (y0 + y1) / 2;
      lcy += seg * my;
    }
    length += len;
    if (len == 0.0 && r.n > 0) add_point(r.x(0), r.y(0));
  }
  template <class S>
  MGPU_DEC void add_ring(const S& r, bool shell) {
    if (shell && r.n > 0 && !has_base) {
      has_base = true;
      bx = r.x(0), by = r.y(0);
    }
    const bool positive = shell ? !is_ccw(r) : is_ccw(r);
    const double sign = positive ? 1.0 : -1.0;
    for (int64_t i = 0; i + 1 < (int64_t)r.n; i++) {
      const double x1 = r.x(i), y1 = r.y(i), x2 = r.x(i + 1), y2 = r.y(i + 1);
      const double tx = bx + x1 + x2, ty = by + y1 + y2;  // centroid3 (times 3)
      const double a2 = (x1 - bx) * (y2 - by) - (x2 - bx) * (y1 - by);
      cgx += sign * a2 * tx;
      cgy += sign * a2 * ty;
      area2 += sign * a2;
    }
    add_line(r);
  }
  MGPU_DEC int result(double* x, double* y) const {
    if (fabs(area2) > 0.0) {
      *x = cgx / 3 / area2;
      *y = cgy / 3 / area2;
    } else if (length > 0.0) {
      *x = lcx / length;
      *y = lcy / length;
    } else if (points > 0) {
      *x = pcx / points;
      *y = pcy / points;
    } else {
      return kDecEmpty;
    }
    return kDecOk;
  }
};

// Centroid of a WKB geometry (any type; collections nested up to 8 deep)
template <class B>
MGPU_DEC int wkb_centroid_any(const B& p, int64_t len, double* x, double* y) {
  Centroid c;
  int64_t o = 0;
  uint32_t left[8];  // components left at each open collection level
  int depth = 0;
  for (;;) {
    bool le;
    uint32_t t;
    int d;
    if (int s = wkb_header(p, len, &o, &le, &t, &d)) return s;
    if (t == 1) {
      if (o + 8 * d > len) return kDecMalformed;
      const double px = rd_f64(p, o, le), py = rd_f64(p, o + 8, le);
      o += 8 * d;
      if (!(px != px && py != py)) c.add_point(px, py);  // (POINT EMPTY is NaN NaN)
    } else if (t == 2 || t == 3) {
      const uint32_t rings = t == 2 ? 1u : (o + 4 <= len ? rd_u32(p, o, le) : 0xFFFFFFFFu);
      if (rings == 0xFFFFFFFFu) return kDecMalformed;
      if (t == 3) o += 4;
      for (uint32_t r = 0; r < rings; r++) {
        if (o + 4 > len) return kDecMalformed;
        WkbSeq<B> q{&p, o + 4, rd_u32(p, o, le), d, le};
        o += 4 + (int64_t)8 * d * q.n;
        if (o > len) return kDecMalformed;
        if (t == 2) {
          // WKBReader (not strict, its default) extends a one-point LineString with its
          // last point (CoordinateSequences.extend): a zero-length line
          if (q.n) c.add_line(Repaired<WkbSeq<B>>{q, q.n == 1 ? 2u : q.n});
          continue;
        }
        if (q.n == 0) {
          if (r == 0) {  // an empty shell: an empty polygon (its holes must be empty too)
            for (uint32_t h = 1; h < rings; h++) {
              if (o + 4 > len || rd_u32(p, o, le) != 0) return kDecMalformed;
              o += 4;
            }
            break;
          }
          continue;
        }
        // WKBReader (not strict) repairs a ring that is not one (CoordinateSequences.
        // ensureValidRing): fewer than 4 points are padded to 4 with the first point, an
        // open ring is closed with it
        const bool closed = q.x(0) == q.x(q.n - 1) && q.y(0) == q.y(q.n - 1);
        c.add_ring(Repaired<WkbSeq<B>>{q, q.n <= 3 ? 4u : (closed ? q.n : q.n + 1)}, r == 0);
      }
    } else if (t >= 4 && t <= 7) {
      if (o + 4 > len) return kDecMalformed;
      const uint32_t k = rd_u32(p, o, le);
      o += 4;
      if (k > 0) {
        if (depth == 8) return kDecUnsupported;
        left[depth++] = k;
        continue;
      }
    } else {
      return kDecUnsupported;
    }
    // one component done: close the collections it finishes
    while (depth > 0 && --left[depth - 1] == 0) depth--;
    if (depth == 0) break;
  }
  return c.result(x, y);
}

MGPU_DEC int wkb_centroid(const uint8_t* p, int64_t len, double* x, double* y) {
  return wkb_centroid_any(BinBytes{p}, len, x, y);
}

MGPU_DEC int hex_centroid(const char* s, int64_t chars, double* x, double* y) {
  if (!hex_valid(s, chars)) return kDecMalformed;
  return wkb_centroid_any(HexBytes{s}, chars / 2, x, y);
}

MGPU_DEC bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
MGPU_DEC void skip_ws(const char* s, int64_t len, int64_t* i) {
  while (*i < len && is_ws(s[*i])) (*i)++;
}
// case-insensitive keyword (followed by a non-letter)
MGPU_DEC bool keyword(const char* s, int64_t len, int64_t* i, const char* kw) {
  int64_t j = *i;
  for (int k = 0; kw[k]; k++, j++)
    if (j >= len || (s[j] | 32) != kw[k]) return false;
  if (j < len && (((s[j] | 32) >= 'a' && (s[j] | 32) <= 'z'))) return false;
  *i = j;
  return true;
}
__attribute__((noinline)) MGPU_DEC bool wkt_number(const char* s, int64_t len, int64_t* i, double* v) {
  skip_ws(s, len, i);
  const int64_t rest = len - *i;
  const int n = dec::parse_number(s + *i, rest > 512 ? 512 : (int)rest, v);
  if (!n) return false;
  *i += n;
  return true;
}
// "x y [z [m]]" -> x, y
MGPU_DEC bool wkt_coord(const char* s, int64_t len, int64_t* i, double* x, double* y) {
  if (!wkt_number(s, len, i, x) || !wkt_number(s, len, i, y)) return false;
  for (int k = 0; k < 2; k++) {
    int64_t j = *i;
    skip_ws(s, len, &j);
    if (j < len && s[j] != ')' && s[j] != ',') {
      double z;
      if (!wkt_number(s, len, i, &z)) return false;
    }
  }
  return true;
}
MGPU_DEC bool wkt_char(const char* s, int64_t len, int64_t* i, char c) {
  skip_ws(s, len, i);
  if (*i < len && s[*i] == c) {
    (*i)++;
    return true;
  }
  return false;
}
MGPU_DEC void wkt_dims(const char* s, int64_t len, int64_t* i) {
  skip_ws(s, len, i);
  if (!keyword(s, len, i, "zm") && !keyword(s, len, i, "z")) keyword(s, len, i, "m");
}

// ---------------------------------------------------------------- GeoJSON (JTS GeoJsonReader)
// A value at *i skipped (string, number, literal, array, object); false if malformed
MGPU_DEC bool json_skip(const char* s, int64_t len, int64_t* i) {
  skip_ws(s, len, i);
  if (*i >= len) return false;
  if (s[*i] == '"') {
    for ((*i)++; *i < len; (*i)++) {
      if (s[*i] == '\\') {
        (*i)++;
        continue;
      }
      if (s[*i] == '"') {
        (*i)++;
        return true;
      }
    }
    return false;
  }
  if (s[*i] == '[' || s[*i] == '{') {
    int depth = 0;
    bool str = false;
    for (; *i < len; (*i)++) {
      const char c = s[*i];
      if (str) {
        if (c == '\\') (*i)++;
        else if (c == '"') str = false;
        continue;
      }
      if (c == '"') str = true;
      else if (c == '[' || c == '{') depth++;
      else if (c == ']' || c == '}') {
        if (--depth == 0) {
          (*i)++;
          return true;
        }
      }
    }
    return false;
  }
  const int64_t b = *i;
  while (*i < len && s[*i] != ',' && s[*i] != '}' && s[*i] != ']' && !is_ws(s[*i])) (*i)++;
  return *i > b;
}
// a JSON string at *i equal to `w` (no escapes in the keys and type names compared)
MGPU_DEC bool json_str_is(const char* s, int64_t len, int64_t i, int64_t e, const char* w) {
  int64_t k = 0;
  for (; w[k]; k++)
    if (i + 1 + k >= e || s[i + 1 + k] != w[k]) return false;
  return i + 1 + k == e - 1;
}
// "[x, y, ...]" -> x, y (n = the count of numbers read, 0 for "[]")
MGPU_DEC bool json_position(const char* s, int64_t len, int64_t* i, double* x, double* y, int* n) {
  *n = 0;
  if (!wkt_char(s, len, i, '[')) return false;
  if (wkt_char(s, len, i, ']')) return true;
  for (;;) {
    double v;
    if (!wkt_number(s, len, i, &v)) return false;
    if (*n == 0) *x = v;
    if (*n == 1) *y = v;
    (*n)++;
    if (wkt_char(s, len, i, ',')) continue;
    return wkt_char(s, len, i, ']') && *n >= 2;
  }
}
// A coordinate sequence in text -- WKT "(x y, x y, ...)" (J = false) or GeoJSON
// "[[x, y], [x, y], ...]" (J = true) -- whose opening bracket is at offset b, n points,
// read by a forward cursor (the Centroid and isCCW walks visit points in order, stepping
// back one at most; an earlier point restarts the cursor).  Validated by text_seq_scan.
template <bool J>
struct TextSeq {
  const char* s;
  int64_t len, b;
  uint32_t n;
  mutable int64_t k = -1, pos = 0;
  mutable double cx = 0, cy = 0, px = 0, py = 0;
  // (out of line: the centroid walks call it from many places, and the decimal parser
  // inlined into each made the device code of the decode kernel ~4x larger)
  __attribute__((noinline)) MGPU_DEC void step() const {
    if (k < 0) pos = b + 1;
    else wkt_char(s, len, &pos, ',');
    px = cx, py = cy;
    if (J) {
      int m;
      json_position(s, len, &pos, &cx, &cy, &m);
    } else {
      wkt_coord(s, len, &pos, &cx, &cy);
    }
    k++;
  }
  __attribute__((noinline)) MGPU_DEC void seek(int64_t i) const {
    if (i < k - 1) k = -1;
    while (k < i) step();
  }
  __attribute__((noinline)) MGPU_DEC double x(int64_t i) const {
    seek(i);
    return i == k ? cx : px;
  }
  __attribute__((noinline)) MGPU_DEC double y(int64_t i) const {
    seek(i);
    return i == k ? cy : py;
  }
};

// The sequence at *i ("(" coords ")" / "[" positions "]"): its offset and point count,
// *i past it; the first and last points (rings: closure).  False if malformed (GeoJSON: a
// position with fewer than two numbers; "[]" is an empty sequence).
template <bool J>
MGPU_DEC bool text_seq_scan(const char* s, int64_t len, int64_t* i, TextSeq<J>* q, double* x0, double* y0,
                            double* x1, double* y1) {
  skip_ws(s, len, i);
  q->s = s, q->len = len, q->b = *i, q->n = 0;
  if (!wkt_char(s, len, i, J ? '[' : '(')) return false;
  if (J && wkt_char(s, len, i, ']')) return true;
  for (;;) {
    double x, y;
    if (J) {
      int m;
      if (!json_position(s, len, i, &x, &y, &m) || m < 2) return false;
    } else if (!wkt_coord(s, len, i, &x, &y)) {
      return false;
    }
    if (q->n == 0) *x0 = x, *y0 = y;
    *x1 = x, *y1 = y;
    q->n++;
    if (wkt_char(s, len, i, ',')) continue;
    return wkt_char(s, len, i, J ? ']' : ')');
  }
}

// A LineString / LinearRing sequence into the accumulator, as JTS's WKTReader and
// GeoJsonReader build them (strict: a LineString of one point and a ring that is not
// closed or has fewer than 4 points throw -- malformed)
template <bool J>
MGPU_DEC int text_line(const char* s, int64_t len, int64_t* i, Centroid& c) {
  TextSeq<J> q;
  double x0, y0, x1, y1;
  if (!text_seq_scan<J>(s, len, i, &q, &x0, &y0, &x1, &y1)) return kDecMalformed;
  if (q.n == 1) return kDecMalformed;
  if (q.n) c.add_line(q);
  return kDecOk;
}
template <bool J>
MGPU_DEC int text_polygon(const char* s, int64_t len, int64_t* i, Centroid& c) {
  if (!wkt_char(s, len, i, J ? '[' : '(')) return kDecMalformed;
  if (J && wkt_char(s, len, i, ']')) return kDecOk;  // an empty polygon
  for (int r = 0;; r++) {
    TextSeq<J> q;
    double x0, y0, x1, y1;
    if (!text_seq_scan<J>(s, len, i, &q, &x0, &y0, &x1, &y1)) return kDecMalformed;
    if (q.n == 0) {
      if (r == 0) return kDecMalformed;  // (an empty shell with holes)
    } else {
      if (q.n < 4 || x0 != x1 || y0 != y1) return kDecMalformed;
      c.add_ring(q, r == 0);
    }
    if (wkt_char(s, len, i, ',')) continue;
    return wkt_char(s, len, i, J ? ']' : ')') ? kDecOk : kDecMalformed;
  }
}

// JTS Centroid of a WKT geometry (WKTReader: every type, Z / M / ZM, EMPTY members,
// collections nested up to 8 deep)
MGPU_DEC int wkt_centroid(const char* s, int64_t len, double* x, double* y) {
  Centroid c;
  int64_t i = 0;
  int depth = 0;  // open GEOMETRYCOLLECTION levels
  for (;;) {
    skip_ws(s, len, &i);
    int t = 0;
    if (keyword(s, len, &i, "point")) t = 1;
    else if (keyword(s, len, &i, "linestring")) t = 2;
    else if (keyword(s, len, &i, "linearring")) t = 8;
    else if (keyword(s, len, &i, "polygon")) t = 3;
    else if (keyword(s, len, &i, "multipoint")) t = 4;
    else if (keyword(s, len, &i, "multilinestring")) t = 5;
    else if (keyword(s, len, &i, "multipolygon")) t = 6;
    else if (keyword(s, len, &i, "geometrycollection")) t = 7;
    else return depth == 0 && i < len && (s[i] | 32) >= 'a' && (s[i] | 32) <= 'z' ? kDecUnsupported : kDecMalformed;
    wkt_dims(s, len, &i);
    skip_ws(s, len, &i);
    if (!keyword(s, len, &i, "empty")) {
      int st = kDecOk;
      if (t == 1) {
        double px, py;
        if (!wkt_char(s, len, &i, '(') || !wkt_coord(s, len, &i, &px, &py) || !wkt_char(s, len, &i, ')')) return kDecMalformed;
        c.add_point(px, py);
      } else if (t == 2) {
        st = text_line<false>(s, len, &i, c);
      } else if (t == 8) {  // a LinearRing: closed, at least 4 points; its centroid is a line's
        TextSeq<false> q;
        double x0, y0, x1, y1;
        if (!text_seq_scan<false>(s, len, &i, &q, &x0, &y0, &x1, &y1) || q.n < 4 || x0 != x1 || y0 != y1) return kDecMalformed;
        c.add_line(q);
      } else if (t == 3) {
        st = text_polygon<false>(s, len, &i, c);
      } else if (t == 7) {
        if (!wkt_char(s, len, &i, '(')) return kDecMalformed;
        if (depth == 8) return kDecUnsupported;
        depth++;
        continue;  // its first member
      } else {
        if (!wkt_char(s, len, &i, '(')) return kDecMalformed;
        for (;;) {
          skip_ws(s, len, &i);
          if (keyword(s, len, &i, "empty")) {
          } else if (t == 4) {
            double px, py;
            const bool paren = wkt_char(s, len, &i, '(');  // MULTIPOINT ((x y), ...) or (x y, ...)
            if (!wkt_coord(s, len, &i, &px, &py) || (paren && !wkt_char(s, len, &i, ')'))) return kDecMalformed;
            c.add_point(px, py);
          } else {
            st = t == 5 ? text_line<false>(s, len, &i, c) : text_polygon<false>(s, len, &i, c);
            if (st) return st;
          }
          if (wkt_char(s, len, &i, ',')) continue;
          if (wkt_char(s, len, &i, ')')) break;
          return kDecMalformed;
        }
      }
      if (st) return st;
    }
    // one geometry done: close the collections it ends
    bool next = false;
    while (depth > 0 && !next) {
      if (wkt_char(s, len, &i, ',')) next = true;
      else if (wkt_char(s, len, &i, ')')) depth--;
      else return kDecMalformed;
    }
    if (!next) break;
  }
  return c.result(x, y);
}


// The members "type" (its string's extent), "coordinates" and "geometries" (value
// offsets, -1 if absent) of the GeoJSON object at *i; *i past it
MGPU_DEC bool json_object(const char* s, int64_t len, int64_t* i, int64_t* type_b, int64_t* type_e, int64_t* coord,
                          int64_t* geoms) {
  *type_b = *type_e = *coord = *geoms = -1;
  if (!wkt_char(s, len, i, '{')) return false;
  if (wkt_char(s, len, i, '}')) return true;
  for (;;) {
    skip_ws(s, len, i);
    const int64_t kb = *i;
    if (!json_skip(s, len, i)) return false;
    const int64_t ke = *i;
    if (!wkt_char(s, len, i, ':')) return false;
    skip_ws(s, len, i);
    const int64_t vb = *i;
    if (!json_skip(s, len, i)) return false;
    if (json_str_is(s, len, kb, ke, "type")) *type_b = vb, *type_e = *i;
    if (json_str_is(s, len, kb, ke, "coordinates")) *coord = vb;
    if (json_str_is(s, len, kb, ke, "geometries")) *geoms = vb;
    if (wkt_char(s, len, i, ',')) continue;
    return wkt_char(s, len, i, '}');
  }
}

// JTS Centroid of a GeoJSON geometry (GeoJsonReader: every type, members in any order,
// GeometryCollection "geometries" nested up to 8 deep)
MGPU_DEC int json_centroid(const char* s, int64_t len, double* x, double* y) {
  Centroid c;
  int64_t stack[8];  // per open collection: the offset of its next member
  int depth = 0;
  int64_t at = 0;
  for (;;) {
    int64_t tb, te, coord, geoms;
    if (!json_object(s, len, &at, &tb, &te, &coord, &geoms)) return kDecMalformed;
    if (tb < 0 || s[tb] != '"') return kDecMalformed;
    int t = 0;
    const char* names[] = {"Point", "LineString", "Polygon", "MultiPoint", "MultiLineString", "MultiPolygon",
                           "GeometryCollection"};
    for (int k = 0; k < 7 && !t; k++)
      if (json_str_is(s, len, tb, te, names[k])) t = k + 1;
    if (!t) return kDecMalformed;
    if (t == 7) {
      if (geoms < 0) return kDecMalformed;
      int64_t j = geoms;
      if (!wkt_char(s, len, &j, '[')) return kDecMalformed;
      if (!wkt_char(s, len, &j, ']')) {
        if (depth == 8) return kDecUnsupported;
        stack[depth++] = at;
        at = j;
        continue;  // its first member
      }
    } else {
      if (coord < 0) return kDecMalformed;
      int64_t j = coord;
      int st = kDecOk;
      if (t == 1) {
        double px, py;
        int m;
        if (!json_position(s, len, &j, &px, &py, &m) || m == 1) return kDecMalformed;
        if (m) c.add_point(px, py);
      } else if (t == 2) {
        st = text_line<true>(s, len, &j, c);
      } else if (t == 3) {
        st = text_polygon<true>(s, len, &j, c);
      } else {
        if (!wkt_char(s, len, &j, '[')) return kDecMalformed;
        if (!wkt_char(s, len, &j, ']')) {
          for (;;) {
            if (t == 4) {
              double px, py;
              int m;
              if (!json_position(s, len, &j, &px, &py, &m) || m == 1) return kDecMalformed;
              if (m) c.add_point(px, py);
            } else {
              st = t == 5 ? text_line<true>(s, len, &j, c) : text_polygon<true>(s, len, &j, c);
              if (st) return st;
            }
            if (wkt_char(s, len, &j, ',')) continue;
            if (wkt_char(s, len, &j, ']')) break;
            return kDecMalformed;
          }
        }
      }
      if (st) return st;
    }
    // one member done: the next one of its collection, or close collections
    bool next = false;
    while (depth > 0 && !next) {
      if (wkt_char(s, len, &at, ',')) next = true;
      else if (wkt_char(s, len, &at, ']')) at = stack[--depth];
      else return kDecMalformed;
    }
    if (!next) break;
  }
  return c.result(x, y);
}

// ---------------------------------------------------------------- Mosaic's InternalGeometryType
// (core/types/model/InternalGeometry.scala: typeId, boundaries, holes; read by
// MosaicGeometryJTS.fromInternal :343-357): flattened -- the row's parts [row_part[r],
// row_part[r + 1]), part q's rings [part_ring[q], part_ring[q + 1]) (the boundary, then
// its holes), ring k's points xy[2 ring_off[k] ..].  Type ids of GeometryTypeEnum:
// POINT 1 (boundaries.head.head), MULTIPOINT 2 (boundaries.head), LINESTRING 3
// (boundaries.head), MULTILINESTRING 4 (each boundary), POLYGON 5 (boundaries.head +
// holes.head), MULTIPOLYGON 6 (each boundary with its holes).
struct FlatSeq {
  const double* xy;
  int64_t b;
  uint32_t n;
  MGPU_DEC double x(int64_t i) const { return xy[2 * (b + i)]; }
  MGPU_DEC double y(int64_t i) const { return xy[2 * (b + i) + 1]; }
};
MGPU_DEC int internal_centroid(int type_id, int64_t p0, int64_t p1, const int64_t* part_ring, const int64_t* ring_off,
                                const double* xy, double* x, double* y) {
  Centroid c;
  if (type_id < 1 || type_id > 6) return kDecUnsupported;
  if (p1 <= p0) return (type_id == 4 || type_id == 6) ? kDecEmpty : kDecMalformed;  // (.head of no boundary)
  const int64_t last = (type_id == 4 || type_id == 6) ? p1 : p0 + 1;
  for (int64_t q = p0; q < last; q++) {
    const int64_t r0 = part_ring[q], r1 = part_ring[q + 1];
    if (r1 <= r0) continue;
    if (type_id <= 4) {
      const FlatSeq seq{xy, ring_off[r0], (uint32_t)(ring_off[r0 + 1] - ring_off[r0])};
      if (type_id == 1) {
        if (seq.n == 0) return kDecMalformed;  // (boundaries.head.head of an empty list)
        c.add_point(seq.x(0), seq.y(0));
      } else if (type_id == 2) {
        for (uint32_t k = 0; k < seq.n; k++) c.add_point(seq.x(k), seq.y(k));
      } else {
        if (seq.n == 1) return kDecMalformed;
        if (seq.n) c.add_line(seq);
      }
      continue;
    }
    for (int64_t r = r0; r < r1; r++) {
      const FlatSeq seq{xy, ring_off[r], (uint32_t)(ring_off[r + 1] - ring_off[r])};
      if (seq.n == 0) {
        if (r == r0) {  // an empty shell: an empty polygon, whose holes must be empty too
          for (int64_t h = r0 + 1; h < r1; h++)
            if (ring_off[h + 1] > ring_off[h]) return kDecMalformed;
          break;
        }
        continue;
      }
      if (seq.n < 4 || seq.x(0) != seq.x(seq.n - 1) || seq.y(0) != seq.y(seq.n - 1)) return kDecMalformed;
      c.add_ring(seq, r == r0);
    }
  }
  return c.result(x, y);
}

}  // namespace geom
}  // namespace mgpu
