// The point of a POINT / MULTIPOINT geometry column, host and device: what
// grid_pointascellid reads before pointToIndex.
//
// Reference: PointIndexGeom.nullSafeEval (expressions/index/PointIndexGeom.scala:33-47)
// decodes the row with GeometryAPI.geometry (core/geometry/api/GeometryAPI.scala:81-89:
// BinaryType -> JTS WKBReader, StringType -> JTS WKTReader) and takes getCentroid.
// For a Point the centroid is the point itself; for a MultiPoint JTS's Centroid sums the
// coordinates in order and divides by the count.  Other geometry types (whose centroid
// is JTS's area / length weighting) are reported as unsupported.  An empty point has
// no X (JTS: IllegalStateException) and is reported as such.
#pragma once
#include <stdint.h>

#include "decimal.h"

namespace mgpu {
namespace geom {

enum DecodeStatus { kDecOk = 0, kDecMalformed = 1, kDecUnsupported = 2, kDecEmpty = 3 };

MGPU_DEC uint32_t rd_u32(const uint8_t* p, bool le) {
  return le ? (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24)
            : (uint32_t)p[3] | ((uint32_t)p[2] << 8) | ((uint32_t)p[1] << 16) | ((uint32_t)p[0] << 24);
}
MGPU_DEC double rd_f64(const uint8_t* p, bool le) {
  uint64_t v = 0;
  for (int i = 0; i < 8; i++) v |= (uint64_t)p[le ? i : 7 - i] << (8 * i);
  union {
    uint64_t u;
    double d;
  } c;
  c.u = v;
  return c.d;
}

// one WKB geometry header at p: byte order, base type, coordinate dimension; advances *o
MGPU_DEC int wkb_header(const uint8_t* p, int64_t len, int64_t* o, bool* le, uint32_t* base, int* dims) {
  if (*o + 5 > len) return kDecMalformed;
  const uint8_t bo = p[*o];
  if (bo > 1) return kDecMalformed;
  *le = bo == 1;
  uint32_t t = rd_u32(p + *o + 1, *le);
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

MGPU_DEC int wkb_point_xy(const uint8_t* p, int64_t len, int64_t* o, double* x, double* y) {
  bool le;
  uint32_t t;
  int d;
  if (int s = wkb_header(p, len, o, &le, &t, &d)) return s;
  if (t != 1) return kDecUnsupported;
  if (*o + 8 * d > len) return kDecMalformed;
  *x = rd_f64(p + *o, le);
  *y = rd_f64(p + *o + 8, le);
  *o += 8 * d;
  if (*x != *x && *y != *y) return kDecEmpty;  // JTS writes POINT EMPTY as NaN NaN
  return kDecOk;
}

// centroid of a WKB Point / MultiPoint
MGPU_DEC int wkb_centroid(const uint8_t* p, int64_t len, double* x, double* y) {
  int64_t o = 0;
  bool le;
  uint32_t t;
  int d;
  if (int s = wkb_header(p, len, &o, &le, &t, &d)) return s;
  if (t == 1) {
    o = 0;
    return wkb_point_xy(p, len, &o, x, y);
  }
  if (t != 4) return kDecUnsupported;
  if (o + 4 > len) return kDecMalformed;
  const uint32_t n = rd_u32(p + o, le);
  o += 4;
  double sx = 0.0, sy = 0.0;
  uint32_t cnt = 0;
  for (uint32_t i = 0; i < n; i++) {
    double px, py;
    const int s = wkb_point_xy(p, len, &o, &px, &py);
    if (s == kDecEmpty) continue;
    if (s) return s;
    sx += px;
    sy += py;
    cnt++;
  }
  if (!cnt) return kDecEmpty;
  *x = sx / cnt;
  *y = sy / cnt;
  return kDecOk;
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
MGPU_DEC bool wkt_number(const char* s, int64_t len, int64_t* i, double* v) {
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

// centroid of a WKT POINT / MULTIPOINT
MGPU_DEC int wkt_centroid(const char* s, int64_t len, double* x, double* y) {
  int64_t i = 0;
  skip_ws(s, len, &i);
  if (keyword(s, len, &i, "point")) {
    wkt_dims(s, len, &i);
    skip_ws(s, len, &i);
    if (keyword(s, len, &i, "empty")) return kDecEmpty;
    if (!wkt_char(s, len, &i, '(') || !wkt_coord(s, len, &i, x, y) || !wkt_char(s, len, &i, ')')) return kDecMalformed;
    return kDecOk;
  }
  if (keyword(s, len, &i, "multipoint")) {
    wkt_dims(s, len, &i);
    skip_ws(s, len, &i);
    if (keyword(s, len, &i, "empty")) return kDecEmpty;
    if (!wkt_char(s, len, &i, '(')) return kDecMalformed;
    double sx = 0.0, sy = 0.0;
    uint32_t cnt = 0;
    for (;;) {
      skip_ws(s, len, &i);
      double px, py;
      if (keyword(s, len, &i, "empty")) {
      } else if (wkt_char(s, len, &i, '(')) {  // MULTIPOINT ((x y), ...)
        if (!wkt_coord(s, len, &i, &px, &py) || !wkt_char(s, len, &i, ')')) return kDecMalformed;
        sx += px, sy += py, cnt++;
      } else {  // MULTIPOINT (x y, ...)
        if (!wkt_coord(s, len, &i, &px, &py)) return kDecMalformed;
        sx += px, sy += py, cnt++;
      }
      if (wkt_char(s, len, &i, ',')) continue;
      if (wkt_char(s, len, &i, ')')) break;
      return kDecMalformed;
    }
    if (!cnt) return kDecEmpty;
    *x = sx / cnt;
    *y = sy / cnt;
    return kDecOk;
  }
  return kDecUnsupported;
}

}  // namespace geom
}  // namespace mgpu
