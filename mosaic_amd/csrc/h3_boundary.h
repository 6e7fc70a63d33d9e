// H3 v3.7 cell geometry on the host: h3ToGeoBoundary (and h3ToGeo) for the chip-table
// builder.  Replaces H3IndexSystem.indexToGeometry (H3IndexSystem.scala:103-111:
// h3.h3ToGeoBoundary(index) closed into a ring), which Mosaic intersects with the polygon
// to make each chip (IndexSystem.getBorderChips / getCoreChips, IndexSystem.scala:178-213).
//
// Restated from H3 v3.7 (com.uber:h3:3.7.0, not vendored in the reference):
//   _h3ToFaceIjk (base cell home FaceIJK + digits, overage onto the face the centre lies
//   on), _faceIjkToVerts / _faceIjkPentToVerts (the aperture-33r(7r) substrate vertices),
//   _adjustOverageClassII (faceNeighbors: rotate + translate into the adjacent face),
//   _faceIjkToGeoBoundary / _faceIjkPentToGeoBoundary (a vertex per substrate vertex, each
//   projected with the gnomonic of the face it lies on, plus a "distortion" vertex where
//   a Class III edge crosses an icosahedron edge), _hex2dToGeo, _geoAzDistanceRads.
// The faceNeighbors table is H3's; tools/check_h3_face_neighbors.py re-derives every
// entry from the icosahedron geometry.  Long-double expressions are emulated exactly
// (h3_exact.h); sin/cos/atan/asin/atan2 are the host's libm, as for H3's JNI library.
#pragma once
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <vector>

#include "h3_core.h"

namespace mgpu {
namespace h3b {

using h3::IJK;
namespace X = mgpu::exact;

struct FaceIJK {
  int face;
  IJK c;
};

// faceNeighbors[face][quadrant]: {neighbour face, translation (res-0 units), ccw 60 rotations}
// quadrants: 0 = central, 1 = IJ, 2 = KI, 3 = JK (H3 faceijk.c)
struct FaceOrient {
  int face;
  int ti, tj, tk;
  int rot;
};
static const FaceOrient kFaceNeighbors[20][4] = {
    {{0, 0, 0, 0, 0}, {4, 2, 0, 2, 1}, {1, 2, 2, 0, 5}, {5, 0, 2, 2, 3}},
    {{1, 0, 0, 0, 0}, {0, 2, 0, 2, 1}, {2, 2, 2, 0, 5}, {6, 0, 2, 2, 3}},
    {{2, 0, 0, 0, 0}, {1, 2, 0, 2, 1}, {3, 2, 2, 0, 5}, {7, 0, 2, 2, 3}},
    {{3, 0, 0, 0, 0}, {2, 2, 0, 2, 1}, {4, 2, 2, 0, 5}, {8, 0, 2, 2, 3}},
    {{4, 0, 0, 0, 0}, {3, 2, 0, 2, 1}, {0, 2, 2, 0, 5}, {9, 0, 2, 2, 3}},
    {{5, 0, 0, 0, 0}, {10, 2, 2, 0, 3}, {14, 2, 0, 2, 3}, {0, 0, 2, 2, 3}},
    {{6, 0, 0, 0, 0}, {11, 2, 2, 0, 3}, {10, 2, 0, 2, 3}, {1, 0, 2, 2, 3}},
    {{7, 0, 0, 0, 0}, {12, 2, 2, 0, 3}, {11, 2, 0, 2, 3}, {2, 0, 2, 2, 3}},
    {{8, 0, 0, 0, 0}, {13, 2, 2, 0, 3}, {12, 2, 0, 2, 3}, {3, 0, 2, 2, 3}},
    {{9, 0, 0, 0, 0}, {14, 2, 2, 0, 3}, {13, 2, 0, 2, 3}, {4, 0, 2, 2, 3}},
    {{10, 0, 0, 0, 0}, {5, 2, 2, 0, 3}, {6, 2, 0, 2, 3}, {15, 0, 2, 2, 3}},
    {{11, 0, 0, 0, 0}, {6, 2, 2, 0, 3}, {7, 2, 0, 2, 3}, {16, 0, 2, 2, 3}},
    {{12, 0, 0, 0, 0}, {7, 2, 2, 0, 3}, {8, 2, 0, 2, 3}, {17, 0, 2, 2, 3}},
    {{13, 0, 0, 0, 0}, {8, 2, 2, 0, 3}, {9, 2, 0, 2, 3}, {18, 0, 2, 2, 3}},
    {{14, 0, 0, 0, 0}, {9, 2, 2, 0, 3}, {5, 2, 0, 2, 3}, {19, 0, 2, 2, 3}},
    {{15, 0, 0, 0, 0}, {16, 2, 0, 2, 1}, {19, 2, 2, 0, 5}, {10, 0, 2, 2, 3}},
    {{16, 0, 0, 0, 0}, {17, 2, 0, 2, 1}, {15, 2, 2, 0, 5}, {11, 0, 2, 2, 3}},
    {{17, 0, 0, 0, 0}, {18, 2, 0, 2, 1}, {16, 2, 2, 0, 5}, {12, 0, 2, 2, 3}},
    {{18, 0, 0, 0, 0}, {19, 2, 0, 2, 1}, {17, 2, 2, 0, 5}, {13, 0, 2, 2, 3}},
    {{19, 0, 0, 0, 0}, {15, 2, 0, 2, 1}, {18, 2, 2, 0, 5}, {14, 0, 2, 2, 3}},
};
enum { kCenter = 0, kIJ = 1, kKI = 2, kJK = 3, kInvalidDir = -1 };

// adjacentFaceDir[from][to]: the quadrant of `from` that borders `to`
inline int adjacent_face_dir(int from, int to) {
  if (from == to) return kCenter;
  for (int q = 1; q <= 3; ++q)
    if (kFaceNeighbors[from][q].face == to) return q;
  return kInvalidDir;
}

static const int kMaxDimByCIIres[17] = {2, -1, 14, -1, 98, -1, 686, -1, 4802, -1, 33614, -1, 235298, -1, 1647086, -1, 11529602};
static const int kUnitScaleByCIIres[17] = {1, -1, 7, -1, 49, -1, 343, -1, 2401, -1, 16807, -1, 117649, -1, 823543, -1, 5764801};

inline IJK ijk_add(IJK a, IJK b) { return IJK{a.i + b.i, a.j + b.j, a.k + b.k}; }
inline IJK ijk_scale(IJK a, int s) { return IJK{a.i * s, a.j * s, a.k * s}; }
// sum of the three unit-vector images, then normalised (H3's _ijk* lattice maps)
inline IJK ijk_map(IJK c, IJK iv, IJK jv, IJK kv) {
  IJK r = ijk_add(ijk_add(ijk_scale(iv, c.i), ijk_scale(jv, c.j)), ijk_scale(kv, c.k));
  h3::ijk_normalize(r);
  return r;
}
inline void rotate60ccw(IJK& c) { c = ijk_map(c, {1, 1, 0}, {0, 1, 1}, {1, 0, 1}); }
inline void rotate60cw(IJK& c) { c = ijk_map(c, {1, 0, 1}, {1, 1, 0}, {0, 1, 1}); }
inline void down_ap3(IJK& c) { c = ijk_map(c, {2, 0, 1}, {1, 2, 0}, {0, 1, 2}); }
inline void down_ap3r(IJK& c) { c = ijk_map(c, {2, 1, 0}, {0, 2, 1}, {1, 0, 2}); }
inline bool class3(int res) { return res & 1; }

enum Overage { kNoOverage = 0, kFaceEdge = 1, kNewFace = 2 };

inline Overage adjust_overage_class2(FaceIJK& f, int res, bool pent_leading4, bool substrate) {
  Overage ov = kNoOverage;
  IJK& ijk = f.c;
  int max_dim = kMaxDimByCIIres[res];
  if (substrate) max_dim *= 3;
  const int sum = ijk.i + ijk.j + ijk.k;
  if (substrate && sum == max_dim) {
    ov = kFaceEdge;
  } else if (sum > max_dim) {
    ov = kNewFace;
    const FaceOrient* o;
    if (ijk.k > 0) {
      if (ijk.j > 0) {
        o = &kFaceNeighbors[f.face][kJK];
      } else {
        o = &kFaceNeighbors[f.face][kKI];
        if (pent_leading4) {  // the pentagon's missing sequence
          IJK origin{max_dim, 0, 0};
          IJK tmp{ijk.i - origin.i, ijk.j - origin.j, ijk.k - origin.k};
          rotate60cw(tmp);
          ijk = ijk_add(tmp, origin);
        }
      }
    } else {
      o = &kFaceNeighbors[f.face][kIJ];
    }
    f.face = o->face;
    for (int i = 0; i < o->rot; i++) rotate60ccw(ijk);
    int unit = kUnitScaleByCIIres[res];
    if (substrate) unit *= 3;
    ijk = ijk_add(ijk, IJK{o->ti * unit, o->tj * unit, o->tk * unit});
    h3::ijk_normalize(ijk);
    if (substrate && ijk.i + ijk.j + ijk.k == max_dim) ov = kFaceEdge;
  }
  return ov;
}

inline bool is_pentagon_base(int bc) { return H3T_BASE_CELL_DATA[bc][4] != 0; }
inline bool is_pentagon(uint64_t h) {
  const int res = (int)((h >> 52) & 15), bc = (int)((h >> 45) & 127);
  return is_pentagon_base(bc) && h3::leading_nonzero(h, res) == 0;
}

// _h3ToFaceIjk
inline FaceIJK h3_to_face_ijk(uint64_t h) {
  const int bc = (int)((h >> 45) & 127);
  const int hres = (int)((h >> 52) & 15);
  if (is_pentagon_base(bc) && h3::leading_nonzero(h, hres) == 5) h = h3::rotate_cw(h, hres);
  FaceIJK f{H3T_BASE_CELL_DATA[bc][0], IJK{H3T_BASE_CELL_DATA[bc][1], H3T_BASE_CELL_DATA[bc][2], H3T_BASE_CELL_DATA[bc][3]}};
  // _h3ToFaceIjkWithInitializedFijk
  bool possible_overage = true;
  if (!is_pentagon_base(bc) && (hres == 0 || (f.c.i == 0 && f.c.j == 0 && f.c.k == 0))) possible_overage = false;
  for (int r = 1; r <= hres; ++r) {
    if (class3(r)) h3::down_ap7(f.c);
    else h3::down_ap7r(f.c);
    const int d = h3::digit_at(h, r);
    if (d > 0 && d < 7) {
      f.c.i += (d >> 2) & 1;
      f.c.j += (d >> 1) & 1;
      f.c.k += d & 1;
      h3::ijk_normalize(f.c);
    }
  }
  if (!possible_overage) return f;
  const IJK orig = f.c;
  int res = hres;
  if (class3(res)) {
    h3::down_ap7r(f.c);
    ++res;
  }
  const bool pent_leading4 = is_pentagon_base(bc) && h3::leading_nonzero(h, hres) == 4;
  if (adjust_overage_class2(f, res, pent_leading4, false) != kNoOverage) {
    if (is_pentagon_base(bc))
      while (adjust_overage_class2(f, res, false, false) != kNoOverage) {
      }
    if (res != hres) h3::up_ap7r(f.c);
  } else if (res != hres) {
    f.c = orig;
  }
  return f;
}

struct V2 {
  double x, y;
};

// _ijkToHex2d (M_SQRT3_2 is a long double)
inline V2 ijk_to_hex2d(IJK c) {
  const int i = c.i - c.k, j = c.j - c.k;
  return V2{i - 0.5 * j, X::ld_mul((double)j, X::kXSin60)};
}

// _geoAzDistanceRads
inline void geo_az_distance(double lat1, double lon1, double az, double dist, double* lat2, double* lon2) {
  const double kPi = 3.14159265358979323846, kPi2 = 1.5707963267948966;
  auto constrain = [&](double l) {
    while (l > kPi) l = l - (2 * kPi);
    while (l < -kPi) l = l + (2 * kPi);
    return l;
  };
  if (X::ld_lt(dist, X::kXEpsilon)) {
    *lat2 = lat1;
    *lon2 = lon1;
    return;
  }
  az = h3::pos_angle(az);
  if (X::ld_lt(az, X::kXEpsilon) || X::ld_lt(std::fabs(az - kPi), X::kXEpsilon)) {
    *lat2 = X::ld_lt(az, X::kXEpsilon) ? lat1 + dist : lat1 - dist;
    if (X::ld_lt(std::fabs(*lat2 - kPi2), X::kXEpsilon)) {
      *lat2 = kPi2;
      *lon2 = 0.0;
    } else if (X::ld_lt(std::fabs(*lat2 + kPi2), X::kXEpsilon)) {
      *lat2 = -kPi2;
      *lon2 = 0.0;
    } else {
      *lon2 = constrain(lon1);
    }
    return;
  }
  double sinlat = std::sin(lat1) * std::cos(dist) + std::cos(lat1) * std::sin(dist) * std::cos(az);
  if (sinlat > 1.0) sinlat = 1.0;
  if (sinlat < -1.0) sinlat = -1.0;
  *lat2 = std::asin(sinlat);
  if (X::ld_lt(std::fabs(*lat2 - kPi2), X::kXEpsilon)) {
    *lat2 = kPi2;
    *lon2 = 0.0;
  } else if (X::ld_lt(std::fabs(*lat2 + kPi2), X::kXEpsilon)) {
    *lat2 = -kPi2;
    *lon2 = 0.0;
  } else {
    double sinlon = std::sin(az) * std::sin(dist) / std::cos(*lat2);
    double coslon = (std::cos(dist) - std::sin(lat1) * std::sin(*lat2)) / std::cos(lat1) / std::cos(*lat2);
    if (sinlon > 1.0) sinlon = 1.0;
    if (sinlon < -1.0) sinlon = -1.0;
    if (coslon > 1.0) coslon = 1.0;
    if (coslon < -1.0) coslon = -1.0;
    *lon2 = constrain(lon1 + std::atan2(sinlon, coslon));
  }
}

// _hex2dToGeo -> (lat, lon) radians
inline void hex2d_to_geo(V2 v, int face, int res, bool substrate, double* lat, double* lon) {
  double r = std::sqrt(v.x * v.x + v.y * v.y);
  if (X::ld_lt(r, X::kXEpsilon)) {
    *lat = H3T_FACE_CENTER_GEO[face][0];
    *lon = H3T_FACE_CENTER_GEO[face][1];
    return;
  }
  double theta = std::atan2(v.y, v.x);
  for (int i = 0; i < res; i++) r = X::ld_div(r, X::kXSqrt7);
  if (substrate) {
    r /= 3.0;
    if (class3(res)) r = X::ld_div(r, X::kXSqrt7);
  }
  r *= h3::kRes0UGnomonic;
  r = std::atan(r);
  if (!substrate && class3(res)) theta = h3::pos_angle(X::ld_add(theta, X::kXAp7Rot));
  theta = h3::pos_angle(H3T_FACE_AXES_AZ_CII[face][0] - theta);
  geo_az_distance(H3T_FACE_CENTER_GEO[face][0], H3T_FACE_CENTER_GEO[face][1], theta, r, lat, lon);
}

// _v2dIntersect (H3 keeps the parameter in a float)
inline V2 v2d_intersect(V2 p0, V2 p1, V2 p2, V2 p3) {
  const V2 s1{p1.x - p0.x, p1.y - p0.y}, s2{p3.x - p2.x, p3.y - p2.y};
  const float t = (float)((s2.x * (p0.y - p2.y) - s2.y * (p0.x - p2.x)) / (-s2.x * s1.y + s1.x * s2.y));
  return V2{p0.x + (t * s1.x), p0.y + (t * s1.y)};
}
inline bool v2d_equals(V2 a, V2 b) { return std::fabs(a.x - b.x) < FLT_EPSILON && std::fabs(a.y - b.y) < FLT_EPSILON; }

// the icosahedron face edge of the substrate triangle in quadrant `dir`
inline void face_edge(int dir, int max_dim, V2* e0, V2* e1) {
  const V2 v0{3.0 * max_dim, 0.0};
  // 3.0 * M_SQRT3_2 * maxDim: long double throughout
  const double yy = X::x80_to_double(X::x80_mul(X::x80_mul(X::x80_from_double(3.0), X::kXSin60),
                                                X::x80_from_double((double)max_dim)));
  const V2 v1{-1.5 * max_dim, yy}, v2{-1.5 * max_dim, -yy};
  if (dir == kIJ) {
    *e0 = v0;
    *e1 = v1;
  } else if (dir == kJK) {
    *e0 = v1;
    *e1 = v2;
  } else {
    *e0 = v2;
    *e1 = v0;
  }
}

// _faceIjkToVerts / _faceIjkPentToVerts: the substrate vertices, *res adjusted to Class II
inline void face_ijk_to_verts(FaceIJK f, int* res, int nv, FaceIJK* out) {
  static const IJK kCII[6] = {{2, 1, 0}, {1, 2, 0}, {0, 2, 1}, {0, 1, 2}, {1, 0, 2}, {2, 0, 1}};
  static const IJK kCIII[6] = {{5, 4, 0}, {1, 5, 0}, {0, 5, 4}, {0, 1, 5}, {4, 0, 5}, {5, 0, 1}};
  const IJK* verts = class3(*res) ? kCIII : kCII;
  down_ap3(f.c);
  down_ap3r(f.c);
  if (class3(*res)) {
    h3::down_ap7r(f.c);
    *res += 1;
  }
  for (int v = 0; v < nv; v++) {
    out[v].face = f.face;
    out[v].c = ijk_add(f.c, verts[v]);
    h3::ijk_normalize(out[v].c);
  }
}

struct LatLon {
  double lat, lon;  // radians
};

// a substrate vertex's position: hex2d_to_geo of its hex2d point (a pure function of the
// face, the normalized ijk and the resolution: callers may memoize it)
struct VertexGeo {
  LatLon operator()(const FaceIJK& f, int adj_res) const {
    LatLon p;
    hex2d_to_geo(ijk_to_hex2d(f.c), f.face, adj_res, true, &p.lat, &p.lon);
    return p;
  }
};

// h3ToGeoBoundary (radians, H3's vertex order, not closed); `vertex` computes the cell's
// own substrate vertices (the distortion vertices on icosahedron edges are computed here)
template <class Vertex = VertexGeo>
inline std::vector<LatLon> cell_boundary(uint64_t h, const Vertex& vertex = Vertex()) {
  const int res = (int)((h >> 52) & 15);
  const FaceIJK center = h3_to_face_ijk(h);
  std::vector<LatLon> g;
  int adj_res = res;
  if (is_pentagon(h)) {
    FaceIJK verts[5];
    face_ijk_to_verts(center, &adj_res, 5, verts);
    FaceIJK last{};
    for (int vert = 0; vert < 5 + 1; vert++) {
      const int v = vert % 5;
      FaceIJK f = verts[v];
      while (adjust_overage_class2(f, adj_res, false, true) == kNewFace) {
      }
      if (class3(res) && vert > 0) {
        // all Class III pentagon edges cross icosahedron edges
        FaceIJK tmp = f;
        const V2 orig0 = ijk_to_hex2d(last.c);
        const int dir = adjacent_face_dir(tmp.face, last.face);
        const FaceOrient& o = kFaceNeighbors[tmp.face][dir];
        tmp.face = o.face;
        for (int i = 0; i < o.rot; i++) rotate60ccw(tmp.c);
        const int unit = kUnitScaleByCIIres[adj_res] * 3;
        tmp.c = ijk_add(tmp.c, IJK{o.ti * unit, o.tj * unit, o.tk * unit});
        h3::ijk_normalize(tmp.c);
        const V2 orig1 = ijk_to_hex2d(tmp.c);
        V2 e0, e1;
        face_edge(adjacent_face_dir(tmp.face, f.face), kMaxDimByCIIres[adj_res], &e0, &e1);
        const V2 inter = v2d_intersect(orig0, orig1, e0, e1);
        LatLon p;
        hex2d_to_geo(inter, tmp.face, adj_res, true, &p.lat, &p.lon);
        g.push_back(p);
      }
      if (vert < 5) g.push_back(vertex(f, adj_res));
      last = f;
    }
    return g;
  }
  FaceIJK verts[6];
  face_ijk_to_verts(center, &adj_res, 6, verts);
  int last_face = -1;
  Overage last_ov = kNoOverage;
  for (int vert = 0; vert < 6 + 1; vert++) {
    const int v = vert % 6;
    FaceIJK f = verts[v];
    const Overage ov = adjust_overage_class2(f, adj_res, false, true);
    if (class3(res) && vert > 0 && f.face != last_face && last_ov != kFaceEdge) {
      const int last_v = (v + 5) % 6;
      const V2 orig0 = ijk_to_hex2d(verts[last_v].c), orig1 = ijk_to_hex2d(verts[v].c);
      const int face2 = last_face == center.face ? f.face : last_face;
      V2 e0, e1;
      face_edge(adjacent_face_dir(center.face, face2), kMaxDimByCIIres[adj_res], &e0, &e1);
      const V2 inter = v2d_intersect(orig0, orig1, e0, e1);
      if (!(v2d_equals(orig0, inter) || v2d_equals(orig1, inter))) {
        LatLon p;
        hex2d_to_geo(inter, center.face, adj_res, true, &p.lat, &p.lon);
        g.push_back(p);
      }
    }
    if (vert < 6) g.push_back(vertex(f, adj_res));
    last_face = f.face;
    last_ov = ov;
  }
  return g;
}

// h3ToGeo: _h3ToFaceIjk then _faceIjkToGeo (radians)
inline LatLon cell_center(uint64_t h) {
  const FaceIJK f = h3_to_face_ijk(h);
  LatLon p;
  hex2d_to_geo(ijk_to_hex2d(f.c), f.face, (int)((h >> 52) & 15), false, &p.lat, &p.lon);
  return p;
}

// JDK 8 Math.toDegrees (H3-Java converts each coordinate)
inline double to_degrees(double rad) { return rad * 180.0 / 3.14159265358979323846; }

}  // namespace h3b
}  // namespace mgpu
