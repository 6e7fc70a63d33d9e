// `st_contains(chip.wkb, point)` on the device-resident chip table.
//
// Replaces (per candidate row): ST_Contains.scala:34-42 ->
// MosaicGeometryIOCodeGenJTS.fromWKB (codegen/format/MosaicGeometryIOCodeGenJTS.scala:23-29)
// -> MosaicGeometryJTS.contains (core/geometry/MosaicGeometryJTS.scala:197) ->
// JTS 1.20 Geometry.contains(Point).  The WKB is parsed ONCE at upload instead of
// per candidate; the decision procedure is JTS's:
//   empty -> false; chip envelope must contain p (inclusive);
//   Polygon.isRectangle -> strictly inside the rectangle;
//   else PointLocator: Polygon = shell, then holes (a ring whose envelope misses p
//   is EXTERIOR); Multi/Collection = Mod-2 rule over the polygons.
//   Ring test = RayCrossingCounter.locatePointInRing (p1 = ring[i], p2 = ring[i-1])
//   with CGAlgorithmsDD.orientationIndex (1e-15 filter, DoubleDouble fallback).
// Built with -ffp-contract=off: every product is rounded separately as on the JVM.
#pragma once
#include "chip_table.h"
#include "jts_orient.h"

namespace mgpu {
namespace pip {

enum { kExterior = 0, kBoundary = 1, kInterior = 2 };

// RayCrossingCounter.countSegment(p1, p2) for one segment, as bits: 1 = the point is
// on the segment (BOUNDARY), 2 = the segment crosses the ray (one crossing).  The
// ring's location is then BOUNDARY if any segment sets bit 1, else INTERIOR iff the
// crossings are odd -- independent of the order the segments are visited in, which
// lets the join test only the edges of the point's y-strip (chip_contains_strips).
MGPU_HDI int count_segment(double p1x, double p1y, double p2x, double p2y, double px, double py) {
  if (p1x < px && p2x < px) return 0;
  if (px == p2x && py == p2y) return 1;
  if (p1y == py && p2y == py) {
    double mn = p1x, mx = p2x;
    if (mn > mx) { mn = p2x; mx = p1x; }
    return (px >= mn && px <= mx) ? 1 : 0;
  }
  if (((p1y > py) && (p2y <= py)) || ((p2y > py) && (p1y <= py))) {
    int o = orientation(p1x, p1y, p2x, p2y, px, py);
    if (o == 0) return 1;
    if (p2y < p1y) o = -o;
    return o == 1 ? 2 : 0;
  }
  return 0;
}

// RayCrossingCounter.locatePointInRing over vertices [vb, ve)
MGPU_HDI int ring_locate(const double* __restrict__ vtx, uint32_t vb, uint32_t ve, double px, double py) {
  if (ve <= vb) return kExterior;
  double prevx = vtx[2 * vb], prevy = vtx[2 * vb + 1];
  int crossings = 0;
  for (uint32_t i = vb + 1; i < ve; i++) {
    double p1x = vtx[2 * i], p1y = vtx[2 * i + 1];
    double p2x = prevx, p2y = prevy;
    prevx = p1x;
    prevy = p1y;
    if (p1x < px && p2x < px) continue;
    if (px == p2x && py == p2y) return kBoundary;
    if (p1y == py && p2y == py) {
      double mn = p1x, mx = p2x;
      if (mn > mx) { mn = p2x; mx = p1x; }
      if (px >= mn && px <= mx) return kBoundary;
      continue;
    }
    if (((p1y > py) && (p2y <= py)) || ((p2y > py) && (p1y <= py))) {
      int o = orientation(p1x, p1y, p2x, p2y, px, py);
      if (o == 0) return kBoundary;
      if (p2y < p1y) o = -o;
      if (o == 1) crossings++;
    }
  }
  return (crossings & 1) ? kInterior : kExterior;
}

MGPU_HDI bool env_has(const double* env, double px, double py) {
  return px >= env[0] && px <= env[2] && py >= env[1] && py <= env[3];
}

// PointLocator.locateInPolygon for part `p`
MGPU_HDI int polygon_locate(const ChipTableView& t, uint32_t p, double px, double py) {
  uint32_t rb = t.part_ring[p], re = t.part_ring[p + 1];
  if (re == rb) return kExterior;
  for (uint32_t r = rb; r < re; r++) {
    uint32_t vb = t.ring_vtx[r], ve = t.ring_vtx[r + 1];
    if (r == rb && ve == vb) return kExterior;  // empty shell = empty polygon
    int loc = env_has(t.ring_env + 4 * r, px, py) ? ring_locate(t.vtx, vb, ve, px, py) : kExterior;
    if (r == rb) {
      if (loc != kInterior) return loc;  // EXTERIOR or BOUNDARY
    } else {
      if (loc == kInterior) return kExterior;
      if (loc == kBoundary) return kBoundary;
    }
  }
  return kInterior;
}

enum RingBits { kRingOnSegment = 1 };

// Geometry.contains(point) == (location == INTERIOR), for sorted chip `c`
MGPU_HDI int chip_locate(const ChipTableView& t, uint32_t c, double px, double py) {
  const uint8_t fl = t.chip_flags[c];
  if (fl & (kChipEmpty | kChipNoGeom)) return kExterior;
  const double* env = t.chip_env + 4 * c;
  if (!env_has(env, px, py)) return kExterior;
  if (fl & kChipRect) {
    if (px == env[0] || px == env[2] || py == env[1] || py == env[3]) return kBoundary;
    return kInterior;
  }
  uint32_t pb = t.chip_part[c], pe = t.chip_part[c + 1];
  if (!(fl & kChipMulti)) return polygon_locate(t, pb, px, py);
  bool is_in = false;
  int n_bnd = 0;
  for (uint32_t p = pb; p < pe; p++) {
    int loc = polygon_locate(t, p, px, py);
    if (loc == kInterior) is_in = true;
    if (loc == kBoundary) n_bnd++;
  }
  if (n_bnd & 1) return kBoundary;
  if (n_bnd > 0 || is_in) return kInterior;
  return kExterior;
}

// Geometry.contains(point) for sorted chip `c` by the strip index (chip_table.h): the
// same decision as chip_locate() -- envelope, rectangle shortcut, PointLocator over
// the rings -- with each ring's RayCrossingCounter run over the edges of the
// point's strip only.  Chips flagged kChipNoStrips go to chip_locate().
// The quick part of contains(): flags, envelope, rectangle shortcut and the
// classification grid.  Returns kQuickNo / kQuickYes, or kQuickStrips (a mixed grid
// cell: chip_contains_mixed decides) / kQuickSequential (chip without strip index).
enum QuickVerdict { kQuickNo = 0, kQuickYes = 1, kQuickStrips = 2, kQuickSequential = 3 };

MGPU_HDI int chip_quick(const ChipTableView& t, uint32_t c, double px, double py, uint64_t* walk = nullptr) {
  const ChipHdr& H = t.chip_hdr[c];
  const double e0 = H.env[0], e1 = H.env[1], e2 = H.env[2], e3 = H.env[3];
  const uint8_t fl = H.flags;
  if (fl & (kChipEmpty | kChipNoGeom)) return kQuickNo;
  if (!(px >= e0 && px <= e2 && py >= e1 && py <= e3)) return kQuickNo;
  if (fl & kChipRect) return (px == e0 || px == e2 || py == e1 || py == e3) ? kQuickNo : kQuickYes;
  if (fl & kChipNoStrips) return kQuickSequential;
  const int gx = grid_index(px, e0, H.sx), gy = grid_index(py, e1, H.sy);
  const uint32_t st = (H.grid[gy] >> (2 * gx)) & 3;
  if (st == kCellMixed && walk) {
    // what a deferred walk needs from this header (chip_contains_strip): the point's
    // strip | flags << 32 | single_ring << 40
    const uint32_t sidx = H.strip_base + (uint32_t)strip_of(py, e1, H.inv_h, (int)H.n_strips);
    *walk = (uint64_t)sidx | ((uint64_t)fl << 32) | ((uint64_t)(H.single_ring ? 1 : 0) << 40);
  }
  return st == kCellMixed ? kQuickStrips : (st == kCellIn ? kQuickYes : kQuickNo);
}

// contains() for a point in a mixed grid cell of chip c: RayCrossingCounter over the
// edges of the point's y-strip (MGPU_EDGE_STEP records in flight per step), then PointLocator
// over the rings' verdicts.
// The walk proper, given what it needs from the chip header: `strip` = the point's
// strip (strip_base + strip_of(...)), `one_ring` and the chip flags.  pip_resolve_kernel
// calls it with the values the streaming kernel already read (no header re-read).
MGPU_HDI bool chip_contains_strip(const ChipTableView& t, uint32_t c, uint32_t strip, bool one_ring, uint8_t fl,
                                  double px, double py, uint32_t* stat_edges = nullptr);

MGPU_HDI bool chip_contains_mixed(const ChipTableView& t, uint32_t c, double px, double py,
                                  uint32_t* stat_edges = nullptr) {
  const ChipHdr& H = t.chip_hdr[c];
  const int s = strip_of(py, H.env[1], H.inv_h, (int)H.n_strips);
  return chip_contains_strip(t, c, H.strip_base + (uint32_t)s, H.single_ring != 0, H.flags, px, py, stat_edges);
}

// RayCrossingCounter over the edges of strip `strip` (MGPU_EDGE_STEP records in flight
// per step): the blocks of MGPU_EDGE_STEP edges first, first + stride, ... (in edges; a
// lane group splitting one walk takes first = lane * STEP, stride = lanes * STEP), each
// ring's boundary / parity bits OR-ed / XOR-ed into *bnd / *par -- order-free, so the
// lanes' partial bits combine by OR / XOR.
MGPU_HDI void strip_bits(const ChipTableView& t, uint32_t strip, bool one_ring, double px, double py, uint32_t first,
                         uint32_t stride, uint32_t* bnd_out, uint32_t* par_out, uint32_t* stat_edges = nullptr) {
  const uint32_t eb = t.strip_edge[strip], ee = t.strip_edge[strip + 1];
  if (stat_edges) *stat_edges = ee - eb;
  const double4* E4 = (const double4*)t.edges;
  uint32_t bnd = 0, par = 0;
#ifndef MGPU_EDGE_STEP
#define MGPU_EDGE_STEP 2
#endif
  for (uint32_t e = eb + first; e < ee; e += stride) {
    const uint32_t l = ee - 1;
    int bits[MGPU_EDGE_STEP];
    double4 R[MGPU_EDGE_STEP];
#pragma unroll
    for (int k = 0; k < MGPU_EDGE_STEP; k++) R[k] = E4[e + k < l ? e + k : l];
#pragma unroll
    for (int k = 0; k < MGPU_EDGE_STEP; k++)
      bits[k] = e + k < ee ? count_segment(R[k].x, R[k].y, R[k].z, R[k].w, px, py) : 0;
#pragma unroll
    for (int k = 0; k < MGPU_EDGE_STEP; k++) {
      if (!bits[k]) continue;
      const uint32_t rb = one_ring ? 1u : 1u << t.edge_ring[e + k];
      if (bits[k] & kRingOnSegment) bnd |= rb;
      if (bits[k] & 2) par ^= rb;
    }
  }
  *bnd_out = bnd;
  *par_out = par;
}

// PointLocator over the rings' RayCrossingCounter verdicts (strip_bits of the point's
// strip): contains() of chip c
MGPU_HDI bool strip_verdict(const ChipTableView& t, uint32_t c, bool one_ring, uint8_t fl, uint32_t bnd, uint32_t par,
                            double px, double py) {
  // one polygon, one ring (its envelope is the chip's): RayCrossingCounter's verdict
  if (one_ring) return !(bnd & 1) && (par & 1);
  const uint32_t pb = t.chip_part[c], pe = t.chip_part[c + 1];
  const uint32_t r0 = t.part_ring[pb];
  bool is_in = false;
  int n_bnd = 0, single = -1;
  for (uint32_t p = pb; p < pe; p++) {
    const uint32_t rb = t.part_ring[p], re = t.part_ring[p + 1];
    int loc = kInterior;
    if (re == rb) loc = kExterior;
    for (uint32_t r = rb; r < re; r++) {
      const uint32_t vb = t.ring_vtx[r], ve = t.ring_vtx[r + 1];
      int l;
      if (r == rb && ve == vb) {
        l = kExterior;  // empty shell = empty polygon
      } else if (!env_has(t.ring_env + 4 * r, px, py)) {
        l = kExterior;
      } else {
        const uint32_t m = 1u << (r - r0);
        l = (bnd & m) ? kBoundary : ((par & m) ? kInterior : kExterior);
      }
      if (r == rb) {
        if (l != kInterior) { loc = l; break; }
      } else {
        if (l == kInterior) { loc = kExterior; break; }
        if (l == kBoundary) { loc = kBoundary; break; }
      }
    }
    if (single < 0) single = loc;
    if (loc == kInterior) is_in = true;
    if (loc == kBoundary) n_bnd++;
  }
  if (!(fl & kChipMulti)) return single == kInterior;
  if (n_bnd & 1) return false;
  return n_bnd > 0 || is_in;
}

MGPU_HDI bool chip_contains_strip(const ChipTableView& t, uint32_t c, uint32_t strip, bool one_ring, uint8_t fl,
                                  double px, double py, uint32_t* stat_edges) {
  uint32_t bnd, par;
  strip_bits(t, strip, one_ring, px, py, 0, MGPU_EDGE_STEP, &bnd, &par, stat_edges);
  return strip_verdict(t, c, one_ring, fl, bnd, par, px, py);
}

// Geometry.contains(point) for sorted chip `c` -- the same decision as chip_locate()
// (envelope, rectangle shortcut, PointLocator over the rings) through the chip's
// classification grid and strip index.
MGPU_HDI bool chip_contains_strips(const ChipTableView& t, uint32_t c, double px, double py,
                                   uint32_t* stat_edges = nullptr) {
  const int q = chip_quick(t, c, px, py);
  if (q == kQuickStrips) return chip_contains_mixed(t, c, px, py, stat_edges);
  if (q == kQuickSequential) return chip_locate(t, c, px, py) == kInterior;
  return q == kQuickYes;
}

}  // namespace pip
}  // namespace mgpu
