// H3 kRing / hexRing on the device (grid_cellkring / grid_cellkloop for H3).
//
// Replaces: H3IndexSystem.kRing / kLoop -> H3Core.kRing / hexRing
//   /root/reference/src/main/scala/com/databricks/labs/mosaic/core/index/H3IndexSystem.scala:182-205
// over com.uber:h3:3.7.0 (not vendored; H3 C v3.7 algos.c: h3NeighborRotations,
// hexRangeDistances, hexRing).  One thread walks one cell's spiral (kRing) or ring
// (hexRing) in the reference's output order.
//
// Scope of this version: walks that stay among hexagon base cells.  A walk that
// reaches a cell of one of the 12 pentagon base cells returns kUnsupported and the
// C-ABI call fails loudly (MGPU_E_UNSUPPORTED); the reference's pentagon handling
// (the K-subsequence rotations, the _kRingInternal hash-set fallback, Mosaic's
// kLoop set-difference fallback) is restated in the oracle only
// (oracle/h3_oracle.c); walks next to the south polar pentagon are not yet consistent there.
#pragma once
#include <stdint.h>

#include "h3_core.h"
#include "h3_neighbors.inc"

namespace mgpu {
namespace h3ring {

constexpr uint64_t kUnsupported = ~0ULL;
constexpr uint64_t kDigitsMask = (1ULL << 45) - 1;

MGPU_HD int res_of(uint64_t h) { return (int)((h >> 52) & 15); }
MGPU_HD int base_of(uint64_t h) { return (int)((h >> 45) & 127); }
MGPU_HD bool pentagon_base(int b) { return H3T_BASE_CELL_DATA[b][4] != 0; }

// all digits rotated 60 degrees ccw n times (unused digits stay 7)
MGPU_HD uint64_t rotate_digits(uint64_t h, int n) {
  uint64_t d = h & kDigitsMask;
  for (int i = 0; i < n; i++) d = h3::rotate60ccw_all(d);
  return (h & ~kDigitsMask) | d;
}

// h3NeighborRotations restricted to hexagon base cells (kUnsupported otherwise).
// The digit walk: from the finest digit up, NEW_DIGIT / NEW_ADJUSTMENT (_II for a
// Class III child resolution, _III for Class II) until no step is carried; a step
// carried past resolution 1 crosses into the neighbouring base cell, whose frame is
// reached by baseCellNeighbor60CCWRots ccw rotations of every digit.
MGPU_HD uint64_t neighbor(uint64_t h, int dir, int* rotations) {
  const int res = res_of(h);
  const int old_base = base_of(h);
  if (pentagon_base(old_base)) return kUnsupported;
  for (int i = 0; i < *rotations; i++) dir = h3::rot60ccw(dir);
  int new_rot = 0;
  for (int r = res - 1;; r--) {
    if (r == -1) {
      const int nb = H3T_BASE_CELL_NEIGHBORS[old_base][dir];
      if (nb == H3T_INVALID_BASE_CELL || pentagon_base(nb)) return kUnsupported;
      h = (h & ~(127ULL << 45)) | ((uint64_t)nb << 45);
      new_rot = H3T_BASE_CELL_NEIGHBOR_ROTS[old_base][dir];
      break;
    }
    const int sh = (h3::kMaxRes - (r + 1)) * 3;
    const int od = (int)((h >> sh) & 7);
    int nd, next;
    if ((r + 1) & 1) {
      nd = H3T_NEW_DIGIT_II[od][dir];
      next = H3T_NEW_ADJUSTMENT_II[od][dir];
    } else {
      nd = H3T_NEW_DIGIT_III[od][dir];
      next = H3T_NEW_ADJUSTMENT_III[od][dir];
    }
    h = (h & ~(7ULL << sh)) | ((uint64_t)nd << sh);
    if (next == 0) break;
    dir = next;
  }
  h = rotate_digits(h, new_rot);
  *rotations = (*rotations + new_rot) % 6;
  return h;
}

// J, JK, K, IK, I, IJ; rings start one step in I
__host__ __device__ constexpr int direction(int i) { return (int)((0x231546u >> (4 * (5 - i))) & 0xF); }
constexpr int kNextRing = 4;

// kRing(h, k) in hexRangeDistances' spiral order: number of ids (written to out when
// out != nullptr), or -1 when the walk is outside this version's scope
MGPU_HD int64_t kring(uint64_t h, int k, int64_t* out) {
  int64_t idx = 0;
  if (out) out[idx] = (int64_t)h;
  idx++;
  if (pentagon_base(base_of(h))) return -1;
  int rot = 0;
  for (int ring = 1; ring <= k; ring++) {
    h = neighbor(h, kNextRing, &rot);
    if (h == kUnsupported) return -1;
    for (int d = 0; d < 6; d++) {
      for (int s = 0; s < ring; s++) {
        h = neighbor(h, direction(d), &rot);
        if (h == kUnsupported) return -1;
        if (out) out[idx] = (int64_t)h;
        idx++;
      }
    }
  }
  return idx;
}

// hexRing(h, k): 6k ids (1 for k = 0) in hexRing's order, or -1 (out of scope)
MGPU_HD int64_t hex_ring(uint64_t h, int k, int64_t* out) {
  if (k == 0) {
    if (out) out[0] = (int64_t)h;
    return 1;
  }
  if (pentagon_base(base_of(h))) return -1;
  int rot = 0;
  for (int ring = 0; ring < k; ring++) {
    h = neighbor(h, kNextRing, &rot);
    if (h == kUnsupported) return -1;
  }
  const uint64_t first = h;
  int64_t idx = 0;
  if (out) out[idx] = (int64_t)h;
  idx++;
  for (int d = 0; d < 6; d++) {
    for (int s = 0; s < k; s++) {
      h = neighbor(h, direction(d), &rot);
      if (h == kUnsupported) return -1;
      if (s != k - 1 || d != 5) {
        if (out) out[idx] = (int64_t)h;
        idx++;
      }
    }
  }
  return h == first ? idx : -1;
}

// structural check of an H3 cell id (mode 1, res, base cell, digits 0..6 then 7s)
MGPU_HD bool valid_cell(uint64_t h) {
  if ((h >> 63) || ((h >> 59) & 15) != 1 || base_of(h) >= 122) return false;
  const int res = res_of(h);
  for (int r = 1; r <= h3::kMaxRes; r++) {
    const int d = (int)((h >> ((h3::kMaxRes - r) * 3)) & 7);
    if ((r <= res) == (d == 7)) return false;
  }
  return true;
}

}  // namespace h3ring
}  // namespace mgpu
