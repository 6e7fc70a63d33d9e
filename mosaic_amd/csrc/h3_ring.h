// H3 kRing / hexRing on the device (grid_cellkring / grid_cellkloop for H3).
//
// Replaces: H3IndexSystem.kRing / kLoop -> H3Core.kRing / hexRing
//   /root/reference/src/main/scala/com/databricks/labs/mosaic/core/index/H3IndexSystem.scala:182-205
// over com.uber:h3:3.7.0 (not vendored; H3 C v3.7 algos.c: h3NeighborRotations,
// hexRangeDistances, hexRing).  One thread walks one cell's spiral (kRing) or ring
// (hexRing) in the reference's output order.
//
// Pentagons as in H3 v3.7: h3NeighborRotations' K-subsequence rotations; a spiral or
// ring that meets a pentagon fails (as hexRangeDistances / hexRing do), and the caller
// then takes the reference's fallbacks -- kring_hash (H3 C's _kRingInternal: a DFS
// into an open-addressing hash set keyed by h % maxKringSize, whose nonzero entries in
// array order are what H3-Java's kRing returns) and kloop_diff (Mosaic's kLoop on
// PentagonEncounteredException: kRing(k).toSet diff kRing(k - 1).toSet, iterated in
// Scala 2.12 HashSet order).  Restated beside the oracle's oracle/h3_oracle.c.
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

MGPU_HD uint64_t with_base(uint64_t h, int b) { return (h & ~(127ULL << 45)) | ((uint64_t)b << 45); }
MGPU_HD bool polar_pentagon(int b) { return b == 4 || b == 117; }
// the first nonzero digit of resolutions 1..res (0: none), without an exit inside the
// loop (lanes of a wave take different paths through these walks; early returns inside
// loops gave wrong per-lane results in mixed waves on gfx950)
MGPU_HD int lead_digit(uint64_t h, int res) {
  int lead = 0;
  for (int r = h3::kMaxRes; r >= 1; r--) {
    const int d = (int)((h >> ((h3::kMaxRes - r) * 3)) & 7);
    lead = (r <= res && d != 0) ? d : lead;
  }
  return lead;
}
// all digits rotated 60 degrees ccw / cw (unused digits 7 stay 7)
MGPU_HD uint64_t rot_ccw(uint64_t h) { return rotate_digits(h, 1); }
MGPU_HD uint64_t rot_cw(uint64_t h) { return rotate_digits(h, 5); }
// H3 _h3RotatePent60ccw: ccw, and once more when the leading digit lands on K
MGPU_HD uint64_t rot_pent_ccw(uint64_t h, int res) {
  h = rot_ccw(h);
  return lead_digit(h, res) == 1 ? rot_ccw(h) : h;
}
MGPU_HD bool is_pentagon(uint64_t h) { return pentagon_base(base_of(h)) && lead_digit(h, res_of(h)) == 0; }

// H3 v3.7 h3NeighborRotations: the neighbour of h in direction dir (after *rotations
// ccw rotations of dir), *rotations updated; 0 where H3 leaves it undefined (the
// deleted K direction of a pentagon).  The digit walk: from the finest digit up,
// NEW_DIGIT / NEW_ADJUSTMENT (_II for a Class III child resolution, _III for Class II)
// until no step is carried; a step carried past resolution 1 crosses into the
// neighbouring base cell, whose frame is reached by baseCellNeighbor60CCWRots rotations.
#if defined(MGPU_RING_NOINLINE) && defined(__HIP_DEVICE_COMPILE__)
#define MGPU_RING_FN __host__ __device__ __attribute__((noinline))
#else
#define MGPU_RING_FN MGPU_HD
#endif
MGPU_RING_FN uint64_t neighbor(uint64_t h, int dir, int* rotations) {
  const int res = res_of(h);
  const int old_base = base_of(h);
  const int old_lead = lead_digit(h, res);
  for (int i = 0; i < *rotations; i++) dir = h3::rot60ccw(dir);
  int new_rot = 0;
  for (int r = res - 1;; r--) {
    if (r == -1) {
      h = with_base(h, H3T_BASE_CELL_NEIGHBORS[old_base][dir]);
      new_rot = H3T_BASE_CELL_NEIGHBOR_ROTS[old_base][dir];
      if (base_of(h) == H3T_INVALID_BASE_CELL) {
        // the deleted K vertex at the base-cell level: the edge borders the IK neighbour
        h = with_base(h, H3T_BASE_CELL_NEIGHBORS[old_base][5]);
        new_rot = H3T_BASE_CELL_NEIGHBOR_ROTS[old_base][5];
        h = rot_ccw(h);
        *rotations += 1;
      }
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
  const int new_base = base_of(h);
  bool undefined = false;
  if (pentagon_base(new_base)) {
    bool adjusted = false;
    if (lead_digit(h, res) == 1) {
      if (old_base != new_base) {
        // into the deleted K subsequence of a pentagon base cell from a neighbour
        const int f = H3T_BASE_CELL_DATA[old_base][0];
        const bool cw = H3T_BASE_CELL_DATA[new_base][5] == f || H3T_BASE_CELL_DATA[new_base][6] == f;
        h = cw ? rot_cw(h) : rot_ccw(h);
        adjusted = true;
      } else if (old_lead == 3) {  // from within the same pentagon
        h = rot_ccw(h);
        *rotations += 1;
      } else if (old_lead == 5) {
        h = rot_cw(h);
        *rotations += 5;
      } else {
        undefined = true;  // the K direction is deleted from here
      }
    }
    for (int i = 0; i < new_rot && !undefined; i++) h = rot_pent_ccw(h, res);
    if (old_base != new_base && !undefined) {
      if (polar_pentagon(new_base)) {
        if (old_base != 118 && old_base != 8 && lead_digit(h, res) != 3) *rotations += 1;
      } else if (lead_digit(h, res) == 5 && !adjusted) {
        *rotations += 1;
      }
    }
  } else {
    h = rotate_digits(h, new_rot);
  }
  *rotations = (*rotations + new_rot) % 6;
  return undefined ? 0 : h;
}

// J, JK, K, IK, I, IJ; rings start one step in I
__host__ __device__ constexpr int direction(int i) { return (int)((0x231546u >> (4 * (5 - i))) & 0xF); }
constexpr int kNextRing = 4;
constexpr int64_t kFallback = -2;  // the walk met a pentagon: take the reference's fallback

MGPU_HD int64_t max_kring(int k) { return 3 * (int64_t)k * (k + 1) + 1; }

// kRing(h, k) in hexRangeDistances' spiral order: number of ids (written to out when
// out != nullptr), or kFallback where hexRangeDistances fails (a pentagon).  (Single
// exit, no return inside the loops: lanes of a wave leave the walk at different steps.)
MGPU_HD int64_t kring(uint64_t h, int k, int64_t* out) {
  int64_t idx = 0;
  if (out) out[idx] = (int64_t)h;
  idx++;
  bool fail = is_pentagon(h);
  int rot = 0;
  for (int ring = 1; ring <= k && !fail; ring++) {
    h = neighbor(h, kNextRing, &rot);
    fail = h == 0 || is_pentagon(h);
    for (int d = 0; d < 6 && !fail; d++) {
      for (int s = 0; s < ring && !fail; s++) {
        h = neighbor(h, direction(d), &rot);
        if (h == 0) {
          fail = true;
        } else {
          if (out) out[idx] = (int64_t)h;
          idx++;
          fail = is_pentagon(h);
        }
      }
    }
  }
  return fail ? kFallback : idx;
}

// hexRing(h, k): 6k ids (1 for k = 0) in hexRing's order, or kFallback where H3-Java
// throws PentagonEncounteredException
MGPU_HD int64_t hex_ring(uint64_t h, int k, int64_t* out) {
  if (k == 0) {
    if (out) out[0] = (int64_t)h;
    return 1;
  }
  bool fail = is_pentagon(h);
  int rot = 0;
  for (int ring = 0; ring < k && !fail; ring++) {
    h = neighbor(h, kNextRing, &rot);
    fail = h == 0 || is_pentagon(h);
  }
  const uint64_t first = h;
  int64_t idx = 0;
  if (!fail) {
    if (out) out[idx] = (int64_t)h;
    idx++;
  }
  for (int d = 0; d < 6 && !fail; d++) {
    for (int s = 0; s < k && !fail; s++) {
      h = neighbor(h, direction(d), &rot);
      if (h == 0) {
        fail = true;
      } else if (s != k - 1 || d != 5) {
        if (out) out[idx] = (int64_t)h;
        idx++;
        fail = is_pentagon(h);
      }
    }
  }
  return (fail || h != first) ? kFallback : idx;
}

// H3 C _kRingInternal from h with k rings into the hash set tab[max_kring(k)] (zeroed
// here) with dist[] -- the same depth-first order as the recursion, on an explicit stack
// of depth k + 1 held in the caller's scratch (stk[k + 2], nxt[k + 2]: any k).  Returns
// false if the set overflowed (only possible with inconsistent tables; H3 would not
// terminate).
MGPU_HD bool kring_hash(uint64_t h, int k, uint64_t* tab, int32_t* dist, uint64_t* stk, int8_t* nxt) {
  const int64_t m = max_kring(k);
  for (int64_t i = 0; i < m; i++) tab[i] = 0, dist[i] = 0;
  int depth = 0;
  stk[0] = h;
  nxt[0] = -1;
  while (depth >= 0) {
    if (nxt[depth] < 0) {  // visit stk[depth] at distance depth
      const uint64_t c = stk[depth];
      bool expand = false;
      if (c != 0) {
        int64_t off = (int64_t)(c % (uint64_t)m), probes = 0;
        while (tab[off] != 0 && tab[off] != c) {
          off = off + 1 == m ? 0 : off + 1;
          if (++probes >= m) return false;
        }
        if (!(tab[off] == c && dist[off] <= depth)) {
          tab[off] = c;
          dist[off] = depth;
          expand = depth < k;
        }
      }
      if (!expand) {
        depth--;
        continue;
      }
      nxt[depth] = 0;
    }
    if (nxt[depth] < 6) {
      int rot = 0;
      const uint64_t child = neighbor(stk[depth], direction(nxt[depth]++), &rot);
      depth++;
      stk[depth] = child;
      nxt[depth] = -1;
    } else {
      depth--;
    }
  }
  return true;
}

// c into the open-addressing set tab[m] (keyed by c % m, as kring_hash)
MGPU_HD void hash_insert(uint64_t* tab, int64_t m, uint64_t c) {
  int64_t off = (int64_t)(c % (uint64_t)m);
  for (int64_t probes = 0; probes < m && tab[off] != 0 && tab[off] != c; probes++) off = off + 1 == m ? 0 : off + 1;
  if (tab[off] == 0) tab[off] = c;
}

// the rank of a cell id in a Scala 2.12 immutable.HashSet's iteration (the trie indexed
// by 5-bit chunks of improve(##), lowest chunk first; ## of an H3 id = Long.hashCode)
MGPU_HD uint64_t scala_set_rank(uint64_t v) {
  uint32_t h = (uint32_t)(v ^ (v >> 32));
  h = h + ~(h << 9);
  h ^= h >> 14;
  h += h << 4;
  h ^= h >> 10;
  uint64_t key = 0;  // 7 chunks of 5 bits, the lowest chunk most significant
  for (int j = 0; j < 7; j++) key = (key << 5) | ((h >> (5 * j)) & 31u);
  return key;
}

// kRing(h, k) entries of tab that kRing(h, k - 1) (tab2) lacks, in Scala HashSet order
// (out, returns the count)
MGPU_HD int64_t kloop_diff(const uint64_t* tab, int64_t m, const uint64_t* tab2, int64_t m2, int64_t* out) {
  int64_t n = 0;
  for (int64_t i = 0; i < m; i++) {
    const uint64_t c = tab[i];
    if (c == 0) continue;
    int64_t off = (int64_t)(c % (uint64_t)m2), probes = 0;
    bool inner = false;
    while (tab2[off] != 0 && probes < m2) {
      if (tab2[off] == c) {
        inner = true;
        break;
      }
      off = off + 1 == m2 ? 0 : off + 1;
      probes++;
    }
    if (inner) continue;
    // insertion by rank (the lists are ~6k long)
    const uint64_t r = scala_set_rank(c);
    int64_t j = n++;
    while (j > 0 && scala_set_rank((uint64_t)out[j - 1]) > r) {
      out[j] = out[j - 1];
      j--;
    }
    out[j] = (int64_t)c;
  }
  return n;
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
