// gfx950 kernels of the grid-indexed point-in-polygon join.
//
//   cells_kernel<IS>     IndexSystem.pointToIndex over a batch (H3 / BNG)
//   pip_join_kernel<IS>  fused: cell id -> chip-table probe -> is_core OR
//                        st_contains -> per-tile pair records
//   tile_scan_kernel     tile pair counts -> output offsets
//   pair_emit_kernel     records -> ordered (point_id, polygon_id) output
//   st_contains_kernel   st_contains(chip.wkb, point) for explicit pairs
//
// Design (DESIGN.md has the roofline analysis): the hot path is one pass over the
// points plus two light launches.  pip_join_kernel gives each one-wave workgroup a
// tile of 256 consecutive points (4 per lane; no workgroup barrier waits); the chip table's cell hash and the
// border chips' strip-indexed edges are small and read-only, so they stay in L2 /
// Infinity Cache while the point stream flows from HBM.  A tile writes its pairs as
// compact records into its own slot -- no workgroup ever waits for another --
// tile_scan_kernel turns the tiles' pair counts into output offsets, and
// pair_emit_kernel writes the pairs ordered by input position (then polygon id).
// Nothing here is a dense contraction, so MFMA is not used.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define H3T_QUAL static __constant__ const
#include "h3_core.h"
#include "bng_core.h"
#include "pip_core.h"
#include "h3_ring.h"
#include "kernels.h"
#include "raster.h"

namespace mgpu {

// the join's tile: one workgroup of kBlock threads, kItems points per thread
#ifndef MGPU_BLOCK
#define MGPU_BLOCK 64
#endif
constexpr int kBlock = MGPU_BLOCK;
constexpr int kItems = 4;
constexpr int kTile = kBlock * kItems;
constexpr int kStreamBlock = 256;  // the per-point kernels (cells, st_contains)
static_assert(kTile <= 1024, "point-in-tile indices are 10 bits");

constexpr uint64_t kNoDst = ~0ULL;
constexpr int kScanGroup = 32;  // tiles per first-level scan group (<= 64)

// ---------------------------------------------------------------- point -> cell

constexpr uint32_t kAllFaces = (1u << 20) - 1;

__device__ __forceinline__ void count_wave(unsigned long long* ctr, bool pred) {
  unsigned long long b = __ballot(pred);
  if (b && (threadIdx.x & 63) == (__ffsll((long long)b) - 1)) atomicAdd(ctr, (unsigned long long)__popcll(b));
}

// The H3 route (h3_core.h route_face_ijk: H3's own formulas, libm calls out of line)
// is needed for ~1 point in 1e6 -- those whose fast-path decisions fall inside the
// tie band.  It is never called from the streaming kernels: a call makes the caller
// allocate the callee-saved VGPRs the route's calls need (84+), which would cap the
// streaming kernels' occupancy.  They hand the rare points to *_fix kernels instead.

// IndexSystem.pointToIndex over a batch.  H3: fast projection; near-ties are queued
// (ties[0] = count, ties[1 ..] = point indices) for cells_fix_kernel.
template <int IS>
__global__ __launch_bounds__(kStreamBlock) void cells_kernel(const double* __restrict__ x, const double* __restrict__ y,
                                                       int64_t n, int res, int64_t* __restrict__ out,
                                                       unsigned long long* __restrict__ counters,
                                                       unsigned long long* __restrict__ ties, int64_t tie_cap,
                                                       const uint8_t* __restrict__ valid, int64_t voff) {
  const double k_res = h3::k_of_res(res);
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    bool ok;
    int64_t c = 0;
    const double px = x[i], py = y[i];
    if (!pt_valid(valid, voff, i)) {
      ok = true;  // a null row: null out (cell 0 here, the caller's validity says null)
    } else if (IS == MGPU_H3) {
      ok = isfinite(px) && isfinite(py);
      if (ok) {
        const h3::FastHex f = h3::fast_hex2d(h3::to_radians_fast(py), h3::to_radians_fast(px), res, k_res, kAllFaces);
        if (f.tie) {
          const unsigned long long q = atomicAdd(&ties[0], 1ull);
          if ((int64_t)q < tie_cap) ties[1 + q] = (unsigned long long)i;
        } else {
          c = (int64_t)h3::face_ijk_to_h3_fast(f.face, f.ijk, res);
        }
      }
    } else {
      ok = bng::point_to_cell(px, py, res, &c);
    }
    out[i] = c;
    count_wave(&counters[2], !ok);
  }
}

// A near-tie of the H3 route, queued for the host's libm pass (JoinArgs.tie_queue)
__device__ __forceinline__ void tie_record(uint64_t* tq, int64_t cap, int64_t pos, double x, double y, uint64_t key) {
  const unsigned long long q = atomicAdd((unsigned long long*)tq, 1ull);
  if ((int64_t)q < cap) {
    uint64_t* r = tq + 2 + 4 * q;
    r[0] = (uint64_t)pos;
    r[1] = (uint64_t)__double_as_longlong(x);
    r[2] = (uint64_t)__double_as_longlong(y);
    r[3] = key;
  }
}

// The queued near-ties by the H3 route; if the queue overflowed, every point again
// (fast path + route where needed).  The route's own near-ties go to tie_queue with
// their (correctly rounded) cell.
__global__ __launch_bounds__(kStreamBlock) void cells_fix_kernel(const double* __restrict__ x, const double* __restrict__ y,
                                                           int64_t n, int res, int64_t* __restrict__ out,
                                                           unsigned long long* __restrict__ counters,
                                                           const unsigned long long* __restrict__ ties,
                                                           int64_t tie_cap, uint64_t* __restrict__ tq, int64_t tq_cap,
                                                           const uint8_t* __restrict__ valid, int64_t voff) {
  const int64_t nt = (int64_t)ties[0];
  const bool all = nt > tie_cap;
  const int64_t m = all ? n : nt;
  const double k_res = h3::k_of_res(res);
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < m; q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = all ? q : (int64_t)ties[1 + q];
    const double px = x[i], py = y[i];
    bool tie = false;
    if (isfinite(px) && isfinite(py) && pt_valid(valid, voff, i)) {
      h3::FastHex f = h3::fast_hex2d(h3::to_radians_fast(py), h3::to_radians_fast(px), res, k_res, kAllFaces);
      if (f.tie) h3::route_face_ijk(h3::to_radians(py), h3::to_radians(px), res, &f.face, &f.ijk, &tie);
      const int64_t c = (int64_t)h3::face_ijk_to_h3_fast(f.face, f.ijk, res);
      out[i] = c;
      if (tie) tie_record(tq, tq_cap, i, px, py, (uint64_t)c);
    }
    count_wave(&counters[1], tie);
  }
}

// wave64 inclusive prefix sum of u32
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t t = __shfl_up(v, d, 64);
    if (lane >= d) v += t;
  }
  return v;
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// One workgroup = one tile of kTile consecutive points, in three phases:
//  1  lane l evaluates points l, l+256, l+512, l+768 (coalesced 8-byte loads): cell
//     -> one hash probe -> the cell's chip range and core-chip mask.  Core chips are
//     matches at once; every border chip becomes a candidate (chip, point, slot j)
//     in the tile's LDS list (a full list: the lane evaluates it on the spot);
//  2  lane per candidate: st_contains by the chip's strip index (pip_core.h
//     chip_contains_strips: envelope, rectangle shortcut, ray crossing over the
//     edges of the point's y-strip only); a hit sets bit j of the point's mask;
//  3  lane l owns points 4l .. 4l+3 (input order): matches = mask bits (chip order
//     == polygon-id order), block scan for positions within the tile, records
//     {point-in-tile, polygon id} staged in LDS and written to the tile's slot as
//     one contiguous run.
// Tiles with a near-tie point, a cell of more than 32 chips or more than kCandCap
// candidates are abandoned by the streaming kernel after phase 1 and redone by
// pip_fix_kernel, which evaluates list overflows on the spot and chips past the
// 32nd of a cell in phase 3.
#ifndef MGPU_CANDCAP
#define MGPU_CANDCAP 512  // (256: BNG res 3's 1.25 candidates per point sent most tiles to the fix kernel)
#endif
constexpr int kCandCap = MGPU_CANDCAP;
constexpr int kMixCap = kTile / 2;  // mixed-cell candidates (phase 2b), after the list in s_buf
// Coordinates phase 1 leaves in LDS for phases 2 / 2b (the rest are re-read), per
// join_tile mode -- A/B r3 (profiles/r3_stash_ab.txt): the fused kernel keeps every
// point with a candidate (BNG res 3's 1.25 candidates per point re-read most coordinates
// with 80 candidate entries: C4 r3 join 3.69 ms per 1e8, 320 entries 2.78, per point
// 2.55; r4 1.75 / 1.71 / 1.67); the binned join the first 160 candidates (C3 3.29 ->
// 3.17; 256 and more cost it occupancy), the split pipeline's mixed tiles 80 (160 and
// more: C5 +4%)
// intermediate arrays written once and read once by a later kernel (classify codes, the
// binned coordinates / perm, the gathered answers): non-temporal stores (A/B r3)
#ifndef MGPU_NT_INTER
#define MGPU_NT_INTER 0
#endif
#if MGPU_NT_INTER
#define MGPU_ST_INTER(v, ptr) __builtin_nontemporal_store((v), (ptr))
#else
#define MGPU_ST_INTER(v, ptr) (*(ptr) = (v))
#endif
// the edge-parallel walk over LDS-staged runs (below): 0 off, 1 every tile mode, 2 the split
// pipeline's mixed tiles only -- A/B round 6 (profiles/r6/ab_edgepar.txt): C5 mixed 0.353 ->
// 0.263 ms per 1e8 points (long fractal strips), C3 binned join 3.49 -> 3.51, C4 fused join
// 1.664 -> 1.683 (short strips: the flat layout costs them registers and an LDS round trip)
#ifndef MGPU_EDGE_PAR
#define MGPU_EDGE_PAR 2
#endif
#ifndef MGPU_SPLIT_WALK
#define MGPU_SPLIT_WALK 1  // (A/B r3, profiles/r3_split_walk_ab.txt: C3 binned join -3.8%, C4 r4 -1.6%)
#endif
#ifndef MGPU_STASH_FUSED
#define MGPU_STASH_FUSED 0
#endif
#ifndef MGPU_STASH_BINNED
#define MGPU_STASH_BINNED 160
#endif
#ifndef MGPU_STASH_MIXED
#define MGPU_STASH_MIXED 80
#endif
// (MGPU_STASH_FUSED 0: the fused kernel keeps EVERY point of the tile that has a
// candidate, by point -- kTile entries, no re-read at all)
template <int G>
constexpr int stash_of() {
  return G == 2 ? MGPU_STASH_MIXED : G == 1 ? MGPU_STASH_BINNED : (MGPU_STASH_FUSED ? MGPU_STASH_FUSED : kTile);
}
template <int G>
constexpr bool point_stash() {
  return G == 0 && MGPU_STASH_FUSED == 0;
}
#ifndef MGPU_OUTCAP
#define MGPU_OUTCAP 896
#endif
constexpr int kOutCap = MGPU_OUTCAP;  // pairs a tile stages in LDS (the fused lists' bytes)
static_assert(kCandCap * 2 + kMixCap * 2 + stash_of<0>() * 16 <= kOutCap * 6, "phase 1-2 lists fit the staging buffer");
constexpr int kMaskBits = 32;
// A tile reserves kSlot records in its slot; more go to the overflow pool.
constexpr int kSlot = 2 * kTile;

// chips of a cell: first, count, core mask (bits < 16)
struct Range {
  uint32_t first;
  uint32_t count;
  uint32_t core;
};

__device__ __forceinline__ Range probe_range(const ChipTableView& t, uint64_t key) {
  uint32_t h = cell_hash(key) & t.hash_mask;
  for (uint32_t k = 0; k <= t.max_probe; k++) {
    const HashSlot s = t.slots[h];
    if (s.count == 0) break;
    if (s.cell == key) return Range{s.first, s.count, s.core_mask};
    h = (h + 1) & t.hash_mask;
  }
  return Range{0, 0, 0};
}

// The chips of the point's cell.  *ok = false for non-finite coordinates.  *tie: in
// the fast kernel (SLOW = false), the projection is in its tie band (the tile goes
// to pip_fix_kernel); in the fix kernel, the H3 route's own near-tie flag (counted).
// A dense-grid probe is left to the caller: *gi = the grid entry to load (the loads of
// a lane's four points then fly together), else *gi = kNoEntry and the range is final.
constexpr uint32_t kNoEntry = 0xFFFFFFFFu;
// binned H3 slot keys (bin_key_of): a grid entry index | kKeyDeep, or one of the codes
constexpr uint32_t kKeyNone = 0xFFFFFFFFu, kKeyBad = 0xFFFFFFFEu, kKeyTie = 0xFFFFFFFDu;
constexpr uint32_t kKeyDeep = 0x80000000u, kKeyIndex = 0x3FFFFFFFu;

__device__ __forceinline__ Range grid_range(uint64_t e, bool ans) {
  return Range{(uint32_t)e, grid_count(e, ans), (uint32_t)(e >> 48)};
}

// The H3 route for a point the fast projection could not decide (fix kernels only).  A
// host override (the reference's libm decided the point) replaces the route's (face,
// ijk) without computing it; else a near-tie of the route itself is queued for the
// host's libm pass.  `p` = the kernel's point index (the binned slot in the binned
// pipeline: a.pos_of maps it to the input position, which keys the queue and the
// overrides).
__device__ __forceinline__ int64_t input_pos(const JoinArgs& a, int64_t p) {
  return a.pos_of ? (int64_t)a.pos_of[p] : p;
}
__device__ __forceinline__ void route_point(const JoinArgs& a, int64_t p, double px, double py, h3::FastHex* f,
                                                      bool* tie) {
  const int64_t pos = input_pos(a, p);
  if (a.n_ovr) {
    int64_t lo = 0, hi = a.n_ovr;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (a.ovr[2 * mid] < (uint64_t)pos)
        lo = mid + 1;
      else
        hi = mid;
    }
    if (lo < a.n_ovr && a.ovr[2 * lo] == (uint64_t)pos) {
      const uint64_t key = a.ovr[2 * lo + 1];
      f->face = (int)(key >> 56);
      h3::IJK c{(int)((key >> 28) & 0xFFFFFFFULL) - (1 << 27), (int)(key & 0xFFFFFFFULL) - (1 << 27), 0};
      h3::ijk_normalize(c);
      f->ijk = c;
      *tie = true;  // (not queued again: the override table is the run's audit list)
      return;
    }
  }
  h3::route_face_ijk(h3::to_radians(py), h3::to_radians(px), a.res, &f->face, &f->ijk, tie);
  if (*tie && a.tie_queue) tie_record(a.tie_queue, a.tie_cap, pos, px, py, h3::lattice_key(f->face, f->ijk));
}

template <int IS, bool SLOW>
__device__ __forceinline__ Range chip_probe(const JoinArgs& a, int64_t p, double px, double py, bool* ok, bool* tie,
                                            uint32_t* gi, bool* deep = nullptr) {
  const ChipTableView& t = a.chips;
  const int res = a.res;
  *tie = false;
  *gi = kNoEntry;
  if (deep) *deep = false;
  if (IS == MGPU_BNG) {
    *ok = px == px && py == py;  // pointToIndex rejects NaN only
    if (!*ok || !a.res_match) return Range{0, 0, 0};
    const int32_t eI = bng::d2i(px), nI = bng::d2i(py);
    // whole-metre coordinates in [0, 1e7): the cell id is a bijection of (eI / edge,
    // nI / edge) (capi.cpp build_bng_dense), so the dense grid replaces id + hash probe
    if (t.probe_mode == kProbeDense && res == t.res && (uint32_t)eI < 10000000u && (uint32_t)nI < 10000000u) {
      const uint32_t ed = t.bng_edge;
      uint32_t col = (uint32_t)((double)eI * t.bng_inv_edge);
      uint32_t row = (uint32_t)((double)nI * t.bng_inv_edge);
      col = col * ed > (uint32_t)eI ? col - 1 : ((col + 1) * ed <= (uint32_t)eI ? col + 1 : col);
      row = row * ed > (uint32_t)nI ? row - 1 : ((row + 1) * ed <= (uint32_t)nI ? row + 1 : row);
      const DenseFace& D = t.dense[0];
      const uint32_t da = col - (uint32_t)D.a0, db = row - (uint32_t)D.b0;
      if (da >= D.w || db >= D.h) return Range{0, 0, 0};
      *gi = D.base + db * D.w + da;
      return Range{0, 0, 0};
    }
    int64_t c;
    bng::point_to_cell(px, py, res, &c);
    return probe_range(t, (uint64_t)c);
  }
  *ok = isfinite(px) && isfinite(py);
  if (!*ok || !a.res_match) return Range{0, 0, 0};
  const double lat = h3::to_radians_fast(py), lon = h3::to_radians_fast(px);
  if (t.probe_mode != kProbeCellId) {
    // outside the chip cells' bounding box no cell can match
    if (!(px >= t.bbox[0] && px <= t.bbox[2] && py >= t.bbox[1] && py <= t.bbox[3])) return Range{0, 0, 0};
    h3::FastHex f = h3::fast_hex2d(lat, lon, res, t.k_res, t.face_mask);
    if (deep) *deep = f.deep;
    if (f.tie) {
      if (a.tie_host) {
        // the host decides: queued with the fast cell, joined with it (a fix kernel
        // redoing the tile for another reason finds the point queued already)
        if (!SLOW) tie_record(a.tie_queue, a.tie_cap, input_pos(a, p), px, py, h3::lattice_key(f.face, f.ijk));
      } else if (!SLOW) {
        *tie = true;
        return Range{0, 0, 0};
      } else {
        route_point(a, p, px, py, &f, tie);
      }
    }
    if (t.probe_mode == kProbeDense) {
      const int32_t ga = f.ijk.i - f.ijk.k, gb = f.ijk.j - f.ijk.k;
      DenseFace D;
      const int fu = __builtin_amdgcn_readfirstlane(f.face);
      if (__all(f.face == fu)) {
        D = t.dense[fu];
      } else {
        D = t.dense[f.face];
      }
      const uint32_t da = (uint32_t)(ga - D.a0), db = (uint32_t)(gb - D.b0);
      if (da >= D.w || db >= D.h) return Range{0, 0, 0};
      *gi = D.base + db * D.w + da;
      return Range{0, 0, 0};
    }
    return probe_range(t, h3::lattice_key(f.face, f.ijk));
  }
  // (cell-id probing: res made opaque here, so the per-resolution predicates of
  // k_of_res / face_ijk_to_h3_fast are computed on this path instead of being hoisted
  // into SGPRs across the callers' point loops -- there they spilled to VGPR lanes)
  int res_o = res;
#ifdef __HIP_DEVICE_COMPILE__
  asm volatile("" : "+s"(res_o));
#endif
  h3::FastHex f = h3::fast_hex2d(lat, lon, res_o, t.k_res > 0 ? t.k_res : h3::k_of_res(res_o), kAllFaces);
  if (f.tie) {
    if (a.tie_host) {
      if (!SLOW) tie_record(a.tie_queue, a.tie_cap, input_pos(a, p), px, py, h3::lattice_key(f.face, f.ijk));
    } else if (!SLOW) {
      *tie = true;
      return Range{0, 0, 0};
    } else {
      route_point(a, p, px, py, &f, tie);
    }
  }
  return probe_range(t, h3::face_ijk_to_h3_fast(f.face, f.ijk, res_o));
}

__device__ __forceinline__ bool chip_is_core(const ChipTableView& t, const Range& r, uint32_t j) {
  return j < 16 ? ((r.core >> j) & 1) : (t.chip_flags[r.first + j] & kChipCore) != 0;
}

// Phase 1 for one point: its core chips match at once; every border chip becomes a
// candidate (chip, point, slot j) in the tile's LDS list (a full list: the fast kernel
// abandons the tile, the fix kernel evaluates the candidate on the spot).
template <bool SLOW, int CAND_CAP, int STASH, bool PT_STASH = false>
__device__ __forceinline__ void phase1_item(const ChipTableView& t, int li, const Range& r, double px, double py,
                                            bool& any_tie, uint32_t* s_ncand, uint16_t* s_cand_pj,
                                            double2* s_cand_xy, uint32_t* s_first, uint16_t* s_cnt,
                                            uint32_t* s_mask, uint32_t answer = kNoCellAns, bool deep = false) {
  // the streaming kernel keeps no sequential PIP path (its registers would cap
  // occupancy): a cell with more than 32 chips sends the tile to pip_fix_kernel
  if (!SLOW && r.count > (uint32_t)kMaskBits) any_tie = true;
  if (deep && r.count == 1 && (r.core & kCoreWhole)) answer = 1u;  // (H3 whole-cell chip, capi.cpp mark_whole_cells)
  if (answer != kNoCellAns) {  // the cell's answer grid decided every chip (BNG)
    s_first[li] = r.first;
    if (SLOW) s_cnt[li] = (uint16_t)r.count;
    s_mask[li] = answer;
    return;
  }
  const uint32_t nj = r.count < (uint32_t)kMaskBits ? r.count : (uint32_t)kMaskBits;
  const uint32_t lowm = nj >= 32 ? 0xFFFFFFFFu : ((1u << nj) - 1);
  uint32_t border = ~r.core & lowm;
  for (uint32_t j = 16; j < nj; j++)
    if (t.chip_flags[r.first + j] & kChipCore) border &= ~(1u << j);
  uint32_t mask = lowm & ~border;
  if (border) {
    if (PT_STASH) s_cand_xy[li] = make_double2(px, py);
    const uint32_t nb = __popc(border);
    uint32_t j0 = atomicAdd(s_ncand, nb);
    for (uint32_t b = border; b; b &= b - 1) {
      const uint32_t j = __builtin_ctz(b);
      if (j0 < (uint32_t)CAND_CAP) {
        s_cand_pj[j0] = (uint16_t)(li | (j << 10));
        if (!PT_STASH && j0 < (uint32_t)STASH) s_cand_xy[j0] = make_double2(px, py);
      } else if (!SLOW) {
        any_tie = true;  // list full: the fix kernel evaluates such tiles
      } else if (pip::chip_contains_strips(t, r.first + j, px, py)) {
        mask |= 1u << j;  // list full: evaluate here
      }
      j0++;
    }
  }
  s_first[li] = r.first;
  // (the streaming kernel reads no counts: its s_cnt doubles as the raster's list)
  if (SLOW) s_cnt[li] = (uint16_t)(r.count > 0xFFFF ? 0xFFFF : r.count);
  s_mask[li] = mask;
}



// Profiling builds (-DMGPU_STAMPS): thread 0 of each tile adds the wall-clock ticks
// (100 MHz) spent in each phase to counters[9 + phase]: 1 = phase 1 (with a pixel index:
// its pass B), 2 = phase 2, 3 = phase 2b, 4 = phase 3 (output), 5 = pixel-index pass A.
#ifdef MGPU_STAMPS
#define MGPU_STAMP(ph)                                                              \
  do {                                                                              \
    if (threadIdx.x == 0) {                                                         \
      const uint64_t now = wall_clock64();                                          \
      if ((ph) > 0) atomicAdd(&a.counters[9 + (ph)], (unsigned long long)(now - st_t)); \
      st_t = now;                                                                   \
    }                                                                               \
  } while (0)
#else
#define MGPU_STAMP(ph) \
  do {             \
  } while (0)
#endif

// the split pipeline's chunk (classify_kernel / split_emit_kernel workgroup): its points
// and at most kChunkTiles tiles of mixed points.  A mixed tile holds kGTile points; mixed
// points lie near chip edges, with ~2 border-chip candidates each, so its candidate
// lists are longer (kGCandCap, kGMixCap).
constexpr int kChunk = 4096;
constexpr int kGTile = kTile;
constexpr int kChunkTiles = kChunk / kGTile;
constexpr int kGCandCap = 3 * kTile;
constexpr int kGMixCap = kTile;


// One tile (see the phase comment above).  SLOW = false: the streaming kernel; a
// tile with a near-tie point is queued for pip_fix_kernel and abandoned after phase 1.
// SLOW = true: the fix kernel; near-ties go through the H3 route.
// G = true: the split pipeline's mixed points -- tile = chunk * kChunkTiles + t covers
// list positions [t * kTile, ...) of the chunk's mixed list; the phases are the same,
// the result is each point's (first chip, match mask) in mixed_res (no pair records).
template <int IS, bool SLOW, int G = 0>
__device__ __forceinline__ void join_tile(const JoinArgs& a, const uint32_t tile) {
  __shared__ uint32_t s_ncand, s_nmix;
  __shared__ uint32_t s_wave_tot[kBlock / 64];
  __shared__ uint32_t s_first[kTile];   // first chip of the point's cell
  __shared__ __attribute__((aligned(16))) uint32_t s_mask[kTile];  // bit j: chip first + j matches (j < 32)
  // chips of the point's cell (0: none) -- read by the fix kernels only; the fused
  // streaming kernel's raster pass lists its mixed points here; the split / binned
  // streaming tiles use none of it (their LDS sets their occupancy)
  __shared__ uint16_t s_cnt[(SLOW || G == 0) ? kTile : 1];
  // phases 1-2: candidate list; phase 3: output staging (same bytes)
  constexpr int kCap = G ? kGCandCap : kCandCap, kMix = G ? kGMixCap : kMixCap;
  constexpr int kStash = stash_of<G>();
  __shared__ __attribute__((aligned(16))) uint8_t s_buf[G ? kStash * 16 + kCap * 2 + kMix * 2 : kOutCap * 6];
  // candidate c = chip s_first[li] + j of point li, s_cand_pj[c] = li | j << 10; the
  // first kStash candidates also keep the point's coordinates (no re-read in phase 2)
  double2* s_cand_xy = (double2*)s_buf;                             // [kStash]
  uint16_t* s_cand_pj = (uint16_t*)(s_buf + kStash * 16);           // [kCandCap]
  uint16_t* s_mix = (uint16_t*)(s_buf + kStash * 16 + kCap * 2);  // [kMix] candidate index
  int32_t* s_out_poly = (int32_t*)s_buf;                          // [kOutCap]
  uint16_t* s_out_li = (uint16_t*)(s_buf + kOutCap * 4);          // [kOutCap]
  // G == 2 (the split pipeline): the tile's slice of its chunk's mixed list, each item's
  // point index within the chunk; G == 1 (binned): the chunk's points in order
  __shared__ uint16_t s_gidx[G == 2 ? kTile : 1];

  const uint32_t chunk = G ? tile / kChunkTiles : 0u;
  const int64_t gbase = (int64_t)chunk * kChunk;                        // first point of the chunk
  const int64_t lbase = gbase + (int64_t)(tile % kChunkTiles) * kGTile;  // first list position
  uint32_t gcount = 0;
  if (G) {
    const int64_t left = a.n - gbase;
    const uint32_t nm = G == 2 ? a.chunk_mixed[chunk] : (uint32_t)(left <= 0 ? 0 : (left < kChunk ? left : kChunk));
    const uint32_t t0 = (tile % kChunkTiles) * kGTile;
    if (nm <= t0) return;
    gcount = nm - t0 < (uint32_t)kGTile ? nm - t0 : (uint32_t)kGTile;
    if (G == 2)
      for (uint32_t li = threadIdx.x; li < (uint32_t)kTile; li += kBlock)
        s_gidx[li] = li < gcount ? a.mixed_idx[lbase + li] : (uint16_t)0;
  }
  // (binned, MGPU_BIN_JOIN_COUNTS: the input positions of slots 4 lane .. 4 lane + 3 load
  // now, with the tile's first loads, and are used only at its end -- each slot's input
  // chunk, for the chunk pair counts)
  uint32_t ckp[G == 1 ? 4 : 1];
  if (G == 1 && a.in_chunk_pairs) {
    const uint32_t s0 = 4u * threadIdx.x;
    if (s0 + 3 < gcount) {
      const uint4 q = *(const uint4*)(a.pos_of + lbase + s0);  // (perm: 256-byte aligned, lbase % 256 == 0)
      ckp[0] = q.x, ckp[1] = q.y, ckp[2] = q.z, ckp[3] = q.w;
    } else {
#pragma unroll
      for (int i = 0; i < 4; i++) ckp[i] = s0 + i < gcount ? a.pos_of[lbase + s0 + i] : 0u;
    }
  }
#define MGPU_PT(li) (G == 2 ? gbase + (int64_t)s_gidx[li] : G == 1 ? lbase + (li) : (int64_t)tile * kTile + (li))
#define MGPU_VALID(li) (G ? (uint32_t)(li) < gcount : (int64_t)tile * kTile + (li) < a.n)


#ifdef MGPU_STAMPS
  uint64_t st_t = 0;
#endif
  if (threadIdx.x == 0) {
    s_ncand = 0;
    s_nmix = 0;
  }
  __syncthreads();
  const ChipTableView& t = a.chips;
  const int64_t base = (int64_t)tile * kTile;
  const bool res_match = a.res_match;

  MGPU_STAMP(0);
  // ---- phase 1: cells, core matches, candidates
  bool any_tie = false, any_bad = false;
  uint32_t n_tie_pts = 0;  // (SLOW: the lane's near-tie points, mgpu_stats.n_near_ties)
#ifndef MGPU_NT_POINTS
#define MGPU_NT_POINTS 1
#endif
#if MGPU_NT_POINTS
#define MGPU_LDPT(ptr) __builtin_nontemporal_load(ptr)
#else
#define MGPU_LDPT(ptr) (*(ptr))
#endif
  if (!G && !SLOW && kBlock == 64 && t.raster_mode != kRasterNone && res_match && (IS == MGPU_H3 || a.res == t.res)) {
    // pass A: the lane's four points load together, then their pixels' classes: a
    // pure pixel's matches are final (no projection, no candidates); the rest are
    // listed (s_cnt is free in the streaming kernel) for pass B
    const int lane = threadIdx.x;
    double bx[kItems], by[kItems];
#pragma unroll
    for (int k = 0; k < kItems; k++) {
      const int64_t p = base + k * kBlock + lane;
      bx[k] = by[k] = 0.0;
      if (p < a.n) {
        bx[k] = MGPU_LDPT(&a.x[p]);
        by[k] = MGPU_LDPT(&a.y[p]);
      }
    }
    uint32_t ri[kItems], gix[kItems], sb[kItems];
#pragma unroll
    for (int k = 0; k < kItems; k++) {
      ri[k] = kNoPixel;
      gix[k] = 0;
      sb[k] = 0;
      if (base + k * kBlock + lane < a.n && pt_valid(a.valid, a.valid_off, base + k * kBlock + lane)) {
        bool ok;
        ri[k] = raster_index<IS>(t, bx[k], by[k], &ok, &gix[k], &sb[k]);
        any_bad |= !ok;
      }
    }
    uint32_t cl[kItems];
    uint64_t ge[kItems];
#pragma unroll
    for (int k = 0; k < kItems; k++) {
      cl[k] = ri[k] < kRasterFull ? raster_class(t, ri[k], sb[k]) : (ri[k] == kRasterFull ? kPixMixed : kPixEmpty);
      if (IS == MGPU_BNG) ge[k] = ri[k] < kRasterFull ? t.grid[gix[k]] : 0ull;  // (independent of the pixel load)
    }
    uint64_t ce[kItems];
#pragma unroll
    for (int k = 0; k < kItems; k++) {
      if (IS == MGPU_BNG)  // the pixel holds the mask of the cell's chips
        ce[k] = (cl[k] != kPixEmpty && cl[k] != kPixMixed) ? ((uint64_t)(uint32_t)ge[k] | ((uint64_t)cl[k] << 32)) : 0ull;
      else
        ce[k] = (cl[k] != kPixEmpty && cl[k] != kPixMixed) ? t.raster_cls[cl[k]] : 0ull;
    }
    uint16_t* s_list = s_cnt;
    uint32_t nlist = 0;
#pragma unroll
    for (int k = 0; k < kItems; k++) {
      const int li = k * kBlock + lane;
      const bool mixed = cl[k] == kPixMixed;
      if (!mixed) {
        s_first[li] = (uint32_t)ce[k];
        s_mask[li] = (uint32_t)(ce[k] >> 32);
      }
      const unsigned long long bal = __ballot(mixed);
      if (mixed) s_list[nlist + __popcll(bal & ((1ull << lane) - 1ull))] = (uint16_t)li;
      nlist += (uint32_t)__popcll(bal);
    }
    __syncthreads();
    MGPU_STAMP(5);  // (profiling: pass A)
    // pass B: the listed points, 64 at a time with every lane busy (coordinates from
    // the owning lane's registers)
    for (uint32_t q0 = 0; q0 < nlist; q0 += kBlock) {
      const uint32_t q = q0 + lane;
      const int li = q < nlist ? (int)s_list[q] : 0;
      const int owner = li & 63, kk = li >> 6;
      double px = 0.0, py = 0.0;
#pragma unroll
      for (int k = 0; k < kItems; k++) {
        const double vx = __shfl(bx[k], owner, 64), vy = __shfl(by[k], owner, 64);
        if (kk == k) {
          px = vx;
          py = vy;
        }
      }
      if (q < nlist) {
        bool ok, tie;
        uint32_t gi;
        Range r = chip_probe<IS, SLOW>(a, base + li, px, py, &ok, &tie, &gi);
        if (gi != kNoEntry) r = grid_range(t.grid[gi], t.cell_ans_row != nullptr);
        any_tie |= tie;
        phase1_item<SLOW, kCap, kStash, point_stash<G>()>(t, li, r, px, py, any_tie, &s_ncand, s_cand_pj, s_cand_xy, s_first, s_cnt, s_mask);
      }
    }
  } else if (IS == MGPU_BNG) {
    // the cell is a few integer ops: the lane's four points load together, then
    // their four grid entries (a wave's loads complete in order, so a load issued
    // behind a point prefetch would wait for it)
    double bx[kItems], by[kItems];
#pragma unroll
    for (int k = 0; k < kItems; k++) {
      const int li = k * kBlock + threadIdx.x;
      bx[k] = by[k] = 0.0;
      if (MGPU_VALID(li)) {
        const int64_t p = MGPU_PT(li);
        bx[k] = MGPU_LDPT(&a.x[p]);
        by[k] = MGPU_LDPT(&a.y[p]);
      }
    }
    Range r[kItems];
    uint32_t gi[kItems];
#pragma unroll
    for (int k = 0; k < kItems; k++) {
      r[k] = Range{0, 0, 0};
      gi[k] = kNoEntry;
      if (MGPU_VALID(k * kBlock + threadIdx.x) && pt_valid(a.valid, a.valid_off, MGPU_PT(k * kBlock + threadIdx.x))) {
        bool ok, tie;
        r[k] = chip_probe<IS, SLOW>(a, MGPU_PT(k * kBlock + threadIdx.x), bx[k], by[k], &ok, &tie, &gi[k]);
        any_bad |= !ok;
      }
    }
    uint64_t ge[kItems];
#pragma unroll
    for (int k = 0; k < kItems; k++) ge[k] = gi[k] != kNoEntry ? t.grid[gi[k]] : 0;
    // a flagged cell's answer grid (chip_table.h cell_ans): its row base (a small table),
    // then the square
    uint32_t av[kItems];
#pragma unroll
    for (int k = 0; k < kItems; k++) {
      av[k] = kNoCellAns;
      if (t.cell_ans_row && (ge[k] & kCellAnsFlag)) {
        const uint32_t eI = (uint32_t)bng::d2i(bx[k]), nI = (uint32_t)bng::d2i(by[k]), ed = t.bng_edge;
        const uint32_t col = div_fix(eI, ed, t.bng_inv_edge), row = div_fix(nI, ed, t.bng_inv_edge);
        const uint32_t u = div_fix(eI - col * ed, t.cell_ans_sw, t.cell_ans_inv_sw);
        const uint32_t v = div_fix(nI - row * ed, t.cell_ans_sw, t.cell_ans_inv_sw);
        const uint32_t ai = t.cell_ans_row[row - (uint32_t)t.dense[0].b0] + cell_ans_index(ge[k]);
        const uint16_t m = t.cell_ans[((size_t)ai * t.cell_ans_g + v) * t.cell_ans_g + u];
        if (m != kCellAnsMixed) av[k] = m;
      }
    }
#pragma unroll
    for (int k = 0; k < kItems; k++) {
      if (gi[k] != kNoEntry) r[k] = grid_range(ge[k], t.cell_ans_row != nullptr);
      phase1_item<SLOW, kCap, kStash, point_stash<G>()>(t, k * kBlock + threadIdx.x, r[k], bx[k], by[k], any_tie, &s_ncand, s_cand_pj,
                        s_cand_xy, s_first, s_cnt, s_mask, av[k]);
    }
  } else if (!SLOW && G == 1 && IS == MGPU_H3 && a.bin_key != nullptr) {
    // binned slots with their grid keys (bin_scatter_kernel): every grid load in flight at
    // once, no projection here
    uint32_t kv[kItems];
    double bx[kItems], by[kItems];
#pragma unroll
    for (int k = 0; k < kItems; k++) {
      const int li = k * kBlock + threadIdx.x;
      kv[k] = kKeyNone;
      bx[k] = by[k] = 0.0;
      if (MGPU_VALID(li)) {
        const int64_t p = MGPU_PT(li);
        kv[k] = MGPU_LDPT(&a.bin_key[p]);
        bx[k] = MGPU_LDPT(&a.x[p]);
        by[k] = MGPU_LDPT(&a.y[p]);
      }
    }
    uint64_t ge[kItems];
#pragma unroll
    for (int k = 0; k < kItems; k++) ge[k] = kv[k] < kKeyTie ? t.grid[kv[k] & kKeyIndex] : 0ull;
#pragma unroll
    for (int k = 0; k < kItems; k++) {
      const bool hit = kv[k] < kKeyTie;
      any_bad |= kv[k] == kKeyBad;
      any_tie |= kv[k] == kKeyTie;
      const Range r = hit ? grid_range(ge[k], t.cell_ans_row != nullptr) : Range{0, 0, 0};
      phase1_item<SLOW, kCap, kStash, point_stash<G>()>(t, k * kBlock + threadIdx.x, r, bx[k], by[k], any_tie, &s_ncand,
                                                        s_cand_pj, s_cand_xy, s_first, s_cnt, s_mask, kNoCellAns,
                                                        hit && (kv[k] & kKeyDeep) != 0u);
    }
  } else {
    // one item ahead: item k + 1's coordinates load while item k projects
    double nx = 0.0, ny = 0.0;
    if (MGPU_VALID(threadIdx.x)) {
      nx = MGPU_LDPT(&a.x[MGPU_PT(threadIdx.x)]);
      ny = MGPU_LDPT(&a.y[MGPU_PT(threadIdx.x)]);
    }
#pragma unroll 1
    for (int k = 0; k < kItems; k++) {
      const int li = k * kBlock + threadIdx.x;
      const int64_t p = MGPU_PT(li);
      Range r{0, 0, 0};
      const double px = nx, py = ny;
      if (k + 1 < kItems && MGPU_VALID(li + kBlock)) {
        nx = MGPU_LDPT(&a.x[MGPU_PT(li + kBlock)]);
        ny = MGPU_LDPT(&a.y[MGPU_PT(li + kBlock)]);
      }
      bool deep = false;
      if (MGPU_VALID(li) && pt_valid(a.valid, a.valid_off, p)) {
        bool ok, tie;
        uint32_t gi;
        r = chip_probe<IS, SLOW>(a, p, px, py, &ok, &tie, &gi, &deep);
        if (gi != kNoEntry) r = grid_range(t.grid[gi], t.cell_ans_row != nullptr);
        n_tie_pts += (SLOW && tie) ? 1u : 0u;
        any_bad |= !ok;
        any_tie |= tie;
      }
      phase1_item<SLOW, kCap, kStash, point_stash<G>()>(t, li, r, px, py, any_tie, &s_ncand, s_cand_pj, s_cand_xy, s_first, s_cnt, s_mask,
                                                        kNoCellAns, deep);
    }
  }
  count_wave(&a.counters[2], any_bad);
  if (SLOW) {
    const uint32_t wt = wave_sum_u32(n_tie_pts);
    if ((threadIdx.x & 63) == 0 && wt) atomicAdd(&a.counters[1], (unsigned long long)wt);
  }
  if (!SLOW && __syncthreads_or(any_tie)) {
    // a near-tie (or a case only the fix kernel handles): the tile is redone there
    if (threadIdx.x == 0) {
      const unsigned int q = atomicAdd(a.n_dirty, 1u);
      a.dirty[q] = tile;
      if (!G) {
        a.tile_count[tile] = 0;
        a.tile_where[tile] = kNoDst;
      }
    }
    return;
  }
  __syncthreads();
  MGPU_STAMP(1);
  const uint32_t ncand = s_ncand < (uint32_t)kCap ? s_ncand : (uint32_t)kCap;
  // per scan group, not one global counter: same-address atomics from every tile serialize
  if (threadIdx.x == 0 && s_ncand) atomicAdd(&a.group_cand[G ? chunk : tile / kScanGroup], s_ncand);

  // ---- phase 2: lane per candidate: envelope / rectangle / classification grid.
  // Candidates in a mixed grid cell (~1 in 8) are listed again and evaluated in
  // phase 2b, so the strip walk runs once per tile instead of in every wave.
  bool redo = false;
  for (uint32_t c = threadIdx.x; c < ncand; c += kBlock) {
    const uint32_t pj = s_cand_pj[c];
    const int li = pj & 1023;
    const uint32_t ch = s_first[li] + (pj >> 10);
    const int64_t p = MGPU_PT(li);
    double px, py;
    if (point_stash<G>() || c < (uint32_t)kStash) {
      const double2 q = s_cand_xy[point_stash<G>() ? (uint32_t)li : c];
      px = q.x;
      py = q.y;
    } else {
      px = a.x[p];
      py = a.y[p];
    }
    const int q = pip::chip_quick(t, ch, px, py, nullptr);
    bool hit = q == pip::kQuickYes;
    if (q >= pip::kQuickStrips) {
      const uint32_t m = atomicAdd(&s_nmix, 1u);
      if (m < (uint32_t)kMix && (SLOW || q == pip::kQuickStrips)) {
        s_mix[m] = (uint16_t)c;
      } else if (!SLOW) {
        redo = true;  // list full / chip without strip index: pip_fix_kernel
      } else {
        hit = q == pip::kQuickStrips ? pip::chip_contains_mixed(t, ch, px, py)
                                     : pip::chip_locate(t, ch, px, py) == pip::kInterior;
      }
    }
    if (hit) atomicOr(&s_mask[li], 1u << (pj >> 10));
  }
  if (!SLOW && __syncthreads_or(redo)) {
    if (threadIdx.x == 0) {
      const unsigned int q = atomicAdd(a.n_dirty, 1u);
      a.dirty[q] = tile;
      if (!G) {
        a.tile_count[tile] = 0;
        a.tile_where[tile] = kNoDst;
      }
    }
    return;
  }
  __syncthreads();
  MGPU_STAMP(2);
  const uint32_t nmix = s_nmix < (uint32_t)kMix ? s_nmix : (uint32_t)kMix;
#ifdef MGPU_STATS
  uint32_t st_edges = 0;
#endif
  bool walked = false;
#if MGPU_EDGE_PAR
  if (MGPU_EDGE_PAR == 1 || G == 2)
  // north_star's ray-crossing test over LDS-staged vertex runs: the walks' strip edge runs
  // (each strip a contiguous run of edge records in JTS's visiting order) are laid end to
  // end in LDS -- per flat position its walk -- and every lane of the wave tests one edge
  // per step, loads for several steps in flight, whatever walk it belongs to; the rings'
  // boundary / parity bits gather per walk by LDS atomics (order-free: OR / XOR), then the
  // walk's lane applies PointLocator's verdict.  s_buf's candidate lists are dead here once
  // each walk lane holds its candidate, so the runs reuse its bytes.
  if (!SLOW && kBlock == 64 && nmix > 0 && nmix <= 64) {
    constexpr uint32_t kBufBytes = sizeof(s_buf);
    constexpr uint32_t kWalkBytes = 64 * (8 + 8 + 4 + 4 + 4 + 4 + 1);
    constexpr uint32_t kFlatCap = kBufBytes > kWalkBytes ? kBufBytes - kWalkBytes : 0;
    const uint32_t lane = threadIdx.x;
    uint32_t pj = 0, ch = 0, eb = 0, ne = 0;
    int li = 0;
    bool one = false;
    uint8_t fl = 0;
    double px = 0.0, py = 0.0;
    if (lane < nmix) {
      const uint32_t c = s_mix[lane];
      pj = s_cand_pj[c];
      li = pj & 1023;
      ch = s_first[li] + (pj >> 10);
      if (point_stash<G>() || c < (uint32_t)kStash) {
        const double2 q = s_cand_xy[point_stash<G>() ? (uint32_t)li : c];
        px = q.x;
        py = q.y;
      } else {
        px = a.x[MGPU_PT(li)];
        py = a.y[MGPU_PT(li)];
      }
      const ChipHdr& H = t.chip_hdr[ch];
      const uint32_t strip = H.strip_base + (uint32_t)strip_of(py, H.env[1], H.inv_h, (int)H.n_strips);
      one = H.single_ring != 0;
      fl = H.flags;
      eb = t.strip_edge[strip];
      ne = t.strip_edge[strip + 1] - eb;
    }
    uint32_t inc = ne;
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t u = (uint32_t)__shfl_up((int)inc, d);
      if ((int)lane >= d) inc += u;
    }
    const uint32_t total = (uint32_t)__shfl((int)inc, 63), off = inc - ne;
    if (total <= kFlatCap) {
      __syncthreads();  // (every walk lane has read its candidate: s_buf is free)
      double* s_wx = (double*)s_buf;
      double* s_wy = s_wx + 64;
      uint32_t* s_web = (uint32_t*)(s_wy + 64);
      uint32_t* s_woff = s_web + 64;
      uint32_t* s_bnd = s_woff + 64;
      uint32_t* s_par = s_bnd + 64;
      uint8_t* s_wone = (uint8_t*)(s_par + 64);
      uint8_t* s_walk = s_wone + 64;  // [kFlatCap]: the walk of each flat edge
      s_wx[lane] = px;
      s_wy[lane] = py;
      s_web[lane] = eb;
      s_woff[lane] = off;
      s_bnd[lane] = 0;
      s_par[lane] = 0;
      s_wone[lane] = one ? 1 : 0;
      for (uint32_t k = 0; k < ne; k++) s_walk[off + k] = (uint8_t)lane;
      __syncthreads();
      const double4* E4 = (const double4*)t.edges;
#ifndef MGPU_EDGE_PAR_STEPS
#define MGPU_EDGE_PAR_STEPS 4
#endif
      constexpr int kS = MGPU_EDGE_PAR_STEPS;
      const uint32_t e_safe = s_web[s_walk[0]];  // (a valid record for the idle lanes' loads)
      for (uint32_t f0 = 0; f0 < total; f0 += 64 * kS) {
        double4 R[kS];
        uint32_t wm[kS], we[kS];
#pragma unroll
        for (int k = 0; k < kS; k++) {
          const uint32_t f = f0 + lane + 64u * k;
          wm[k] = f < total ? s_walk[f] : 0u;
          we[k] = f < total ? s_web[wm[k]] + (f - s_woff[wm[k]]) : 0u;
          R[k] = E4[f < total ? we[k] : e_safe];
        }
#pragma unroll
        for (int k = 0; k < kS; k++) {
          const uint32_t f = f0 + lane + 64u * k;
          if (f >= total) continue;
          const int bits = pip::count_segment(R[k].x, R[k].y, R[k].z, R[k].w, s_wx[wm[k]], s_wy[wm[k]]);
          if (!bits) continue;
          const uint32_t rb = s_wone[wm[k]] ? 1u : 1u << t.edge_ring[we[k]];
          if (bits & pip::kRingOnSegment) atomicOr(&s_bnd[wm[k]], rb);
          if (bits & 2) atomicXor(&s_par[wm[k]], rb);
        }
      }
      __syncthreads();
      if (lane < nmix && pip::strip_verdict(t, ch, one, fl, s_bnd[lane], s_par[lane], px, py))
        atomicOr(&s_mask[li], 1u << (pj >> 10));
      walked = true;
    }
  }
#endif
  if (!walked) {
#if MGPU_SPLIT_WALK
  // few walks (binned tiles: ~16): a group of 4 (<= 16 walks) or 2 (<= 32) lanes shares
  // each walk, every lane taking every L-th block of the strip's edges; the partial
  // ring bits combine by OR / XOR across the group
  if (!SLOW && kBlock == 64 && nmix > 0 && nmix <= 32) {
    const uint32_t lg = nmix <= 16 ? 2u : 1u;  // (8 lanes at <= 8 walks: no gain, r3)
    const uint32_t lane = threadIdx.x, m = lane >> lg, sub = lane & ((1u << lg) - 1u);
    uint32_t bnd = 0, par = 0, pj = 0, ch = 0;
    int li = 0;
    bool one = false;
    uint8_t fl = 0;
    double px = 0.0, py = 0.0;
    if (m < nmix) {
      const uint32_t c = s_mix[m];
      pj = s_cand_pj[c];
      li = pj & 1023;
      ch = s_first[li] + (pj >> 10);
      if (point_stash<G>() || c < (uint32_t)kStash) {
        const double2 q = s_cand_xy[point_stash<G>() ? (uint32_t)li : c];
        px = q.x;
        py = q.y;
      } else {
        px = a.x[MGPU_PT(li)];
        py = a.y[MGPU_PT(li)];
      }
      const ChipHdr& H = t.chip_hdr[ch];
      const uint32_t strip = H.strip_base + (uint32_t)strip_of(py, H.env[1], H.inv_h, (int)H.n_strips);
      one = H.single_ring != 0;
      fl = H.flags;
      pip::strip_bits(t, strip, one, px, py, sub * MGPU_EDGE_STEP, MGPU_EDGE_STEP << lg, &bnd, &par);
    }
    for (uint32_t o = 1; o < (1u << lg); o <<= 1) {
      bnd |= (uint32_t)__shfl_xor((int)bnd, (int)o);
      par ^= (uint32_t)__shfl_xor((int)par, (int)o);
    }
    if (m < nmix && sub == 0 && pip::strip_verdict(t, ch, one, fl, bnd, par, px, py))
      atomicOr(&s_mask[li], 1u << (pj >> 10));
  } else
#endif
  for (uint32_t m = threadIdx.x; m < nmix; m += kBlock) {
    const uint32_t c = s_mix[m];
    const uint32_t pj = s_cand_pj[c];
    const int li = pj & 1023;
    const uint32_t ch = s_first[li] + (pj >> 10);
    const int64_t p = MGPU_PT(li);
    double px, py;
    if (point_stash<G>() || c < (uint32_t)kStash) {
      const double2 q = s_cand_xy[point_stash<G>() ? (uint32_t)li : c];
      px = q.x;
      py = q.y;
    } else {
      px = a.x[p];
      py = a.y[p];
    }
    bool hit;
    if (SLOW && (t.chip_hdr[ch].flags & kChipNoStrips)) {
      hit = pip::chip_locate(t, ch, px, py) == pip::kInterior;
    } else {
#ifdef MGPU_STATS
      uint32_t ne = 0;
      hit = pip::chip_contains_mixed(t, ch, px, py, &ne);
      st_edges += ne;
#else
      hit = pip::chip_contains_mixed(t, ch, px, py);
#endif
    }
    if (hit) atomicOr(&s_mask[li], 1u << (pj >> 10));
  }
  }  // (!walked)
#ifdef MGPU_STATS
  if (threadIdx.x == 0) {
    atomicAdd(&a.counters[8], (unsigned long long)s_nmix);
  }
  atomicAdd(&a.counters[9], (unsigned long long)st_edges);
#endif
  __syncthreads();

  MGPU_STAMP(3);
  if (G) {
    // the split pipeline: each listed point's answer, and the chunk's pair count
    // the binned pipeline: one match is answered by its polygon id (the chip is local
    // here; in input order, where the emit runs, every lookup would be a random line);
    // the lane's lookups are issued together, then its answers stored
    uint64_t v[kItems];
    uint32_t mine[kItems];
#pragma unroll
    for (int k = 0; k < kItems; k++) {
      const uint32_t li = threadIdx.x + k * kBlock;
      v[k] = 0;
      mine[k] = 0;
      if (li < gcount) {
        const uint32_t m = s_mask[li];
        v[k] = (uint64_t)s_first[li] | ((uint64_t)m << 32);
        if (a.poly_answers && m && !(m & (m - 1)))
          v[k] = (uint64_t)(uint32_t)t.chip_poly[s_first[li] + __builtin_ctz(m)] | (1ull << 32);
        mine[k] = __popc(m);
      }
    }
#pragma unroll
    for (int k = 0; k < kItems; k++) {
      const uint32_t li = threadIdx.x + k * kBlock;
      if (li < gcount) a.mixed_res[lbase + li] = v[k];  // (the slot: the list position / binned point)
    }
    if (G == 1 && a.in_chunk_pairs) {
      // per input chunk pair counts: slots are bin-major, chunk-minor, so the tile's 256
      // slots hold a few runs of one input chunk each.  Lane l takes slots 4l .. 4l + 3
      // (their masks from LDS): one wave scan gives every slot's prefix, and the last slot
      // of each run adds the run's sum -- one atomic per run (kBlock == 64: one wave)
      const int lane = threadIdx.x & 63;
      const uint32_t s0 = 4u * (uint32_t)lane;
      const uint4 mq = *(const uint4*)(s_mask + s0);
      const uint32_t mv[4] = {mq.x, mq.y, mq.z, mq.w};
      uint32_t c[4], loc[4], nn[4];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const bool act = s0 + i < gcount;
        c[i] = act ? ckp[i] / (uint32_t)kChunk : 0xFFFFFFFFu;  // (kBinChunk == kChunk)
        nn[i] = act ? (uint32_t)__popc(mv[i]) : 0u;
        loc[i] = (i ? loc[i - 1] : 0u) + nn[i];
      }
      const uint32_t lane_excl = wave_incl_scan(loc[3]) - loc[3];
      const uint32_t prev_c = __shfl_up(c[3], 1, 64), next_c = __shfl_down(c[0], 1, 64);
      bool head[4];
      uint32_t hpre = 0;  // the prefix before the lane's last run head
#pragma unroll
      for (int i = 0; i < 4; i++) {
        head[i] = c[i] != 0xFFFFFFFFu && (i ? c[i] != c[i - 1] : (lane == 0 || prev_c != c[0]));
        if (head[i]) hpre = lane_excl + loc[i] - nn[i];
      }
      const unsigned long long hl = __ballot(head[0] || head[1] || head[2] || head[3]);
      const unsigned long long lower = hl & ((1ull << lane) - 1ull);
      uint32_t start = __shfl(hpre, lower ? 63 - __clzll(lower) : 0, 64);  // (the run in progress)
#pragma unroll
      for (int i = 0; i < 4; i++) {
        if (head[i]) start = lane_excl + loc[i] - nn[i];
        const bool tail = c[i] != 0xFFFFFFFFu && (i < 3 ? c[i + 1] != c[i] : (lane == 63 || next_c != c[3]));
        const uint32_t run = lane_excl + loc[i] - start;
        if (tail && run) atomicAdd(&a.in_chunk_pairs[c[i]], run);
      }
    }
    uint32_t tm = 0;
#pragma unroll
    for (int k = 0; k < kItems; k++) tm += mine[k];
    const unsigned long long tot = wave_sum_u64(tm);
    if ((threadIdx.x & 63) == 0 && tot) atomicAdd(&a.group_sum[chunk], (uint32_t)tot);
    return;
  }
  // ---- phase 3: lane l owns points 4l .. 4l+3 (input order)
  const int l0 = threadIdx.x * kItems;
  uint32_t mine = 0;
#pragma unroll
  for (int k = 0; k < kItems; k++) {
    const int li = l0 + k;
    mine += __popc(s_mask[li]);
    const uint32_t cnt = s_cnt[li];
    if (SLOW && cnt > (uint32_t)kMaskBits) {  // chips past the 32nd of the cell
      const int64_t p = MGPU_PT(li);
      const Range r{s_first[li], cnt, 0};
      for (uint32_t j = kMaskBits; j < cnt; j++)
        mine += (chip_is_core(t, r, j) || pip::chip_contains_strips(t, r.first + j, a.x[p], a.y[p])) ? 1 : 0;
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t incl = wave_incl_scan(mine);
  if (lane == 63) s_wave_tot[wave] = incl;
  __syncthreads();
  uint32_t wave_off = 0, agg = 0;
#pragma unroll
  for (int w = 0; w < kBlock / 64; w++) {
    uint32_t v = s_wave_tot[w];
    if (w < wave) wave_off += v;
    agg += v;
  }
  const uint32_t excl = wave_off + incl - mine;

  // the tile's records go to its own slot (kSlot records), or -- when it has more --
  // to space reserved in the overflow pool
  __shared__ uint64_t s_dst;
  if (threadIdx.x == 0) {
    uint64_t dst = (uint64_t)tile * kSlot;
    if (agg > (uint32_t)kSlot) {
      const unsigned long long off = atomicAdd(a.pool_used, (unsigned long long)agg);
      dst = off + agg <= (unsigned long long)a.pool_cap ? (uint64_t)a.n_tiles * kSlot + off : kNoDst;
    }
    a.tile_count[tile] = agg;
    a.tile_where[tile] = dst;
    if (agg) atomicAdd(&a.group_sum[tile / kScanGroup], agg);
    s_dst = dst;
  }
  const bool staged = agg <= (uint32_t)kOutCap;
  __syncthreads();
  const uint64_t dst = s_dst;
  uint64_t* const rec = dst == kNoDst ? nullptr : a.recs + dst;

  // this lane's pairs {li << 32 | polygon id}: staged in LDS (then written as
  // contiguous runs) or direct
  uint32_t pos = excl;
#pragma unroll 1
  for (int k = 0; k < kItems; k++) {
    const int li = l0 + k;
    if (!SLOW) {
      // every match is a mask bit
      const uint32_t first = s_first[li];
      for (uint32_t m = s_mask[li]; m; m &= m - 1) {
        const int32_t poly = t.chip_poly[first + __builtin_ctz(m)];
        if (staged) {
          s_out_poly[pos] = poly;
          s_out_li[pos] = (uint16_t)li;
        } else if (rec) {
          rec[pos] = ((uint64_t)li << 32) | (uint32_t)poly;
        }
        pos++;
      }
      continue;
    }
    const uint32_t cnt = s_cnt[li];
    if (!cnt) continue;
    const uint32_t first = s_first[li];
    const int64_t p = MGPU_PT(li);
    uint32_t m = s_mask[li];
    const uint32_t nj = cnt < (uint32_t)kMaskBits ? cnt : (uint32_t)kMaskBits;
    for (uint32_t j = 0; j < cnt; j++) {
      bool hit;
      if (!SLOW || j < nj) {
        hit = (m >> j) & 1;
      } else {
        const Range r{first, cnt, 0};
        hit = chip_is_core(t, r, j) || pip::chip_contains_strips(t, first + j, a.x[p], a.y[p]);
      }
      if (!hit) continue;
      const int32_t poly = t.chip_poly[first + j];
      if (staged) {
        s_out_poly[pos] = poly;
        s_out_li[pos] = (uint16_t)li;
      } else if (rec) {
        rec[pos] = ((uint64_t)li << 32) | (uint32_t)poly;
      }
      pos++;
    }
  }
  MGPU_STAMP(4);
  if (!staged || !rec) return;
  __syncthreads();
#ifndef MGPU_NT_RECS
#define MGPU_NT_RECS 1
#endif
  for (uint32_t i = threadIdx.x; i < agg; i += kBlock) {
    const uint64_t v = ((uint64_t)s_out_li[i] << 32) | (uint32_t)s_out_poly[i];
#if MGPU_NT_RECS
    __builtin_nontemporal_store(v, &rec[i]);
#else
    rec[i] = v;
#endif
  }
  MGPU_STAMP(4);
}

// One workgroup per tile (a persistent grid walking the tiles measured 25% slower in
// round 1: workgroups that carry a tile of real work hide their dispatch).
// 8 waves per SIMD: the kernel is held to 64 VGPRs (the fused tile's LDS, ~8 KB with its
// per-point stash, allows 20 workgroups per CU; the binned tile's ~7 KB, 22) (it is latency-bound: the 8th wave measured -7% on C2,
// -10% on C5)
#ifndef MGPU_WAVES_PER_EU
#define MGPU_WAVES_PER_EU 8
#endif
#if MGPU_WAVES_PER_EU
#define MGPU_JOIN_ATTR __attribute__((amdgpu_waves_per_eu(MGPU_WAVES_PER_EU)))
#else
#define MGPU_JOIN_ATTR
#endif
template <int IS>
__global__ __launch_bounds__(kBlock) MGPU_JOIN_ATTR void pip_join_kernel(JoinArgs a) {
  join_tile<IS, false>(a, blockIdx.x);
}

// The tiles queued by pip_join_kernel, with the H3 route for their near-ties.
template <int IS>
__global__ __launch_bounds__(kBlock) void pip_fix_kernel(JoinArgs a) {
  const uint32_t nd = *a.n_dirty;
  for (uint32_t q = blockIdx.x; q < nd; q += gridDim.x) {
    join_tile<IS, true>(a, a.dirty[q]);
    __syncthreads();
  }
}

// ---------------------------------------------------------------- split pipeline
// (kernels.h SplitArgs).  A chip table with a pixel index answers most points from their
// pixel; the fused kernel still pays a tile's full phase structure (and its memory round
// trips) for them.  The split pipeline streams instead: classify_kernel touches every
// point once (16 B read, one pixel load, a 2- or 4-byte code written), the few mixed
// points go through join_tile's phases gathered into full tiles, and split_emit_kernel
// writes the ordered pairs from the codes.
#ifndef MGPU_CLS_BLOCK
#define MGPU_CLS_BLOCK 256  // threads per chunk in the emit kernels (16 points each; 512: 8)
#endif
constexpr int kClsBlock = MGPU_CLS_BLOCK;
constexpr int kClsItems = kChunk / kClsBlock;  // points per thread
static_assert(kClsItems * (kClsBlock / 64) == 64, "one wave scans a chunk's ballots");
constexpr uint32_t kCodeMixed32 = 0xFFFFFFFFu;

template <int IS>
struct CodeOf {
  using T = uint16_t;  // H3: the pixel class (kPixMixed: mixed)
};
template <>
struct CodeOf<MGPU_BNG> {
  using T = uint32_t;  // BNG: first chip << 8 | match mask (0: none, ~0: mixed)
};


// BNG without a pixel index (option bng_split): the point's dense grid entry is its code.
// A cell whose chips are all core (at most 8) answers every point in it; a cell flagged
// with an answer grid (chip_table.h cell_ans) answers from the point's square unless that
// square is mixed; the other cells' points (border chips) are mixed -- the mixed tiles run
// the whole join for them.  Cells off the dense box go through the id + hash probe.
// Returns the match mask over the chips from *first, or kPixMixed.
__device__ __forceinline__ uint32_t bng_grid_class(const JoinArgs& a, int64_t p, double px, double py, bool* ok,
                                                     uint32_t* first) {
  const ChipTableView& t = a.chips;
  bool tie = false;
  uint32_t gi = kNoEntry;
  Range r = chip_probe<MGPU_BNG, false>(a, p, px, py, ok, &tie, &gi);
  if (!*ok) return kPixEmpty;
  uint64_t e = 0;
  if (gi != kNoEntry) {
    e = t.grid[gi];
    r = grid_range(e, t.cell_ans_row != nullptr);
  }
  *first = r.first;
  if (r.count == 0) return kPixEmpty;
  if (r.count <= 8 && (r.core & ((1u << r.count) - 1u)) == (1u << r.count) - 1u) return (1u << r.count) - 1u;
  if (t.cell_ans_row && (e & kCellAnsFlag)) {
    const uint32_t eI = (uint32_t)bng::d2i(px), nI = (uint32_t)bng::d2i(py), ed = t.bng_edge;
    const uint32_t col = div_fix(eI, ed, t.bng_inv_edge), row = div_fix(nI, ed, t.bng_inv_edge);
    const uint32_t u = div_fix(eI - col * ed, t.cell_ans_sw, t.cell_ans_inv_sw);
    const uint32_t v = div_fix(nI - row * ed, t.cell_ans_sw, t.cell_ans_inv_sw);
    const uint32_t ai = t.cell_ans_row[row - (uint32_t)t.dense[0].b0] + cell_ans_index(e);
    const uint16_t m = t.cell_ans[((size_t)ai * t.cell_ans_g + v) * t.cell_ans_g + u];
    if (m != kCellAnsMixed && m < 256u) return m;
  }
  return kPixMixed;
}

// One wave per chunk of kChunk points: a lane takes every 64th point of the chunk
// (item-major, so consecutive lanes read consecutive points), and the chunk's mixed
// points are ranked in point order by a running wave count plus the item's ballot -- no
// workgroup barrier per chunk, no LDS scan.  The workgroup (512 threads: four share a
// CU) copies the pixel block table (chip_table.h raster_blk) into LDS once; a point in a
// uniform block takes its class from there, the rest load their pixel (and sub-pixel)
// class.  Waves take chunks blockIdx.x * W + wave, then + gridDim.x * W ...
// (Measured and rejected, r3: a software pipeline over the wave's batches -- batch g's
// pixel and rank loads, batch g - 1's sub-pixel loads, batch g + 1's coordinates in
// flight before any wait: 0.806 ms vs 0.765 on C2 at batch 4 (6 waves/SIMD), 0.841 at
// batch 2; the speculative rank loads add requests and the chain is not the limit.)
#ifndef MGPU_CFY_BLOCK
#define MGPU_CFY_BLOCK 512
#endif
constexpr int kCfyBlock = MGPU_CFY_BLOCK;
#ifndef MGPU_CFY_BATCH
#define MGPU_CFY_BATCH 4
#endif
#ifndef MGPU_CFY_WAVES
#define MGPU_CFY_WAVES 1  // (8 = at most 64 VGPRs: spills, slower on C2 / C5)
#endif
constexpr int kCfyBatch = MGPU_CFY_BATCH;
template <int IS>
__global__ __launch_bounds__(kCfyBlock) __attribute__((amdgpu_waves_per_eu(MGPU_CFY_WAVES))) void classify_wave_kernel(SplitArgs sa, int64_t n_chunks) {
  using Code = typename CodeOf<IS>::T;
  constexpr int kW = kCfyBlock / 64;        // waves per workgroup
  constexpr int kItems = kChunk / 64;       // points per lane per chunk
  static_assert(kItems % kCfyBatch == 0, "MGPU_CFY_BATCH must divide the points per lane of a chunk");
  const JoinArgs& a = sa.j;
  const ChipTableView& t = a.chips;
  extern __shared__ uint16_t s_blk[];       // [raster_bny * raster_bnx] (IS == H3), then the row bands
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool use_blk = IS == MGPU_H3 && t.raster_blk != nullptr;
  const bool bng_grid = IS == MGPU_BNG && t.raster_mode == kRasterNone;  // (bng_grid_class)
  const uint32_t nblk = use_blk ? t.raster_bnx * t.raster_bny : 0u;
  uint32_t* s_band = (uint32_t*)(s_blk + ((nblk + 1) & ~1u));
  if (use_blk)
    for (uint32_t i = threadIdx.x; i < nblk; i += kCfyBlock) s_blk[i] = t.raster_blk[i];
  if (IS == MGPU_H3)
    for (uint32_t i = threadIdx.x; i < t.raster_nband; i += kCfyBlock) s_band[i] = t.raster_band[i];
  __syncthreads();
  Code* codes = (Code*)sa.codes;
  const unsigned long long below = (1ull << lane) - 1ull;
  bool any_bad = false;
  const int64_t ch_step = (int64_t)gridDim.x * kW;
  double bx[kCfyBatch], by[kCfyBatch];
  auto load_batch = [&](int64_t ch, int b, double* X, double* Y) {
#pragma unroll
    for (int k = 0; k < kCfyBatch; k++) {
      const int64_t p = ch * kChunk + (int64_t)(b + k) * 64 + lane;
      X[k] = Y[k] = 0.0;
      if (ch < n_chunks && p < a.n) {
        X[k] = __builtin_nontemporal_load(&a.x[p]);
        Y[k] = __builtin_nontemporal_load(&a.y[p]);
      }
    }
  };
  for (int64_t ch = (int64_t)blockIdx.x * kW + wave; ch < n_chunks; ch += ch_step) {
    const int64_t c0 = ch * kChunk;
    uint32_t pairs = 0, nmixed = 0;  // nmixed: wave-uniform
    for (int b = 0; b < kItems; b += kCfyBatch) {
      load_batch(ch, b, bx, by);
      uint32_t ri[kCfyBatch], gix[kCfyBatch], sb[kCfyBatch], bi[kCfyBatch];
#pragma unroll
      for (int k = 0; k < kCfyBatch; k++) {
        ri[k] = kNoPixel;
        gix[k] = 0;
        sb[k] = 0;
        bi[k] = kNoPixel;
        const int64_t pk = c0 + (int64_t)(b + k) * 64 + lane;
        if (pk < a.n && pt_valid(a.valid, a.valid_off, pk)) {
          bool ok = true;
          uint32_t g_ = 0, s_ = 0, b_ = kNoPixel;
          if (IS == MGPU_BNG && bng_grid) {
            const uint32_t m = bng_grid_class(a, pk, bx[k], by[k], &ok, &g_);
            ri[k] = m == kPixMixed ? kRasterFull : m;  // (the class itself, below)
          } else {
            ri[k] = raster_index<IS>(t, bx[k], by[k], &ok, &g_, &s_, &b_);  // (see classify_pair_kernel)
          }
          gix[k] = g_;
          sb[k] = s_;
          bi[k] = use_blk ? b_ : kNoPixel;
          any_bad |= !ok;
        }
      }
      uint32_t cl[kCfyBatch];
      uint64_t ge[kCfyBatch];
#ifndef MGPU_CFY_ABLATE
#define MGPU_CFY_ABLATE 0  // profiling only (wrong answers): 1 no lookups, 2 LDS blocks only, 3 no sub-pixels
#endif
#pragma unroll
      for (int k = 0; k < kCfyBatch; k++) {
#if MGPU_CFY_ABLATE == 1
        cl[k] = ri[k] < kRasterFull ? (ri[k] & 1) : kPixEmpty;
#elif MGPU_CFY_ABLATE == 2
        cl[k] = ri[k] < kRasterFull && bi[k] != kNoPixel && s_blk[bi[k]] != kPixMixed ? s_blk[bi[k]] : kPixEmpty;
#elif MGPU_CFY_ABLATE == 3
        cl[k] = ri[k] < kRasterFull ? (bi[k] != kNoPixel && s_blk[bi[k]] != kPixMixed ? s_blk[bi[k]] : t.raster[ri[k]])
                                    : kPixEmpty;
#elif MGPU_CFY_ABLATE == 4
        cl[k] = ri[k] < kRasterFull ? t.raster[ri[k]] : kPixEmpty;  // every lane loads its pixel
#elif MGPU_CFY_ABLATE == 5
        cl[k] = ri[k] < kRasterFull ? (bi[k] != kNoPixel && s_blk[bi[k]] != kPixMixed ? s_blk[bi[k]] : kPixMixed)
                                    : kPixEmpty;  // (LDS, then every non-uniform block point mixed: no global loads)
#else
        if (IS == MGPU_BNG && bng_grid)
          cl[k] = ri[k] == kRasterFull ? kPixMixed : (ri[k] == kNoPixel ? kPixEmpty : ri[k]);
        else
          cl[k] = ri[k] < kRasterFull ? raster_class_blk(t, s_blk, ri[k], bi[k], sb[k], s_band)
                                      : (ri[k] == kRasterFull ? kPixMixed : kPixEmpty);
#endif
        if (IS == MGPU_BNG && bng_grid) ge[k] = gix[k];  // (the first chip)
        else ge[k] = (IS == MGPU_BNG && ri[k] < kRasterFull) ? t.grid[gix[k]] : 0ull;
      }
#pragma unroll
      for (int k = 0; k < kCfyBatch; k++) {
        const int64_t p = c0 + (int64_t)(b + k) * 64 + lane;
        const bool valid = p < a.n;
        bool mixed = cl[k] == kPixMixed;
        Code code;
        if (IS == MGPU_H3) {
          code = (Code)cl[k];
          if (!mixed && cl[k] != kPixEmpty) {
            const uint32_t c = cl[k];
            pairs += c < t.raster_pc[0] ? 1u : c < t.raster_pc[1] ? 2u : c < t.raster_pc[2] ? 3u : c < t.raster_pc[3] ? 4u
                     : (uint32_t)__popc((uint32_t)(t.raster_cls[c] >> 32));
          }
        } else {
          const uint32_t first = (uint32_t)ge[k], m = cl[k];
          if (!mixed && m && !(m < 256u && first < (1u << 24))) mixed = true;
          code = (Code)(mixed ? kCodeMixed32 : (m ? (first << 8) | m : 0u));
          if (!mixed) pairs += __popc(m);
        }
        if (valid) MGPU_ST_INTER(code, &codes[p]);
        mixed = mixed && valid;
        const unsigned long long bal = __ballot(mixed);
        if (mixed) sa.mixed_idx[c0 + nmixed + (uint32_t)__popcll(bal & below)] = (uint16_t)((b + k) * 64 + lane);
        nmixed += (uint32_t)__popcll(bal);
      }
    }
    pairs = wave_sum_u32(pairs);
    if (lane == 0) {
      sa.chunk_pairs[ch] = pairs;
      sa.chunk_mixed[ch] = nmixed;
    }
  }
  count_wave(&a.counters[2], any_bad);
}


// classify_wave_kernel with two consecutive points per lane: each coordinate array is
// read 16 bytes per lane (one global_load_dwordx4 for a lane's two x, one for its two y)
// and the two codes are stored together.  A wave's item covers 128 points; a mixed
// point's rank in the chunk is the wave's running count plus the mixed points of the
// lower lanes (both halves) plus, for the second point, the first's.  Launched when x and
// y are 16-byte aligned (else classify_wave_kernel).
#ifndef MGPU_CFY_PAIR
#define MGPU_CFY_PAIR 1
#endif
typedef double dbl2_t __attribute__((ext_vector_type(2)));
template <int IS>
__global__ __launch_bounds__(kCfyBlock) __attribute__((amdgpu_waves_per_eu(MGPU_CFY_WAVES))) void classify_pair_kernel(SplitArgs sa, int64_t n_chunks) {
  using Code = typename CodeOf<IS>::T;
  constexpr int kW = kCfyBlock / 64;
  constexpr int kPairItems = kChunk / 128;                       // pair items per lane per chunk
  constexpr int kPB = kCfyBatch / 2 > 0 ? kCfyBatch / 2 : 1;      // pair items in flight
  constexpr int kPts = 2 * kPB;
  static_assert(kPairItems % kPB == 0, "MGPU_CFY_BATCH / 2 must divide the pair items per lane of a chunk");
  const JoinArgs& a = sa.j;
  const ChipTableView& t = a.chips;
  extern __shared__ uint16_t s_blk[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool use_blk = IS == MGPU_H3 && t.raster_blk != nullptr;
  const bool bng_grid = IS == MGPU_BNG && t.raster_mode == kRasterNone;  // (bng_grid_class)
  const uint32_t nblk = use_blk ? t.raster_bnx * t.raster_bny : 0u;
  uint32_t* s_band = (uint32_t*)(s_blk + ((nblk + 1) & ~1u));
  if (use_blk)
    for (uint32_t i = threadIdx.x; i < nblk; i += kCfyBlock) s_blk[i] = t.raster_blk[i];
  if (IS == MGPU_H3)
    for (uint32_t i = threadIdx.x; i < t.raster_nband; i += kCfyBlock) s_band[i] = t.raster_band[i];
  __syncthreads();
  Code* codes = (Code*)sa.codes;
  const unsigned long long below = (1ull << lane) - 1ull;
  bool any_bad = false;
  const int64_t ch_step = (int64_t)gridDim.x * kW;
  for (int64_t ch = (int64_t)blockIdx.x * kW + wave; ch < n_chunks; ch += ch_step) {
    const int64_t c0 = ch * kChunk;
    uint32_t pairs = 0, nmixed = 0;
    for (int b = 0; b < kPairItems; b += kPB) {
      double X[kPts], Y[kPts];
#pragma unroll
      for (int k = 0; k < kPB; k++) {
        const int64_t p = c0 + (int64_t)(b + k) * 128 + 2 * lane;
        if (p + 1 < a.n) {
          const dbl2_t vx = __builtin_nontemporal_load((const dbl2_t*)(a.x + p));
          const dbl2_t vy = __builtin_nontemporal_load((const dbl2_t*)(a.y + p));
          X[2 * k] = vx.x, X[2 * k + 1] = vx.y, Y[2 * k] = vy.x, Y[2 * k + 1] = vy.y;
        } else {
          X[2 * k] = Y[2 * k] = X[2 * k + 1] = Y[2 * k + 1] = 0.0;
          if (p < a.n) X[2 * k] = a.x[p], Y[2 * k] = a.y[p];
        }
      }
      uint32_t ri[kPts], gix[kPts], sb[kPts], bi[kPts];
#pragma unroll
      for (int j = 0; j < kPts; j++) {
        ri[j] = kNoPixel;
        gix[j] = 0;
        sb[j] = 0;
        bi[j] = kNoPixel;
        const int64_t pj = c0 + (int64_t)(b + j / 2) * 128 + 2 * lane + (j & 1);
        if (pj < a.n && pt_valid(a.valid, a.valid_off, pj)) {
          bool ok = true;
          uint32_t g_ = 0, s_ = 0, b_ = kNoPixel;
          if (IS == MGPU_BNG && bng_grid) {
            const uint32_t m = bng_grid_class(a, pj, X[j], Y[j], &ok, &g_);
            ri[j] = m == kPixMixed ? kRasterFull : m;
          } else {
            // (always a local's address: a pointer chosen at run time put b_ in scratch)
            ri[j] = raster_index<IS>(t, X[j], Y[j], &ok, &g_, &s_, &b_);
          }
          gix[j] = g_;
          sb[j] = s_;
          bi[j] = use_blk ? b_ : kNoPixel;
          any_bad |= !ok;
        }
      }
      uint32_t cl[kPts];
      uint64_t ge[kPts];
#pragma unroll
      for (int j = 0; j < kPts; j++) {
        if (IS == MGPU_BNG && bng_grid) {
          cl[j] = ri[j] == kRasterFull ? kPixMixed : (ri[j] == kNoPixel ? kPixEmpty : ri[j]);
          ge[j] = gix[j];  // (the first chip)
        } else {
          cl[j] = ri[j] < kRasterFull ? raster_class_blk(t, s_blk, ri[j], bi[j], sb[j], s_band)
                                      : (ri[j] == kRasterFull ? kPixMixed : kPixEmpty);
          ge[j] = (IS == MGPU_BNG && ri[j] < kRasterFull) ? t.grid[gix[j]] : 0ull;
        }
      }
      Code code[kPts];
      bool mixed[kPts];
#pragma unroll
      for (int j = 0; j < kPts; j++) {
        const int64_t pj = c0 + (int64_t)(b + j / 2) * 128 + 2 * lane + (j & 1);
        bool m = cl[j] == kPixMixed;
        if (IS == MGPU_H3) {
          code[j] = (Code)cl[j];
          if (!m && cl[j] != kPixEmpty) {
            const uint32_t c = cl[j];
            pairs += c < t.raster_pc[0] ? 1u : c < t.raster_pc[1] ? 2u : c < t.raster_pc[2] ? 3u : c < t.raster_pc[3] ? 4u
                     : (uint32_t)__popc((uint32_t)(t.raster_cls[c] >> 32));
          }
        } else {
          const uint32_t first = (uint32_t)ge[j], mm = cl[j];
          if (!m && mm && !(mm < 256u && first < (1u << 24))) m = true;
          code[j] = (Code)(m ? kCodeMixed32 : (mm ? (first << 8) | mm : 0u));
          if (!m) pairs += __popc(mm);
        }
        mixed[j] = m && pj < a.n;
      }
#pragma unroll
      for (int k = 0; k < kPB; k++) {
        const int64_t p = c0 + (int64_t)(b + k) * 128 + 2 * lane;
        if (p + 1 < a.n) {
          if (sizeof(Code) == 2) {
            MGPU_ST_INTER((uint32_t)code[2 * k] | ((uint32_t)code[2 * k + 1] << 16), (uint32_t*)(codes + p));
          } else {
            typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
            u32x2_t v;
            v.x = (uint32_t)code[2 * k];
            v.y = (uint32_t)code[2 * k + 1];
            MGPU_ST_INTER(v, (u32x2_t*)(codes + p));
          }
        } else if (p < a.n) {
          MGPU_ST_INTER(code[2 * k], &codes[p]);
        }
        const unsigned long long b0 = __ballot(mixed[2 * k]), b1 = __ballot(mixed[2 * k + 1]);
        const uint32_t r0 = nmixed + (uint32_t)__popcll(b0 & below) + (uint32_t)__popcll(b1 & below);
        const uint16_t li = (uint16_t)((b + k) * 128 + 2 * lane);
        if (mixed[2 * k]) sa.mixed_idx[c0 + r0] = li;
        if (mixed[2 * k + 1]) sa.mixed_idx[c0 + r0 + (mixed[2 * k] ? 1u : 0u)] = (uint16_t)(li + 1);
        nmixed += (uint32_t)(__popcll(b0) + __popcll(b1));
      }
    }
    pairs = wave_sum_u32(pairs);
    if (lane == 0) {
      sa.chunk_pairs[ch] = pairs;
      sa.chunk_mixed[ch] = nmixed;
    }
  }
  count_wave(&a.counters[2], any_bad);
}

// The mixed points of one chunk per workgroup: its first tile of kTile; a chunk with
// more queues its further tiles for pip_mixed_more_kernel (a loop over tiles here pinned
// 23 more VGPRs: 5 waves/SIMD instead of 7).  (Measured and rejected, r3: the chunks'
// lists packed into full tiles walked by a resident grid -- C2 mixed 0.22 -> 0.35 ms,
// C5 0.60 -> 0.87: a full tile's phases take longer, and fewer tiles are in flight.)
template <int IS>
__global__ __launch_bounds__(kBlock) MGPU_JOIN_ATTR void pip_mixed_kernel(JoinArgs a) {
  const uint32_t nm = a.chunk_mixed[blockIdx.x];
  if (threadIdx.x == 0 && nm > (uint32_t)kGTile) {
    const uint32_t more = (nm - 1) / kGTile;
    const uint32_t q = atomicAdd(a.n_extra, more);
    for (uint32_t t = 0; t < more; t++) a.extra[q + t] = blockIdx.x * kChunkTiles + 1 + t;
  }
  join_tile<IS, false, 2>(a, blockIdx.x * kChunkTiles);
}

template <int IS>
__global__ __launch_bounds__(kBlock) void pip_mixed_more_kernel(JoinArgs a) {
  const uint32_t n = *a.n_extra;
  for (uint32_t q = blockIdx.x; q < n; q += gridDim.x) {
    join_tile<IS, false, 2>(a, a.extra[q]);
    __syncthreads();
  }
}

template <int IS, int G>
__global__ __launch_bounds__(kBlock) void pip_mixed_fix_kernel(JoinArgs a) {
  const uint32_t nd = *a.n_dirty;
  for (uint32_t q = blockIdx.x; q < nd; q += gridDim.x) {
    join_tile<IS, true, G>(a, a.dirty[q]);
    __syncthreads();
  }
}

// Ordered output.  Thread i handles the chunk's points 16 i .. 16 i + 15 (their codes:
// one or two 16-byte loads); a block scan of the threads' mixed counts gives each mixed
// point its rank in the chunk's mixed list (classify_kernel ranks them in point order
// too), a second scan of the pair counts each thread's first output slot.  The chunk's
// pairs are one contiguous output range: staged in LDS (polygon id, point) a window of
// kEmitWin pairs at a time, then written by consecutive lanes.
// A workgroup barrier that orders LDS only: __syncthreads() also waits for the wave's
// outstanding global loads and stores (its release fence), which would hold the emit
// kernels' output stores and the next chunk's prefetched loads at every barrier.
#ifndef MGPU_EMIT_LDSBAR
#define MGPU_EMIT_LDSBAR 1
#endif
__device__ __forceinline__ void lds_barrier() {
#if MGPU_EMIT_LDSBAR
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#else
  __syncthreads();
#endif
}

__device__ __forceinline__ uint32_t chunk_excl_scan(uint32_t v, uint32_t* s_w, uint32_t* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t incl = wave_incl_scan(v);
  if (lane == 63) s_w[wave] = incl;
  lds_barrier();
  uint32_t before = 0, all = 0;
#pragma unroll
  for (int w = 0; w < kClsBlock / 64; w++) {
    before += w < wave ? s_w[w] : 0u;
    all += s_w[w];
  }
  *total = all;
  return before + incl - v;
}

constexpr int kEmitWin = 2048;  // pairs staged at a time
// A thread stages its points' pairs at consecutive slots, so at one item the lanes write
// slots a thread's pair count apart (~16 at one pair per point: the lanes fall on 4 of
// the 64 LDS banks).  The slot index is swizzled within its 64-slot row -- the row's
// index XORed into the low bits -- which spreads those writes over the banks and keeps
// the reads (consecutive slots: one row per wave) conflict-free.
#ifndef MGPU_EMIT_SWZ
#define MGPU_EMIT_SWZ 1
#endif
__device__ __forceinline__ uint32_t emit_swz(uint32_t q) { return MGPU_EMIT_SWZ ? q ^ ((q >> 6) & 63u) : q; }
// the split emit's ordered pairs with non-temporal stores (A/B r3, profiles/r3_emit_nt_ab.txt:
// C2 emit 0.362 -> 0.328 ms, C5 0.397 -> 0.355); bin_emit_kernel / pair_emit_kernel with
// plain stores (non-temporal: C3 emit +0.09 ms, C4 +0.06)
#ifndef MGPU_EMIT_NT
#define MGPU_EMIT_NT 1
#endif
#ifndef MGPU_EMIT_NT_OTHER
#define MGPU_EMIT_NT_OTHER 0
#endif
#ifndef MGPU_EMIT_WAVES
#define MGPU_EMIT_WAVES 5  // (8: 64 VGPRs, spills; 5: none, A/B equal or better)
#endif
// lonlat one-match classes answer from an LDS copy of raster_cls_poly, and the chunk's
// mixed results (with the polygon of each one-chip match) are staged in LDS by one
// cooperative load at the start: the per-item loops below then touch no global memory
// for the common cases.  (A/B r4, profiles/r4_emit_ab.txt: the loops' per-item global
// loads -- mixed_res, chip_poly -- serialised ~16 dependent L2 round trips per wave; with
// staging skipped entirely the kernel took 0.19 ms instead of 0.34.  A resident-grid
// variant prefetching the next chunk measured slower, 0.45 ms.)
constexpr int kEmitCls = 2048;  // classes staged in LDS (8 KB)
constexpr int kEmitMres = 512;  // mixed results of a chunk staged in LDS (the rest: global)
#ifndef MGPU_EMIT_MR
#define MGPU_EMIT_MR 1
#endif
template <int IS>
__global__ __launch_bounds__(kClsBlock) __attribute__((amdgpu_waves_per_eu(MGPU_EMIT_WAVES))) void split_emit_kernel(SplitArgs sa) {
  using Code = typename CodeOf<IS>::T;
  constexpr int kWords = kClsItems * (int)sizeof(Code) / 4;  // 32-bit words of a thread's codes
  static_assert(kWords % 4 == 0 && kWords >= 4, "whole 16-byte code loads per thread (MGPU_CLS_BLOCK 256 or 512)");
  const JoinArgs& a = sa.j;
  const ChipTableView& t = a.chips;
  __shared__ uint32_t s_w[2][kClsBlock / 64];
  __shared__ uint32_t s_poly[kEmitWin];  // staging: polygon id
  __shared__ uint16_t s_pt[kEmitWin];    // staging: point of the chunk
  __shared__ int32_t s_cp[IS == MGPU_H3 ? kEmitCls : 1];
  __shared__ uint64_t s_mr[MGPU_EMIT_MR ? kEmitMres : 1];  // mixed results: first chip | mask << 32
  __shared__ int32_t s_mp[MGPU_EMIT_MR ? kEmitMres : 1];   // ... the polygon of a one-chip match
  // (an override rerun: the chunks before the first whose count changed keep their
  // output, but for the rerun ones)
  if (sa.redo_affected && blockIdx.x < *sa.redo_first && !sa.redo_affected[blockIdx.x]) return;
  const int64_t c0 = (int64_t)blockIdx.x * kChunk;
  const int64_t p0 = c0 + (int64_t)threadIdx.x * kClsItems;
  const Code kMixed = IS == MGPU_H3 ? (Code)kPixMixed : (Code)kCodeMixed32;
  uint32_t cw[kWords];
  if (p0 + kClsItems <= a.n) {
    const uint4* src = (const uint4*)((const Code*)sa.codes + p0);
#pragma unroll
    for (int i = 0; i < kWords / 4; i++) {
      const uint4 v = src[i];
      cw[4 * i] = v.x, cw[4 * i + 1] = v.y, cw[4 * i + 2] = v.z, cw[4 * i + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < kWords; i++) cw[i] = 0;
    const Code* cs = (const Code*)sa.codes;
    for (int k = 0; k < kClsItems; k++)
      if (p0 + k < a.n) {
        const uint32_t c = cs[p0 + k];
        if (sizeof(Code) == 2)
          cw[k >> 1] |= c << ((k & 1) * 16);
        else
          cw[k] = c;
      }
  }
  // (the chunk scans below order these LDS stores before the reads)
  uint32_t ncp = 0;
  if (IS == MGPU_H3) {
    ncp = min(min(t.raster_ncls, t.raster_pc[0]), (uint32_t)kEmitCls);
    for (uint32_t i = threadIdx.x; i < ncp; i += kClsBlock) s_cp[i] = t.raster_cls_poly[i];
  }
  constexpr uint32_t kMr = MGPU_EMIT_MR ? (uint32_t)kEmitMres : 0u;
#if MGPU_EMIT_MR
  {
    const uint32_t nm = sa.chunk_mixed[blockIdx.x], nms = nm < kMr ? nm : kMr;
    for (uint32_t i = threadIdx.x; i < nms; i += kClsBlock) {
      const uint64_t v = a.mixed_res[c0 + i];
      const uint32_t m = (uint32_t)(v >> 32);
      s_mr[i] = v;
      s_mp[i] = __popc(m) == 1 ? t.chip_poly[(uint32_t)v + __builtin_ctz(m)] : 0;
    }
  }
#endif
  auto code = [&](int k) -> Code {
    return sizeof(Code) == 2 ? (Code)(cw[k >> 1] >> ((k & 1) * 16)) : (Code)cw[k];
  };
  // a pure code's answer (first chip | match mask << 32)
  auto pure = [&](Code c) -> uint64_t {
    if (IS == MGPU_H3) return t.raster_cls[(uint32_t)c];
    return (uint64_t)((uint32_t)c >> 8) | ((uint64_t)((uint32_t)c & 0xFFu) << 32);
  };
  auto mres = [&](uint32_t r) -> uint64_t { return r < kMr ? s_mr[r] : a.mixed_res[c0 + r]; };
  uint32_t nmix = 0;
#pragma unroll
  for (int k = 0; k < kClsItems; k++) nmix += code(k) == kMixed;
  uint32_t all_mixed;
  const uint32_t rank0 = chunk_excl_scan(nmix, s_w[0], &all_mixed);
  uint32_t npair = 0, r = rank0;
#pragma unroll
  for (int k = 0; k < kClsItems; k++) {
    const Code c = code(k);
    if (c == kMixed)
      npair += __popc((uint32_t)(mres(r++) >> 32));
    else if (c != 0) {
      if (IS == MGPU_H3)  // the match count from the class order (raster_pc)
        npair += c < t.raster_pc[0]   ? 1u
                 : c < t.raster_pc[1] ? 2u
                 : c < t.raster_pc[2] ? 3u
                 : c < t.raster_pc[3] ? 4u
                                      : (uint32_t)__popc((uint32_t)(pure(c) >> 32));
      else
        npair += (uint32_t)__popc((uint32_t)c & 0xFFu);
    }
  }
  uint32_t total;
  const uint32_t off0 = chunk_excl_scan(npair, s_w[1], &total);
  const uint64_t base = sa.chunk_off[blockIdx.x];
  for (uint32_t w0 = 0; w0 < total; w0 += kEmitWin) {
    if (off0 < w0 + kEmitWin && off0 + npair > w0) {
      uint32_t q = off0;
      r = rank0;
#pragma unroll
      for (int k = 0; k < kClsItems; k++) {
        const Code c = code(k);
        uint64_t v = 0;
        bool has_one = false;  // one match, its polygon from LDS (any int32 id, negative too)
        int32_t one = 0;
        if (c == kMixed) {
          const uint32_t rr = r++;
          if (rr < kMr && __popc((uint32_t)(s_mr[rr] >> 32)) == 1)
            has_one = true, one = s_mp[rr];
          else
            v = mres(rr);
        } else if (IS == MGPU_H3 && c != 0 && (uint32_t)c < ncp)
          has_one = true, one = s_cp[(uint32_t)c];  // classes below raster_pc[0] match once
        else if (c != 0)
          v = pure(c);
        if (has_one) {
          if (q >= w0 && q < w0 + kEmitWin) {
            s_poly[emit_swz(q - w0)] = (uint32_t)one;
            s_pt[emit_swz(q - w0)] = (uint16_t)(threadIdx.x * kClsItems + k);
          }
          q++;
        }
        const uint32_t first = (uint32_t)v;
        for (uint32_t m = (uint32_t)(v >> 32); m; m &= m - 1, q++)
          if (q >= w0 && q < w0 + kEmitWin) {
            s_poly[emit_swz(q - w0)] = (uint32_t)t.chip_poly[first + __builtin_ctz(m)];
            s_pt[emit_swz(q - w0)] = (uint16_t)(threadIdx.x * kClsItems + k);
          }
      }
    }
    lds_barrier();
    const uint32_t cnt = total - w0 < (uint32_t)kEmitWin ? total - w0 : (uint32_t)kEmitWin;
    for (uint32_t i = threadIdx.x; i < cnt; i += kClsBlock) {
      const uint64_t q = base + w0 + i;
      if ((int64_t)q >= sa.capacity) break;
      const int64_t p = c0 + s_pt[emit_swz(i)];
#if MGPU_EMIT_NT
      __builtin_nontemporal_store(sa.point_id ? sa.point_id[p] : sa.id_base + p, &sa.out_point[q]);
      __builtin_nontemporal_store((int32_t)s_poly[emit_swz(i)], &sa.out_poly[q]);
#else
      sa.out_point[q] = sa.point_id ? sa.point_id[p] : sa.id_base + p;
      sa.out_poly[q] = (int32_t)s_poly[emit_swz(i)];
#endif
    }
    lds_barrier();
  }
}

// Output offsets, in two levels: pip_join_kernel / pip_fix_kernel add each tile's pair
// count to its group of kScanGroup tiles; this one workgroup scans the group sums
// (~3e3 per 1e8 points, coalesced chunks of 1024) and pair_emit_kernel adds the counts
// of the tile's predecessors inside its group.  counters[0] = total pairs.
constexpr int kScanBlock = 1024;
constexpr int kScanLds = 24576;  // counts staged in LDS (96 KB): 1e8 points in 4096-point chunks
__global__ __launch_bounds__(kScanBlock) void tile_scan_kernel(const uint32_t* __restrict__ gsum,
                                                               const uint32_t* __restrict__ gcand, int64_t ng,
                                                               uint64_t* __restrict__ goff,
                                                               unsigned long long* __restrict__ counters,
                                                               const uint32_t* only_if = nullptr) {
  if (only_if && *only_if == 0) return;  // (a rerun that changed no count: the offsets stand)
  // thread i owns the contiguous run [i * per, (i + 1) * per): every load is issued
  // before the one workgroup scan of the run sums (a loop of block scans waits on each)
  __shared__ unsigned long long s_w[kScanBlock / 64];
  __shared__ uint32_t s_v[kScanLds];          // the counts, loaded coalesced (ng <= kScanLds)
  __shared__ unsigned long long s_base[kScanBlock];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t per = (ng + kScanBlock - 1) / kScanBlock;
  const int64_t b = threadIdx.x * per, e = b + per < ng ? b + per : ng;
  unsigned long long cand = 0, sum = 0;
  const bool lds = ng <= kScanLds;
  if (lds) {
    // coalesced loads (every count in flight at once), then each thread's contiguous run
    // from LDS; offsets written back coalesced
    for (int64_t i = threadIdx.x; i < ng; i += kScanBlock) {
      cand += gcand[i];
      s_v[i] = gsum[i];
    }
    __syncthreads();
    for (int64_t i = b; i < e; i++) sum += s_v[i];
  } else {
    for (int64_t i = b; i < e; i++) {
      cand += gcand[i];
      sum += gsum[i];
    }
  }
  cand = wave_sum_u64(cand);
  if (lane == 0 && cand) atomicAdd(&counters[3], cand);
  unsigned long long incl = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned long long u = __shfl_up(incl, d, 64);
    if (lane >= d) incl += u;
  }
  if (lane == 63) s_w[wave] = incl;
  __syncthreads();
  unsigned long long run = incl - sum, tot = 0;
  for (int w = 0; w < kScanBlock / 64; w++) {
    if (w < wave) run += s_w[w];
    tot += s_w[w];
  }
  if (lds) {
    // s_v[i] = the offset of i within its thread's run (< 2^32), s_base = the run's base
    s_base[threadIdx.x] = run;
    uint32_t rel = 0;
    for (int64_t i = b; i < e; i++) {
      const uint32_t v = s_v[i];
      s_v[i] = rel;
      rel += v;
    }
    __syncthreads();
    for (int64_t i = threadIdx.x; i < ng; i += kScanBlock) goff[i] = s_base[i / per] + s_v[i];
  } else {
    for (int64_t i = b; i < e; i++) {
      goff[i] = run;
      run += gsum[i];
    }
  }
  if (threadIdx.x == 0) counters[0] = tot;
}

// Ordered output: the records of kEmitTiles consecutive tiles (their output ranges are
// contiguous) -> out[offset of the first ...] with point ids, as one flat stream over
// the workgroup's lanes.
constexpr int kEmitBlock = 256;
constexpr int kEmitTiles = 4096 / kTile;  // 4 tiles of 1024 points, 16 of 256
static_assert(kScanGroup % kEmitTiles == 0 && kEmitTiles <= 64, "emit groups inside scan groups");
__global__ __launch_bounds__(kEmitBlock) void pair_emit_kernel(EmitArgs a, int64_t n_tiles) {
  __shared__ uint32_t s_pref[kEmitTiles + 1];
  __shared__ uint64_t s_where[kEmitTiles];
  __shared__ int64_t s_off;
  const int64_t t0 = (int64_t)blockIdx.x * kEmitTiles;
  if (a.redo_affected && t0 + kEmitTiles <= (int64_t)*a.redo_first) {  // (an override rerun: as split_emit_kernel)
    bool any = false;
    for (int k = 0; k < kEmitTiles && t0 + k < n_tiles; k++) any |= a.redo_affected[t0 + k] != 0;
    if (!any) return;
  }
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    // this block's tiles: counts, slots, in-block prefix
    const int64_t t = t0 + lane;
    const bool in = lane < kEmitTiles && t < n_tiles;
    const uint32_t cnt = in ? a.tile_count[t] : 0u;
    if (lane < kEmitTiles) s_where[lane] = in ? a.tile_where[t] : kNoDst;
    const uint32_t incl = wave_incl_scan(cnt);
    if (lane < kEmitTiles) s_pref[lane + 1] = incl;
    if (lane == 0) s_pref[0] = 0;
    // predecessors of t0 inside its scan group
    const int64_t g0 = t0 - t0 % kScanGroup;
    const int64_t j = g0 + lane;
    unsigned long long v = (lane < kScanGroup && j < t0) ? a.tile_count[j] : 0u;
    v = wave_sum_u64(v);
    if (lane == 0) s_off = (int64_t)(a.group_off[t0 / kScanGroup] + v);
  }
  __syncthreads();
  const int64_t off = s_off;
  const uint32_t total = s_pref[kEmitTiles];
  for (uint32_t i = threadIdx.x; i < total; i += kEmitBlock) {
    const int64_t q = off + i;
    if (q >= a.capacity) break;
    int k = 0;
#pragma unroll
    for (int step = kEmitTiles / 2; step >= 1; step >>= 1)
      if (s_pref[k + step] <= i) k += step;
    const uint64_t where = s_where[k];
    if (where == kNoDst) continue;  // pool exhausted: the total exceeds the capacity
    const uint64_t r = a.recs[where + (i - s_pref[k])];
    const int64_t p = (t0 + k) * kTile + (int64_t)(r >> 32);
#if MGPU_EMIT_NT_OTHER
    __builtin_nontemporal_store(a.point_id ? a.point_id[p] : a.id_base + p, &a.out_point[q]);
    __builtin_nontemporal_store((int32_t)(uint32_t)r, &a.out_poly[q]);
#else
    a.out_point[q] = a.point_id ? a.point_id[p] : a.id_base + p;
    a.out_poly[q] = (int32_t)(uint32_t)r;
#endif
  }
}

__global__ __launch_bounds__(kStreamBlock) void st_contains_kernel(ChipTableView t, const int64_t* __restrict__ row,
                                                             const double* __restrict__ x,
                                                             const double* __restrict__ y, int64_t n,
                                                             int8_t* __restrict__ out,
                                                             unsigned long long* __restrict__ counters) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t r = i < n ? row[i] : 0;
  const bool bad = i < n && (r < 0 || r >= (int64_t)t.n_chips);
  count_wave(&counters[2], bad);  // the call fails with MGPU_E_INVALID_ARG
  if (i >= n) return;
  if (bad) {
    out[i] = -2;
    return;
  }
  uint32_t c = t.row_to_chip[r];
  if (t.chip_flags[c] & kChipNoGeom) {
    out[i] = -1;
    return;
  }
  out[i] = pip::chip_locate(t, c, x[i], y[i]) == pip::kInterior ? 1 : 0;
}

// ---------------------------------------------------------------- StringType cell ids
// IndexSystem.serializeCellId for StringType (IndexSystem.scala:61-70): BNG
// BNGIndexSystem.format (BNGIndexSystem.scala:119-134; bng_core.h format_cell_packed, the
// code the host formatter runs) and H3 h3ToString (H3IndexSystem.format = Long.toHexString,
// lowercase, no leading zeros).  Three passes, chunked by kFmtChunk ids per workgroup:
//   fmt_count_kernel  lengths -> one total per chunk (8 B read per id)
//   scan_sums_kernel  exclusive scan of the chunk totals
//   fmt_write_kernel  lengths again, workgroup scan per 256-id slice, offsets (8 B per
//                     id) and the characters (LDS-staged, coalesced 4-byte stores)
constexpr int kFmtBlock = 256;
constexpr int kFmtSlices = 16;
constexpr int kFmtChunk = kFmtBlock * kFmtSlices;

template <int IS>
__device__ __forceinline__ int format_id(int64_t id, uint64_t* lo, uint64_t* hi) {
  if (IS == MGPU_BNG) return bng::format_cell_packed(id, lo, hi);
  const uint64_t v = (uint64_t)id;
  const int nd = v ? (64 - __clzll((long long)v) + 3) / 4 : 1;
  *lo = *hi = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    if (i < nd) {
      const uint32_t d = (uint32_t)(v >> (4 * (nd - 1 - i))) & 15u;
      bng::put_char(lo, hi, i, d < 10 ? '0' + d : 'a' + d - 10);
    }
  }
  return nd;
}

// workgroup-wide exclusive scan of one value per thread; returns the total too
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_w, uint32_t* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t incl = wave_incl_scan(v);
  if (lane == 63) s_w[wave] = incl;
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kFmtBlock / 64; w++) {
    const uint32_t x = s_w[w];
    if (w < wave) off += x;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return off + incl - v;
}

template <int IS>
__global__ __launch_bounds__(kFmtBlock) void fmt_count_kernel(const int64_t* __restrict__ cells, int64_t n,
                                                            int64_t* __restrict__ chunk_tot,
                                                            unsigned long long* __restrict__ counters) {
  __shared__ uint32_t s_w[kFmtBlock / 64];
  const int64_t c0 = (int64_t)blockIdx.x * kFmtChunk;
  uint32_t sum = 0;
  bool bad = false;
#pragma unroll 4
  for (int sl = 0; sl < kFmtSlices; sl++) {
    const int64_t i = c0 + sl * kFmtBlock + threadIdx.x;
    if (i < n) {
      uint64_t lo, hi;
      const int len = format_id<IS>(cells[i], &lo, &hi);
      sum += len < 0 ? 0u : (uint32_t)len;
      bad |= len < 0;
    }
  }
  count_wave(&counters[2], bad);
  uint32_t tot;
  block_excl_scan(sum, s_w, &tot);
  if (threadIdx.x == 0) chunk_tot[blockIdx.x] = tot;
}

template <int IS>
__global__ __launch_bounds__(kFmtBlock) void fmt_write_kernel(const int64_t* __restrict__ cells, int64_t n,
                                                            const int64_t* __restrict__ chunk_off,
                                                            int64_t* __restrict__ offsets, char* __restrict__ out,
                                                            int64_t out_bytes) {
  __shared__ uint32_t s_w[kFmtBlock / 64];
  __shared__ __attribute__((aligned(16))) char s_c[kFmtBlock * 16 + 8];
  const int64_t c0 = (int64_t)blockIdx.x * kFmtChunk;
  int64_t carry = chunk_off[blockIdx.x];
  for (int sl = 0; sl < kFmtSlices; sl++) {
    const int64_t s0 = c0 + sl * kFmtBlock;
    if (s0 >= n) break;
    const int64_t i = s0 + threadIdx.x;
    uint64_t lo = 0, hi = 0;
    int len = 0;
    if (i < n) {
      len = format_id<IS>(cells[i], &lo, &hi);
      if (len < 0) len = 0;
    }
    uint32_t tot;
    const uint32_t ex = block_excl_scan((uint32_t)len, s_w, &tot);
    if (i < n) {
      offsets[i] = carry + ex;
      if (i == n - 1) offsets[n] = carry + ex + len;
#pragma unroll
      for (int k = 0; k < 16; k++)
        if (k < len) s_c[ex + k] = (char)((k < 8 ? lo >> (8 * k) : hi >> (8 * (k - 8))) & 0xFF);
    }
    __syncthreads();
    // [base, end): head bytes up to 4-byte alignment, words, tail bytes
    const int64_t base = carry, end = carry + tot < out_bytes ? carry + tot : out_bytes;
    const int64_t a0 = (base + 3) & ~(int64_t)3, a1 = end & ~(int64_t)3;
    if (a0 >= a1) {
      for (int64_t q = base + threadIdx.x; q < end; q += kFmtBlock) out[q] = s_c[q - base];
    } else {
      if (base + threadIdx.x < a0) out[base + threadIdx.x] = s_c[threadIdx.x];
      for (int64_t q = a0 + 4 * (int64_t)threadIdx.x; q < a1; q += 4 * kFmtBlock) {
        const int64_t r = q - base;
        const uint32_t w = (uint32_t)(uint8_t)s_c[r] | ((uint32_t)(uint8_t)s_c[r + 1] << 8) |
                           ((uint32_t)(uint8_t)s_c[r + 2] << 16) | ((uint32_t)(uint8_t)s_c[r + 3] << 24);
        *(uint32_t*)(out + q) = w;
      }
      if (a1 + threadIdx.x < end) out[a1 + threadIdx.x] = s_c[a1 + threadIdx.x - base];
    }
    carry += tot;
    __syncthreads();
  }
}

constexpr int kScan = 1024;
// exclusive scan of v[0, nb) in place (one workgroup)
__global__ __launch_bounds__(kScan) void scan_sums_kernel(int64_t* __restrict__ bsum, int64_t nb) {
  __shared__ int64_t s_w[kScan / 64];
  __shared__ int64_t s_carry;
  if (threadIdx.x == 0) s_carry = 0;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int64_t b = 0; b < nb; b += kScan) {
    const int64_t i = b + threadIdx.x;
    const int64_t x = i < nb ? bsum[i] : 0;
    int64_t incl = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int64_t u = __shfl_up(incl, d, 64);
      if (lane >= d) incl += u;
    }
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    int64_t run = s_carry + incl - x, tot = 0;
    for (int w = 0; w < kScan / 64; w++) {
      if (w < wave) run += s_w[w];
      tot += s_w[w];
    }
    if (i < nb) bsum[i] = run;
    __syncthreads();
    if (threadIdx.x == 0) s_carry += tot;
    __syncthreads();
  }
}

// ---------------------------------------------------------------- BNG kRing / kLoop
// BNGIndexSystem.kRing / kLoop (BNGIndexSystem.scala:221-252) over a device column of
// cells (grid_cellkring / grid_cellkloop, expressions/index/CellKRing.scala:68,
// CellKLoop.scala:63): the candidates of every loop are pointToIndex of the corners
// around the cell's south-west corner (bng_core.h kloop_xy), kept when isValid; kRing =
// the cell, then loops 1..k.  Same three-pass layout as the string ids: counts per
// chunk, chunk scan, then per 256-cell slice a workgroup scan, offsets and the ids.
// one loop's kept ids (-1: a candidate's isValid throws in the reference)
__device__ __forceinline__ int64_t bng_loop(int r, int32_t e, int32_t x, int32_t y, int k, int64_t* out) {
  int64_t m = 0;
  for (int c = 0; c < 8 * k; c++) {
    int32_t px, py;
    bng::kloop_xy(x, y, e, k, c, &px, &py);
    int64_t nb = 0;
    bng::point_to_cell((double)px, (double)py, r, &nb);
    const int v = bng::valid_state(nb);
    if (v < 0) return -1;
    if (v) {
      if (out) out[m] = nb;
      m++;
    }
  }
  return m;
}

// entries of one cell's list (-1: the reference throws -- the id is no BNG cell, or
// a loop candidate cannot be parsed by isValid)
__device__ __forceinline__ int64_t bng_kring(int64_t id, int k, bool loop_only, int64_t* out) {
  int r, xl, yl;
  int32_t e, x, y;
  if (!bng::cell_corner(id, &r, &e, &x, &y, &xl, &yl)) return -1;
  if (loop_only) return bng_loop(r, e, x, y, k, out);
  int64_t m = 1;
  if (out) out[0] = id;
  for (int j = 1; j <= k; j++) {
    const int64_t l = bng_loop(r, e, x, y, j, out ? out + m : nullptr);
    if (l < 0) return -1;
    m += l;
  }
  return m;
}

// one cell's list for either index system: H3 kRing / hexRing (h3_ring.h) or BNG.
// -1: not a cell of the system (BNG: or isValid throws); -2: H3 walk reaches a
// pentagon base cell (outside this version's scope)
__device__ __forceinline__ int64_t cell_kring(int is, int64_t id, int k, bool loop_only, int64_t* out) {
  if (is == MGPU_BNG) return bng_kring(id, k, loop_only, out);
  if (!h3ring::valid_cell((uint64_t)id)) return -1;
  const int64_t m = loop_only ? h3ring::hex_ring((uint64_t)id, k, out) : h3ring::kring((uint64_t)id, k, out);
  return m < 0 ? h3ring::kFallback : m;
}

// per cell: mc[i] = its list length, -1 (not a cell of the index system) or kFallback
// (an H3 walk that met a pentagon: kring_fallback_kernel decides it); the fallback cells
// are listed in fb_idx (counters[3] = their number); chunk_tot = the direct lists' sums
__global__ __launch_bounds__(kFmtBlock) void kring_count_kernel(int is, const int64_t* __restrict__ cells, int64_t n, int k,
                                                              int loop_only, int64_t* __restrict__ mc,
                                                              int64_t* __restrict__ chunk_tot, uint32_t* __restrict__ fb_idx,
                                                              unsigned long long* __restrict__ counters) {
  __shared__ unsigned long long s_w[kFmtBlock / 64];
  const int64_t c0 = (int64_t)blockIdx.x * kFmtChunk;
  const int lane = threadIdx.x & 63;
  unsigned long long sum = 0;
  bool bad = false;
  for (int sl = 0; sl < kFmtSlices; sl++) {
    const int64_t i = c0 + sl * kFmtBlock + threadIdx.x;
    bool fb = false;
    if (i < n) {
      const int64_t m = cell_kring(is, cells[i], k, loop_only != 0, nullptr);
      mc[i] = m;
      sum += m < 0 ? 0ull : (unsigned long long)m;
      bad |= m == -1;
      fb = m == h3ring::kFallback;
    }
    const unsigned long long bal = __ballot(fb);
    if (bal) {
      const int leader = __ffsll((long long)bal) - 1;
      unsigned long long base = 0;
      if (lane == leader) base = atomicAdd(&counters[3], (unsigned long long)__popcll(bal));
      base = __shfl(base, leader, 64);
      if (fb) fb_idx[base + __popcll(bal & ((1ull << lane) - 1ull))] = (uint32_t)i;
    }
  }
  count_wave(&counters[2], bad);
  sum = wave_sum_u64(sum);
  if (lane == 0) s_w[threadIdx.x >> 6] = sum;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < kFmtBlock / 64; w++) t += s_w[w];
    chunk_tot[blockIdx.x] = (int64_t)t;
  }
}

// The H3 cells whose walk met a pentagon, fb_idx[j0 .. j1), one thread each, with the
// reference's fallbacks (h3_ring.h kring_hash / kloop_diff) in kring_fallback_words(k)
// words of scratch per cell.  Count mode: mc[i] = -(length + 3), chunk_tot += length;
// write mode: the list at out[offsets[i]] (when it fits the capacity).  counters[4] +=
// walks whose hash set overflowed (inconsistent tables; never expected).
__host__ __device__ constexpr int64_t kring_fb_words(int k) {
  return 2 * (3 * (int64_t)k * (k + 1) + 1) + (3 * (int64_t)k * (k + 1) + 2) / 2 +
         (k > 0 ? (3 * (int64_t)(k - 1) * k + 1) + (3 * (int64_t)(k - 1) * k + 2) / 2 : 0) + 2 +
         (k + 2) + (k + 2 + 7) / 8;  // + the walk's stack (cells, next direction)
}
__global__ __launch_bounds__(64) void kring_fallback_kernel(const int64_t* __restrict__ cells, const uint32_t* __restrict__ fb_idx,
                                                            int64_t j0, int64_t j1, int k, int loop_only,
                                                            int64_t* __restrict__ mc, int64_t* __restrict__ chunk_tot,
                                                            const int64_t* __restrict__ offsets, int64_t* __restrict__ out,
                                                            int64_t capacity, uint64_t* __restrict__ scratch, int write,
                                                            unsigned long long* __restrict__ counters) {
  const int64_t j = j0 + (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (j >= j1) return;
  const int64_t i = fb_idx[j];
  const uint64_t h = (uint64_t)cells[i];
  const int64_t m = h3ring::max_kring(k), m2 = k > 0 ? h3ring::max_kring(k - 1) : 1;
  uint64_t* tab = scratch + (j - j0) * kring_fb_words(k);
  int32_t* dist = (int32_t*)(tab + m);
  uint64_t* tab2 = tab + m + (m + 1) / 2;
  int32_t* dist2 = (int32_t*)(tab2 + m2);
  int64_t* list = (int64_t*)(tab2 + m2 + (m2 + 1) / 2);
  uint64_t* stk = tab + kring_fb_words(k) - ((k + 2) + (k + 2 + 7) / 8);
  int8_t* nxt = (int8_t*)(stk + k + 2);
  bool ok = true;
  int64_t cnt = 0;
  if (!loop_only) {  // (here the spiral failed: H3's _kRingInternal)
    ok = h3ring::kring_hash(h, k, tab, dist, stk, nxt);
    for (int64_t q = 0; q < m; q++)
      if (tab[q]) list[cnt++] = (int64_t)tab[q];
  } else {
    // kRing(h, k) and kRing(h, k - 1) as H3-Java gives them -- the spiral where it
    // succeeds (its cells put into a hash set: toSet), else the hash-set walk
    const int64_t ma = h3ring::kring(h, k, list);
    if (ma >= 0) {
      for (int64_t q = 0; q < m; q++) tab[q] = 0;
      for (int64_t q = 0; q < ma; q++) h3ring::hash_insert(tab, m, (uint64_t)list[q]);
    } else {
      ok = h3ring::kring_hash(h, k, tab, dist, stk, nxt);
    }
    const int64_t ms = h3ring::kring(h, k - 1, list);
    if (ms >= 0) {
      for (int64_t q = 0; q < m2; q++) tab2[q] = 0;
      for (int64_t q = 0; q < ms; q++) h3ring::hash_insert(tab2, m2, (uint64_t)list[q]);
    } else {
      ok = ok && h3ring::kring_hash(h, k - 1, tab2, dist2, stk, nxt);
    }
    cnt = ok ? h3ring::kloop_diff(tab, m, tab2, m2, list) : 0;
  }
  if (!ok) {
    atomicAdd(&counters[4], 1ull);
    cnt = 0;
  }
  if (!write) {
    mc[i] = -(cnt + 3);
    atomicAdd((unsigned long long*)&chunk_tot[i / kFmtChunk], (unsigned long long)cnt);
    return;
  }
  const int64_t o = offsets[i];
  if (o + cnt <= capacity)
    for (int64_t q = 0; q < cnt; q++) out[o + q] = list[q];
}

__global__ __launch_bounds__(kFmtBlock) void kring_write_kernel(int is, const int64_t* __restrict__ cells, int64_t n, int k,
                                                              int loop_only, const int64_t* __restrict__ mc,
                                                              const int64_t* __restrict__ chunk_off,
                                                              int64_t* __restrict__ offsets, int64_t* __restrict__ out,
                                                              int64_t capacity) {
  __shared__ uint32_t s_w[kFmtBlock / 64];
  const int64_t c0 = (int64_t)blockIdx.x * kFmtChunk;
  int64_t carry = chunk_off[blockIdx.x];
  for (int sl = 0; sl < kFmtSlices; sl++) {
    const int64_t s0 = c0 + sl * kFmtBlock;
    if (s0 >= n) break;
    const int64_t i = s0 + threadIdx.x;
    int64_t m = 0, v = 0;
    if (i < n) {
      v = mc[i];
      m = v >= 0 ? v : (v <= -3 ? -(v + 3) : 0);
    }
    uint32_t tot;
    const uint32_t ex = block_excl_scan((uint32_t)m, s_w, &tot);
    if (i < n) {
      const int64_t o = carry + ex;
      offsets[i] = o;
      if (i == n - 1) offsets[n] = o + m;
      // (fallback cells are written by kring_fallback_kernel in write mode)
      if (v > 0 && o + m <= capacity) cell_kring(is, cells[i], k, loop_only != 0, out + o);
    }
    carry += tot;
  }
}

int64_t format_chunks(int64_t n) { return (n + kFmtChunk - 1) / kFmtChunk; }

hipError_t launch_kring_count(int is, const int64_t* cells, int64_t n, int k, int loop_only, int64_t* mc,
                              int64_t* chunk, uint32_t* fb_idx, unsigned long long* counters, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(kring_count_kernel, dim3((unsigned)format_chunks(n)), dim3(kFmtBlock), 0, s, is, cells, n, k,
                     loop_only, mc, chunk, fb_idx, counters);
  return hipGetLastError();
}

int64_t kring_fallback_words(int k) { return kring_fb_words(k); }
int32_t kring_fallback_max_k() { return 1024; }  // (the entry's own bound on k)

hipError_t launch_kring_fallback(const int64_t* cells, const uint32_t* fb_idx, int64_t j0, int64_t j1, int k,
                                 int loop_only, int64_t* mc, int64_t* chunk, const int64_t* offsets, int64_t* out,
                                 int64_t capacity, uint64_t* scratch, int write, unsigned long long* counters,
                                 hipStream_t s) {
  if (j1 <= j0) return hipSuccess;
  hipLaunchKernelGGL(kring_fallback_kernel, dim3((unsigned)((j1 - j0 + 63) / 64)), dim3(64), 0, s, cells, fb_idx, j0, j1,
                     k, loop_only, mc, chunk, offsets, out, capacity, scratch, write, counters);
  return hipGetLastError();
}

hipError_t launch_kring_write(int is, const int64_t* cells, int64_t n, int k, int loop_only, const int64_t* mc,
                              int64_t* chunk, int64_t* offsets, int64_t* out, int64_t capacity, hipStream_t s) {
  hipError_t e = hipMemsetAsync(offsets, 0, sizeof(int64_t), s);
  if (e != hipSuccess || n <= 0) return e;
  const int64_t nc = format_chunks(n);
  hipLaunchKernelGGL(scan_sums_kernel, dim3(1), dim3(kScan), 0, s, chunk, nc);
  hipLaunchKernelGGL(kring_write_kernel, dim3((unsigned)nc), dim3(kFmtBlock), 0, s, is, cells, n, k, loop_only, mc, chunk,
                     offsets, out, capacity);
  return hipGetLastError();
}

hipError_t launch_format_cells(int is, const int64_t* cells, int64_t n, char* out, int64_t out_bytes,
                               int64_t* offsets, int64_t* chunk, unsigned long long* counters, hipStream_t s) {
  hipError_t e = hipMemsetAsync(offsets, 0, sizeof(int64_t), s);
  if (e != hipSuccess || n <= 0) return e;
  const int64_t nc = format_chunks(n);
  if (is == MGPU_BNG)
    hipLaunchKernelGGL(fmt_count_kernel<MGPU_BNG>, dim3((unsigned)nc), dim3(kFmtBlock), 0, s, cells, n, chunk, counters);
  else
    hipLaunchKernelGGL(fmt_count_kernel<MGPU_H3>, dim3((unsigned)nc), dim3(kFmtBlock), 0, s, cells, n, chunk, counters);
  hipLaunchKernelGGL(scan_sums_kernel, dim3(1), dim3(kScan), 0, s, chunk, nc);
  if (is == MGPU_BNG)
    hipLaunchKernelGGL(fmt_write_kernel<MGPU_BNG>, dim3((unsigned)nc), dim3(kFmtBlock), 0, s, cells, n, chunk, offsets,
                       out, out_bytes);
  else
    hipLaunchKernelGGL(fmt_write_kernel<MGPU_H3>, dim3((unsigned)nc), dim3(kFmtBlock), 0, s, cells, n, chunk, offsets,
                       out, out_bytes);
  return hipGetLastError();
}

// ---------------------------------------------------------------- binned pipeline
// (kernels.h BinArgs).  With a chip table far beyond the caches (C3: 9.4M chips, 1.2 GB
// of border-chip headers, a 60 MB lattice grid) a uniform point stream makes every point
// fetch its own random grid line and, per candidate, two random header lines -- 8-16x
// the algorithmic bytes.  A counting sort of the points by a coarse spatial bin (one
// histogram pass, one scatter pass: no full sort, the order inside a bin is irrelevant)
// lets the join walk the table bin by bin: the tiles of a bin run on one XCD and share
// its chips in that XCD's L2.  The answers are per binned slot; the emit gathers them
// back in input order (a chunk's slots fall in one short run per bin).
constexpr int kBinBlock = 512;
constexpr int kBinChunk = 4096;                   // points per histogram / scatter workgroup
constexpr int kBinItems = kBinChunk / kBinBlock;  // per thread, all in flight
constexpr int kBinMax = 512;                      // bins
constexpr int kBinGroup = 64;                     // chunk rows per first-level column scan
static_assert(kBinMax == kBinBlock, "one bin per thread in the workgroup scans");

__device__ __forceinline__ uint32_t bin_of(const BinArgs& b, double x, double y) {
  // NaN and points outside the extent clamp to an edge bin (the bin only orders the work)
  const double fx = (x - b.x0) * b.inv_bx, fy = (y - b.y0) * b.inv_by;
  const int ix = fx >= 0.0 ? (fx < (double)b.nbx ? (int)fx : b.nbx - 1) : 0;
  const int iy = fy >= 0.0 ? (fy < (double)b.nby ? (int)fy : b.nby - 1) : 0;
  // boustrophedon rows: consecutive bins are neighbours
  return (uint32_t)(iy * b.nbx + ((iy & 1) ? b.nbx - 1 - ix : ix));
}

// per chunk of kBinChunk points: its row of bin counts
__global__ __launch_bounds__(kBinBlock) void bin_hist_kernel(BinArgs b) {
  __shared__ uint32_t s_h[kBinMax];
  const int nb = b.nbx * b.nby;
  if ((int)threadIdx.x < nb) s_h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t n = b.s.j.n, c0 = (int64_t)blockIdx.x * kBinChunk;
  double px[kBinItems], py[kBinItems];
#pragma unroll
  for (int k = 0; k < kBinItems; k++) {
    const int64_t p = c0 + (int64_t)k * kBinBlock + threadIdx.x;
    px[k] = py[k] = 0.0;
    if (p < n) {
      px[k] = __builtin_nontemporal_load(&b.x[p]);
      py[k] = __builtin_nontemporal_load(&b.y[p]);
    }
  }
  // one LDS atomic per distinct bin of the wave (as bin_scatter_kernel's ranks)
  const int nbits = nb > 1 ? 32 - __clz(nb - 1) : 0;
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < kBinItems; k++) {
    const bool act = c0 + (int64_t)k * kBinBlock + threadIdx.x < n;
    const uint32_t bi = act ? bin_of(b, px[k], py[k]) : 0u;
    unsigned long long peers = __ballot(act);
    for (int bit = 0; bit < nbits; bit++) {
      const bool on = (bi >> bit) & 1u;
      const unsigned long long m = __ballot(on);
      peers &= on ? m : ~m;
    }
    if (act && lane == __ffsll((unsigned long long)peers) - 1) atomicAdd(&s_h[bi], (uint32_t)__popcll(peers));
  }
  __syncthreads();
  if ((int)threadIdx.x < nb) b.cnt[(int64_t)blockIdx.x * nb + threadIdx.x] = s_h[threadIdx.x];
}

// pre[chunk][bin] = the exclusive prefix of cnt over the chunks of its group of
// kBinGroup; gsum[group][bin] = the group's sum
__global__ __launch_bounds__(256) void bin_colscan_kernel(BinArgs b, int64_t n_chunks) {
  const int nb = b.nbx * b.nby;
  const int bin = blockIdx.x * 256 + threadIdx.x;
  if (bin >= nb) return;
  const int64_t k0 = (int64_t)blockIdx.y * kBinGroup;
  uint32_t v[kBinGroup];
#pragma unroll
  for (int k = 0; k < kBinGroup; k++) v[k] = k0 + k < n_chunks ? b.cnt[(k0 + k) * nb + bin] : 0u;
  uint32_t run = 0;
#pragma unroll
  for (int k = 0; k < kBinGroup; k++) {
    if (k0 + k < n_chunks) b.pre[(k0 + k) * nb + bin] = run;
    run += v[k];
  }
  b.gsum[(int64_t)blockIdx.y * nb + bin] = run;
}

// one workgroup: each bin's total, the bins' exclusive scan (slots are bin-major), then
// gsum[group][bin] = the first slot of the bin's points of that group of chunks.  Each
// bin's column of group sums is cut into kBaseBlock / bins parts, one thread each (one
// thread per bin walked ~400 groups serially: 83 us per 1e8 points on C3).
constexpr int kBaseBlock = 1024;
__global__ __launch_bounds__(kBaseBlock) void bin_base_kernel(BinArgs b, int64_t n_groups) {
  __shared__ uint32_t s_part[kBaseBlock];
  __shared__ uint32_t s_base[kBinMax];
  __shared__ uint32_t s_w[kBaseBlock / 64];
  const int nb = b.nbx * b.nby;
  const int parts = kBaseBlock / nb > 0 ? kBaseBlock / nb : 1;
  const int bin = threadIdx.x / parts, part = threadIdx.x % parts;
  const int64_t per = (n_groups + parts - 1) / parts;
  const int64_t g0 = part * per, g1 = g0 + per < n_groups ? g0 + per : n_groups;
  uint32_t mine = 0;
  if (bin < nb)
    for (int64_t g = g0; g < g1; g++) mine += b.gsum[g * nb + bin];
  s_part[threadIdx.x] = mine;
  __syncthreads();
  // the bins' totals, scanned (thread t < nb: bin t)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t tot = 0;
  if ((int)threadIdx.x < nb)
    for (int q = 0; q < parts; q++) tot += s_part[threadIdx.x * parts + q];
  const uint32_t incl = wave_incl_scan(tot);
  if (lane == 63) s_w[wave] = incl;
  __syncthreads();
  if ((int)threadIdx.x < nb) {
    uint32_t run = incl - tot;
    for (int w = 0; w < wave; w++) run += s_w[w];
    s_base[threadIdx.x] = run;
  }
  __syncthreads();
  if (bin < nb) {
    uint32_t run = s_base[bin];
    for (int q = 0; q < part; q++) run += s_part[bin * parts + q];
    for (int64_t g = g0; g < g1; g++) {
      const uint32_t v = b.gsum[g * nb + bin];
      b.gsum[g * nb + bin] = run;
      run += v;
    }
  }
}

// The chunk's bin runs: s_off[bin] = its first binned slot, s_loc[bin] = its first
// position in the chunk's bin-sorted order (the scan of the chunk's counts); every lane
// of the workgroup ends holding nothing, the tables are in LDS after the barrier.
__device__ __forceinline__ void bin_runs(const BinArgs& b, int64_t k, uint32_t* s_off, uint32_t* s_loc,
                                         uint32_t* s_w) {
  const int nb = b.nbx * b.nby;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t g = k / kBinGroup;
  const int bin = threadIdx.x;
  uint32_t c = 0;
  if (bin < nb) {
    c = b.cnt[k * nb + bin];
    s_off[bin] = b.gsum[g * nb + bin] + b.pre[k * nb + bin];
  }
  const uint32_t incl = wave_incl_scan(c);
  if (lane == 63) s_w[wave] = incl;
  __syncthreads();
  uint32_t before = incl - c;
  for (int w = 0; w < wave; w++) before += s_w[w];
  if (bin < nb) s_loc[bin] = before;
  __syncthreads();
}

// the bin of position lp of the chunk's bin-sorted order (the last bin starting at or
// before it; empty bins start where the next one does)
__device__ __forceinline__ uint32_t bin_at(const uint32_t* s_loc, int nb, uint32_t lp) {
  uint32_t lo = 0, hi = (uint32_t)nb;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (s_loc[mid] <= lp)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

// Binned H3 joins over a dense lattice grid: the scatter kernel, which holds every point
// anyway, projects it (the streaming fast path, h3::fast_hex2d, as chip_probe) and writes
// the point's grid entry index per binned slot; the join's phase 1 then issues all of a
// lane's grid loads at once instead of one projection -> grid load chain per item.  A
// near-tie is queued here (tie_host) or sends the join's tile to the fix kernel (kKeyTie).
__device__ __forceinline__ uint32_t bin_key_of(const JoinArgs& a, int64_t pos, double px, double py) {
  const ChipTableView& t = a.chips;
  if (!(isfinite(px) && isfinite(py))) return kKeyBad;
  if (!a.res_match || !(px >= t.bbox[0] && px <= t.bbox[2] && py >= t.bbox[1] && py <= t.bbox[3])) return kKeyNone;
  const h3::FastHex f = h3::fast_hex2d(h3::to_radians_fast(py), h3::to_radians_fast(px), a.res, t.k_res, t.face_mask);
  if (f.tie) {
    if (!a.tie_host) return kKeyTie;
    tie_record(a.tie_queue, a.tie_cap, pos, px, py, h3::lattice_key(f.face, f.ijk));
  }
  const int32_t ga = f.ijk.i - f.ijk.k, gb = f.ijk.j - f.ijk.k;
  const DenseFace& D = t.dense[f.face];
  const uint32_t da = (uint32_t)(ga - D.a0), db = (uint32_t)(gb - D.b0);
  if (da >= D.w || db >= D.h) return kKeyNone;
  return (D.base + db * D.w + da) | (f.deep ? kKeyDeep : 0u);
}

// Per chunk: each point's rank among the chunk's points of its bin (LDS atomics -- any
// order inside a bin will do: perm[slot] records where each point came from), the
// chunk's points sorted by bin in LDS, then written as contiguous runs (one per bin) by
// consecutive lanes: whole cache lines, not one scattered 8-byte store per point.
template <bool KEY>
__global__ __launch_bounds__(kBinBlock) void bin_scatter_kernel(BinArgs b) {
  // (the chunk indices through s_val in a third pass, 8 KB less LDS -- 4 workgroups per CU
  // instead of 3 -- measured equal: profiles/r5/ab_c3_join_counts.txt)
  __shared__ double s_val[kBinChunk];   // x, then y, in the chunk's bin-sorted order
  __shared__ uint16_t s_li[kBinChunk];  // the point's index in the chunk
  __shared__ uint32_t s_off[kBinMax];
  __shared__ uint32_t s_loc[kBinMax];
  __shared__ uint32_t s_rank[kBinMax];
  __shared__ uint32_t s_w[kBinBlock / 64];
  const int nb = b.nbx * b.nby;
  const int64_t k = blockIdx.x;
  const int64_t n = b.s.j.n, c0 = k * kBinChunk;
  // the chunk's points load while the run tables are built
  double px[kBinItems], py[kBinItems];
#pragma unroll
  for (int q = 0; q < kBinItems; q++) {
    const int64_t p = c0 + (int64_t)q * kBinBlock + threadIdx.x;
    px[q] = py[q] = 0.0;
    if (p < n) {
      px[q] = __builtin_nontemporal_load(&b.x[p]);
      py[q] = __builtin_nontemporal_load(&b.y[p]);
    }
  }
  if ((int)threadIdx.x < nb) s_rank[threadIdx.x] = 0;
  bin_runs(b, k, s_off, s_loc, s_w);
  // ranks: the wave's lanes with the same bin found by one ballot per bin bit; one LDS
  // atomic per distinct bin (its lowest lane adds the group's size) -- not one per point,
  // whose same-address collisions serialised (r4: 45M LDS conflict cycles per 1e8 points)
  const int nbits = nb > 1 ? 32 - __clz(nb - 1) : 0;
  const int lane = threadIdx.x & 63;
  const unsigned long long below = (1ull << lane) - 1ull;
  uint32_t lps[kBinItems];
#pragma unroll
  for (int q = 0; q < kBinItems; q++) {
    const int64_t p = c0 + (int64_t)q * kBinBlock + threadIdx.x;
    const bool act = p < n;
    const uint32_t bi = act ? bin_of(b, px[q], py[q]) : 0u;
    unsigned long long peers = __ballot(act);
    for (int bit = 0; bit < nbits; bit++) {
      const bool on = (bi >> bit) & 1u;
      const unsigned long long m = __ballot(on);
      peers &= on ? m : ~m;
    }
    const int leader = act ? __ffsll((unsigned long long)peers) - 1 : lane;
    uint32_t base = 0;
    if (act && lane == leader) base = atomicAdd(&s_rank[bi], (uint32_t)__popcll(peers));
    base = __shfl(base, leader, 64);
    lps[q] = 0xFFFFFFFFu;
    if (act) {
      lps[q] = s_loc[bi] + base + (uint32_t)__popcll(peers & below);
      s_val[lps[q]] = px[q];
      s_li[lps[q]] = (uint16_t)(q * kBinBlock + threadIdx.x);
    }
  }
  __syncthreads();
  const int64_t left = n - c0;
  const uint32_t m = left < kBinChunk ? (uint32_t)left : (uint32_t)kBinChunk;
  uint32_t sls[kBinItems];
#pragma unroll
  for (int q = 0; q < kBinItems; q++) {
    const uint32_t lp = q * kBinBlock + threadIdx.x;
    sls[q] = 0xFFFFFFFFu;
    if (lp < m) {
      const uint32_t bi = bin_at(s_loc, nb, lp);
      sls[q] = s_off[bi] + (lp - s_loc[bi]);
      MGPU_ST_INTER(s_val[lp], &b.bx[sls[q]]);
      MGPU_ST_INTER((uint32_t)(c0 + s_li[lp]), &b.perm[sls[q]]);
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kBinItems; q++)
    if (lps[q] != 0xFFFFFFFFu) s_val[lps[q]] = py[q];
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kBinItems; q++)
    if (sls[q] != 0xFFFFFFFFu) MGPU_ST_INTER(s_val[q * kBinBlock + threadIdx.x], &b.by[sls[q]]);
  if (KEY) {
    // the grid keys, through the same LDS order (the first half of s_val as u32)
    uint32_t* s_key = (uint32_t*)s_val;
    uint32_t kv[kBinItems];
#pragma unroll
    for (int q = 0; q < kBinItems; q++)
      kv[q] = lps[q] != 0xFFFFFFFFu ? bin_key_of(b.s.j, c0 + (int64_t)q * kBinBlock + threadIdx.x, px[q], py[q]) : kKeyNone;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kBinItems; q++)
      if (lps[q] != 0xFFFFFFFFu) s_key[lps[q]] = kv[q];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kBinItems; q++)
      if (sls[q] != 0xFFFFFFFFu) MGPU_ST_INTER(s_key[q * kBinBlock + threadIdx.x], &b.key[sls[q]]);
  }
}

// the join over the binned points: join_tile's phases (G mode, no mixed list: every
// point of the chunk), the answers per slot in mixed_res.  xcd_runs: block b runs tile
// (b % 8) * per_xcd + b / 8 -- blocks b and b + 8 share an XCD, so each XCD walks one
// contiguous run of tiles (= of bins) and a bin's chips are fetched into one L2
template <int IS>
__global__ __launch_bounds__(kBlock) MGPU_JOIN_ATTR void pip_binned_kernel(JoinArgs a, uint32_t per_xcd, uint32_t n_tiles) {
  const uint32_t tile = per_xcd ? (blockIdx.x & 7u) * per_xcd + (blockIdx.x >> 3) : blockIdx.x;
  if (tile < n_tiles) join_tile<IS, false, 1>(a, tile);
}

// The answers back in input order, per chunk of kBinChunk input points: the chunk's bin
// runs are read run by run (consecutive lanes, consecutive slots: coalesced, one page
// per run) and placed by perm[] into LDS, then written out in input order; the pairs of
// each split_chunk() of input points are counted on the way (the emit's offsets).
constexpr int kBinEmitItems = kChunk / kClsBlock;
static_assert(kBinEmitItems % 2 == 0, "16-byte answer loads per thread");
static_assert(kBinChunk % kChunk == 0 && kBinChunk / kChunk <= kBinBlock / 64, "emit chunks inside a bin chunk");
// A bin chunk's answers into LDS in input order: its bin runs read whole (consecutive
// lanes, consecutive slots: coalesced, one page per run), placed by perm[]; every load of
// a thread's kBgItems slots in flight before its LDS stores
constexpr int kBgItems = kBinChunk / kBinBlock;  // slots per thread
__device__ __forceinline__ void bin_gather_lds(const BinArgs& b, int64_t c0, uint32_t m, int nb,
                                               const uint32_t* s_off, const uint32_t* s_loc, uint64_t* s_v) {
  uint32_t pp[kBgItems];
  uint64_t rv[kBgItems];
#pragma unroll
  for (int q = 0; q < kBgItems; q++) {
    const uint32_t lp = q * kBinBlock + threadIdx.x;
    pp[q] = 0xFFFFFFFFu;
    if (lp < m) {
      const uint32_t bi = bin_at(s_loc, nb, lp);
      const uint32_t sl = s_off[bi] + (lp - s_loc[bi]);
      pp[q] = b.perm[sl];
      rv[q] = b.s.j.mixed_res[sl];
    }
  }
#pragma unroll
  for (int q = 0; q < kBgItems; q++)
    if (pp[q] != 0xFFFFFFFFu) s_v[pp[q] - (uint32_t)c0] = rv[q];
}

__global__ __launch_bounds__(kBinBlock) void bin_gather_kernel(BinArgs b) {
  __shared__ uint64_t s_v[kBinChunk];
  __shared__ uint32_t s_off[kBinMax];
  __shared__ uint32_t s_loc[kBinMax];
  __shared__ uint32_t s_w[kBinBlock / 64];
  const int nb = b.nbx * b.nby;
  const int64_t k = blockIdx.x;
  const int64_t n = b.s.j.n, c0 = k * kBinChunk;
  bin_runs(b, k, s_off, s_loc, s_w);
  const int64_t left = n - c0;
  const uint32_t m = left < kBinChunk ? (uint32_t)left : (uint32_t)kBinChunk;
#ifndef MGPU_GATHER_UNROLL
#define MGPU_GATHER_UNROLL 1
#endif
  if (MGPU_GATHER_UNROLL) {
    bin_gather_lds(b, c0, m, nb, s_off, s_loc, s_v);
  } else {
    for (uint32_t lp = threadIdx.x; lp < m; lp += kBinBlock) {
      const uint32_t bi = bin_at(s_loc, nb, lp);
      const uint32_t sl = s_off[bi] + (lp - s_loc[bi]);
      s_v[b.perm[sl] - (uint32_t)c0] = b.s.j.mixed_res[sl];
    }
  }
  __syncthreads();
  constexpr int kPerWave = kChunk / (kBinBlock / 64) * (kBinChunk / kChunk);  // points per wave
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t np = 0;
  for (int i = wave * kPerWave + lane; i < (wave + 1) * kPerWave; i += 64)
    if ((uint32_t)i < m) {
      const uint64_t v = s_v[i];
      MGPU_ST_INTER(v, &b.res[c0 + i]);
      np += __popc((uint32_t)(v >> 32));
    }
  np = wave_sum_u32(np);
  // waves w .. w + W/E - 1 cover emit chunk (w * E / W): their sums meet in s_w
  __syncthreads();
  if (lane == 0) s_w[wave] = np;
  __syncthreads();
  constexpr int kE = kBinChunk / kChunk, kWpe = (kBinBlock / 64) / kE;  // emit chunks, waves per emit chunk
  if ((int)threadIdx.x < kE) {
    const int64_t e = k * kE + threadIdx.x;
    if (e * kChunk < n) {
      uint32_t t = 0;
      for (int w = 0; w < kWpe; w++) t += s_w[threadIdx.x * kWpe + w];
      b.s.chunk_pairs[e] = t;
    }
  }
}

// the answers of input points p0 .. p0 + 15, in input order
__device__ __forceinline__ void bin_answers(const BinArgs& b, int64_t p0, uint64_t* v) {
  const int64_t n = b.s.j.n;
  if (p0 + kBinEmitItems <= n) {
    const ulonglong2* src = (const ulonglong2*)(b.res + p0);
#pragma unroll
    for (int i = 0; i < kBinEmitItems / 2; i++) {
      const ulonglong2 q = src[i];
      v[2 * i] = q.x, v[2 * i + 1] = q.y;
    }
  } else {
#pragma unroll
    for (int k = 0; k < kBinEmitItems; k++) v[k] = p0 + k < n ? b.res[p0 + k] : 0ull;
  }
}

// ordered output of one input chunk (as split_emit_kernel: the chunk's pairs are one
// contiguous range, staged in LDS a window at a time, written by consecutive lanes)
__global__ __launch_bounds__(kClsBlock) __attribute__((amdgpu_waves_per_eu(MGPU_EMIT_WAVES))) void bin_emit_kernel(BinArgs b) {
  const SplitArgs& sa = b.s;
  const ChipTableView& t = sa.j.chips;
  __shared__ uint32_t s_w[kClsBlock / 64];
  __shared__ uint32_t s_poly[kEmitWin];
  __shared__ uint16_t s_pt[kEmitWin];
  const int64_t c0 = (int64_t)blockIdx.x * kChunk;
  const int l0 = threadIdx.x * kBinEmitItems;
  uint64_t v[kBinEmitItems];
  bin_answers(b, c0 + l0, v);
  uint32_t npair = 0;
#pragma unroll
  for (int k = 0; k < kBinEmitItems; k++) npair += __popc((uint32_t)(v[k] >> 32));
  uint32_t total;
  const uint32_t off0 = chunk_excl_scan(npair, s_w, &total);
  const uint64_t base = sa.chunk_off[blockIdx.x];
  for (uint32_t w0 = 0; w0 < total; w0 += kEmitWin) {
    if (off0 < w0 + kEmitWin && off0 + npair > w0) {
      uint32_t q = off0;
#pragma unroll
      for (int k = 0; k < kBinEmitItems; k++) {
        const uint32_t first = (uint32_t)v[k], msk = (uint32_t)(v[k] >> 32);
        if (msk == 1u) {  // one match: first is the polygon id (JoinArgs.poly_answers)
          if (q >= w0 && q < w0 + kEmitWin) {
            s_poly[emit_swz(q - w0)] = first;
            s_pt[emit_swz(q - w0)] = (uint16_t)(l0 + k);
          }
          q++;
          continue;
        }
        for (uint32_t m = msk; m; m &= m - 1, q++)
          if (q >= w0 && q < w0 + kEmitWin) {
            s_poly[emit_swz(q - w0)] = (uint32_t)t.chip_poly[first + __builtin_ctz(m)];
            s_pt[emit_swz(q - w0)] = (uint16_t)(l0 + k);
          }
      }
    }
    __syncthreads();
    const uint32_t cnt = total - w0 < (uint32_t)kEmitWin ? total - w0 : (uint32_t)kEmitWin;
    for (uint32_t i = threadIdx.x; i < cnt; i += kClsBlock) {
      const uint64_t q = base + w0 + i;
      if ((int64_t)q >= sa.capacity) break;
      const int64_t p = c0 + s_pt[emit_swz(i)];
#if MGPU_EMIT_NT_OTHER
      __builtin_nontemporal_store(sa.point_id ? sa.point_id[p] : sa.id_base + p, &sa.out_point[q]);
      __builtin_nontemporal_store((int32_t)s_poly[emit_swz(i)], &sa.out_poly[q]);
#else
      sa.out_point[q] = sa.point_id ? sa.point_id[p] : sa.id_base + p;
      sa.out_poly[q] = (int32_t)s_poly[emit_swz(i)];
#endif
    }
    __syncthreads();
  }
}

// The binned answers straight to ordered pairs (MGPU_BIN_JOIN_COUNTS: the join counted
// each input chunk's pairs, the scan made the offsets): per input chunk, its bin runs of
// answers are read whole (coalesced, one page per run) and placed by perm[] into LDS in
// input order -- bin_gather_kernel's front half, without writing the answers back out --
// then emitted as bin_emit_kernel does, 8 consecutive points per thread.
#ifndef MGPU_BIN_JOIN_COUNTS
#define MGPU_BIN_JOIN_COUNTS 1
#endif
static_assert(kBinChunk == kChunk, "one emit chunk per bin chunk");
__global__ __launch_bounds__(kBinBlock) void bin_emit_gather_kernel(BinArgs b) {
  const SplitArgs& sa = b.s;
  const ChipTableView& t = sa.j.chips;
  __shared__ uint64_t s_v[kBinChunk];
  __shared__ uint32_t s_off[kBinMax];
  __shared__ uint32_t s_loc[kBinMax];
  __shared__ uint32_t s_w[kBinBlock / 64];
  __shared__ uint32_t s_poly[kEmitWin];
  __shared__ uint16_t s_pt[kEmitWin];
  const int nb = b.nbx * b.nby;
  const int64_t k = blockIdx.x, n = sa.j.n, c0 = k * kBinChunk;
  bin_runs(b, k, s_off, s_loc, s_w);
  const int64_t left = n - c0;
  const uint32_t m = left < kBinChunk ? (uint32_t)left : (uint32_t)kBinChunk;
  bin_gather_lds(b, c0, m, nb, s_off, s_loc, s_v);
  __syncthreads();
  const int l0 = threadIdx.x * kBgItems;
  uint64_t v[kBgItems];
  uint32_t npair = 0;
#pragma unroll
  for (int q = 0; q < kBgItems; q++) {
    v[q] = (uint32_t)(l0 + q) < m ? s_v[l0 + q] : 0ull;
    npair += __popc((uint32_t)(v[q] >> 32));
  }
  // the thread's first pair within the chunk: a block scan of npair
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t incl = wave_incl_scan(npair);
  __syncthreads();  // (bin_runs' s_w reads are done)
  if (lane == 63) s_w[wave] = incl;
  __syncthreads();
  uint32_t off0 = incl - npair, total = 0;
#pragma unroll
  for (int w = 0; w < kBinBlock / 64; w++) {
    off0 += w < wave ? s_w[w] : 0u;
    total += s_w[w];
  }
  const uint64_t base = sa.chunk_off[k];
  for (uint32_t w0 = 0; w0 < total; w0 += kEmitWin) {
    if (off0 < w0 + kEmitWin && off0 + npair > w0) {
      uint32_t q = off0;
#pragma unroll
      for (int i = 0; i < kBgItems; i++) {
        const uint32_t first = (uint32_t)v[i], msk = (uint32_t)(v[i] >> 32);
        if (msk == 1u) {  // one match: first is the polygon id (JoinArgs.poly_answers)
          if (q >= w0 && q < w0 + kEmitWin) {
            s_poly[emit_swz(q - w0)] = first;
            s_pt[emit_swz(q - w0)] = (uint16_t)(l0 + i);
          }
          q++;
          continue;
        }
        for (uint32_t mm = msk; mm; mm &= mm - 1, q++)
          if (q >= w0 && q < w0 + kEmitWin) {
            s_poly[emit_swz(q - w0)] = (uint32_t)t.chip_poly[first + __builtin_ctz(mm)];
            s_pt[emit_swz(q - w0)] = (uint16_t)(l0 + i);
          }
      }
    }
    __syncthreads();
    const uint32_t cnt = total - w0 < (uint32_t)kEmitWin ? total - w0 : (uint32_t)kEmitWin;
    for (uint32_t i = threadIdx.x; i < cnt; i += kBinBlock) {
      const uint64_t q = base + w0 + i;
      if ((int64_t)q >= sa.capacity) break;
      const int64_t p = c0 + s_pt[emit_swz(i)];
      sa.out_point[q] = sa.point_id ? sa.point_id[p] : sa.id_base + p;
      sa.out_poly[q] = (int32_t)s_poly[emit_swz(i)];
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void scatter_i64_kernel(const int64_t* __restrict__ pos, const int64_t* __restrict__ val,
                                                          int64_t n, int64_t* __restrict__ out) {
  for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < n; k += (int64_t)gridDim.x * 256) out[pos[k]] = val[k];
}

__global__ __launch_bounds__(256) void gather_xy_kernel(const double* __restrict__ x, const double* __restrict__ y,
                                                        const int64_t* __restrict__ pos, int64_t n,
                                                        double* __restrict__ xy) {
  for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < n; k += (int64_t)gridDim.x * 256) {
    xy[2 * k] = x[pos[k]];
    xy[2 * k + 1] = y[pos[k]];
  }
}

// ---------------------------------------------------------------- launchers

hipError_t launch_cells(int is, int res, const double* x, const double* y, int64_t n, int64_t* out,
                        unsigned long long* counters, unsigned long long* ties, int64_t tie_cap, uint64_t* tie_queue,
                        int64_t tq_cap, hipStream_t s, const uint8_t* valid, int64_t voff) {
  if (n <= 0) return hipSuccess;
  int64_t blocks = (n + kStreamBlock - 1) / kStreamBlock;
  if (blocks > 256 * 64) blocks = 256 * 64;
  if (is == MGPU_H3) {
    hipLaunchKernelGGL(cells_kernel<MGPU_H3>, dim3((unsigned)blocks), dim3(kStreamBlock), 0, s, x, y, n, res, out, counters,
                       ties, tie_cap, valid, voff);
    hipLaunchKernelGGL(cells_fix_kernel, dim3(256), dim3(kStreamBlock), 0, s, x, y, n, res, out, counters, ties, tie_cap,
                       tie_queue, tq_cap, valid, voff);
  } else {
    hipLaunchKernelGGL(cells_kernel<MGPU_BNG>, dim3((unsigned)blocks), dim3(kStreamBlock), 0, s, x, y, n, res, out,
                       counters, ties, tie_cap, valid, voff);
  }
  return hipGetLastError();
}

hipError_t launch_scatter_i64(const int64_t* pos, const int64_t* val, int64_t n, int64_t* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(scatter_i64_kernel, dim3((unsigned)blocks), dim3(256), 0, s, pos, val, n, out);
  return hipGetLastError();
}

hipError_t launch_gather_xy(const double* x, const double* y, const int64_t* pos, int64_t n, double* xy, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(gather_xy_kernel, dim3((unsigned)blocks), dim3(256), 0, s, x, y, pos, n, xy);
  return hipGetLastError();
}

__global__ __launch_bounds__(kStreamBlock) void valid_and_kernel(const uint8_t* __restrict__ a, int64_t aoff,
                                                               const uint8_t* __restrict__ b, int64_t boff, int64_t n,
                                                               uint8_t* __restrict__ out) {
  const int64_t byte = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (byte * 8 >= n) return;
  uint8_t v = 0;
  for (int k = 0; k < 8; k++) {
    const int64_t p = byte * 8 + k;
    if (p < n && pt_valid(a, aoff, p) && pt_valid(b, boff, p)) v |= (uint8_t)(1u << k);
  }
  out[byte] = v;
}

hipError_t launch_valid_and(const uint8_t* a, int64_t aoff, const uint8_t* b, int64_t boff, int64_t n, uint8_t* out,
                            hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t bytes = (n + 7) / 8;
  hipLaunchKernelGGL(valid_and_kernel, dim3((unsigned)((bytes + kStreamBlock - 1) / kStreamBlock)), dim3(kStreamBlock), 0,
                     s, a, aoff, b, boff, n, out);
  return hipGetLastError();
}

int64_t join_tiles(int64_t n) { return (n + kTile - 1) / kTile; }
int64_t join_tile_points() { return kTile; }
int64_t join_slot_records() { return kSlot; }

#ifndef MGPU_FIX_GRID
#define MGPU_FIX_GRID 8192
#endif
constexpr int64_t kFixGrid = MGPU_FIX_GRID;  // fix-kernel workgroups (one wave each; idle ones exit at once)
hipError_t launch_join(int is, const JoinArgs& a, const EmitArgs& e, hipStream_t s, hipEvent_t after_stream) {
  if (a.n_tiles <= 0) return hipSuccess;
  // BNG has no near-ties, but its tiles still go dirty on a cell of more than 32
  // chips, a candidate-list overflow or a chip without a strip index
  // (the fix kernel walks the dirty list grid-stride; a grid that fills the GPU, since a
  // workload with many border-chip candidates per point -- BNG res 3 -- dirties most tiles)
  const unsigned fix_blocks = (unsigned)(a.n_tiles < kFixGrid ? a.n_tiles : kFixGrid);
  if (is == MGPU_H3) {
    hipLaunchKernelGGL(pip_join_kernel<MGPU_H3>, dim3((unsigned)a.n_tiles), dim3(kBlock), 0, s, a);
    if (after_stream) hipEventRecord(after_stream, s);
    hipLaunchKernelGGL(pip_fix_kernel<MGPU_H3>, dim3(fix_blocks), dim3(kBlock), 0, s, a);
  } else {
    hipLaunchKernelGGL(pip_join_kernel<MGPU_BNG>, dim3((unsigned)a.n_tiles), dim3(kBlock), 0, s, a);
    if (after_stream) hipEventRecord(after_stream, s);
    hipLaunchKernelGGL(pip_fix_kernel<MGPU_BNG>, dim3(fix_blocks), dim3(kBlock), 0, s, a);
  }
  hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(kScanBlock), 0, s, a.group_sum, a.group_cand,
                     (a.n_tiles + kScanGroup - 1) / kScanGroup, e.group_off, a.counters);
  hipLaunchKernelGGL(pair_emit_kernel, dim3((unsigned)((a.n_tiles + kEmitTiles - 1) / kEmitTiles)),
                     dim3(kEmitBlock), 0, s, e, a.n_tiles);
  return hipGetLastError();
}

// The override pass (capi.cpp launch_override_pass): a rerun of only the units -- fused
// tiles, split chunks -- holding points whose H3 cell the host's libm moved (R.list[0 ..
// n)).  Each unit's pairs leave its count first (the old count kept in R.old), the fix
// kernel redoes it with the overrides; when no unit's count changed (a point moved to a
// cell of the same polygons) the offsets stand and only the rerun units are emitted
// again, else the scan runs and the units from the first changed one on are emitted.
__global__ __launch_bounds__(256) void tile_unpair_kernel(JoinArgs a, RedoArgs R, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t tile = R.list[i];
  const uint32_t c = a.tile_count[tile];
  R.old[i] = c;
  if (c) atomicSub(&a.group_sum[tile / kScanGroup], c);
  a.tile_count[tile] = 0;
  a.tile_where[tile] = kNoDst;
  R.affected[tile] = 1;
  a.dirty[i] = tile;
}

__global__ __launch_bounds__(256) void chunk_unpair_kernel(JoinArgs a, RedoArgs R) {
  __shared__ uint32_t s_w[4];
  const uint32_t chunk = R.list[blockIdx.x];
  const uint32_t nm = a.chunk_mixed[chunk];
  uint32_t mine = 0;
  for (uint32_t i = threadIdx.x; i < nm; i += 256) mine += __popc((uint32_t)(a.mixed_res[(int64_t)chunk * kChunk + i] >> 32));
  mine = wave_sum_u32(mine);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = mine;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t tot = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    R.old[blockIdx.x] = a.group_sum[chunk];
    a.group_sum[chunk] -= tot;
    a.group_cand[chunk] = 0;  // (recounted by the rerun)
    R.affected[chunk] = 1;
    const uint32_t nt = (nm + kGTile - 1) / kGTile;  // the chunk's mixed tiles
    const uint32_t q = atomicAdd(a.n_dirty, nt);
    for (uint32_t t = 0; t < nt; t++) a.dirty[q + t] = chunk * kChunkTiles + t;
  }
}

__global__ __launch_bounds__(256) void redo_compare_kernel(const uint32_t* counts, RedoArgs R, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n && counts[R.list[i]] != R.old[i]) {
    atomicOr(R.changed, 1u);
    atomicMin(R.first, R.list[i]);
  }
}

hipError_t launch_join_redo(int is, const JoinArgs& a, const EmitArgs& e, const RedoArgs& R, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const unsigned g = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(tile_unpair_kernel, dim3(g), dim3(256), 0, s, a, R, n);
  const unsigned fix_blocks = (unsigned)(n < kFixGrid ? n : kFixGrid);
  if (is == MGPU_H3)
    hipLaunchKernelGGL(pip_fix_kernel<MGPU_H3>, dim3(fix_blocks), dim3(kBlock), 0, s, a);
  else
    hipLaunchKernelGGL(pip_fix_kernel<MGPU_BNG>, dim3(fix_blocks), dim3(kBlock), 0, s, a);
  hipLaunchKernelGGL(redo_compare_kernel, dim3(g), dim3(256), 0, s, (const uint32_t*)a.tile_count, R, n);
  hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(kScanBlock), 0, s, a.group_sum, a.group_cand,
                     (a.n_tiles + kScanGroup - 1) / kScanGroup, e.group_off, a.counters, (const uint32_t*)R.changed);
  EmitArgs er = e;
  er.redo_first = R.first;
  er.redo_affected = R.affected;
  hipLaunchKernelGGL(pair_emit_kernel, dim3((unsigned)((a.n_tiles + kEmitTiles - 1) / kEmitTiles)),
                     dim3(kEmitBlock), 0, s, er, a.n_tiles);
  return hipGetLastError();
}

int64_t split_chunk() { return kChunk; }
int64_t split_chunk_tiles() { return kChunkTiles; }
int64_t split_chunks(int64_t n) { return (n + kChunk - 1) / kChunk; }

// workgroups of `block` threads with `lds` dynamic LDS bytes resident on the whole GPU at once
static int resident_blocks(const void* kernel, int block, size_t lds) {
  int dev = 0, cus = 0, per = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, block, lds) != hipSuccess || per < 1) per = 1;
  return std::max(cus, 1) * per;
}

template <int IS>
static void launch_emit(const SplitArgs& a, int64_t nc, hipStream_t s) {
  // (A/B r5, profiles/r5/ab_classify_pair_emit_wave.txt: one wave per chunk -- wave scans,
  // no workgroup barrier, the class table loaded once per workgroup -- took the C2 emit
  // 0.255 -> 0.467 ms: rejected)
  hipLaunchKernelGGL(split_emit_kernel<IS>, dim3((unsigned)nc), dim3(kClsBlock), 0, s, a);
}

template <int IS>
static void launch_split_t(const SplitArgs& a, hipStream_t s, hipEvent_t after_classify, hipEvent_t after_mixed) {
  const int64_t nc = split_chunks(a.j.n);
  const ChipTableView& ct = a.j.chips;
  const size_t nblk = (IS == MGPU_H3 && ct.raster_blk) ? (size_t)ct.raster_bnx * ct.raster_bny : 0;
  const size_t lds = IS == MGPU_H3 ? ((nblk + 1) & ~(size_t)1) * 2 + (size_t)ct.raster_nband * 4 : 0;
  const int64_t wg = (nc + kCfyBlock / 64 - 1) / (kCfyBlock / 64);
  if (lds > 64 * 1024) {  // (a block table beyond 64 KB: one workgroup per CU)
    hipFuncSetAttribute((const void*)classify_pair_kernel<IS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipFuncSetAttribute((const void*)classify_wave_kernel<IS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  }
  if (MGPU_CFY_PAIR && ((((uintptr_t)a.j.x) | ((uintptr_t)a.j.y)) & 15) == 0) {
    const int64_t grid = std::min<int64_t>(wg, (int64_t)resident_blocks((const void*)classify_pair_kernel<IS>, kCfyBlock, lds));
    hipLaunchKernelGGL(classify_pair_kernel<IS>, dim3((unsigned)grid), dim3(kCfyBlock), lds, s, a, nc);
  } else {
    const int64_t grid = std::min<int64_t>(wg, (int64_t)resident_blocks((const void*)classify_wave_kernel<IS>, kCfyBlock, lds));
    hipLaunchKernelGGL(classify_wave_kernel<IS>, dim3((unsigned)grid), dim3(kCfyBlock), lds, s, a, nc);
  }
  if (after_classify) hipEventRecord(after_classify, s);
  // (one workgroup per chunk walking its mixed tiles; one workgroup per tile measured 8x
  // slower on C2: ~6 ns per dispatched workgroup, most of them empty)
  hipLaunchKernelGGL(pip_mixed_kernel<IS>, dim3((unsigned)nc), dim3(kBlock), 0, s, a.j);
  const int64_t more = std::min<int64_t>(nc, (int64_t)resident_blocks((const void*)pip_mixed_more_kernel<IS>, kBlock, 0));
  hipLaunchKernelGGL(pip_mixed_more_kernel<IS>, dim3((unsigned)more), dim3(kBlock), 0, s, a.j);
  const int64_t fix = nc * kChunkTiles < kFixGrid ? nc * kChunkTiles : kFixGrid;
  hipLaunchKernelGGL((pip_mixed_fix_kernel<IS, 2>), dim3((unsigned)fix), dim3(kBlock), 0, s, a.j);
  if (after_mixed) hipEventRecord(after_mixed, s);
  hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(kScanBlock), 0, s, a.chunk_pairs, a.j.group_cand, nc,
                     a.chunk_off, a.j.counters);
  launch_emit<IS>(a, nc, s);
}

hipError_t launch_split(int is, const SplitArgs& a, hipStream_t s, hipEvent_t after_classify, hipEvent_t after_mixed) {
  if (a.j.n <= 0) return hipSuccess;
  if (is == MGPU_H3)
    launch_split_t<MGPU_H3>(a, s, after_classify, after_mixed);
  else
    launch_split_t<MGPU_BNG>(a, s, after_classify, after_mixed);
  return hipGetLastError();
}

// the split pipeline's override pass (launch_join_redo): R.list = the chunks, n of them
hipError_t launch_split_redo(int is, const SplitArgs& sa, const RedoArgs& R, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t nc = split_chunks(sa.j.n);
  hipLaunchKernelGGL(chunk_unpair_kernel, dim3((unsigned)n), dim3(256), 0, s, sa.j, R);
  const int64_t most = n * kChunkTiles;
  const unsigned fix = (unsigned)(most < kFixGrid ? most : kFixGrid);
  if (is == MGPU_H3)
    hipLaunchKernelGGL((pip_mixed_fix_kernel<MGPU_H3, 2>), dim3(fix), dim3(kBlock), 0, s, sa.j);
  else
    hipLaunchKernelGGL((pip_mixed_fix_kernel<MGPU_BNG, 2>), dim3(fix), dim3(kBlock), 0, s, sa.j);
  hipLaunchKernelGGL(redo_compare_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                     (const uint32_t*)sa.chunk_pairs, R, n);
  hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(kScanBlock), 0, s, sa.chunk_pairs, sa.j.group_cand, nc,
                     sa.chunk_off, sa.j.counters, (const uint32_t*)R.changed);
  SplitArgs sr = sa;
  sr.redo_first = R.first;
  sr.redo_affected = R.affected;
  if (is == MGPU_H3)
    launch_emit<MGPU_H3>(sr, nc, s);
  else
    launch_emit<MGPU_BNG>(sr, nc, s);
  return hipGetLastError();
}

// only the ordered output of a split join already computed (mgpu_pip_join_fetch)
hipError_t launch_split_emit(int is, const SplitArgs& a, hipStream_t s) {
  if (a.j.n <= 0) return hipSuccess;
  const int64_t nc = split_chunks(a.j.n);
  if (is == MGPU_H3)
    launch_emit<MGPU_H3>(a, nc, s);
  else
    launch_emit<MGPU_BNG>(a, nc, s);
  return hipGetLastError();
}

int64_t bin_chunk() { return kBinChunk; }
int64_t bin_chunks(int64_t n) { return (n + kBinChunk - 1) / kBinChunk; }
int64_t bin_groups(int64_t n) { return (bin_chunks(n) + kBinGroup - 1) / kBinGroup; }
int32_t bin_max() { return kBinMax; }

// the binned answers -> ordered pairs: fused (one resident-grid pass with a look-back) or
// gather, scan, emit
// (A/B r5, profiles/r5/ab_c3_fused_output.txt: the three in one resident-grid pass with
// a decoupled look-back over the chunks took 11.1 ms instead of 1.0 on C3 -- a chunk's
// look-back walks back through the whole grid's round one dependent load at a time)
static void launch_bin_output(const BinArgs& a, hipStream_t s) {
  const int64_t n = a.s.j.n, K = bin_chunks(n), nc = split_chunks(n);
  if (!MGPU_BIN_JOIN_COUNTS)
    hipLaunchKernelGGL(bin_gather_kernel, dim3((unsigned)K), dim3(kBinBlock), 0, s, a);
  hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(kScanBlock), 0, s, a.s.chunk_pairs, a.s.j.group_cand, nc,
                     a.s.chunk_off, a.s.j.counters);
  if (MGPU_BIN_JOIN_COUNTS)
    hipLaunchKernelGGL(bin_emit_gather_kernel, dim3((unsigned)K), dim3(kBinBlock), 0, s, a);
  else
    hipLaunchKernelGGL(bin_emit_kernel, dim3((unsigned)nc), dim3(kClsBlock), 0, s, a);
}

template <int IS>
static void launch_binned_t(const BinArgs& a, hipStream_t s, hipEvent_t after_bin, hipEvent_t after_join) {
  const int64_t n = a.s.j.n, K = bin_chunks(n), G = bin_groups(n), nb = (int64_t)a.nbx * a.nby;
  hipLaunchKernelGGL(bin_hist_kernel, dim3((unsigned)K), dim3(kBinBlock), 0, s, a);
  hipLaunchKernelGGL(bin_colscan_kernel, dim3((unsigned)((nb + 255) / 256), (unsigned)G), dim3(256), 0, s, a, K);
  hipLaunchKernelGGL(bin_base_kernel, dim3(1), dim3(kBaseBlock), 0, s, a, G);
  if (IS == MGPU_H3 && a.key) {
    hipLaunchKernelGGL(bin_scatter_kernel<true>, dim3((unsigned)K), dim3(kBinBlock), 0, s, a);
  } else {
    // (a resident grid prefetching its next chunk's points behind the current one's
    // ranking measured 1.80 vs 1.75 ms on C3: profiles/r5/ab_c3_scatter_pf.txt)
    hipLaunchKernelGGL(bin_scatter_kernel<false>, dim3((unsigned)K), dim3(kBinBlock), 0, s, a);
  }
  const int64_t nc = split_chunks(n), tiles = nc * kChunkTiles;
  JoinArgs j = a.s.j;
  if (MGPU_BIN_JOIN_COUNTS) {  // the join counts each input chunk's pairs (the emit's offsets)
    hipMemsetAsync(a.s.chunk_pairs, 0, (size_t)nc * sizeof(uint32_t), s);
    j.in_chunk_pairs = a.s.chunk_pairs;
  }
  if (after_bin) hipEventRecord(after_bin, s);
  const uint32_t per = a.xcd_runs ? (uint32_t)((tiles + 7) / 8) : 0u;
  const int64_t grid = per ? 8 * (int64_t)per : tiles;
  hipLaunchKernelGGL(pip_binned_kernel<IS>, dim3((unsigned)grid), dim3(kBlock), 0, s, j, per, (uint32_t)tiles);
  if (after_join) hipEventRecord(after_join, s);
  const int64_t fix = tiles < kFixGrid ? tiles : kFixGrid;
  hipLaunchKernelGGL((pip_mixed_fix_kernel<IS, 1>), dim3((unsigned)fix), dim3(kBlock), 0, s, j);
  launch_bin_output(a, s);
}

hipError_t launch_binned(int is, const BinArgs& a, hipStream_t s, hipEvent_t after_bin, hipEvent_t after_join) {
  if (a.s.j.n <= 0) return hipSuccess;
  if (a.nbx < 1 || a.nby < 1 || (int64_t)a.nbx * a.nby > kBinMax) return hipErrorInvalidValue;
  if (is == MGPU_H3)
    launch_binned_t<MGPU_H3>(a, s, after_bin, after_join);
  else
    launch_binned_t<MGPU_BNG>(a, s, after_bin, after_join);
  return hipGetLastError();
}

// only the ordered output of a binned join already computed (mgpu_pip_join_fetch)
hipError_t launch_bin_emit(const BinArgs& a, hipStream_t s) {
  if (a.s.j.n <= 0) return hipSuccess;
  if (MGPU_BIN_JOIN_COUNTS)
    hipLaunchKernelGGL(bin_emit_gather_kernel, dim3((unsigned)bin_chunks(a.s.j.n)), dim3(kBinBlock), 0, s, a);
  else
    hipLaunchKernelGGL(bin_emit_kernel, dim3((unsigned)split_chunks(a.s.j.n)), dim3(kClsBlock), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_emit(const EmitArgs& e, int64_t n_tiles, hipStream_t s) {
  if (n_tiles <= 0) return hipSuccess;
  hipLaunchKernelGGL(pair_emit_kernel, dim3((unsigned)((n_tiles + kEmitTiles - 1) / kEmitTiles)), dim3(kEmitBlock), 0, s, e,
                     n_tiles);
  return hipGetLastError();
}

hipError_t launch_st_contains(const ChipTableView& t, const int64_t* row, const double* x, const double* y, int64_t n,
                              int8_t* out, unsigned long long* counters, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(st_contains_kernel, dim3((unsigned)((n + kStreamBlock - 1) / kStreamBlock)), dim3(kStreamBlock), 0, s, t, row, x,
                     y, n, out, counters);
  return hipGetLastError();
}

}  // namespace mgpu
