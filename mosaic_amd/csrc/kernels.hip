// gfx950 kernels of the grid-indexed point-in-polygon join.
//
//   cells_kernel<IS>     IndexSystem.pointToIndex over a batch (H3 / BNG)
//   pip_join_kernel<IS>  fused: cell id -> chip-table probe -> is_core OR
//                        st_contains -> ordered (point_id, polygon_id) output
//   st_contains_kernel   st_contains(chip.wkb, point) for explicit pairs
//
// Design (DESIGN.md has the roofline analysis): the hot path is one pass over the
// points.  Each 256-thread workgroup owns a tile of 1024 consecutive points (4 per
// lane, loaded as 32 contiguous bytes per lane per coordinate).  The chip table's
// cell hash (16 B slots) and the border-chip vertex runs are small and read-only;
// they stay in L2 / Infinity Cache while the point stream flows from HBM.  Output
// positions come from a single-pass decoupled look-back scan over tiles (tile
// ids taken from an atomic ticket, so every predecessor tile is already running),
// which keeps the output ordered by input position without a second pass or a
// sort.  Nothing here is a dense contraction, so MFMA is not used.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define H3T_QUAL static __constant__ const
#include "h3_core.h"
#include "bng_core.h"
#include "pip_core.h"
#include "kernels.h"

namespace mgpu {

constexpr int kBlock = 256;
constexpr int kItems = 4;
constexpr int kTile = kBlock * kItems;
constexpr int kKeep = 2;  // matches per point kept in registers between the passes

constexpr uint64_t kFlagAgg = 1ULL << 62;
constexpr uint64_t kFlagPrefix = 2ULL << 62;
constexpr uint64_t kValueMask = (1ULL << 62) - 1;
constexpr uint32_t kSpinLimit = 1u << 22;

// ---------------------------------------------------------------- point -> cell

constexpr uint32_t kAllFaces = (1u << 20) - 1;

// H3IndexSystem.pointToIndex: fast closed-form projection, H3 route on near-ties
__device__ __forceinline__ uint64_t h3_cell(double lon_deg, double lat_deg, int res, double k_res, bool* ok,
                                           bool* tie) {
  const double lat = h3::to_radians(lat_deg), lon = h3::to_radians(lon_deg);
  *tie = false;
  if (!isfinite(lat) || !isfinite(lon)) {
    *ok = false;
    return 0;
  }
  *ok = true;
  h3::FastHex f = h3::fast_hex2d(lat, lon, res, k_res, kAllFaces);
  if (f.tie) {
    h3::route_face_ijk(lat, lon, res, &f.face, &f.ijk, tie);
  }
  return h3::face_ijk_to_h3(f.face, f.ijk, res);
}

// probe the hash with `key`; returns the chip range [first, first + count)
__device__ __forceinline__ uint2 probe(const ChipTableView& t, uint64_t key) {
  uint32_t h = cell_hash(key) & t.hash_mask;
  for (uint32_t k = 0; k <= t.max_probe; k++) {
    HashSlot s = t.slots[h];
    if (s.count == 0) break;
    if (s.cell == key) return make_uint2(s.first, s.count);
    h = (h + 1) & t.hash_mask;
  }
  return make_uint2(0, 0);
}

// The chips of the point's cell.  *ok = false for invalid coordinates (NaN), *tie
// when the H3 route itself sits in its near-tie band (reported).
template <int IS>
__device__ __forceinline__ uint2 chips_of(const ChipTableView& t, double px, double py, int res, bool res_match,
                                          bool* ok, bool* tie) {
  *tie = false;
  if (IS == MGPU_BNG) {
    int64_t c;
    *ok = bng::point_to_cell(px, py, res, &c);
    if (!*ok || !res_match) return make_uint2(0, 0);
    return probe(t, (uint64_t)c);
  }
  const double lat = h3::to_radians(py), lon = h3::to_radians(px);
  if (!isfinite(lat) || !isfinite(lon)) {
    *ok = false;
    return make_uint2(0, 0);
  }
  *ok = true;
  if (!res_match) return make_uint2(0, 0);
  if (t.probe_mode == kProbeLattice) {
    // outside the chip cells' bounding box no cell can match
    if (!(px >= t.bbox[0] && px <= t.bbox[2] && py >= t.bbox[1] && py <= t.bbox[3])) return make_uint2(0, 0);
    h3::FastHex f = h3::fast_hex2d(lat, lon, res, t.k_res, t.face_mask);
    if (f.tie) h3::route_face_ijk(lat, lon, res, &f.face, &f.ijk, tie);
    return probe(t, h3::lattice_key(f.face, f.ijk));
  }
  h3::FastHex f = h3::fast_hex2d(lat, lon, res, t.k_res > 0 ? t.k_res : h3::k_of_res(res), kAllFaces);
  if (f.tie) h3::route_face_ijk(lat, lon, res, &f.face, &f.ijk, tie);
  return probe(t, h3::face_ijk_to_h3(f.face, f.ijk, res));
}

__device__ __forceinline__ void count_wave(unsigned long long* ctr, bool pred) {
  unsigned long long b = __ballot(pred);
  if (b && (threadIdx.x & 63) == (__ffsll((long long)b) - 1)) atomicAdd(ctr, (unsigned long long)__popcll(b));
}

template <int IS>
__global__ __launch_bounds__(kBlock) void cells_kernel(const double* __restrict__ x, const double* __restrict__ y,
                                                       int64_t n, int res, int64_t* __restrict__ out,
                                                       unsigned long long* __restrict__ counters) {
  const double k_res = h3::k_of_res(res);
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    bool ok, tie = false;
    int64_t c = 0;
    if (IS == MGPU_H3) {
      c = (int64_t)h3_cell(x[i], y[i], res, k_res, &ok, &tie);
    } else {
      ok = bng::point_to_cell(x[i], y[i], res, &c);
    }
    out[i] = c;
    count_wave(&counters[1], tie);
    count_wave(&counters[2], !ok);
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

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// One workgroup = one tile of kTile consecutive points, in six phases:
//  1  lane l evaluates points l, l+256, l+512, l+768 (coalesced 8-byte loads): cell
//     -> chip range; every border chip of the point is appended to the tile's
//     candidate list (LDS);
//  2  per candidate: chip envelope / rectangle shortcuts, else one "ring entry" per
//     ring of the chip (edge count, or skipped when the ring envelope misses);
//  3  exclusive scan of the ring entries' edge counts;
//  4  edge-parallel ray crossing: every lane tests one (candidate, edge) pair per
//     step -- no divergence on ring length, consecutive lanes read consecutive
//     vertices -- and ORs / XORs its result bits into the ring entry (LDS atomics);
//  5  per candidate: PointLocator over its rings' bits -> contains?;
//  6  lane l owns points 4l .. 4l+3 (input order): count matches (chip order ==
//     polygon-id order), block scan + decoupled look-back over tiles, write pairs.
// Tiles whose candidates or ring entries overflow the LDS lists evaluate the
// overflowing points with the sequential PointLocator (pip::chip_locate).
constexpr int kCandCap = 1536;
constexpr int kRingCap = 1536;
constexpr uint16_t kNoCand = 0xFFFF;
constexpr uint32_t kNoChip = 0xFFFFFFFFu;
enum CandRes : uint8_t { kResExterior = 0, kResInterior = 1, kResPending = 2, kResSequential = 3 };

__device__ __forceinline__ int64_t tile_point(const JoinArgs& a, int64_t base, int li) { return base + li; }

template <int IS>
__global__ __launch_bounds__(kBlock) void pip_join_kernel(JoinArgs a) {
  __shared__ uint32_t s_tile, s_ncand, s_nring, s_nedge;
  __shared__ uint32_t s_wave_tot[kBlock / 64];
  __shared__ unsigned long long s_prefix;
  __shared__ uint2 s_range[kTile];               // chip range of each point
  __shared__ uint16_t s_pfirst[kTile];           // first candidate of each point (kNoCand: sequential)
  __shared__ uint32_t s_cand_chip[kCandCap];
  __shared__ uint16_t s_cand_pt[kCandCap];
  __shared__ uint16_t s_cand_ring[kCandCap];     // first ring entry of the candidate
  __shared__ uint8_t s_cand_res[kCandCap];
  __shared__ uint32_t s_ring_id[kRingCap];       // global ring index
  __shared__ uint32_t s_ring_pref[kRingCap + 1]; // edge counts, then their exclusive scan
  __shared__ uint32_t s_ring_bits[kRingCap];
  __shared__ uint16_t s_ring_cand[kRingCap];

  if (threadIdx.x == 0) {
    s_tile = atomicAdd(a.tile_ticket, 1u);
    s_ncand = 0;
    s_nring = 0;
  }
  __syncthreads();
  const uint32_t tile = s_tile;
  const ChipTableView& t = a.chips;
  const int64_t base = (int64_t)tile * kTile;
  const bool res_match = a.res_match;

  // ---- phase 1: cells and candidates
  bool any_tie = false, any_bad = false;
#pragma unroll 1
  for (int k = 0; k < kItems; k++) {
    const int li = k * kBlock + threadIdx.x;
    const int64_t p = base + li;
    uint2 r = make_uint2(0, 0);
    uint16_t first = 0;
    if (p < a.n) {
      bool ok, tie;
      r = chips_of<IS>(t, a.x[p], a.y[p], a.res, res_match, &ok, &tie);
      if (a.ablate == 2) r = make_uint2(0, 0);
      any_bad |= !ok;
      any_tie |= tie;
      uint32_t nb = 0;
      for (uint32_t c = r.x; c < r.x + r.y; c++) nb += (t.chip_flags[c] & kChipCore) ? 0 : 1;
      if (nb) {
        uint32_t c0 = atomicAdd(&s_ncand, nb);
        if (c0 + nb <= (uint32_t)kCandCap) {
          first = (uint16_t)c0;
          uint32_t j = c0;
          for (uint32_t c = r.x; c < r.x + r.y; c++) {
            if (t.chip_flags[c] & kChipCore) continue;
            s_cand_chip[j] = c;
            s_cand_pt[j] = (uint16_t)li;
            j++;
          }
        } else {
          first = kNoCand;
          // the part of the reservation inside the list must still be defined
          for (uint32_t j = c0; j < c0 + nb && j < (uint32_t)kCandCap; j++) s_cand_chip[j] = kNoChip;
        }
      }
    }
    s_range[li] = r;
    s_pfirst[li] = first;
  }
  count_wave(&a.counters[1], any_tie);
  count_wave(&a.counters[2], any_bad);
  __syncthreads();
  const uint32_t ncand = s_ncand < (uint32_t)kCandCap ? s_ncand : (uint32_t)kCandCap;
  if (threadIdx.x == 0 && ncand) atomicAdd(&a.counters[3], (unsigned long long)ncand);

  // ---- phase 2: per candidate, shortcuts or ring entries
  for (uint32_t c = threadIdx.x; c < ncand; c += kBlock) {
    const uint32_t ch = s_cand_chip[c];
    if (ch == kNoChip) continue;  // slot of an overflowed reservation (never read back)
    const int64_t p = base + s_cand_pt[c];
    const double px = a.x[p], py = a.y[p];
    const uint8_t fl = t.chip_flags[ch];
    uint8_t res = kResExterior;
    if (a.ablate == 1 || (fl & (kChipEmpty | kChipNoGeom))) {
      res = kResExterior;
    } else if (!pip::env_has(t.chip_env + 4 * ch, px, py)) {
      res = kResExterior;
    } else if (fl & kChipRect) {
      const double* e = t.chip_env + 4 * ch;
      res = (px == e[0] || px == e[2] || py == e[1] || py == e[3]) ? kResExterior : kResInterior;
    } else {
      const uint32_t rb = t.part_ring[t.chip_part[ch]], re = t.part_ring[t.chip_part[ch + 1]];
      const uint32_t nr = re - rb;
      const uint32_t r0 = atomicAdd(&s_nring, nr);
      if (r0 + nr <= (uint32_t)kRingCap) {
        res = kResPending;
        s_cand_ring[c] = (uint16_t)r0;
        for (uint32_t q = 0; q < nr; q++) {
          const uint32_t ring = rb + q;
          const uint32_t vb = t.ring_vtx[ring], ve = t.ring_vtx[ring + 1];
          const bool use = ve - vb >= 2 && pip::env_has(t.ring_env + 4 * ring, px, py);
          s_ring_id[r0 + q] = ring;
          s_ring_pref[r0 + q] = use ? ve - vb - 1 : 0;
          s_ring_bits[r0 + q] = use ? 0u : (uint32_t)pip::kRingSkipped;
          s_ring_cand[r0 + q] = (uint16_t)c;
        }
      } else {
        res = kResSequential;
        for (uint32_t q = r0; q < r0 + nr && q < (uint32_t)kRingCap; q++) {
          s_ring_id[q] = rb;
          s_ring_pref[q] = 0;
          s_ring_bits[q] = (uint32_t)pip::kRingSkipped;
          s_ring_cand[q] = (uint16_t)c;
        }
      }
    }
    s_cand_res[c] = res;
  }
  __syncthreads();

  // ---- phase 3: exclusive scan of the ring entries' edge counts (one wave)
  const uint32_t nring = s_nring < (uint32_t)kRingCap ? s_nring : (uint32_t)kRingCap;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    uint32_t carry = 0;
    for (uint32_t b0 = 0; b0 < nring; b0 += 64) {
      const uint32_t i = b0 + lane;
      const uint32_t v = i < nring ? s_ring_pref[i] : 0;
      const uint32_t inc = wave_incl_scan(v);
      if (i < nring) s_ring_pref[i] = carry + inc - v;
      carry += __shfl(inc, 63, 64);
    }
    if (lane == 0) {
      s_ring_pref[nring] = carry;
      s_nedge = carry;
    }
  }
  __syncthreads();

  // ---- phase 4: edge-parallel ray crossing
  const uint32_t nedge = s_nedge;
  for (uint32_t f = threadIdx.x; f < nedge; f += kBlock) {
    uint32_t lo = 0, hi = nring;  // last entry with pref <= f
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (s_ring_pref[mid] <= f) lo = mid; else hi = mid;
    }
    const uint32_t ring = s_ring_id[lo];
    const uint32_t i = t.ring_vtx[ring] + 1 + (f - s_ring_pref[lo]);
    const int64_t p = base + s_cand_pt[s_ring_cand[lo]];
    const double px = a.x[p], py = a.y[p];
    const double* v = t.vtx + 2 * (size_t)i;
    const int bits = pip::count_segment(v[0], v[1], v[-2], v[-1], px, py);
    if (bits & pip::kRingOnSegment) atomicOr(&s_ring_bits[lo], (uint32_t)pip::kRingOnSegment);
    if (bits & 2) atomicXor(&s_ring_bits[lo], (uint32_t)pip::kRingParity);
  }
  __syncthreads();

  // ---- phase 5: PointLocator per pending candidate
  for (uint32_t c = threadIdx.x; c < ncand; c += kBlock) {
    if (s_cand_res[c] != kResPending) continue;
    const int loc = pip::chip_locate_from_rings(t, s_cand_chip[c], &s_ring_bits[s_cand_ring[c]]);
    s_cand_res[c] = loc == pip::kInterior ? kResInterior : kResExterior;
  }
  __syncthreads();

  // ---- phase 6: lane l owns points 4l .. 4l+3 (input order)
  const int l0 = threadIdx.x * kItems;
  uint32_t mine = 0;
#pragma unroll 1
  for (int k = 0; k < kItems; k++) {
    const int li = l0 + k;
    const uint2 r = s_range[li];
    if (!r.y) continue;
    uint32_t cj = s_pfirst[li];
    const int64_t p = base + li;
    for (uint32_t q = r.x; q < r.x + r.y; q++) {
      bool m;
      if (t.chip_flags[q] & kChipCore) {
        m = true;
      } else {
        const uint8_t res = cj != kNoCand ? s_cand_res[cj++] : kResSequential;
        m = res == kResInterior ||
            (res == kResSequential && a.ablate != 1 && pip::chip_locate(t, q, a.x[p], a.y[p]) == pip::kInterior);
      }
      mine += m ? 1 : 0;
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

  // decoupled look-back (wave 0): status word = {2-bit flag, 62-bit count}
  if (wave == 0) {
    unsigned long long prefix = 0;
    if (tile == 0) {
      if (lane == 0) __hip_atomic_store(&a.tile_status[0], kFlagPrefix | (uint64_t)agg, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane == 0) __hip_atomic_store(&a.tile_status[tile], kFlagAgg | (uint64_t)agg, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
      int64_t top = (int64_t)tile - 1;
      uint32_t spins = 0;
      while (true) {
        const int64_t idx = top - lane;
        uint64_t st = idx >= 0 ? __hip_atomic_load(&a.tile_status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                               : kFlagPrefix;
        const uint32_t flag = (uint32_t)(st >> 62);
        if (__any(flag == 0)) {
          if (++spins > kSpinLimit) {
            if (lane == 0) atomicAdd(&a.counters[4], 1ull);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        const unsigned long long pb = __ballot(flag == 2);
        const int first = pb ? (__ffsll((long long)pb) - 1) : 64;
        unsigned long long v = (lane <= first) ? (st & kValueMask) : 0ull;
        prefix += wave_sum_u64(v);
        if (pb) break;
        top -= 64;
      }
      if (lane == 0)
        __hip_atomic_store(&a.tile_status[tile], kFlagPrefix | (uint64_t)(prefix + agg), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) {
      s_prefix = prefix;
      if (tile == a.n_tiles - 1) a.counters[0] = prefix + agg;
    }
  }
  __syncthreads();

  int64_t pos = (int64_t)s_prefix + excl;
#pragma unroll 1
  for (int k = 0; k < kItems; k++) {
    const int li = l0 + k;
    const uint2 r = s_range[li];
    if (!r.y) continue;
    uint32_t cj = s_pfirst[li];
    const int64_t p = base + li;
    const int64_t pid = a.point_id ? a.point_id[p] : a.id_base + p;
    for (uint32_t q = r.x; q < r.x + r.y; q++) {
      bool m;
      if (t.chip_flags[q] & kChipCore) {
        m = true;
      } else {
        const uint8_t res = cj != kNoCand ? s_cand_res[cj++] : kResSequential;
        m = res == kResInterior ||
            (res == kResSequential && a.ablate != 1 && pip::chip_locate(t, q, a.x[p], a.y[p]) == pip::kInterior);
      }
      if (m) {
        if (pos < a.capacity) {
          a.out_point[pos] = pid;
          a.out_poly[pos] = t.chip_poly[q];
        }
        pos++;
      }
    }
  }
}

__global__ __launch_bounds__(kBlock) void st_contains_kernel(ChipTableView t, const int64_t* __restrict__ row,
                                                             const double* __restrict__ x,
                                                             const double* __restrict__ y, int64_t n,
                                                             int8_t* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int64_t r = row[i];
  if (r < 0 || r >= (int64_t)t.n_chips) {
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

// ---------------------------------------------------------------- launchers

hipError_t launch_cells(int is, int res, const double* x, const double* y, int64_t n, int64_t* out,
                        unsigned long long* counters, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  int64_t blocks = (n + kBlock - 1) / kBlock;
  if (blocks > 256 * 64) blocks = 256 * 64;
  if (is == MGPU_H3)
    hipLaunchKernelGGL(cells_kernel<MGPU_H3>, dim3((unsigned)blocks), dim3(kBlock), 0, s, x, y, n, res, out, counters);
  else
    hipLaunchKernelGGL(cells_kernel<MGPU_BNG>, dim3((unsigned)blocks), dim3(kBlock), 0, s, x, y, n, res, out, counters);
  return hipGetLastError();
}

int64_t join_tiles(int64_t n) { return (n + kTile - 1) / kTile; }

hipError_t launch_join(int is, const JoinArgs& a, hipStream_t s) {
  if (a.n_tiles <= 0) return hipSuccess;
  if (is == MGPU_H3)
    hipLaunchKernelGGL(pip_join_kernel<MGPU_H3>, dim3((unsigned)a.n_tiles), dim3(kBlock), 0, s, a);
  else
    hipLaunchKernelGGL(pip_join_kernel<MGPU_BNG>, dim3((unsigned)a.n_tiles), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_st_contains(const ChipTableView& t, const int64_t* row, const double* x, const double* y, int64_t n,
                              int8_t* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(st_contains_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, t, row, x,
                     y, n, out);
  return hipGetLastError();
}

}  // namespace mgpu
