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

template <int IS>
__device__ __forceinline__ bool cell_of(double x, double y, int res, uint64_t* cell, bool* tie) {
  if (IS == MGPU_H3) {
    uint64_t c = h3::point_to_cell(x, y, res, tie);
    *cell = c;
    return c != 0;
  } else {
    int64_t c;
    *tie = false;
    bool ok = bng::point_to_cell(x, y, res, &c);
    *cell = (uint64_t)c;
    return ok;
  }
}

// probe the cell hash; returns the chip range [first, first + count)
__device__ __forceinline__ uint2 probe(const ChipTableView& t, uint64_t cell) {
  uint32_t h = cell_hash(cell) & t.hash_mask;
  for (uint32_t k = 0; k <= t.max_probe; k++) {
    HashSlot s = t.slots[h];
    if (s.count == 0) break;
    if (s.cell == cell) return make_uint2(s.first, s.count);
    h = (h + 1) & t.hash_mask;
  }
  return make_uint2(0, 0);
}

__device__ __forceinline__ void count_wave(unsigned long long* ctr, bool pred) {
  unsigned long long b = __ballot(pred);
  if (b && (threadIdx.x & 63) == (__ffsll((long long)b) - 1)) atomicAdd(ctr, (unsigned long long)__popcll(b));
}

template <int IS>
__global__ __launch_bounds__(kBlock) void cells_kernel(const double* __restrict__ x, const double* __restrict__ y,
                                                       int64_t n, int res, int64_t* __restrict__ out,
                                                       unsigned long long* __restrict__ counters) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    uint64_t c = 0;
    bool tie = false;
    bool ok = cell_of<IS>(x[i], y[i], res, &c, &tie);
    out[i] = (int64_t)c;
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

template <int IS>
__global__ __launch_bounds__(kBlock) void pip_join_kernel(JoinArgs a) {
  __shared__ uint32_t s_tile;
  __shared__ uint32_t s_wave_tot[kBlock / 64];
  __shared__ unsigned long long s_prefix;

  if (threadIdx.x == 0) s_tile = atomicAdd(a.tile_ticket, 1u);
  __syncthreads();
  const uint32_t tile = s_tile;
  const ChipTableView& t = a.chips;
  const int64_t p0 = (int64_t)tile * kTile + (int64_t)threadIdx.x * kItems;

  int cnt[kItems];
  int32_t keep[kItems][kKeep];
  uint32_t mine = 0, cand = 0;
  bool any_tie = false, any_bad = false;

#pragma unroll
  for (int k = 0; k < kItems; k++) {
    cnt[k] = 0;
    const int64_t p = p0 + k;
    if (p >= a.n) continue;
    const double px = a.x[p], py = a.y[p];
    uint64_t cell;
    bool tie;
    if (!cell_of<IS>(px, py, a.res, &cell, &tie)) {
      any_bad = true;
      continue;
    }
    any_tie |= tie;
    uint2 r = probe(t, cell);
    for (uint32_t c = r.x; c < r.x + r.y; c++) {
      bool m = (t.chip_flags[c] & kChipCore) != 0;
      if (!m) {
        cand++;
        m = pip::chip_locate(t, c, px, py) == pip::kInterior;
      }
      if (m) {
        if (cnt[k] < kKeep) keep[k][cnt[k]] = t.chip_poly[c];
        cnt[k]++;
      }
    }
    mine += cnt[k];
  }
  count_wave(&a.counters[1], any_tie);
  count_wave(&a.counters[2], any_bad);
  {
    unsigned long long cs = wave_sum_u64(cand);
    if ((threadIdx.x & 63) == 0 && cs) atomicAdd(&a.counters[3], cs);
  }

  // ---- block exclusive scan of per-lane match counts (lane order == point order)
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

  // ---- decoupled look-back (wave 0): status word = {2-bit flag, 62-bit count}
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
        uint64_t s = idx >= 0 ? __hip_atomic_load(&a.tile_status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                              : kFlagPrefix;
        const uint32_t flag = (uint32_t)(s >> 62);
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
        unsigned long long v = (lane <= first) ? (s & kValueMask) : 0ull;
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

  // ---- write this lane's pairs at their global positions
  int64_t pos = (int64_t)s_prefix + excl;
#pragma unroll
  for (int k = 0; k < kItems; k++) {
    if (cnt[k] == 0) continue;
    const int64_t p = p0 + k;
    const int64_t pid = a.point_id ? a.point_id[p] : a.id_base + p;
    if (cnt[k] <= kKeep) {
      for (int q = 0; q < cnt[k]; q++) {
        if (pos + q < a.capacity) {
          a.out_point[pos + q] = pid;
          a.out_poly[pos + q] = keep[k][q];
        }
      }
    } else {
      // more matches than kept: re-evaluate this point's chips in order
      const double px = a.x[p], py = a.y[p];
      uint64_t cell;
      bool tie;
      cell_of<IS>(px, py, a.res, &cell, &tie);
      uint2 r = probe(t, cell);
      int q = 0;
      for (uint32_t c = r.x; c < r.x + r.y; c++) {
        bool m = (t.chip_flags[c] & kChipCore) != 0;
        if (!m) m = pip::chip_locate(t, c, px, py) == pip::kInterior;
        if (m) {
          if (pos + q < a.capacity) {
            a.out_point[pos + q] = pid;
            a.out_poly[pos + q] = t.chip_poly[c];
          }
          q++;
        }
      }
    }
    pos += cnt[k];
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
