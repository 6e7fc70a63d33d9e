// The grid-ring neighbour join of SpatialKNN (models/knn/GridRingNeighbours.scala,
// SpatialKNN.scala) for point landmarks and point candidates, one iteration on the GPU.
//
// Reference, one iteration (GridRingNeighbours.transform, :121, and resultTransform):
//   left  = the landmark's cells: iteration 1 grid_geometrykringexplode(geom, res, 1) --
//           for a point, kRing(pointToIndex(point), 1) (Mosaic.geometryKRing,
//           core/Mosaic.scala:123-128: a point is one border chip); iteration k > 1
//           grid_geometrykloopexplode(geom, res, k) -- kLoop(cell, k) minus kRing(cell,
//           k - 1), i.e. kLoop(cell, k) (Mosaic.geometryKLoop :142-156)
//   right = the candidates' chips, grid_tessellateexplode(keepCoreGeometries = false)
//           (SpatialKNN.transform :~160): for a point one chip at pointToIndex(point)
//           (Mosaic.pointChip :48-59)
//   join  = left cell == right chip index_id; st_intersects_agg is true for a left chip
//           wrapped with isCore = true (ST_IntersectsAgg.update), so every (landmark,
//           candidate) sharing a cell is a pair, once; distance = st_distance (JTS
//           Coordinate.distance, Math.hypot); self matches (the same geometry) dropped;
//           neighbour_number = row_number over (landmark, distance ascending);
//           SpatialKNN keeps neighbour_number <= kNeighbours and distance <= threshold.
// Here: cells of both sides by mgpu_points_to_cells (the reference's cells, near-ties
// included), ring lists by mgpu_grid_kring (H3's pentagon handling included), the
// candidates in an open-addressing hash of their cells (each slot heads a list of its
// candidates), one thread per landmark probing its ring cells; pairs per landmark
// ordered by (distance, candidate index) -- the reference's window leaves distance ties
// unordered; this order is the oracle's.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <unordered_set>
#include <vector>

#include "capi_internal.h"
#include "geom_decode.h"

namespace {

#define RJ_TRY(expr)                                                                                     \
  do {                                                                                                   \
    hipError_t _e = (expr);                                                                              \
    if (_e != hipSuccess) return mgpu::set_error(MGPU_E_DEVICE, "%s: %s", #expr, hipGetErrorString(_e)); \
  } while (0)

struct RjArgs {
  const double *lx, *ly, *rx, *ry;
  const int64_t* ring;        // ring cells of every landmark, [ring_off[i], ring_off[i + 1])
  const int64_t* ring_off;    // [n_left + 1]
  const uint64_t* slot_cell;  // candidate-cell hash: the cell (0: empty slot)
  const int64_t* slot_head;   // its first candidate (a list through next[])
  const int64_t* next;        // [n_right] the next candidate of the same cell (-1: end)
  uint64_t mask;              // slots - 1
  int64_t n_left;
  double max_dist;            // < 0: no threshold
};

__device__ __forceinline__ uint64_t rj_hash(uint64_t c) {
  c ^= c >> 33;
  c *= 0xff51afd7ed558ccdULL;
  c ^= c >> 33;
  return c;
}

// the candidates into the hash: slot of the cell (claimed by CAS), candidate pushed on its
// list (the list order does not matter: segments are sorted afterwards)
__global__ __launch_bounds__(256) void rj_insert_kernel(const int64_t* __restrict__ rc, int64_t n, uint64_t* slot_cell,
                                                        unsigned long long* slot_head, int64_t* __restrict__ next,
                                                        uint64_t mask) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint64_t c = (uint64_t)rc[j];
  uint64_t h = rj_hash(c) & mask;
  for (;;) {
    const unsigned long long prev = atomicCAS((unsigned long long*)&slot_cell[h], 0ull, (unsigned long long)c);
    if (prev == 0ull || prev == c) break;
    h = (h + 1) & mask;
  }
  next[j] = (int64_t)atomicExch(&slot_head[h], (unsigned long long)j);
}

__device__ __forceinline__ bool same_bits(double a, double b) {
  return __double_as_longlong(a) == __double_as_longlong(b);
}

// per landmark: the candidates sharing one of its ring cells, minus itself (the same
// coordinates: the reference's hash of the same geometry), within the threshold --
// counted (WRITE = false) or written from off[i] (WRITE = true)
// (WRITE = false also flags, in nul[i], a landmark with a ring cell holding no candidate:
// the left_outer join's null row, GridRingNeighbours.scala:128,151)
template <bool WRITE>
__global__ __launch_bounds__(256) void rj_pairs_kernel(RjArgs a, int64_t* __restrict__ cnt, const int64_t* __restrict__ off,
                                                      int64_t* __restrict__ out_right, double* __restrict__ out_dist,
                                                      int8_t* __restrict__ nul) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n_left) return;
  const double px = a.lx[i], py = a.ly[i];
  int64_t m = 0, q = WRITE ? off[i] : 0;
  bool empty_cell = false;
  for (int64_t r = a.ring_off[i]; r < a.ring_off[i + 1]; r++) {
    const uint64_t c = (uint64_t)a.ring[r];
    uint64_t h = rj_hash(c) & a.mask;
    while (a.slot_cell[h] != 0 && a.slot_cell[h] != c) h = (h + 1) & a.mask;
    if (a.slot_cell[h] != c) {
      empty_cell = true;
      continue;
    }
    for (int64_t k = a.slot_head[h]; k >= 0; k = a.next[k]) {
      const double qx = a.rx[k], qy = a.ry[k];
      if (same_bits(px, qx) && same_bits(py, qy)) continue;
      const double d = mgpu::geom::jhypot(px - qx, py - qy);
      if (a.max_dist >= 0.0 && !(d <= a.max_dist)) continue;
      if (WRITE) {
        out_right[q] = k;
        out_dist[q] = d;
        q++;
      }
      m++;
    }
  }
  if (!WRITE) {
    cnt[i] = m;
    nul[i] = empty_cell ? 1 : 0;
  }
}

__device__ __forceinline__ bool rj_less(double da, int64_t ia, double db, int64_t ib) {
  return da < db || (da == db && ia < ib);
}

// each landmark's segment in (distance, candidate) order -- the first `keep` of it by
// selection when keep is small, else all of it by a Shell sort -- and its kept count
__global__ __launch_bounds__(256) void rj_sort_kernel(const int64_t* __restrict__ off, int64_t n, int64_t keep,
                                                      int64_t* __restrict__ right, double* __restrict__ dist,
                                                      int64_t* __restrict__ kept, const int8_t* __restrict__ nul) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t b = off[i], m = off[i + 1] - b;
  int64_t* R = right + b;
  double* D = dist + b;
  const int64_t want = keep > 0 && keep < m ? keep : m;
  if (keep > 0 && keep < m && keep <= 32) {
    for (int64_t r = 0; r < want; r++) {
      int64_t best = r;
      for (int64_t j = r + 1; j < m; j++)
        if (rj_less(D[j], R[j], D[best], R[best])) best = j;
      const double td = D[r];
      const int64_t tr = R[r];
      D[r] = D[best], R[r] = R[best];
      D[best] = td, R[best] = tr;
    }
  } else {
    int64_t gap = 1;
    while (gap < m / 3) gap = 3 * gap + 1;
    for (; gap > 0; gap /= 3)
      for (int64_t j = gap; j < m; j++) {
        const double td = D[j];
        const int64_t tr = R[j];
        int64_t q = j;
        while (q >= gap && rj_less(td, tr, D[q - gap], R[q - gap])) {
          D[q] = D[q - gap];
          R[q] = R[q - gap];
          q -= gap;
        }
        D[q] = td;
        R[q] = tr;
      }
  }
  if (kept) kept[i] = want + (nul ? nul[i] : 0);
}

// kept[i]: the landmark's output rows -- its pairs cut to `keep` (0: all), plus its null row
__global__ __launch_bounds__(256) void rj_kept_kernel(const int64_t* __restrict__ off, int64_t n, int64_t keep,
                                                      const int8_t* __restrict__ nul, int64_t* __restrict__ kept) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t m = off[i + 1] - off[i];
  kept[i] = (keep > 0 && keep < m ? keep : m) + (nul ? nul[i] : 0);
}

// out[i] = off[i] - base (a batch's segment offsets relative to its first pair)
__global__ __launch_bounds__(256) void rj_rebase_kernel(const int64_t* __restrict__ off, int64_t n, int64_t base,
                                                        int64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = off[i] - base;
}

// exclusive scan of v[0 .. n) into out[0 .. n] (out[n] = the total), three launches:
// per-block scans with block sums, the block sums scanned by one workgroup, added back
constexpr int kScanB = 1024;
__global__ __launch_bounds__(kScanB) void rj_scan_block_kernel(const int64_t* __restrict__ v, int64_t n,
                                                              int64_t* __restrict__ out, int64_t* __restrict__ bsum) {
  __shared__ int64_t s[kScanB];
  const int64_t i = (int64_t)blockIdx.x * kScanB + threadIdx.x;
  const int64_t x = i < n ? v[i] : 0;
  s[threadIdx.x] = x;
  __syncthreads();
  for (int d = 1; d < kScanB; d <<= 1) {
    const int64_t t = threadIdx.x >= (unsigned)d ? s[threadIdx.x - d] : 0;
    __syncthreads();
    s[threadIdx.x] += t;
    __syncthreads();
  }
  if (i < n) out[i] = s[threadIdx.x] - x;
  if (threadIdx.x == kScanB - 1) bsum[blockIdx.x] = s[kScanB - 1];
}
__global__ __launch_bounds__(kScanB) void rj_scan_sums_kernel(int64_t* __restrict__ bsum, int64_t nb) {
  __shared__ int64_t s[kScanB];
  int64_t carry = 0;
  for (int64_t b0 = 0; b0 < nb; b0 += kScanB) {
    const int64_t i = b0 + threadIdx.x;
    const int64_t x = i < nb ? bsum[i] : 0;
    s[threadIdx.x] = x;
    __syncthreads();
    for (int d = 1; d < kScanB; d <<= 1) {
      const int64_t t = threadIdx.x >= (unsigned)d ? s[threadIdx.x - d] : 0;
      __syncthreads();
      s[threadIdx.x] += t;
      __syncthreads();
    }
    if (i < nb) bsum[i] = carry + s[threadIdx.x] - x;
    const int64_t tot = s[kScanB - 1];
    __syncthreads();
    carry += tot;
  }
  if (threadIdx.x == 0) bsum[nb] = carry;
}
__global__ __launch_bounds__(kScanB) void rj_scan_add_kernel(int64_t* __restrict__ out, int64_t n,
                                                            const int64_t* __restrict__ bsum, int64_t nb) {
  const int64_t i = (int64_t)blockIdx.x * kScanB + threadIdx.x;
  if (i < n) out[i] += bsum[blockIdx.x];
  if (i == 0) out[n] = bsum[nb];
}

// the first kept[i] pairs of landmark i's sorted segment to its output range
__global__ __launch_bounds__(256) void rj_copy_kernel(const int64_t* __restrict__ off, const int64_t* __restrict__ koff,
                                                      int64_t n, const int64_t* __restrict__ right,
                                                      const double* __restrict__ dist, int64_t left_base,
                                                      int64_t capacity, int64_t* __restrict__ out_left,
                                                      int64_t* __restrict__ out_right, double* __restrict__ out_dist,
                                                      const int8_t* __restrict__ nul) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t b = off[i], e = koff[i + 1];
  int64_t o = koff[i];
  if (nul && nul[i]) {  // the null row first (Spark orders nulls first in an ascending window)
    if (o < capacity) {
      out_left[o] = left_base + i;
      out_right[o] = -1;
      out_dist[o] = __longlong_as_double(0x7FF8000000000000LL);
    }
    o++;
  }
  for (int64_t q = o; q < e && q < capacity; q++) {
    out_left[q] = left_base + i;
    out_right[q] = right[b + q - o];
    out_dist[q] = dist[b + q - o];
  }
}

unsigned grid_of(int64_t n) { return (unsigned)std::max<int64_t>(1, (n + 255) / 256); }

// device scratch freed on every return path
struct Scratch {
  std::vector<void*> ptrs;
  ~Scratch() {
    for (void* p : ptrs) (void)hipFree(p);
  }
  template <class T>
  hipError_t get(T** p, size_t count) {
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, std::max<size_t>(count, 1) * sizeof(T));
    if (e == hipSuccess) ptrs.push_back(q);
    *p = (T*)q;
    return e;
  }
};

}  // namespace

// The join proper over given landmark cell lists (device CSR ring / ring_off): the
// candidates' cells and hash, pairs, per-landmark order and cut, output.  flags:
// MGPU_RING_LEFT_OUTER adds the null row of a landmark with a cell that holds no candidate.
static int32_t cells_join(mgpu_ctx* ctx, hipStream_t s, Scratch& S, int32_t index_system, int32_t res, const double* lx,
                          const double* ly, int64_t n_left, const int64_t* ring, const int64_t* ring_off,
                          const double* rx, const double* ry, int64_t n_right, int64_t left_id_base,
                          int32_t max_per_left, double max_distance, int32_t flags, int64_t capacity, int64_t* out_n,
                          int64_t* out_left, int64_t* out_right, double* out_dist) {
  void* stream = (void*)s;
  int64_t* rc;
  RJ_TRY(S.get(&rc, n_right));
  if (n_right)
    if (int32_t st = mgpu_points_to_cells(ctx, index_system, res, rx, ry, n_right, rc, stream, nullptr)) return st;
  // the candidates' cell hash (cell ids are never 0)
  uint64_t slots = 16;
  while (slots < 2 * (uint64_t)std::max<int64_t>(n_right, 1)) slots <<= 1;
  uint64_t* slot_cell;
  int64_t *slot_head, *next;
  RJ_TRY(S.get(&slot_cell, slots));
  RJ_TRY(S.get(&slot_head, slots));
  RJ_TRY(S.get(&next, n_right));
  RJ_TRY(hipMemsetAsync(slot_cell, 0, slots * 8, s));
  RJ_TRY(hipMemsetAsync(slot_head, 0xFF, slots * 8, s));
  if (n_right)
    hipLaunchKernelGGL(rj_insert_kernel, dim3(grid_of(n_right)), dim3(256), 0, s, rc, n_right, slot_cell,
                       (unsigned long long*)slot_head, next, slots - 1);
  const int64_t nb = (n_left + kScanB - 1) / kScanB;
  int64_t* bsum;
  RJ_TRY(S.get(&bsum, nb + 1));
  auto scan = [&](const int64_t* v, int64_t* out) {
    hipLaunchKernelGGL(rj_scan_block_kernel, dim3((unsigned)nb), dim3(kScanB), 0, s, v, n_left, out, bsum);
    hipLaunchKernelGGL(rj_scan_sums_kernel, dim3(1), dim3(kScanB), 0, s, bsum, nb);
    hipLaunchKernelGGL(rj_scan_add_kernel, dim3((unsigned)nb), dim3(kScanB), 0, s, out, n_left, bsum, nb);
  };
  // pairs: counts, offsets, the pairs; each landmark's segment ordered by (distance,
  // candidate) and cut to max_per_left; kept counts, offsets, the output
  RjArgs a{lx, ly, rx, ry, ring, ring_off, slot_cell, slot_head, next, slots - 1, n_left, max_distance};
  int64_t *cnt, *off;
  int8_t* nul;
  RJ_TRY(S.get(&cnt, n_left));
  RJ_TRY(S.get(&off, n_left + 1));
  RJ_TRY(S.get(&nul, n_left));
  hipLaunchKernelGGL(rj_pairs_kernel<false>, dim3(grid_of(n_left)), dim3(256), 0, s, a, cnt, nullptr, nullptr, nullptr,
                     nul);
  scan(cnt, off);
  // the kept counts follow from the counts (the cut and the null row), so the output
  // offsets are known before any pair is written
  int64_t *kept, *koff;
  RJ_TRY(S.get(&kept, n_left));
  RJ_TRY(S.get(&koff, n_left + 1));
  const int8_t* nul_out = (flags & MGPU_RING_LEFT_OUTER) ? nul : nullptr;
  hipLaunchKernelGGL(rj_kept_kernel, dim3(grid_of(n_left)), dim3(256), 0, s, off, n_left, (int64_t)max_per_left, nul_out,
                     kept);
  scan(kept, koff);
  // the output's size (kept pairs) and the candidate pairs' total: a short output fails
  // here, before any pair is generated (the caller retries at the reported size)
  int64_t n_out = 0, n_pairs = 0;
  RJ_TRY(hipMemcpyAsync(&n_out, koff + n_left, 8, hipMemcpyDeviceToHost, s));
  RJ_TRY(hipMemcpyAsync(&n_pairs, off + n_left, 8, hipMemcpyDeviceToHost, s));
  RJ_TRY(hipStreamSynchronize(s));
  if (out_n) *out_n = n_out;
  if (n_out > capacity)
    return mgpu::set_error(MGPU_E_CAPACITY, "ring_join: %lld pairs, capacity %lld", (long long)n_out, (long long)capacity);
  if (n_out == 0) return MGPU_OK;
  // the pairs, sorted and cut per landmark, in batches of landmarks holding at most
  // kBatchPairs candidate pairs (a landmark with more is a batch of its own), so the
  // scratch stays bounded whatever the density; the per-landmark offsets come to the host
  // only when the pairs need more than one batch
  const int64_t kBatchPairs = ctx->opt.ring_batch;  // (option ring_batch)
  std::vector<int64_t> hoff;
  int64_t biggest = 0;
  if (n_pairs > kBatchPairs) {
    hoff.resize(n_left + 1);
    RJ_TRY(hipMemcpyAsync(hoff.data(), off, (n_left + 1) * 8, hipMemcpyDeviceToHost, s));
    RJ_TRY(hipStreamSynchronize(s));
    for (int64_t i = 0; i < n_left; i++) biggest = std::max(biggest, hoff[i + 1] - hoff[i]);
  }
  int64_t *pr, *roff;
  double* pd;
  RJ_TRY(S.get(&roff, n_left + 1));
  RJ_TRY(S.get(&pr, std::min(n_pairs, std::max(kBatchPairs, biggest))));
  RJ_TRY(S.get(&pd, std::min(n_pairs, std::max(kBatchPairs, biggest))));
  for (int64_t b0 = 0; b0 < n_left;) {
    int64_t b1 = n_left;
    if (!hoff.empty()) {
      b1 = b0 + 1;
      while (b1 < n_left && hoff[b1 + 1] - hoff[b0] <= std::max(kBatchPairs, biggest)) b1++;
    }
    RjArgs ab = a;
    ab.lx = a.lx + b0, ab.ly = a.ly + b0, ab.ring_off = a.ring_off + b0, ab.n_left = b1 - b0;
    // (offsets relative to the batch: the batch's segment starts at pr[0])
    hipLaunchKernelGGL(rj_rebase_kernel, dim3(grid_of(b1 - b0 + 1)), dim3(256), 0, s, off + b0, b1 - b0 + 1,
                       hoff.empty() ? (int64_t)0 : hoff[b0], roff);
    hipLaunchKernelGGL(rj_pairs_kernel<true>, dim3(grid_of(b1 - b0)), dim3(256), 0, s, ab, nullptr, roff, pr, pd,
                       nullptr);
    hipLaunchKernelGGL(rj_sort_kernel, dim3(grid_of(b1 - b0)), dim3(256), 0, s, roff, b1 - b0, (int64_t)max_per_left,
                       pr, pd, nullptr, nullptr);
    if (capacity > 0)
      hipLaunchKernelGGL(rj_copy_kernel, dim3(grid_of(b1 - b0)), dim3(256), 0, s, roff, koff + b0, b1 - b0, pr, pd,
                         left_id_base + b0, capacity, out_left, out_right, out_dist, nul_out ? nul_out + b0 : nullptr);
    RJ_TRY(hipGetLastError());
    RJ_TRY(hipStreamSynchronize(s));
    b0 = b1;
  }
  return MGPU_OK;
}

static int32_t check_join_args(mgpu_ctx* ctx, int32_t index_system, int32_t res, const double* lx, const double* ly,
                               int64_t n_left, const double* rx, const double* ry, int64_t n_right,
                               int32_t max_per_left, int32_t flags, int64_t capacity, int64_t* out_left,
                               int64_t* out_right, double* out_dist) {
  if (!ctx || n_left < 0 || n_right < 0 || (n_left && (!lx || !ly)) || (n_right && (!rx || !ry)) || capacity < 0 ||
      (capacity > 0 && (!out_left || !out_right || !out_dist)) || max_per_left < 0 || (flags & ~MGPU_RING_LEFT_OUTER))
    return mgpu::set_error(MGPU_E_INVALID_ARG, "ring_join: bad arguments");
  return mgpu_check_resolution(index_system, res);
}

extern "C" int32_t mgpu_ring_join_ex(mgpu_ctx* ctx, int32_t index_system, int32_t res, int32_t k, int32_t loop_only,
                                     const double* lx, const double* ly, int64_t n_left, const double* rx,
                                     const double* ry, int64_t n_right, int64_t left_id_base, int32_t max_per_left,
                                     double max_distance, int32_t flags, int64_t capacity, int64_t* out_n,
                                     int64_t* out_left, int64_t* out_right, double* out_dist, void* stream) {
  if (int32_t st = check_join_args(ctx, index_system, res, lx, ly, n_left, rx, ry, n_right, max_per_left, flags,
                                   capacity, out_left, out_right, out_dist))
    return st;
  if (k < 0 || k > 1024) return mgpu::set_error(MGPU_E_INVALID_ARG, "ring_join: k must be in [0, 1024]");
  RJ_TRY(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  if (out_n) *out_n = 0;
  if (n_left == 0) return MGPU_OK;
  Scratch S;
  int64_t* lc;
  RJ_TRY(S.get(&lc, n_left));
  // the landmarks' cells, the reference's (near-ties by its libm): IndexSystem.pointToIndex
  if (int32_t st = mgpu_points_to_cells(ctx, index_system, res, lx, ly, n_left, lc, stream, nullptr)) return st;
  // their ring cells (IndexSystem.kRing / kLoop through mgpu_grid_kring)
  int64_t *ring_off, *ring;
  RJ_TRY(S.get(&ring_off, n_left + 1));
  // (first guess bounded at 2^24 cells; mgpu_grid_kring reports the exact total when short)
  const int64_t per = loop_only ? (k == 0 ? 1 : 6 * (int64_t)k) : 3 * (int64_t)k * (k + 1) + 1;
  int64_t ring_cap = std::min<int64_t>(n_left * per + 1024, (int64_t)1 << 24), ring_total = 0;
  RJ_TRY(S.get(&ring, ring_cap));
  int32_t st = mgpu_grid_kring(ctx, index_system, lc, n_left, k, loop_only, ring, ring_cap, ring_off, &ring_total, stream);
  if (st == MGPU_E_CAPACITY) {
    ring_cap = ring_total;
    RJ_TRY(S.get(&ring, ring_cap));
    st = mgpu_grid_kring(ctx, index_system, lc, n_left, k, loop_only, ring, ring_cap, ring_off, &ring_total, stream);
  }
  if (st) return st;
  return cells_join(ctx, s, S, index_system, res, lx, ly, n_left, ring, ring_off, rx, ry, n_right, left_id_base,
                    max_per_left, max_distance, flags, capacity, out_n, out_left, out_right, out_dist);
}

extern "C" int32_t mgpu_ring_join(mgpu_ctx* ctx, int32_t index_system, int32_t res, int32_t k, int32_t loop_only,
                                  const double* lx, const double* ly, int64_t n_left, const double* rx,
                                  const double* ry, int64_t n_right, int64_t left_id_base, int32_t max_per_left,
                                  double max_distance, int64_t capacity, int64_t* out_n, int64_t* out_left,
                                  int64_t* out_right, double* out_dist, void* stream) {
  return mgpu_ring_join_ex(ctx, index_system, res, k, loop_only, lx, ly, n_left, rx, ry, n_right, left_id_base,
                           max_per_left, max_distance, 0, capacity, out_n, out_left, out_right, out_dist, stream);
}

// JTS OffsetSegmentGenerator.createCircle (the buffer of a point, 8 quadrant segments):
// the start (x + r, y), then the fillet from angle 0 clockwise through 2 pi in 32 equal
// steps (its first point repeats the start and is dropped), closed
static void jts_circle(double x, double y, double r, std::vector<double>& xy) {
  const double inc = 2.0 * M_PI / 32;
  xy.push_back(x + r);
  xy.push_back(y);
  for (int i = 1; i < 32; i++) {
    const double a = -(double)i * inc;
    xy.push_back(x + r * std::cos(a));
    xy.push_back(y + r * std::sin(a));
  }
  xy.push_back(x + r);
  xy.push_back(y);
}

// SpatialKNN's last iteration (GridRingNeighbours.leftTransform with iterationID = -1,
// models/knn/GridRingNeighbours.scala:82-90): per landmark, the cells of
// grid_tessellate(st_buffer(landmark, radius[i]), res) not in grid_geometrykring(landmark,
// res, k[i]) (array_except), joined with the candidates as every iteration is.  The
// buffers are tessellated on the host by mgpu_tessellate (mosaicFill's sets, chips of
// every cell meeting the circle); radius[i] NaN or <= 0 gives the landmark no cells.
extern "C" int32_t mgpu_ring_join_final(mgpu_ctx* ctx, int32_t index_system, int32_t res, const double* lx,
                                        const double* ly, const double* radius, const int32_t* k_iterated,
                                        int64_t n_left, const double* rx, const double* ry, int64_t n_right,
                                        int64_t left_id_base, int32_t max_per_left, double max_distance,
                                        int32_t flags, int64_t capacity, int64_t* out_n, int64_t* out_left,
                                        int64_t* out_right, double* out_dist, void* stream) {
  if (int32_t st = check_join_args(ctx, index_system, res, lx, ly, n_left, rx, ry, n_right, max_per_left, flags,
                                   capacity, out_left, out_right, out_dist))
    return st;
  if (n_left && (!radius || !k_iterated)) return mgpu::set_error(MGPU_E_INVALID_ARG, "ring_join_final: bad arguments");
  if (n_left >= ((int64_t)1 << 31)) return mgpu::set_error(MGPU_E_INVALID_ARG, "ring_join_final: too many landmarks");
  for (int64_t i = 0; i < n_left; i++)
    if (k_iterated[i] < 0 || k_iterated[i] > 1024)
      return mgpu::set_error(MGPU_E_INVALID_ARG, "ring_join_final: k must be in [0, 1024]");
  RJ_TRY(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  if (out_n) *out_n = 0;
  if (n_left == 0) return MGPU_OK;
  Scratch S;
  // the landmarks on the host (their circles), and their cells
  std::vector<double> hx(n_left), hy(n_left);
  RJ_TRY(hipMemcpyAsync(hx.data(), lx, n_left * 8, hipMemcpyDeviceToHost, s));
  RJ_TRY(hipMemcpyAsync(hy.data(), ly, n_left * 8, hipMemcpyDeviceToHost, s));
  int64_t* lc;
  RJ_TRY(S.get(&lc, n_left));
  if (int32_t st = mgpu_points_to_cells(ctx, index_system, res, lx, ly, n_left, lc, stream, nullptr)) return st;
  RJ_TRY(hipStreamSynchronize(s));
  // st_buffer(landmark, radius) -> grid_tessellate (mosaicFill's cells)
  std::vector<int32_t> pid;
  std::vector<int64_t> poff{0}, roff{0}, voff{0};
  std::vector<double> xy;
  for (int64_t i = 0; i < n_left; i++) {
    if (!(radius[i] > 0) || !std::isfinite(radius[i]) || !std::isfinite(hx[i]) || !std::isfinite(hy[i])) continue;
    pid.push_back((int32_t)i);
    jts_circle(hx[i], hy[i], radius[i], xy);
    voff.push_back((int64_t)xy.size() / 2);
    roff.push_back((int64_t)voff.size() - 1);
    poff.push_back((int64_t)roff.size() - 1);
  }
  std::vector<std::vector<int64_t>> cells(n_left);
  if (!pid.empty()) {
    mgpu_tess* t = nullptr;
    if (int32_t st = mgpu_tessellate_ex(index_system, res, (int64_t)pid.size(), pid.data(), poff.data(), roff.data(),
                                        voff.data(), xy.data(), 0, MGPU_CORE_MOSAICFILL, &t))
      return st;
    int64_t nc = 0, wb = 0;
    mgpu_tess_result_sizes(t, &nc, &wb);
    std::vector<int64_t> cell(nc), woff(nc + 1);
    std::vector<int32_t> cpoly(nc);
    std::vector<uint8_t> core(nc), wkb(std::max<int64_t>(wb, 1));
    mgpu_tess_result_copy(t, cell.data(), cpoly.data(), core.data(), woff.data(), wkb.data());
    mgpu_tess_destroy(t);
    for (int64_t c = 0; c < nc; c++) cells[cpoly[c]].push_back(cell[c]);
  }
  // minus kRing(landmark cell, k[i]), per distinct k
  std::vector<int64_t> hlc(n_left);
  RJ_TRY(hipMemcpy(hlc.data(), lc, n_left * 8, hipMemcpyDeviceToHost));
  std::vector<int32_t> ks(k_iterated, k_iterated + n_left);
  std::sort(ks.begin(), ks.end());
  ks.erase(std::unique(ks.begin(), ks.end()), ks.end());
  std::vector<std::vector<int64_t>> iterated(n_left);
  for (int32_t k : ks) {
    std::vector<int64_t> who;
    for (int64_t i = 0; i < n_left; i++)
      if (k_iterated[i] == k && !cells[i].empty()) who.push_back(i);
    if (who.empty()) continue;
    std::vector<int64_t> sub(who.size());
    for (size_t q = 0; q < who.size(); q++) sub[q] = hlc[who[q]];
    int64_t *dsub, *doff, *dring;
    RJ_TRY(S.get(&dsub, sub.size()));
    RJ_TRY(S.get(&doff, sub.size() + 1));
    RJ_TRY(hipMemcpy(dsub, sub.data(), sub.size() * 8, hipMemcpyHostToDevice));
    // (first guess bounded at 2^24 cells, as mgpu_ring_join_ex's; the exact total on a retry)
    int64_t cap = std::min<int64_t>((int64_t)sub.size() * (3 * (int64_t)k * (k + 1) + 1) + 1024, (int64_t)1 << 24),
            total = 0;
    RJ_TRY(S.get(&dring, cap));
    int32_t st = mgpu_grid_kring(ctx, index_system, dsub, (int64_t)sub.size(), k, 0, dring, cap, doff, &total, stream);
    if (st == MGPU_E_CAPACITY) {
      cap = total;
      RJ_TRY(S.get(&dring, cap));
      st = mgpu_grid_kring(ctx, index_system, dsub, (int64_t)sub.size(), k, 0, dring, cap, doff, &total, stream);
    }
    if (st) return st;
    std::vector<int64_t> hr(total), ho(sub.size() + 1);
    RJ_TRY(hipMemcpy(hr.data(), dring, total * 8, hipMemcpyDeviceToHost));
    RJ_TRY(hipMemcpy(ho.data(), doff, ho.size() * 8, hipMemcpyDeviceToHost));
    for (size_t q = 0; q < who.size(); q++) iterated[who[q]].assign(hr.begin() + ho[q], hr.begin() + ho[q + 1]);
  }
  // array_except: the distinct tessellation cells outside the iterated ring, in their
  // first-seen order (a hash set of the cells seen: linear per landmark)
  std::vector<int64_t> ring, ring_off{0};
  std::unordered_set<int64_t> seen;
  for (int64_t i = 0; i < n_left; i++) {
    std::vector<int64_t> it = iterated[i];
    std::sort(it.begin(), it.end());
    seen.clear();
    for (int64_t c : cells[i]) {
      if (std::binary_search(it.begin(), it.end(), c)) continue;
      if (!seen.insert(c).second) continue;
      ring.push_back(c);
    }
    ring_off.push_back((int64_t)ring.size());
  }
  int64_t *dring, *droff;
  RJ_TRY(S.get(&dring, ring.size()));
  RJ_TRY(S.get(&droff, ring_off.size()));
  if (!ring.empty()) RJ_TRY(hipMemcpy(dring, ring.data(), ring.size() * 8, hipMemcpyHostToDevice));
  RJ_TRY(hipMemcpy(droff, ring_off.data(), ring_off.size() * 8, hipMemcpyHostToDevice));
  return cells_join(ctx, s, S, index_system, res, lx, ly, n_left, dring, droff, rx, ry, n_right, left_id_base,
                    max_per_left, max_distance, flags, capacity, out_n, out_left, out_right, out_dist);
}
