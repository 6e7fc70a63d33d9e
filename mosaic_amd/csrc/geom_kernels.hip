// grid_pointascellid's decode step on the GPU: the centroid of every row of a geometry
// column (geom_decode.h: WKB / HEX / WKT / GeoJSON readers and JTS's Centroid) and of
// Mosaic's InternalGeometryType rows.  Its own translation unit: the text readers are
// the heaviest device code of the library and compile in parallel with kernels.hip.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define H3T_QUAL static __constant__ const
#include "kernels.h"
#include "raster.h"
#include "geom_decode.h"

namespace mgpu {

constexpr int kStreamBlock = 256;

__device__ __forceinline__ void count_wave(unsigned long long* ctr, bool pred) {
  unsigned long long b = __ballot(pred);
  if (b && (threadIdx.x & 63) == (__ffsll((long long)b) - 1)) atomicAdd(ctr, (unsigned long long)__popcll(b));
}

// ---------------------------------------------------------------- geometry columns
__global__ __launch_bounds__(kStreamBlock) void decode_points_kernel(int format, const uint8_t* __restrict__ data,
                                                                   const void* __restrict__ off, int off32,
                                                                   const uint8_t* __restrict__ valid, int64_t voff,
                                                                   int64_t n, double* __restrict__ ox,
                                                                   double* __restrict__ oy,
                                                                   unsigned long long* __restrict__ counters) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int st = geom::kDecOk;
  if (i < n) {
    double x = NAN, y = NAN;
    if (pt_valid(valid, voff, i)) {
      const int64_t b = off32 ? ((const int32_t*)off)[i] : ((const int64_t*)off)[i];
      const int64_t e = off32 ? ((const int32_t*)off)[i + 1] : ((const int64_t*)off)[i + 1];
      if (e < b) {
        st = geom::kDecMalformed;
      } else if (format == MGPU_GEOM_WKB) {
        st = geom::wkb_centroid(data + b, e - b, &x, &y);
      } else if (format == MGPU_GEOM_WKT) {
        st = geom::wkt_centroid((const char*)data + b, e - b, &x, &y);
      } else if (format == MGPU_GEOM_HEX) {
        st = geom::hex_centroid((const char*)data + b, e - b, &x, &y);
      } else {
        st = geom::json_centroid((const char*)data + b, e - b, &x, &y);
      }
      if (st) x = y = NAN;
    }
    ox[i] = x;
    oy[i] = y;
  }
  count_wave(&counters[4], st == geom::kDecMalformed);
  count_wave(&counters[5], st == geom::kDecUnsupported);
  count_wave(&counters[6], st == geom::kDecEmpty);
}

// Mosaic's InternalGeometryType rows (geom_decode.h internal_centroid) -> their centroids
__global__ __launch_bounds__(kStreamBlock) void decode_internal_kernel(const int32_t* __restrict__ type_id,
                                                                     const int64_t* __restrict__ row_part,
                                                                     const int64_t* __restrict__ part_ring,
                                                                     const int64_t* __restrict__ ring_off,
                                                                     const double* __restrict__ xy,
                                                                     const uint8_t* __restrict__ valid, int64_t voff,
                                                                     int64_t n, double* __restrict__ ox,
                                                                     double* __restrict__ oy,
                                                                     unsigned long long* __restrict__ counters) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int st = geom::kDecOk;
  if (i < n) {
    double x = NAN, y = NAN;
    if (pt_valid(valid, voff, i)) {
      st = geom::internal_centroid(type_id[i], row_part[i], row_part[i + 1], part_ring, ring_off, xy, &x, &y);
      if (st) x = y = NAN;
    }
    ox[i] = x;
    oy[i] = y;
  }
  count_wave(&counters[4], st == geom::kDecMalformed);
  count_wave(&counters[5], st == geom::kDecUnsupported);
  count_wave(&counters[6], st == geom::kDecEmpty);
}

hipError_t launch_decode_internal(const int32_t* type_id, const int64_t* row_part, const int64_t* part_ring,
                                  const int64_t* ring_off, const double* xy, const uint8_t* valid, int64_t voff,
                                  int64_t n, double* x, double* y, unsigned long long* counters, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(decode_internal_kernel, dim3((unsigned)((n + kStreamBlock - 1) / kStreamBlock)), dim3(kStreamBlock),
                     0, s, type_id, row_part, part_ring, ring_off, xy, valid, voff, n, x, y, counters);
  return hipGetLastError();
}

hipError_t launch_decode_points(int format, const uint8_t* data, const void* offsets, int off32, const uint8_t* valid,
                                int64_t voff, int64_t n, double* x, double* y, unsigned long long* counters,
                                hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(decode_points_kernel, dim3((unsigned)((n + kStreamBlock - 1) / kStreamBlock)), dim3(kStreamBlock), 0,
                     s, format, data, offsets, off32, valid, voff, n, x, y, counters);
  return hipGetLastError();
}


}  // namespace mgpu
