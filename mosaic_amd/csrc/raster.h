// Pixel index lookup (chip_table.h "Pixel index"; built by capi.cpp build_raster_*),
// shared by the streaming join kernel and the host-side certificate test
// (mgpu_test_raster_host).
#pragma once
#include <math.h>
#include <stdint.h>

#include "bng_core.h"
#include "chip_table.h"
#include "../../include/mosaic_gpu.h"

namespace mgpu {

constexpr uint32_t kNoPixel = 0xFFFFFFFFu;

// Pixel index (chip_table.h) of a point: the pixel, kNoPixel (no chip can match: outside
// the chip cells' box -- or a non-finite coordinate, *ok = false) or kRasterFull (BNG
// coordinates outside [0, 1e7): the id + hash path).  BNG: *gi = the cell's dense grid
// entry (the pixel holds the match mask of that cell's chips).
constexpr uint32_t kRasterFull = 0xFFFFFFFEu;
MGPU_HDI uint32_t div_fix(uint32_t v, uint32_t d, double inv) {
  const uint32_t q = (uint32_t)((double)v * inv);
  return q * d > v ? q - 1 : ((q + 1) * d <= v ? q + 1 : q);
}
template <int IS>
MGPU_HDI uint32_t raster_index(const ChipTableView& t, double px, double py, bool* ok, uint32_t* gi) {
  if (IS == MGPU_BNG) {
    *ok = px == px && py == py;  // pointToIndex rejects NaN only
    if (!*ok) return kNoPixel;
    const int32_t eI = bng::d2i(px), nI = bng::d2i(py);
    if (!((uint32_t)eI < 10000000u && (uint32_t)nI < 10000000u)) return kRasterFull;
    const uint32_t col = div_fix((uint32_t)eI, t.raster_pix, t.raster_inv_dx);
    const uint32_t row = div_fix((uint32_t)nI, t.raster_pix, t.raster_inv_dy);
    const uint32_t ix = col - (uint32_t)t.raster_px0, iy = row - (uint32_t)t.raster_py0;
    if (ix >= t.raster_nx || iy >= t.raster_ny) return kNoPixel;  // outside the dense box: no chip cell
    const DenseFace& D = t.dense[0];
    *gi = D.base + (div_fix((uint32_t)nI, t.bng_edge, t.bng_inv_edge) - (uint32_t)D.b0) * D.w +
          (div_fix((uint32_t)eI, t.bng_edge, t.bng_inv_edge) - (uint32_t)D.a0);
    return iy * t.raster_nx + ix;
  }
  *ok = isfinite(px) && isfinite(py);
  if (!*ok || !(px >= t.bbox[0] && px <= t.bbox[2] && py >= t.bbox[1] && py <= t.bbox[3])) return kNoPixel;
  uint32_t ix = (uint32_t)((px - t.raster_x0) * t.raster_inv_dx), iy = (uint32_t)((py - t.raster_y0) * t.raster_inv_dy);
  ix = ix < t.raster_nx ? ix : t.raster_nx - 1;
  iy = iy < t.raster_ny ? iy : t.raster_ny - 1;
  return iy * t.raster_nx + ix;
}

}  // namespace mgpu
