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

// Arrow-style validity bitmap (bit (off + p), LSB first); null = every row valid.  A null
// point matches nothing (the reference's expressions are NullIntolerant: null in, null out).
MGPU_HDI bool pt_valid(const uint8_t* v, int64_t off, int64_t p) {
  if (!v) return true;
  const int64_t b = off + p;
  return (v[b >> 3] >> (b & 7)) & 1;
}

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
MGPU_HDI uint32_t raster_index(const ChipTableView& t, double px, double py, bool* ok, uint32_t* gi, uint32_t* sub,
                               uint32_t* blk = nullptr) {
  if (blk) *blk = kNoPixel;
  if (IS == MGPU_BNG) {
    *ok = px == px && py == py;  // pointToIndex rejects NaN only
    if (!*ok) return kNoPixel;
    const int32_t eI = bng::d2i(px), nI = bng::d2i(py);
    if (!((uint32_t)eI < 10000000u && (uint32_t)nI < 10000000u)) return kRasterFull;
    const uint32_t col = div_fix((uint32_t)eI, t.raster_pix, t.raster_inv_dx);
    const uint32_t row = div_fix((uint32_t)nI, t.raster_pix, t.raster_inv_dy);
    const uint32_t ix = col - (uint32_t)t.raster_px0, iy = row - (uint32_t)t.raster_py0;
    if (ix >= t.raster_nx || iy >= t.raster_ny) return kNoPixel;  // outside the dense box: no chip cell
    if (t.raster_sub_n) {
      const double inv_w = 1.0 / (double)t.raster_sub_w;
      const uint32_t u = div_fix((uint32_t)eI - col * t.raster_pix, t.raster_sub_w, inv_w);
      const uint32_t v = div_fix((uint32_t)nI - row * t.raster_pix, t.raster_sub_w, inv_w);
      *sub = v * t.raster_sub_n + u;
    }
    const DenseFace& D = t.dense[0];
    *gi = D.base + (div_fix((uint32_t)nI, t.bng_edge, t.bng_inv_edge) - (uint32_t)D.b0) * D.w +
          (div_fix((uint32_t)eI, t.bng_edge, t.bng_inv_edge) - (uint32_t)D.a0);
    return iy * t.raster_nx + ix;
  }
  *ok = isfinite(px) && isfinite(py);
  if (!*ok || !(px >= t.bbox[0] && px <= t.bbox[2] && py >= t.bbox[1] && py <= t.bbox[3])) return kNoPixel;
  const double tx = (px - t.raster_x0) * t.raster_inv_dx, ty = (py - t.raster_y0) * t.raster_inv_dy;
  uint32_t ix = (uint32_t)tx, iy = (uint32_t)ty;
  ix = ix < t.raster_nx ? ix : t.raster_nx - 1;
  iy = iy < t.raster_ny ? iy : t.raster_ny - 1;
  if (blk && t.raster_bshift) *blk = (iy >> t.raster_bshift) * t.raster_bnx + (ix >> t.raster_bshift);
  if (t.raster_sub_n) {
    const double S = (double)t.raster_sub_n;
    uint32_t u = (uint32_t)((tx - (double)ix) * S), v = (uint32_t)((ty - (double)iy) * S);
    u = u < t.raster_sub_n ? u : t.raster_sub_n - 1;
    v = v < t.raster_sub_n ? v : t.raster_sub_n - 1;
    *sub = v * t.raster_sub_n + u;
    if (t.raster_band) *sub |= (iy >> t.raster_band_shift) << 16;  // the row band (raster_class)
  }
  return iy * t.raster_nx + ix;
}

// The class of pixel ri (a raster_index result below kRasterFull), refined by its
// second level when the pixel is mixed (`band`: raster_band or its LDS copy).
#ifndef MGPU_RANK_SPEC
#define MGPU_RANK_SPEC 0
#endif
MGPU_HDI uint32_t raster_class(const ChipTableView& t, uint32_t ri, uint32_t sub, const uint32_t* band = nullptr) {
  if (t.raster_band) {
    uint32_t cl = t.raster[ri];
    if (cl >= 0x8000u && cl != kPixMixed) {
      const uint64_t b = (uint64_t)(band ? band : t.raster_band)[sub >> 16] + (cl & 0x7FFFu);
      const uint32_t i = sub & 0xFFFFu, s2 = t.raster_sub_n * t.raster_sub_n;
      if (t.raster_pal) {
        // (the palette word and the index byte load together: both hang off b)
        const uint64_t P = t.raster_pal[b];
        const uint32_t q = t.raster_idx2[b * (s2 >> 2) + (i >> 2)];
        const uint32_t c = (uint32_t)(P >> (16 * ((q >> (2 * (i & 3))) & 3))) & 0x7FFFu;
        cl = (P & kPalFull) ? t.raster_sub[(P & 0xFFFFFFFFull) * s2 + i] : (c == 0x7FFFu ? kPixMixed : c);
      } else {
        cl = t.raster_sub[b * s2 + i];
      }
    }
    return cl;
  }
#if MGPU_RANK_SPEC
  // the rank word loads beside the pixel's class (no second round trip for mixed pixels)
  const RankWord w = t.raster_rank ? t.raster_rank[ri >> 5] : RankWord{0u, 0u};
  uint32_t cl = t.raster[ri];
  if (cl == kPixMixed) {
#else
  uint32_t cl = t.raster[ri];
  if (cl == kPixMixed && t.raster_rank) {
    const RankWord w = t.raster_rank[ri >> 5];
#endif
    const uint32_t bit = 1u << (ri & 31);
    if (w.bits & bit) {
      const uint64_t b = (uint64_t)w.base + (uint64_t)__builtin_popcount(w.bits & (bit - 1));
      cl = t.raster_sub[b * t.raster_sub_n * t.raster_sub_n + sub];
    }
  }
  return cl;
}

// raster_class with the block table first (`blk_table`: raster_blk or its LDS copy; bi
// from raster_index, kNoPixel: no block)
MGPU_HDI uint32_t raster_class_blk(const ChipTableView& t, const uint16_t* blk_table, uint32_t ri, uint32_t bi,
                                   uint32_t sub, const uint32_t* band = nullptr) {
  const uint32_t c = bi != kNoPixel ? blk_table[bi] : kPixMixed;
  return c != kPixMixed ? c : raster_class(t, ri, sub, band);
}

}  // namespace mgpu
