// Device-resident chip table: the ChipType rows `(is_core, index_id, wkb)` of
// `grid_tessellateexplode` (reference core/types/ChipType.scala:17-29,
// core/types/model/MosaicChip.scala:20-83), plus the owning polygon id, flattened
// to structure-of-arrays in ONE device allocation (so it can be replicated to
// other GPUs with a single RCCL broadcast).
//
// Layout (all arrays 16-byte aligned inside the blob):
//   cell hash  : open addressing, linear probing, `hash_cap` slots of
//                {u64 cell, u32 first_chip, u32 n_chips}; n_chips == 0 = empty
//   chips      : sorted by (cell, polygon id, input row)  -> matches come out in
//                polygon-id order for every point
//                chip_poly[i32], chip_flags[u8], chip_part[u32 n_chips+1],
//                chip_env[double4 minx,miny,maxx,maxy], chip_row[i64 input row]
//   geometry   : part_ring[u32 n_parts+1], ring_vtx[u32 n_rings+1],
//                ring_env[double4], vtx[double2 x,y]
//   row map    : row_to_chip[u32 n_chips] (input row -> sorted position)
//   strips     : per border chip, its envelope's y-range cut into S equal strips;
//                chip_strip[u32 n_chips+1] (first strip of each chip), chip_sy
//                [double2 y0, S/height], strip_edge[u32 n_strips+1] -> edge records
//                edges[double4 p1x,p1y,p2x,p2y] + edge_ring[u8 ring within chip].
//                A strip lists every chip edge whose closed y-range meets it (the
//                strip of a y value is computed by strip_of() on host and device
//                alike, which is monotone in y).  Exactness: RayCrossingCounter's
//                countSegment contributes nothing for a segment whose closed y-range
//                misses p.y, so the strip's edges give the same crossing parity and
//                on-boundary bit as the whole ring (pip_core.h chip_contains_strips).
// For H3 tables the hash is keyed by the (face, i, j) lattice position that the
// kernel's projection yields, not by the 64-bit cell id: the kernel then never
// assembles H3 digits.  Every lattice position of every chip cell on every face a
// point of that cell can project to is present (built and verified at upload with
// face_ijk_to_h3, mosaic_amd/csrc/capi.cpp build_lattice).
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#define MGPU_HDI_FWD __host__ __device__ __forceinline__
#else
#define MGPU_HDI_FWD inline
#endif

namespace mgpu {

enum ChipFlags : uint8_t {
  kChipCore = 1,       // is_core: every point of the cell matches
  kChipRect = 2,       // Polygon.isRectangle(): RectangleContains shortcut
  kChipMulti = 4,      // MultiPolygon / GeometryCollection: Mod-2 PointLocator
  kChipEmpty = 8,      // no coordinates: contains nothing
  kChipNoGeom = 16,    // WKB was NULL (core chip with keep_core_geometries=false)
  kChipNoStrips = 32,  // more than 32 rings: evaluated by the sequential PointLocator
};

constexpr int kMaxStrips = 64;
constexpr int kStripRings = 32;

// strip of y within a chip of `S` strips (y >= y0 whenever it is used on a point,
// since the chip envelope test comes first); monotone non-decreasing in y
MGPU_HDI_FWD int strip_of(double y, double y0, double inv_h, int S) {
  double v = (y - y0) * inv_h;
  int s = v < (double)S ? (int)v : S - 1;
  return s < 0 ? 0 : s;
}

// cell (or lattice key) -> its chips [first, first + count).  core_mask bit j: chip
// first + j is a core chip (j < 16; chips past 16 are looked up in chip_flags).
struct alignas(16) HashSlot {
  uint64_t cell;
  uint32_t first;
  uint16_t count;
  uint16_t core_mask;
};

// Everything the join's PIP step needs about one border chip, in two 64-byte lines
// (the per-array form above stays for st_contains and the sequential PointLocator).
//
// Classification grid: the chip envelope cut into kGrid x kGrid cells, cell (gx, gy)
// = the points whose computed indices gx = (int)((x - minx) * sx), gy likewise
// (clamped) are gx, gy.  State 1 / 0: every such point is INTERIOR / EXTERIOR, so
// contains() is decided by one lookup; 2: mixed, use the strip's edges.  A cell is
// given state 0 / 1 only if its rectangle, widened by a margin far above the index
// rounding error, meets no chip edge: all its points then lie in one connected
// component of the plane minus the chip boundary, at a positive distance from it,
// where JTS's robust PointLocator returns the topological location -- the one it
// returns for the cell centre (evaluated at upload with the same PointLocator).
constexpr int kGrid = 16;
struct alignas(64) ChipHdr {
  double env[4];        // minx, miny, maxx, maxy
  double sx, sy;        // grid scales kGrid / width, kGrid / height (0: one cell)
  double inv_h;         // strip scale S / height (strip_of with y0 = miny)
  uint32_t strip_base;  // first strip (index into strip_edge)
  uint16_t n_strips;
  uint8_t flags;        // ChipFlags
  uint8_t single_ring;  // one polygon with one ring, not a collection
  uint32_t grid[kGrid]; // row gy: 2 bits per cell gx (0 out, 1 in, 2 mixed)
};
static_assert(sizeof(ChipHdr) == 128, "ChipHdr is two lines");

enum GridState { kCellOut = 0, kCellIn = 1, kCellMixed = 2 };

MGPU_HDI_FWD int grid_index(double v, double v0, double scale) {
  double g = (v - v0) * scale;
  int i = g < (double)kGrid ? (int)g : kGrid - 1;
  return i < 0 ? 0 : i;
}

struct DenseFace {
  int32_t a0, b0;
  uint32_t w, h;
  uint32_t base;
};

struct alignas(8) RankWord {
  uint32_t bits;  // pixels 32 w .. 32 w + 31 that are mixed
  uint32_t base;  // mixed pixels before pixel 32 w
};

struct ChipTableView {
  const HashSlot* slots;
  uint32_t hash_mask;
  uint32_t max_probe;
  uint32_t n_chips;
  uint32_t n_cells;
  const int32_t* chip_poly;
  const uint8_t* chip_flags;
  const uint32_t* chip_part;   // [n_chips + 1]
  const double* chip_env;      // 4 per chip
  const int64_t* chip_row;     // input row of each sorted chip
  const uint32_t* part_ring;   // [n_parts + 1]
  const uint32_t* ring_vtx;    // [n_rings + 1]
  const double* ring_env;      // 4 per ring
  const double* vtx;           // 2 per vertex
  const uint32_t* row_to_chip; // [n_chips]
  const uint32_t* chip_strip;  // [n_chips + 1]
  const double* chip_sy;       // 2 per chip: y0, S / height
  const uint32_t* strip_edge;  // [n_strips + 1]
  const double* edges;         // 4 per edge record: p1x, p1y, p2x, p2y (p1 = ring[i], p2 = ring[i-1])
  const uint8_t* edge_ring;    // ring index of the edge within its chip
  const ChipHdr* chip_hdr;     // [n_chips]
  // probing (lattice: H3 only; dense grid: H3 lattice or BNG column/row)
  int32_t probe_mode;          // ProbeMode: hash by cell id / hash by lattice key / dense grid
  int32_t res;                 // resolution of the chip cells (H3), -1 if mixed / unknown
  uint32_t face_mask;          // icosahedron faces a point inside `bbox` can be nearest to
  double bbox[4];              // lon_min, lat_min, lon_max, lat_max (deg): points outside match no chip
  double k_res;                // sqrt7^res / RES0_U_GNOMONIC
  // kProbeDense: per face f, grid[base + (b - b0) * w + (a - a0)] for the axial
  // lattice coordinates a = i - k, b = j - k inside [a0, a0 + w) x [b0, b0 + h);
  // entry = first | count << 32 | core_mask << 48 (count 0: no chip cell there)
  // BNG (kProbeDense): dense[0] spans the chip cells' (column, row) box, column =
  // easting / bng_edge and row = northing / bng_edge in whole metres (bng_edge = the
  // cell edge, halved for quadrant resolutions); the same entry format
  const uint64_t* grid;
  DenseFace dense[20];
  uint32_t bng_edge;
  double bng_inv_edge;
  // Pixel index (kRaster*, capi.cpp build_raster): a raster of the chip cells' box in the
  // point coordinates whose pixel p holds a class: kPixEmpty (no point of the pixel has a
  // match), kPixMixed (the streaming kernel projects and tests the point), or k >= 1 =
  // raster_cls[k] = first chip | match mask << 32 -- every point of the pixel lies in
  // ONE chip cell (certified at build time, with margins, for the whole pixel) and in the
  // interior / exterior of each of its chips (no chip edge meets the pixel), so its
  // matches are the chips first + j for the mask bits j.
  //   H3: pixel (ix, iy) = ((lon - x0) * inv_dx, (lat - y0) * inv_dy) truncated, clamped
  //       to the last pixel (the raster spans `bbox`);
  //   BNG: pixel = (easting / pix, northing / pix) in whole metres, minus (px0, py0); pix
  //       divides the cell edge, so every pixel lies in one cell.
  uint32_t max_cell_chips;     // chips of the fullest cell
  int32_t raster_mode;         // kRasterNone / kRasterLonLat / kRasterBng
  uint32_t raster_nx, raster_ny;
  uint32_t raster_pix;         // BNG pixel edge (metres)
  int32_t raster_px0, raster_py0;
  double raster_x0, raster_y0, raster_inv_dx, raster_inv_dy;
  uint32_t raster_pc[4];       // lonlat: classes are ordered by match count; class c has k + 1
                               // matches for raster_pc[k - 1] <= c < raster_pc[k] (k < 4)
  const uint16_t* raster;      // [ny * nx] classes
  const uint64_t* raster_cls;  // [classes]
  // raster_cls_poly[c] = the polygon of class c when it has one match (c < raster_pc[0]),
  // else -1: the emit kernels copy it to LDS and answer a one-match pixel without the
  // raster_cls / chip_poly gathers
  const int32_t* raster_cls_poly;  // [raster_ncls]
  uint32_t raster_ncls;
  // second level: every mixed pixel p is cut into sub_n x sub_n sub-pixels whose classes
  // are raster_sub[b * sub_n^2 + v * sub_n + u], b = the number of mixed pixels before p
  // (lonlat: u = the truncated sub_n * fractional pixel position, clamped; BNG: (metres
  // into the pixel) / raster_sub_w).  b comes from raster_rank (a bitmap of the mixed
  // pixels with a running count per 32-pixel word: one 8-byte load per mixed point, a
  // table 1/8 the size of the pixel classes -- it stays in L2 beside them -- that the
  // streaming kernel loads together with the pixel's class).
  uint32_t raster_sub_n, raster_sub_w;
  const RankWord* raster_rank;  // [ceil(ny * nx / 32)], or null: no second level / bands
  // lonlat, instead of raster_rank (capi.cpp raster_bands): a refined mixed pixel's class
  // is 0x8000 | its index within its band of 2^raster_band_shift rows, b = raster_band[iy
  // >> raster_band_shift] + (class & 0x7FFF); every other class is below 0x7FFF
  uint32_t raster_band_shift, raster_nband;
  const uint32_t* raster_band;  // [raster_nband], or null
  // BNG dense grid: per-cell answer grids (capi.cpp build_cell_answers).  A cell with
  // border chips (at most kCellAnsChips) is cut into cell_ans_g x cell_ans_g squares of
  // cell_ans_sw whole metres; its grid entry carries kCellAnsFlag (bit 47: such tables
  // have no cell of 2^15 chips) and its index k among the dense row's answer cells (bits
  // 36-46 and 63 -- the count takes bits 32-35, the core mask no bit 15), and
  // cell_ans[((cell_ans_row[row] + k) * g + v) * g + u] = the match mask of the cell's
  // chips for every point of square (u, v) (certified like a pixel), or kCellAnsMixed:
  // the candidates' path.  Only flagged cells cost a load.
  uint32_t cell_ans_g, cell_ans_sw;
  double cell_ans_inv_sw;
  const uint32_t* cell_ans_row;  // [dense rows], or null: no answer grids
  const uint16_t* cell_ans;
  const uint16_t* raster_sub;
  // lonlat with bands, palette-compressed (capi.cpp raster_palette; null: raster_sub holds
  // every block): block b's sub-pixel i has class (raster_pal[b] >> 16 k) & 0x7FFF (0x7FFF
  // = kPixMixed), k = the 2 bits (i & 3) of byte raster_idx2[b * sub_n^2 / 4 + i / 4];
  // raster_pal[b] with kPalFull: its classes are raster_sub[(raster_pal[b] & 0xFFFFFFFF) *
  // sub_n^2 + i]
  const uint64_t* raster_pal;
  const uint8_t* raster_idx2;
  // lonlat: blocks of 2^bshift x 2^bshift pixels, raster_blk[(iy >> bshift) * bnx + (ix >>
  // bshift)] = the class all of the block's pixels share, else kPixMixed (a table small
  // enough for LDS: the streaming kernels answer most points without a global load);
  // bshift = 0: none
  uint32_t raster_bshift, raster_bnx, raster_bny;
  const uint16_t* raster_blk;
};

enum RasterMode { kRasterNone = 0, kRasterLonLat = 1, kRasterBng = 2 };
constexpr uint32_t kCellAnsChips = 15;      // chips of a cell with an answer grid, at most
constexpr uint16_t kCellAnsMixed = 0xFFFF;
constexpr uint32_t kNoCellAns = 0xFFFFFFFFu;
constexpr uint64_t kCellAnsFlag = 1ull << 47;
// H3: core-mask bit 15 of a one-chip cell whose chip is the cell's own hexagon (capi.cpp
// mark_whole_cells): a point deep inside the cell (FastHex::deep) matches it
constexpr uint32_t kCoreWhole = 0x8000u;
// the chip count of a dense grid entry (first | count << 32 | core mask << 48); `ans`: the
// table has answer grids (ChipTableView::cell_ans_row)
MGPU_HDI_FWD uint32_t grid_count(uint64_t e, bool ans) {
  return (uint32_t)(e >> 32) & ((ans && (e & kCellAnsFlag)) ? 0xFu : 0xFFFFu);
}
MGPU_HDI_FWD uint32_t cell_ans_index(uint64_t e) { return (uint32_t)((e >> 36) & 0x7FF) | (uint32_t)(e >> 63) << 11; }
constexpr uint16_t kPixEmpty = 0;
constexpr uint16_t kPixMixed = 0xFFFF;
constexpr uint64_t kPalFull = 1ull << 63;

enum ProbeMode { kProbeCellId = 0, kProbeLattice = 1, kProbeDense = 2 };

#ifdef __HIPCC__
#define MGPU_HDI __host__ __device__ __forceinline__
#else
#define MGPU_HDI inline
#endif

MGPU_HDI uint32_t cell_hash(uint64_t cell) {
  uint64_t z = cell * 0x9E3779B97F4A7C15ULL;
  z ^= z >> 29;
  z *= 0xBF58476D1CE4E5B9ULL;
  return (uint32_t)(z >> 32);
}

}  // namespace mgpu
