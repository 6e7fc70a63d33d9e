// C-ABI of the MI355X point-in-polygon join (include/mosaic_gpu.h).
//
// Host-side responsibilities: argument validation with the reference's error
// classes, chip-table construction (WKB -> SoA + cell hash, one device blob),
// workspace management and kernel launches.  No computation on the data path
// happens here; every per-point operation runs in kernels.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <unordered_map>
#include <unordered_set>
#include <chrono>
#include <sched.h>
#include <array>
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <limits>
#include <string>
#include <map>
#include <functional>
#include <tuple>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/mosaic_arrow.h"
#include "../../include/mosaic_gpu.h"
#include "bng_core.h"
#include "chip_table.h"
#include "error.h"
#include "h3_core.h"
#include "kernels.h"
#include "parallel.h"
#include "pip_core.h"
#include "raster.h"
#include "wkb.h"
#include "capi_internal.h"
#include "geom_decode.h"
#include "h3_glibc.h"
#include "h3_boundary.h"

namespace {

thread_local std::string g_err;

int32_t fail(int32_t code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                          \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess) return fail(MGPU_E_DEVICE, "%s: %s", #expr, hipGetErrorString(_e)); \
  } while (0)

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// The chip-table blob is self-describing: a header at offset 0 records the array
// offsets, so a byte copy of the blob on another GPU (RCCL broadcast) is a
// complete chip table there.
constexpr uint64_t kBlobMagic = 0x4d4f534149434850ULL;  // "MOSAICHP"
constexpr int kBlobArrays = 29;
constexpr uint32_t kBlobVersion = 13;  // 12: BNG cell answer grids; 13: palette-compressed second level
struct BlobHeader {
  uint64_t magic;
  uint32_t version, hash_mask, max_probe, n_chips, n_cells;
  int32_t index_system;  // MGPU_H3 / MGPU_BNG: the system the chip cells belong to
  int64_t n_vertices;
  uint64_t off[kBlobArrays];
  int32_t probe_mode, res;
  uint32_t face_mask, pad2;
  double bbox[4];
  double k_res;
  mgpu::DenseFace dense[20];
  uint32_t bng_edge, pad3;
  double bng_inv_edge;
  int32_t raster_mode;
  uint32_t raster_nx, raster_ny, raster_pix;
  int32_t raster_px0, raster_py0;
  double raster_x0, raster_y0, raster_inv_dx, raster_inv_dy;
  uint64_t blob_bytes;  // the whole blob (header included)
  uint32_t max_cell_chips, pad4;
  uint32_t raster_pc[4];
  uint32_t raster_sub_n, raster_sub_w;
  uint32_t raster_bshift, raster_bnx, raster_bny, raster_ncls;
  uint32_t raster_band_shift, raster_nband;
  uint32_t cell_ans_g, cell_ans_sw;
  uint32_t raster_pal, pad5;  // 1: the second level is palette-compressed
};
constexpr size_t kBlobHeaderBytes = 1024;
static_assert(sizeof(BlobHeader) <= kBlobHeaderBytes, "header too large");

mgpu::ChipTableView view_from_header(const BlobHeader& h, uint8_t* base) {
  mgpu::ChipTableView v;
  v.slots = (const mgpu::HashSlot*)(base + h.off[0]);
  v.hash_mask = h.hash_mask;
  v.max_probe = h.max_probe;
  v.n_chips = h.n_chips;
  v.n_cells = h.n_cells;
  v.chip_poly = (const int32_t*)(base + h.off[1]);
  v.chip_flags = (const uint8_t*)(base + h.off[2]);
  v.chip_part = (const uint32_t*)(base + h.off[3]);
  v.chip_env = (const double*)(base + h.off[4]);
  v.chip_row = (const int64_t*)(base + h.off[5]);
  v.part_ring = (const uint32_t*)(base + h.off[6]);
  v.ring_vtx = (const uint32_t*)(base + h.off[7]);
  v.ring_env = (const double*)(base + h.off[8]);
  v.vtx = (const double*)(base + h.off[9]);
  v.row_to_chip = (const uint32_t*)(base + h.off[10]);
  v.chip_strip = (const uint32_t*)(base + h.off[11]);
  v.chip_sy = (const double*)(base + h.off[12]);
  v.strip_edge = (const uint32_t*)(base + h.off[13]);
  v.edges = (const double*)(base + h.off[14]);
  v.edge_ring = (const uint8_t*)(base + h.off[15]);
  v.chip_hdr = (const mgpu::ChipHdr*)(base + h.off[16]);
  v.grid = (const uint64_t*)(base + h.off[17]);
  for (int f = 0; f < 20; f++) v.dense[f] = h.dense[f];
  v.probe_mode = h.probe_mode;
  v.res = h.res;
  v.face_mask = h.face_mask;
  for (int k = 0; k < 4; k++) v.bbox[k] = h.bbox[k];
  v.k_res = h.k_res;
  v.bng_edge = h.bng_edge;
  v.bng_inv_edge = h.bng_inv_edge;
  v.max_cell_chips = h.max_cell_chips;
  v.raster_mode = h.raster_mode;
  v.raster_nx = h.raster_nx;
  v.raster_ny = h.raster_ny;
  v.raster_pix = h.raster_pix;
  v.raster_px0 = h.raster_px0;
  v.raster_py0 = h.raster_py0;
  v.raster_x0 = h.raster_x0;
  v.raster_y0 = h.raster_y0;
  v.raster_inv_dx = h.raster_inv_dx;
  v.raster_inv_dy = h.raster_inv_dy;
  for (int k = 0; k < 4; k++) v.raster_pc[k] = h.raster_pc[k];
  v.raster = (const uint16_t*)(base + h.off[18]);
  v.raster_cls = (const uint64_t*)(base + h.off[19]);
  v.raster_sub_n = h.raster_sub_n;
  v.raster_sub_w = h.raster_sub_w;
  v.raster_band_shift = h.raster_band_shift;
  v.raster_nband = h.raster_nband;
  v.raster_band = h.raster_nband ? (const uint32_t*)(base + h.off[24]) : nullptr;
  v.raster_rank = h.raster_sub_n && !h.raster_nband ? (const mgpu::RankWord*)(base + h.off[20]) : nullptr;
  v.cell_ans_g = h.cell_ans_g;
  v.cell_ans_sw = h.cell_ans_sw;
  v.cell_ans_inv_sw = h.cell_ans_sw ? 1.0 / h.cell_ans_sw : 0.0;
  v.cell_ans_row = h.cell_ans_g ? (const uint32_t*)(base + h.off[25]) : nullptr;
  v.cell_ans = (const uint16_t*)(base + h.off[26]);
  v.raster_sub = (const uint16_t*)(base + h.off[21]);
  v.raster_pal = h.raster_pal ? (const uint64_t*)(base + h.off[27]) : nullptr;
  v.raster_idx2 = (const uint8_t*)(base + h.off[28]);
  v.raster_bshift = h.raster_bshift;
  v.raster_bnx = h.raster_bnx;
  v.raster_bny = h.raster_bny;
  v.raster_blk = h.raster_bshift ? (const uint16_t*)(base + h.off[22]) : nullptr;
  v.raster_ncls = h.raster_ncls;
  v.raster_cls_poly = (const int32_t*)(base + h.off[23]);
  return v;
}

// BNG dense probing.  For one resolution r (nPositions p, BNGIndexSystem.scala:
// 284-298, encode :540-553) a cell id is 10^(2p+3) + eLetter 10^(2p+1) + nLetter
// 10^(2p-1) + eBin 10^p + nBin 10 + quadrant with eBin, nBin < 10^(p-1): for whole-metre
// eastings / northings in [0, 1e7) (letters < 100, ids < 2^53) it is a bijection of
// (column, row) = (e / edge, n / edge), edge = the cell edge (halved for the quadrant
// resolutions r <= -2, whose quadrant digit is the column / row parity).  Every chip
// cell is decoded and re-encoded by point_to_cell at its centre; any cell that does
// not round-trip (negative coordinates, mixed resolutions, r = -1) keeps the hash.
bool build_bng_dense(const std::vector<mgpu::HashSlot>& cells, int32_t* res_out, mgpu::DenseFace* D,
                     uint32_t* edge_out, std::vector<uint64_t>& grid) {
  if (cells.empty()) return false;
  auto p10 = [](int k) {
    int64_t v = 1;
    while (k-- > 0) v *= 10;
    return v;
  };
  int p = -1;
  for (int q = 1; q <= 6; q++)
    if ((int64_t)cells[0].cell >= p10(2 * q + 3) && (int64_t)cells[0].cell < 2 * p10(2 * q + 3)) p = q;
  if (p < 0) return false;
  const bool quad = cells[0].cell % 10 != 0;
  if (quad && p > 5) return false;
  const int res = quad ? -(p + 1) : p;
  const int64_t d = p10(6 - p);  // metres per (column, row) of the id's bins
  const int64_t edge = quad ? d / 2 : d;
  const int64_t B = p10(p - 1);
  std::vector<std::pair<int64_t, int64_t>> cr(cells.size());
  int64_t c0 = INT64_MAX, c1 = INT64_MIN, r0 = INT64_MAX, r1 = INT64_MIN;
  for (size_t k = 0; k < cells.size(); k++) {
    const int64_t id = (int64_t)cells[k].cell;
    int64_t rem = id - p10(2 * p + 3);
    if (rem < 0 || rem >= p10(2 * p + 3)) return false;
    const int64_t eL = rem / p10(2 * p + 1);
    rem %= p10(2 * p + 1);
    const int64_t nL = rem / p10(2 * p - 1);
    rem %= p10(2 * p - 1);
    const int64_t eB = rem / p10(p);
    rem %= p10(p);
    const int64_t nB = rem / 10, q = rem % 10;
    if (eB >= B || nB >= B || (quad ? (q < 1 || q > 4) : q != 0)) return false;
    int64_t col = eL * B + eB, row = nL * B + nB;
    if (quad) col = 2 * col + (q == 3 || q == 4), row = 2 * row + (q == 2 || q == 3);
    int64_t back = 0;
    mgpu::bng::point_to_cell((col + 0.5) * (double)edge, (row + 0.5) * (double)edge, res, &back);
    if (back != id || (col + 1) * edge > 10000000 || (row + 1) * edge > 10000000) return false;
    cr[k] = {col, row};
    c0 = std::min(c0, col), c1 = std::max(c1, col), r0 = std::min(r0, row), r1 = std::max(r1, row);
  }
  const int64_t total = (c1 - c0 + 1) * (r1 - r0 + 1);
  if (total > std::max<int64_t>(16 * (int64_t)cells.size(), 1 << 20) || total > (1LL << 26)) return false;
  memset(D, 0, sizeof(mgpu::DenseFace));
  D->a0 = (int32_t)c0;
  D->b0 = (int32_t)r0;
  D->w = (uint32_t)(c1 - c0 + 1);
  D->h = (uint32_t)(r1 - r0 + 1);
  D->base = 0;
  grid.assign((size_t)total, 0);
  for (size_t k = 0; k < cells.size(); k++) {
    const mgpu::HashSlot& e = cells[k];
    grid[(size_t)((cr[k].second - r0) * D->w + (cr[k].first - c0))] =
        (uint64_t)e.first | ((uint64_t)e.count << 32) | ((uint64_t)e.core_mask << 48);
  }
  *res_out = res;
  *edge_out = (uint32_t)edge;
  return true;
}

constexpr double kPi = 3.14159265358979323846;

double angle_between(const double* a, const double* b) {
  double d = a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
  d = d > 1 ? 1 : (d < -1 ? -1 : d);
  return acos(d);
}

// H3 lattice probing (chip_table.h).  For every distinct chip cell: its centre (home
// face lattice -> sphere), every face a point of the cell can be nearest to (angle
// within 3 rho of the nearest, rho = circumradius bound), and on each such face the
// lattice positions within hex distance 3 of the centre's projection whose
// face_ijk_to_h3 IS the cell.  Points outside the chip cells' bounding box match
// nothing; inside it, only faces that can be nearest somewhere in the box are
// tested (65 x 65 sampling with a 2-Lipschitz margin).  Returns false (caller keeps
// cell-id probing) for mixed resolutions, res < 5, or pentagon base cells.
// H3's maxDimByCIIres: the face triangle at Class II resolution r is normalized
// i + j + k <= this
constexpr int64_t kMaxDimCII[17] = {2, -1, 14, -1, 98, -1, 686, -1, 4802, -1, 33614, -1, 235298, -1, 1647086, -1, 11529602};

bool build_lattice(const std::vector<mgpu::HashSlot>& cells, std::vector<std::pair<uint64_t, uint32_t>>& keys,
                   int* res_out, uint32_t* face_mask, double bbox[4], std::vector<uint8_t>* interior_out = nullptr) {
  namespace H = mgpu::h3;
  if (cells.empty()) return false;
  int res = (int)((cells[0].cell >> 52) & 15);
  if (res < 5) return false;
  const double rho = 0.3 / pow(H::kSqrt7, res);
  double k_res = H::k_of_res(res);
  // cells are independent: per-thread key lists and extents, merged afterwards (the
  // caller sorts the keys, so the merge order does not matter)
  if (interior_out) interior_out->assign(cells.size(), 0);
  const int64_t grain = 4096;
  const int T = mgpu::parallel_slots((int64_t)cells.size(), grain);
  std::vector<std::vector<std::pair<uint64_t, uint32_t>>> tkeys(T);
  std::vector<std::array<double, 4>> text(T, std::array<double, 4>{1e9, -1e9, 1e9, -1e9});
  std::atomic<bool> bad{false};
  mgpu::parallel_for((int64_t)cells.size(), grain, [&](int64_t cb, int64_t ce, int t) {
    auto& tk = tkeys[t];
    auto& ex = text[t];
    for (int64_t ci = cb; ci < ce; ci++) {
      uint64_t h = cells[ci].cell;
      if (((h >> 59) & 15) != 1 || (int)((h >> 52) & 15) != res || (h >> 63)) {
        bad = true;
        return;
      }
      int face, r;
      H::IJK ijk;
      if (!H::h3_home_face_ijk(h, &face, &ijk, &r)) {
        bad = true;
        return;
      }
      double hx, hy, lat, lon;
      H::ijk_to_hex2d(ijk, &hx, &hy);
      H::hex2d_to_geo(hx, hy, face, res, &lat, &lon);
      double v[3] = {cos(lat) * cos(lon), cos(lat) * sin(lon), sin(lat)};
      // faces within 3 rho of the nearest face centre, by dot products (angle <= amin + 3
      // rho  <=>  dot >= cos(amin + 3 rho): one acos and one cos per cell instead of 20 acos)
      double dot[20], dmax = -2.0;
      for (int f = 0; f < 20; f++) {
        const double* c = H3T_FACE_CENTER_POINT[f];
        dot[f] = v[0] * c[0] + v[1] * c[1] + v[2] * c[2];
        dmax = std::max(dmax, dot[f]);
      }
      const double amin = acos(std::min(1.0, std::max(-1.0, dmax)));
      const double cthr = cos(std::min(kPi, amin + 3 * rho));
      // a cell deep inside its home face (the only face within 3 rho, every lattice
      // position within hex distance 3 of its own strictly inside the face triangle --
      // normalized i + j + k below the face's maxDim, for Class III compared after the
      // aperture-7 step to the next Class II resolution, which at most quadruples the sum)
      // is reached at its own position only: positions inside one face are distinct cells
      int near = 0;
      for (int f = 0; f < 20; f++) near += dot[f] >= cthr;
      const int64_t sum = (int64_t)ijk.i + ijk.j + ijk.k;
      const bool interior = near == 1 && dot[face] >= cthr &&
                            ((res & 1) ? 4 * (sum + 6) < kMaxDimCII[res + 1] : sum + 6 < kMaxDimCII[res]);
      if (interior) tk.push_back({H::lattice_key(face, ijk), (uint32_t)ci});
      if (interior_out) (*interior_out)[ci] = interior ? 1 : 0;
      for (int f = 0; f < 20 && !interior; f++) {
        if (dot[f] < cthr) continue;
        const double(*F)[3] = H3T_FACE_FRAME[f][res & 1];
        double dc = v[0] * F[2][0] + v[1] * F[2][1] + v[2] * F[2][2];
        if (dc <= 0.5) continue;
        double x = k_res * (v[0] * F[0][0] + v[1] * F[0][1] + v[2] * F[0][2]) / dc;
        double y = k_res * (v[0] * F[1][0] + v[1] * F[1][1] + v[2] * F[1][2]) / dc;
        double mg;
        H::IJK c0 = H::hex2d_to_ijk(x, y, &mg);
        int i0 = c0.i - c0.k, j0 = c0.j - c0.k;
        for (int di = -3; di <= 3; di++)
          for (int dj = -3; dj <= 3; dj++) {
            if (std::abs(di) + std::abs(dj) + std::abs(di - dj) > 6) continue;  // hex distance <= 3
            H::IJK n{i0 + di, j0 + dj, 0};
            H::ijk_normalize(n);
            if (H::face_ijk_to_h3(f, n, res) == h) tk.push_back({H::lattice_key(f, n), (uint32_t)ci});
          }
      }
      double latd = lat * 180 / kPi, lond = lon * 180 / kPi;
      ex[0] = std::min(ex[0], latd);
      ex[1] = std::max(ex[1], latd);
      ex[2] = std::min(ex[2], lond);
      ex[3] = std::max(ex[3], lond);
    }
  });
  if (bad) return false;
  double lat_lo = 1e9, lat_hi = -1e9, lon_lo = 1e9, lon_hi = -1e9;
  for (int t = 0; t < T; t++) {
    keys.insert(keys.end(), tkeys[t].begin(), tkeys[t].end());
    lat_lo = std::min(lat_lo, text[t][0]);
    lat_hi = std::max(lat_hi, text[t][1]);
    lon_lo = std::min(lon_lo, text[t][2]);
    lon_hi = std::max(lon_hi, text[t][3]);
  }
  // bounding box of every chip cell (centre +- 2 rho), or the whole sphere
  double m = 2 * rho * 180 / kPi;
  double latmax = std::max(std::fabs(lat_lo), std::fabs(lat_hi)) + m;
  if (latmax < 80.0 && lon_hi - lon_lo < 180.0) {
    double ml = m / cos(latmax * kPi / 180);
    bbox[0] = lon_lo - ml;
    bbox[1] = lat_lo - m;
    bbox[2] = lon_hi + ml;
    bbox[3] = lat_hi + m;
    // faces that can be nearest somewhere in the box
    const int G = 65;
    double s_ang = 0;
    uint32_t mask = 0;
    std::vector<double> pts;
    for (int a = 0; a < G; a++)
      for (int b = 0; b < G; b++) {
        double lond = bbox[0] + (bbox[2] - bbox[0]) * a / (G - 1), latd = bbox[1] + (bbox[3] - bbox[1]) * b / (G - 1);
        double la = latd * kPi / 180, lo = lond * kPi / 180;
        pts.push_back(cos(la) * cos(lo));
        pts.push_back(cos(la) * sin(lo));
        pts.push_back(sin(la));
      }
    // sample spacing (angle) bound: the box diagonal cell
    {
      double la0 = bbox[1] * kPi / 180, lo0 = bbox[0] * kPi / 180;
      double la1 = (bbox[1] + (bbox[3] - bbox[1]) / (G - 1)) * kPi / 180,
             lo1 = (bbox[0] + (bbox[2] - bbox[0]) / (G - 1)) * kPi / 180;
      double p0[3] = {cos(la0) * cos(lo0), cos(la0) * sin(lo0), sin(la0)};
      double p1[3] = {cos(la1) * cos(lo1), cos(la1) * sin(lo1), sin(la1)};
      s_ang = angle_between(p0, p1);
      // the equator-side rows are wider: scale by the cosine ratio
      s_ang /= std::max(0.05, cos(latmax * kPi / 180) / std::max(cos(bbox[1] * kPi / 180), cos(bbox[3] * kPi / 180)));
    }
    for (size_t q = 0; q < pts.size(); q += 3) {
      double ang[20], amin = 1e9;
      for (int f = 0; f < 20; f++) {
        ang[f] = angle_between(&pts[q], H3T_FACE_CENTER_POINT[f]);
        amin = std::min(amin, ang[f]);
      }
      for (int f = 0; f < 20; f++)
        if (ang[f] <= amin + 2 * s_ang + 1e-12) mask |= 1u << f;
    }
    *face_mask = mask;
  } else {
    bbox[0] = -1e300;
    bbox[1] = -1e300;
    bbox[2] = 1e300;
    bbox[3] = 1e300;
    *face_mask = (1u << 20) - 1;
  }
  *res_out = res;
  return true;
}

// Strip index of the border chips (chip_table.h "strips"): for chip c with E edges,
// S = clamp(E / 2, 1, kMaxStrips) equal strips over its envelope's y-range; edge e
// (p1 = ring[i], p2 = ring[i-1], as RayCrossingCounter visits it) is listed in the
// strips strip_of(min y) .. strip_of(max y) -- the same function the kernel applies
// to the point, so a point whose y lies in the edge's closed y-range always finds
// the edge in its strip.
// An allocator whose resize() leaves new elements uninitialised (the builders write every
// element, in parallel; a zero-filling resize of a GB-sized array is a serial pass).
// the builder's per-chip arrays (huge_alloc.h)
template <class T>
using HVec = std::vector<T, mgpu::HugeAlloc<T>>;
template <class T>
struct NoInit : mgpu::HugeAlloc<T> {
  template <class U>
  struct rebind {
    using other = NoInit<U>;
  };
  NoInit() = default;
  template <class U>
  NoInit(const NoInit<U>&) {}
  template <class U>
  void construct(U* p) noexcept {
    ::new ((void*)p) U;
  }
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    ::new ((void*)p) U(std::forward<A>(a)...);
  }
};

struct Strips {
  HVec<uint32_t> chip_strip;
  HVec<double> chip_sy;
  HVec<uint32_t> strip_edge{0};
  std::vector<double, NoInit<double>> edges;
  HVec<uint8_t> edge_ring;
};

void build_strips(int64_t n_chips, HVec<uint8_t>& cflags, const HVec<uint32_t>& cpart,
                  const HVec<double>& cenv, const mgpu::wkb::Flat& geo, Strips& st, int64_t G) {
  st.chip_strip.assign(n_chips + 1, 0);
  st.chip_sy.assign(2 * (size_t)n_chips, 0.0);
  // chunks of G chips in parallel, each into its own strip / edge lists (chip_strip then
  // local), concatenated with the offsets shifted
  const int64_t NC = (n_chips + G - 1) / G;
  std::vector<Strips> cs(NC);
  mgpu::parallel_for(NC, 1, [&](int64_t kb, int64_t ke, int) {
    // (per chip: each edge's strip range, a count per strip, then the edges placed by a
    // counting sort -- no per-strip vectors)
    std::vector<uint32_t> cnt, pos;
    for (int64_t kc = kb; kc < ke; kc++) {
      Strips& L = cs[kc];
      for (int64_t c = kc * G; c < std::min(n_chips, (kc + 1) * G); c++) {
        st.chip_strip[c] = (uint32_t)(L.strip_edge.size() - 1);
        uint8_t fl = cflags[c];
        if (fl & (mgpu::kChipCore | mgpu::kChipEmpty | mgpu::kChipNoGeom | mgpu::kChipRect)) {
          if (!(fl & (mgpu::kChipEmpty | mgpu::kChipNoGeom | mgpu::kChipRect))) cflags[c] |= mgpu::kChipNoStrips;
          continue;
        }
        const uint32_t r0 = geo.part_ring[cpart[c]], r1 = geo.part_ring[cpart[c + 1]];
        if (r1 - r0 > (uint32_t)mgpu::kStripRings) {
          cflags[c] |= mgpu::kChipNoStrips;
          continue;
        }
        int64_t E = 0;
        for (uint32_t r = r0; r < r1; r++) {
          uint32_t nv = geo.ring_vtx[r + 1] - geo.ring_vtx[r];
          if (nv >= 2) E += nv - 1;
        }
        int S = (int)std::min<int64_t>(mgpu::kMaxStrips, std::max<int64_t>(1, E / 2));
        const double y0 = cenv[4 * c + 1], H = cenv[4 * c + 3] - y0;
        if (!(H > 0)) S = 1;
        const double inv_h = (H > 0) ? (double)S / H : 0.0;
        st.chip_sy[2 * c] = y0;
        st.chip_sy[2 * c + 1] = inv_h;
        // (two passes over the chip's edges: counts per strip, then each edge placed in
        // every strip it spans -- in ring order within each strip)
        cnt.assign(S + 1, 0);
        for (uint32_t r = r0; r < r1; r++) {
          const uint32_t vb = geo.ring_vtx[r], ve = geo.ring_vtx[r + 1];
          for (uint32_t i = vb + 1; i < ve; i++) {
            const double p1y = geo.vtx[2 * i + 1], p2y = geo.vtx[2 * i - 1];
            const int sa = mgpu::strip_of(std::min(p1y, p2y), y0, inv_h, S);
            const int sb = mgpu::strip_of(std::max(p1y, p2y), y0, inv_h, S);
            for (int q = sa; q <= sb; q++) cnt[q + 1]++;
          }
        }
        for (int q = 0; q < S; q++) cnt[q + 1] += cnt[q];
        const size_t e_base = L.edge_ring.size();
        L.edges.resize(4 * (e_base + cnt[S]));
        L.edge_ring.resize(e_base + cnt[S]);
        pos.assign(cnt.begin(), cnt.end() - 1);
        for (uint32_t r = r0; r < r1; r++) {
          const uint32_t vb = geo.ring_vtx[r], ve = geo.ring_vtx[r + 1];
          for (uint32_t i = vb + 1; i < ve; i++) {
            const double p1x = geo.vtx[2 * i], p1y = geo.vtx[2 * i + 1];
            const double p2x = geo.vtx[2 * i - 2], p2y = geo.vtx[2 * i - 1];
            const int sa = mgpu::strip_of(std::min(p1y, p2y), y0, inv_h, S);
            const int sb = mgpu::strip_of(std::max(p1y, p2y), y0, inv_h, S);
            for (int q = sa; q <= sb; q++) {
              const size_t d = e_base + pos[q]++;
              double* o = L.edges.data() + 4 * d;
              o[0] = p1x, o[1] = p1y, o[2] = p2x, o[3] = p2y;
              L.edge_ring[d] = (uint8_t)(r - r0);
            }
          }
        }
        for (int q = 0; q < S; q++) L.strip_edge.push_back((uint32_t)(e_base + cnt[q + 1]));
      }
    }
  });
  std::vector<size_t> s0(NC + 1, 0), e0(NC + 1, 0);
  for (int64_t k = 0; k < NC; k++) {
    s0[k + 1] = s0[k] + cs[k].strip_edge.size() - 1;
    e0[k + 1] = e0[k] + cs[k].edge_ring.size();
  }
  st.strip_edge.assign(s0[NC] + 1, 0);
  st.edges.resize(4 * e0[NC]);
  st.edge_ring.resize(e0[NC]);
  mgpu::parallel_for(NC, 1, [&](int64_t kb, int64_t ke, int) {
    for (int64_t k = kb; k < ke; k++) {
      const Strips& L = cs[k];
      for (size_t q = 1; q < L.strip_edge.size(); q++) st.strip_edge[s0[k] + q] = (uint32_t)(L.strip_edge[q] + e0[k]);
      std::copy(L.edges.begin(), L.edges.end(), st.edges.begin() + 4 * e0[k]);
      std::copy(L.edge_ring.begin(), L.edge_ring.end(), st.edge_ring.begin() + e0[k]);
      for (int64_t c = k * G; c < std::min(n_chips, (k + 1) * G); c++) st.chip_strip[c] += (uint32_t)s0[k];
    }
  });
  st.chip_strip[n_chips] = (uint32_t)s0[NC];
}

// Does segment a-b meet the closed box [x0, x1] x [y0, y1]?  (The callers widen the
// box by a margin that dwarfs the rounding of this test.)
bool seg_hits_box(double ax, double ay, double bx, double by, double x0, double y0, double x1, double y1) {
  if (std::max(ax, bx) < x0 || std::min(ax, bx) > x1 || std::max(ay, by) < y0 || std::min(ay, by) > y1) return false;
  const double dx = bx - ax, dy = by - ay;
  const double cx[4] = {x0, x1, x0, x1}, cy[4] = {y0, y0, y1, y1};
  int pos = 0, neg = 0;
  for (int k = 0; k < 4; k++) {
    const double cr = dx * (cy[k] - ay) - dy * (cx[k] - ax);
    pos += cr > 0;
    neg += cr < 0;
  }
  return !(pos == 4 || neg == 4);
}

// Classification grid of chip c (chip_table.h ChipHdr): cell state 2 where a widened
// cell rectangle meets an edge, else the PointLocator's verdict at the cell centre.
void build_grid(const mgpu::ChipTableView& hv, uint32_t c, const mgpu::wkb::Flat& geo, mgpu::ChipHdr& h) {
  using namespace mgpu;
  const double e0 = h.env[0], e1 = h.env[1], e2 = h.env[2], e3 = h.env[3];
  const double W = e2 - e0, H = e3 - e1;
  h.sx = W > 0 ? kGrid / W : 0.0;
  h.sy = H > 0 ? kGrid / H : 0.0;
  uint8_t st[kGrid][kGrid];
  memset(st, 0xFF, sizeof st);  // 0xFF: not yet known
  if (!(W > 0) || !(H > 0)) {
    for (int gy = 0; gy < kGrid; gy++) h.grid[gy] = 0xAAAAAAAAu;  // all mixed
    return;
  }
  // margin in cell units: far above the rounding of grid_index and of this test
  const double mag = std::max(std::max(std::fabs(e0), std::fabs(e2)), std::max(std::fabs(e1), std::fabs(e3)));
  const double ulp = std::nextafter(mag, INFINITY) - mag;
  const double mu_x = 1e-6 + 64 * ulp * h.sx, mu_y = 1e-6 + 64 * ulp * h.sy;
  const uint32_t r0 = hv.part_ring[hv.chip_part[c]], r1 = hv.part_ring[hv.chip_part[c + 1]];
  // the widened cells' bounds, once per chip (the same expressions as per cell)
  double bx0[kGrid], bx1[kGrid], by0[kGrid], by1[kGrid];
  for (int g = 0; g < kGrid; g++) {
    bx0[g] = e0 + (g - mu_x) / h.sx, bx1[g] = e0 + (g + 1 + mu_x) / h.sx;
    by0[g] = e1 + (g - mu_y) / h.sy, by1[g] = e1 + (g + 1 + mu_y) / h.sy;
  }
  for (uint32_t r = r0; r < r1; r++) {
    for (uint32_t i = geo.ring_vtx[r] + 1; i < geo.ring_vtx[r + 1]; i++) {
      const double ax = geo.vtx[2 * i - 2], ay = geo.vtx[2 * i - 1], bx = geo.vtx[2 * i], by = geo.vtx[2 * i + 1];
      // candidate cells: the segment's bounding box, one cell of slack each way
      int gx0 = (int)std::floor((std::min(ax, bx) - e0) * h.sx) - 1, gx1 = (int)std::floor((std::max(ax, bx) - e0) * h.sx) + 1;
      int gy0 = (int)std::floor((std::min(ay, by) - e1) * h.sy) - 1, gy1 = (int)std::floor((std::max(ay, by) - e1) * h.sy) + 1;
      gx0 = std::max(gx0, 0), gy0 = std::max(gy0, 0), gx1 = std::min(gx1, kGrid - 1), gy1 = std::min(gy1, kGrid - 1);
      // seg_hits_box per cell (cell gx spans [e0 + gx / sx, e0 + (gx + 1) / sx]; the
      // clamped last cell also takes everything up to the envelope edge), its terms
      // dy (cx - ax) per column and dx (cy - ay) per row computed once: the same roundings
      const double dx = bx - ax, dy = by - ay;
      const double lx = std::min(ax, bx), hx = std::max(ax, bx), ly = std::min(ay, by), hy = std::max(ay, by);
      double tx0[kGrid], tx1[kGrid];
      bool cok[kGrid];
      for (int gx = gx0; gx <= gx1; gx++) {
        cok[gx] = !(hx < bx0[gx] || lx > bx1[gx]);
        tx0[gx] = dy * (bx0[gx] - ax);
        tx1[gx] = dy * (bx1[gx] - ax);
      }
      for (int gy = gy0; gy <= gy1; gy++) {
        if (hy < by0[gy] || ly > by1[gy]) continue;
        const double u0 = dx * (by0[gy] - ay), u1 = dx * (by1[gy] - ay);
        for (int gx = gx0; gx <= gx1; gx++) {
          if (st[gy][gx] == kCellMixed || !cok[gx]) continue;
          const double c0 = u0 - tx0[gx], c1 = u0 - tx1[gx], c2 = u1 - tx0[gx], c3 = u1 - tx1[gx];
          const int pos = (c0 > 0) + (c1 > 0) + (c2 > 0) + (c3 > 0), neg = (c0 < 0) + (c1 < 0) + (c2 < 0) + (c3 < 0);
          if (!(pos == 4 || neg == 4)) st[gy][gx] = kCellMixed;
        }
      }
    }
  }
  // The rest: PointLocator's verdict at the cell centre, which lies at a positive distance
  // from every edge (its widened cell meets none), so RayCrossingCounter's per-ring
  // crossing parity there is the count of the ring's edges that straddle the centre's
  // row (half-open, as countSegment) and cross it to the right of the centre -- computed
  // per row for the row's 16 centres at once instead of a ring walk per centre.  A part
  // is entered when its shell's parity is odd and no hole's is; the chip when some part
  // is (a point on no boundary: the Mod-2 rule does not arise).
  // (per row: each ring's parity as a 16-column mask -- a crossing at x flips the
  // columns whose centre lies left of x, a prefix as the centres ascend)
  double cxp[kGrid];
  for (int gx = 0; gx < kGrid; gx++) cxp[gx] = e0 + (gx + 0.5) / h.sx;
  uint32_t par[kStripRings];
  const uint32_t p0 = hv.chip_part[c], p1 = hv.chip_part[c + 1];
  for (int gy = 0; gy < kGrid; gy++) {
    uint32_t row = 0;
    bool any = false;
    for (int gx = 0; gx < kGrid && !any; gx++) any = st[gy][gx] != kCellMixed;
    if (any) {
      const double cyp = e1 + (gy + 0.5) / h.sy;
      for (uint32_t r = r0; r < r1; r++) {
        uint32_t m = 0;
        for (uint32_t i = geo.ring_vtx[r] + 1; i < geo.ring_vtx[r + 1]; i++) {
          const double p1x = geo.vtx[2 * i], p1y = geo.vtx[2 * i + 1], p2x = geo.vtx[2 * i - 2], p2y = geo.vtx[2 * i - 1];
          if (((p1y > cyp) && (p2y <= cyp)) || ((p2y > cyp) && (p1y <= cyp))) {
            const double x = p1x + (cyp - p1y) * (p2x - p1x) / (p2y - p1y);
            int k = 0;
            while (k < kGrid && cxp[k] < x) k++;
            m ^= (1u << k) - 1u;
          }
        }
        par[r - r0] = m;
      }
      uint32_t in = 0;
      for (uint32_t p = p0; p < p1; p++) {
        const uint32_t rb = hv.part_ring[p], re = hv.part_ring[p + 1];
        if (re == rb || geo.ring_vtx[rb + 1] == geo.ring_vtx[rb]) continue;
        uint32_t holes = 0;
        for (uint32_t q = rb + 1; q < re; q++) holes |= par[q - r0];
        in |= par[rb - r0] & ~holes;
      }
      for (int gx = 0; gx < kGrid; gx++) {
        uint32_t v = st[gy][gx];
        if (v != kCellMixed) {
          v = ((in >> gx) & 1u) ? kCellIn : kCellOut;
#ifdef MGPU_GRID_VERIFY
          const int loc = pip::chip_locate(hv, c, cxp[gx], cyp);
          if (loc != (((in >> gx) & 1u) ? pip::kInterior : pip::kExterior)) {
            fprintf(stderr, "grid verify: chip %u cell (%d, %d) row parity %d, PointLocator %d\n", c, gx, gy, (int)((in >> gx) & 1u), loc);
            abort();
          }
#endif
        }
        row |= v << (2 * gx);
      }
    }
    h.grid[gy] = any ? row : 0xAAAAAAAAu;
  }
}

// ------------------------------------------------------------------ pixel index
// (chip_table.h "Pixel index").  A pixel gets a class only when its answer is the same
// for every point in it, by a certificate with margins that dwarf rounding:
//  1. one chip cell: H3 -- the four corners of the (widened) pixel are nearest to the
//     same icosahedron face with a squared-chord gap above delta_f, and take the same
//     decision path of _hex2dToCoordIJK (same (m1, m2), same branch outcomes, same
//     quadrant signs) with every compared quantity at least delta_h from its
//     threshold.  Each path's region is an intersection of half-planes of the face's
//     gnomonic plane (the face choice likewise: v.(c_g - c_f) >= 0 per face g), hence
//     convex; the pixel's image there lies within the sagitta of its parallels of the
//     corners' hull (meridians are straight lines), and delta_h, delta_f are taken 8x
//     above that bound -- so every point of the pixel takes the corners' cell, in exact
//     arithmetic and in the reference's (its error is ~1e-12 of a hex unit).  BNG --
//     pixels tile the cells exactly (the pixel edge divides the cell edge, whole metres).
//  2. each chip of that cell: core -> match; else no chip edge meets the widened pixel
//     (seg_hits_box, the classification grid's test), so all its points lie in one
//     component of the plane minus the chip boundary, where JTS's PointLocator returns
//     the verdict of the pixel centre (interior -> match).
// Anything else is kPixMixed and takes the full path in the kernel.
// the second level's rank table over the (ascending) mixed pixels of an n-pixel raster
static void mixed_rank(const std::vector<uint32_t>& mixed, size_t n, std::vector<mgpu::RankWord>& rank) {
  rank.assign((n + 31) / 32, mgpu::RankWord{0, 0});
  for (uint32_t p : mixed) rank[p >> 5].bits |= 1u << (p & 31);
  uint32_t c = 0;
  for (auto& w : rank) {
    w.base = c;
    c += (uint32_t)__builtin_popcount(w.bits);
  }
}

struct Raster {
  int32_t mode = mgpu::kRasterNone;
  uint32_t nx = 0, ny = 0, pix = 0;
  int32_t px0 = 0, py0 = 0;
  double x0 = 0, y0 = 0, inv_dx = 0, inv_dy = 0;
  std::vector<uint16_t> cells;
  std::vector<uint64_t> cls;
  uint32_t pc[4] = {0, 0, 0, 0};
  // second level: ref[pixel] = 1 + block of a refined mixed pixel (0: none); block b's
  // sub_n x sub_n sub-pixel classes at sub[b * sub_n^2 ..] (BNG: sub-pixel edge sub_w metres)
  uint32_t sub_n = 0, sub_w = 0;
  std::vector<mgpu::RankWord> rank;
  std::vector<uint16_t, NoInit<uint16_t>> sub;
  // lonlat: band[k] = the refined pixels before raster rows k << band_shift (rank unused)
  uint32_t band_shift = 0;
  std::vector<uint32_t> band;
  // lonlat with bands, palette-compressed second level (raster_palette): per refined block
  // pal[b] = its <= 4 classes (16 bits each) or kPalFull | the index of its full block in
  // sub (which then keeps only those); idx2[b * sub_n^2 / 4 ..] = 2-bit palette indices
  std::vector<uint64_t> pal;
  std::vector<uint8_t> idx2;
  // blocks of 2^bshift x 2^bshift pixels: the class when all of them share it, else mixed
  uint32_t bshift = 0, bnx = 0, bny = 0;
  std::vector<uint16_t> blk;
  int64_t n_pure = 0;
};

constexpr int64_t kPixAnswerMixed = -1;

// the matches of every point in the widened pixel [x0, x1] x [y0, y1] among the chips
// of grid entry `e` (first | count << 32 | core_mask << 48): a mask, or kPixAnswerMixed
// (edges: when given, the chips' edges whose bounding boxes meet a box holding this one --
// the widened pixel of a sub-pixel -- per chip, filled on first use; an edge outside it
// cannot meet this box, so the answer is the same)
struct PixelEdges {
  std::vector<uint32_t> chip, start, items;  // chip k's edges (end vertex index) items[start[k] .. start[k + 1])
  // chip k's PointLocator verdict when no edge of it meets the box (-1: not yet computed):
  // the whole box then lies in one component of the plane minus the chip's boundary, where
  // the (exact) predicate gives every point the same answer
  std::vector<int> locate;
  // chip k with edges in the box, a sub-box none of them meets: the PointLocator verdict at
  // its centre from the rings' crossings of the centre's row (as build_grid: the centre
  // lies off every edge by far more than the rounding of a crossing), kept per row
  std::vector<double> row_y;
  std::vector<std::vector<double>> xs;
  std::vector<std::vector<uint32_t>> ring_first;
  double x0 = 0, y0 = 0, x1 = 0, y1 = 0;
  void reset(double a0, double b0, double a1, double b1) {
    chip.clear();
    start.assign(1, 0);
    items.clear();
    locate.clear();
    row_y.clear();
    x0 = a0, y0 = b0, x1 = a1, y1 = b1;
  }
};
int64_t pixel_answer(const mgpu::ChipTableView& hv, uint64_t e, double x0, double y0, double x1, double y1,
                     PixelEdges* pe = nullptr) {
  using namespace mgpu;
  const uint32_t first = (uint32_t)e, count = mgpu::grid_count(e, false);  // (before the answer grids)
  if (count == 0) return 0;
  if (count > 32) return kPixAnswerMixed;
  uint64_t mask = 0;
  for (uint32_t j = 0; j < count; j++) {
    const uint32_t c = first + j;
    const uint8_t fl = hv.chip_flags[c];
    if (fl & kChipCore) {
      mask |= 1ull << j;
      continue;
    }
    if (fl & (kChipEmpty | kChipNoGeom)) continue;
    const double* env = hv.chip_env + 4 * c;
    if (x1 < env[0] || x0 > env[2] || y1 < env[1] || y0 > env[3]) continue;  // outside the envelope
    if (pe) {
      size_t k = 0;
      while (k < pe->chip.size() && pe->chip[k] != c) k++;
      if (k == pe->chip.size()) {
        for (uint32_t p = hv.chip_part[c]; p < hv.chip_part[c + 1]; p++)
          for (uint32_t r = hv.part_ring[p]; r < hv.part_ring[p + 1]; r++)
            for (uint32_t i = hv.ring_vtx[r] + 1; i < hv.ring_vtx[r + 1]; i++) {
              const double ax = hv.vtx[2 * i - 2], ay = hv.vtx[2 * i - 1], bx = hv.vtx[2 * i], by = hv.vtx[2 * i + 1];
              if (!(std::max(ax, bx) < pe->x0 || std::min(ax, bx) > pe->x1 || std::max(ay, by) < pe->y0 ||
                    std::min(ay, by) > pe->y1))
                pe->items.push_back(i);
            }
        pe->chip.push_back(c);
        pe->start.push_back((uint32_t)pe->items.size());
        pe->locate.push_back(-1);
        pe->row_y.push_back(NAN);
        if (pe->xs.size() < pe->chip.size()) {
          pe->xs.resize(pe->chip.size());
          pe->ring_first.resize(pe->chip.size());
        }
      }
      for (uint32_t q = pe->start[k]; q < pe->start[k + 1]; q++) {
        const uint32_t i = pe->items[q];
        if (seg_hits_box(hv.vtx[2 * i - 2], hv.vtx[2 * i - 1], hv.vtx[2 * i], hv.vtx[2 * i + 1], x0, y0, x1, y1))
          return kPixAnswerMixed;
      }
      if (pe->start[k] == pe->start[k + 1]) {
        if (pe->locate[k] < 0) pe->locate[k] = pip::chip_locate(hv, c, 0.5 * (x0 + x1), 0.5 * (y0 + y1));
        const int loc = pe->locate[k];
        if (loc == pip::kBoundary) return kPixAnswerMixed;
        if (loc == pip::kInterior) mask |= 1ull << j;
        continue;
      }
      const double cxp = 0.5 * (x0 + x1), cyp = 0.5 * (y0 + y1);
      const uint32_t r0 = hv.part_ring[hv.chip_part[c]], r1 = hv.part_ring[hv.chip_part[c + 1]];
      std::vector<double>& xs = pe->xs[k];
      std::vector<uint32_t>& rf = pe->ring_first[k];
      if (!(pe->row_y[k] == cyp)) {
        pe->row_y[k] = cyp;
        xs.clear();
        rf.clear();
        for (uint32_t r = r0; r < r1; r++) {
          rf.push_back((uint32_t)xs.size());
          for (uint32_t i = hv.ring_vtx[r] + 1; i < hv.ring_vtx[r + 1]; i++) {
            const double p1x = hv.vtx[2 * i], p1y = hv.vtx[2 * i + 1], p2x = hv.vtx[2 * i - 2], p2y = hv.vtx[2 * i - 1];
            if (((p1y > cyp) && (p2y <= cyp)) || ((p2y > cyp) && (p1y <= cyp)))
              xs.push_back(p1x + (cyp - p1y) * (p2x - p1x) / (p2y - p1y));
          }
          std::sort(xs.begin() + rf.back(), xs.end());
        }
        rf.push_back((uint32_t)xs.size());
      }
      auto odd = [&](uint32_t r) {  // ring r (index within the chip): crossings right of cxp
        const auto b = xs.begin() + rf[r], e = xs.begin() + rf[r + 1];
        return ((e - std::upper_bound(b, e, cxp)) & 1) != 0;
      };
      bool in = false;
      for (uint32_t p = hv.chip_part[c]; p < hv.chip_part[c + 1] && !in; p++) {
        const uint32_t rb = hv.part_ring[p], re = hv.part_ring[p + 1];
        if (re == rb || hv.ring_vtx[rb + 1] == hv.ring_vtx[rb] || !odd(rb - r0)) continue;
        bool hole = false;
        for (uint32_t q = rb + 1; q < re && !hole; q++) hole = odd(q - r0);
        in = !hole;
      }
#ifdef MGPU_GRID_VERIFY
      if (pip::chip_locate(hv, c, cxp, cyp) != (in ? pip::kInterior : pip::kExterior)) {
        fprintf(stderr, "pixel verify: chip %u row parity %d differs from PointLocator\n", c, (int)in);
        abort();
      }
#endif
      if (in) mask |= 1ull << j;
      continue;
    } else {
      for (uint32_t p = hv.chip_part[c]; p < hv.chip_part[c + 1]; p++)
        for (uint32_t r = hv.part_ring[p]; r < hv.part_ring[p + 1]; r++)
          for (uint32_t i = hv.ring_vtx[r] + 1; i < hv.ring_vtx[r + 1]; i++)
            if (seg_hits_box(hv.vtx[2 * i - 2], hv.vtx[2 * i - 1], hv.vtx[2 * i], hv.vtx[2 * i + 1], x0, y0, x1, y1))
              return kPixAnswerMixed;
    }
    const int loc = pip::chip_locate(hv, c, 0.5 * (x0 + x1), 0.5 * (y0 + y1));
    if (loc == pip::kBoundary) return kPixAnswerMixed;
    if (loc == pip::kInterior) mask |= 1ull << j;
  }
  return (int64_t)mask;
}

// One corner of an H3 pixel: nearest face (and the squared-chord gap to the next),
// hex2d position on that face.
struct Corner {
  int face = -1;
  double gap = 0, x = 0, y = 0;
  bool ok = false;
};

struct SinCos {
  double s = 0, c = 0;
};
SinCos deg_sincos(double deg) {
  SinCos o;
  mgpu::h3::sincos_fast(mgpu::h3::to_radians_fast(deg), &o.s, &o.c);
  return o;
}
// (from the sines and cosines of the corner's longitude and latitude: a grid of corners
// shares them per column and per row)
Corner h3_corner_sc(const SinCos& lon, const SinCos& lat, int res, double k_res) {
  Corner o;
  const double slat = lat.s, clat = lat.c, slon = lon.s, clon = lon.c;
  const double vx = clon * clat, vy = slon * clat, vz = slat;
  // the squared chords to the 20 face centres (a vector loop over the centres' columns),
  // then the nearest (the first of equals) and the next -- the second smallest of the 20
  struct FaceCols {
    double x[20], y[20], z[20];
    FaceCols() {
      for (int f = 0; f < 20; f++) x[f] = H3T_FACE_CENTER_POINT[f][0], y[f] = H3T_FACE_CENTER_POINT[f][1], z[f] = H3T_FACE_CENTER_POINT[f][2];
    }
  };
  static const FaceCols FC;
  double sq[20];
  for (int f = 0; f < 20; f++) {
    const double dx = FC.x[f] - vx, dy = FC.y[f] - vy, dz = FC.z[f] - vz;
    sq[f] = dx * dx + dy * dy + dz * dz;
  }
  double best = 5.0, second = 5.0;
  for (int f = 0; f < 20; f++) {
    const double s = sq[f];
    if (s < best) {
      second = best;
      best = s;
      o.face = f;
    } else if (s < second) {
      second = s;
    }
  }
  o.gap = second - best;
  const double(*F)[3] = H3T_FACE_FRAME[o.face][res & 1];
  const double dc = vx * F[2][0] + vy * F[2][1] + vz * F[2][2];
  if (!(dc > 0.5)) return o;
  o.x = k_res * (vx * F[0][0] + vy * F[0][1] + vz * F[0][2]) / dc;
  o.y = k_res * (vx * F[1][0] + vy * F[1][1] + vz * F[1][2]) / dc;
  o.ok = std::fabs(o.x) < 1e8 && std::fabs(o.y) < 1e8;
  return o;
}
Corner h3_corner(double lond, double latd, int res, double k_res) {
  return h3_corner_sc(deg_sincos(lond), deg_sincos(latd), res, k_res);
}

// Does the hexagon of axial lattice position (a, b) -- H3's _hex2dToCoordIJK rounds to
// the nearest lattice centre (checked by tests/cpp), so a cell is the hexagon of
// apothem 1/2 around (a - b/2, b sin60) -- come within `d` of the convex quad q?
// (separating axes: the hexagon's three edge normals and the quad's four)
struct HexFrame {  // the hexagon's vertex offsets (circumradius R at 30 + 60 k degrees), edge normals
  double off[6][2], nrm[3][2];
  HexFrame() {
    const double R = 0.57735026918962576451;  // circumradius
    for (int k = 0; k < 6; k++) {
      const double t = (30.0 + 60.0 * k) * kPi / 180.0;
      off[k][0] = R * std::cos(t);
      off[k][1] = R * std::sin(t);
    }
    for (int k = 0; k < 3; k++) {
      const double t = 60.0 * k * kPi / 180.0;
      nrm[k][0] = std::cos(t);
      nrm[k][1] = std::sin(t);
    }
  }
};
// the quad's side of the separating-axis test, shared by the seven hexagons tested
// against it: the hexagon's three edge normals and the quad's four (valid[k]: a non-zero
// edge), and the quad's extent along each
struct QuadAxes {
  double n[7][2], lo[7], hi[7];
  bool valid[7];
  // (el[e]: the length of edge q[e] -> q[(e + 1) % 4], as std::hypot gives it)
  QuadAxes(const double q[4][2], const HexFrame& F, const double el[4]) {
    for (int k = 0; k < 7; k++) {
      valid[k] = true;
      if (k < 3) {
        n[k][0] = F.nrm[k][0], n[k][1] = F.nrm[k][1];
      } else {
        const int e = k - 3;
        const double ex = q[(e + 1) % 4][0] - q[e][0], ey = q[(e + 1) % 4][1] - q[e][1];
        const double l = el[e];
        valid[k] = l > 0;
        n[k][0] = valid[k] ? -ey / l : 0.0, n[k][1] = valid[k] ? ex / l : 0.0;
      }
      double q0 = 1e300, q1 = -1e300;
      for (int p = 0; p < 4; p++) {
        const double v = q[p][0] * n[k][0] + q[p][1] * n[k][1];
        q0 = std::min(q0, v), q1 = std::max(q1, v);
      }
      lo[k] = q0, hi[k] = q1;
    }
  }
};
// (first: the axis tried first -- the hexagon normal facing a neighbour separates it from
// a quad inside the centre cell at once; the answer does not depend on the order)
bool hex_meets_quad(int64_t a, int64_t b, const QuadAxes& Q, const HexFrame& F, double d, int first = 0) {
  const double cx = (double)a - 0.5 * (double)b, cy = (double)b * mgpu::h3::kSin60;
  double hv[6][2];
  for (int k = 0; k < 6; k++) {
    hv[k][0] = cx + F.off[k][0];
    hv[k][1] = cy + F.off[k][1];
  }
  for (int i = 0; i < 7; i++) {
    const int k = i == 0 ? first : (i <= first ? i - 1 : i);
    if (!Q.valid[k]) continue;
    double h0 = 1e300, h1 = -1e300;
    for (int p = 0; p < 6; p++) {
      const double v = hv[p][0] * Q.n[k][0] + hv[p][1] * Q.n[k][1];
      h0 = std::min(h0, v), h1 = std::max(h1, v);
    }
    if (h1 + d < Q.lo[k] || Q.hi[k] + d < h0) return false;
  }
  return true;
}

// The hexagon side of the test on the hexagon's own three normals does not depend on the
// quad: the seven hexagons around one lattice position keep their extents along them in
// a per-thread cache (neighbouring sub-pixels mostly share that position), computed by
// hex_meets_quad's own expressions, so the answers are the same.
struct HexAxisCache {
  int64_t a0 = INT64_MIN, b0 = INT64_MIN;
  double lo[7][3], hi[7][3];
};
static const int kHexDa[7] = {0, 1, -1, 0, 0, 1, -1}, kHexDb[7] = {0, 0, 0, 1, -1, 1, -1};
void hex_axis_fill(HexAxisCache& C, int64_t a0, int64_t b0, const HexFrame& F) {
  C.a0 = a0, C.b0 = b0;
  for (int h = 0; h < 7; h++) {
    const int64_t a = a0 + kHexDa[h], b = b0 + kHexDb[h];
    const double cx = (double)a - 0.5 * (double)b, cy = (double)b * mgpu::h3::kSin60;
    double hv[6][2];
    for (int k = 0; k < 6; k++) {
      hv[k][0] = cx + F.off[k][0];
      hv[k][1] = cy + F.off[k][1];
    }
    for (int k = 0; k < 3; k++) {
      double h0 = 1e300, h1 = -1e300;
      for (int p = 0; p < 6; p++) {
        const double v = hv[p][0] * F.nrm[k][0] + hv[p][1] * F.nrm[k][1];
        h0 = std::min(h0, v), h1 = std::max(h1, v);
      }
      C.lo[h][k] = h0, C.hi[h][k] = h1;
    }
  }
}
// hex_meets_quad for hexagon h of the cache's position (the same axes in the same order)
bool hex_meets_quad_cached(const HexAxisCache& C, int h, const QuadAxes& Q, const HexFrame& F, double d, int first) {
  bool have_hv = false;
  double hv[6][2];
  for (int i = 0; i < 7; i++) {
    const int k = i == 0 ? first : (i <= first ? i - 1 : i);
    if (!Q.valid[k]) continue;
    double h0, h1;
    if (k < 3) {
      h0 = C.lo[h][k], h1 = C.hi[h][k];
    } else {
      if (!have_hv) {
        const int64_t a = C.a0 + kHexDa[h], b = C.b0 + kHexDb[h];
        const double cx = (double)a - 0.5 * (double)b, cy = (double)b * mgpu::h3::kSin60;
        for (int p = 0; p < 6; p++) {
          hv[p][0] = cx + F.off[p][0];
          hv[p][1] = cy + F.off[p][1];
        }
        have_hv = true;
      }
      h0 = 1e300, h1 = -1e300;
      for (int p = 0; p < 6; p++) {
        const double v = hv[p][0] * Q.n[k][0] + hv[p][1] * Q.n[k][1];
        h0 = std::min(h0, v), h1 = std::max(h1, v);
      }
    }
    if (h1 + d < Q.lo[k] || Q.hi[k] + d < h0) return false;
  }
  return true;
}

// pixel budget and size (mgpu_build_opts): raster = 0 disables the index; raster_milli =
// pixel edge as a fraction of the cell edge (default 1/4); raster_sub = sub-pixels per
// mixed pixel edge (default 8; 0: no second level)
double raster_fraction(const mgpu_build_opts& o) { return o.raster_milli / 1000.0; }
int raster_sub_wanted(const mgpu_build_opts& o) { return o.raster_sub >= 2 && o.raster_sub <= 16 ? o.raster_sub : 0; }
constexpr int64_t kRasterMaxPixels = 1LL << 24;
constexpr int64_t kRasterMaxSub = 1LL << 26;

constexpr uint64_t kAnsMixed = ~0ULL;

// classes over the answers of both levels (first | mask << 32; 0 = empty; kAnsMixed):
// class 0 = empty, kPixMixed = mixed, the rest one per distinct ordered polygon list
// (chip_poly of the mask's chips -- answers from different cells with the same polygons
// share a class, represented by the first such answer), ordered by their number of
// matches so a class id tells its pair count (pc[k]: the first class with more than
// k + 1 matches)
using AnsVec = std::vector<uint64_t, NoInit<uint64_t>>;  // (level 2's answers: every one written, in parallel)
void raster_classes(const mgpu::ChipTableView& hv, const std::vector<uint64_t>& a1, const AnsVec& a2, Raster& R) {
  R.cells.assign(a1.size(), mgpu::kPixMixed);
  R.sub.clear();
  R.sub.resize(a2.size());  // (every slot written below)
  R.cls.assign(1, 0);
  auto slot = [&](size_t i) -> uint16_t& { return i < a1.size() ? R.cells[i] : R.sub[i - a1.size()]; };
  auto polys_of = [&](uint64_t v) {
    std::vector<int32_t> ps;
    for (uint32_t m = (uint32_t)(v >> 32); m; m &= m - 1) ps.push_back(hv.chip_poly[(uint32_t)v + __builtin_ctz(m)]);
    return ps;
  };
  // distinct answers -> their polygon lists -> classes
  // (a hash of the distinct answers; neighbouring pixels mostly repeat the previous one).
  // The classes and their representatives follow the answers' first appearance in pixel
  // order: each chunk lists its distinct answers in the order they first appear in it,
  // and the chunks' lists, read in chunk order with the ones seen dropped, are that order.
  const size_t n_all = a1.size() + a2.size();
  constexpr int64_t kChunk = 1 << 20;
  std::vector<std::vector<uint64_t>> firsts((n_all + kChunk - 1) / kChunk);
  mgpu::parallel_for((int64_t)firsts.size(), 1, [&](int64_t cb, int64_t ce, int) {
    for (int64_t ch = cb; ch < ce; ch++) {
      std::unordered_set<uint64_t> seen;
      uint64_t last = kAnsMixed;
      for (size_t i = (size_t)ch * kChunk; i < std::min(n_all, (size_t)(ch + 1) * kChunk); i++) {
        const uint64_t v = i < a1.size() ? a1[i] : a2[i - a1.size()];
        if (v == last) continue;
        last = v;
        if (v == kAnsMixed || (v >> 32) == 0 || !seen.insert(v).second) continue;
        firsts[ch].push_back(v);
      }
    }
  });
  std::unordered_map<uint64_t, int32_t> answer_key;
  answer_key.reserve(1 << 16);
  std::map<std::vector<int32_t>, int32_t> list_key;
  std::vector<uint64_t> rep;  // per list: the representative answer
  std::vector<std::vector<int32_t>> lists;
  for (const auto& fc : firsts)
  for (const uint64_t v : fc) {
    if (answer_key.count(v)) continue;
    auto ps = polys_of(v);
    auto it = list_key.find(ps);
    if (it == list_key.end()) {
      it = list_key.emplace(ps, (int32_t)lists.size()).first;
      lists.push_back(ps);
      rep.push_back(v);
    }
    answer_key[v] = it->second;
  }
  std::vector<int32_t> order(lists.size());
  for (size_t k = 0; k < order.size(); k++) order[k] = (int32_t)k;
  std::sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
    return lists[a].size() != lists[b].size() ? lists[a].size() < lists[b].size() : lists[a] < lists[b];
  });
  std::vector<int32_t> cls_of(lists.size(), -1);
  for (int32_t k : order) {
    if (R.cls.size() >= mgpu::kPixMixed) break;  // out of classes: the rest stay mixed
    cls_of[k] = (int32_t)R.cls.size();
    R.cls.push_back(rep[k]);
  }
  mgpu::parallel_for((int64_t)n_all, 1 << 16, [&](int64_t b, int64_t e, int) {
    uint64_t lv = kAnsMixed;
    int32_t lc = -1;
    for (int64_t i = b; i < e; i++) {
      const uint64_t v = (size_t)i < a1.size() ? a1[i] : a2[i - a1.size()];
      uint16_t out = mgpu::kPixMixed;
      if (v != kAnsMixed && (v >> 32) == 0) {
        out = mgpu::kPixEmpty;
      } else if (v != kAnsMixed) {
        if (v != lv) {
          lv = v;
          lc = cls_of[answer_key.find(v)->second];
        }
        if (lc >= 0) out = (uint16_t)lc;
      }
      slot((size_t)i) = out;
    }
  });
  auto pc = [](uint64_t v) { return __builtin_popcountll(v >> 32); };
  for (int k = 0; k < 4; k++) {
    uint32_t c = 1;
    while (c < R.cls.size() && pc(R.cls[c]) <= k + 1) c++;
    R.pc[k] = c;
  }
  R.n_pure = 0;
  for (uint16_t v : R.cells) R.n_pure += v != mgpu::kPixMixed;
}

// The lonlat second level without the rank table: a refined mixed pixel holds 0x8000 |
// its index among the refined pixels of its band of 2^band_shift raster rows, band[k] the
// refined pixels before band k (a table small enough for LDS), so a mixed point's
// sub-pixel block is band[row >> band_shift] + (class & 0x7FFF) -- one dependent load
// fewer than the rank word (chip_table.h).  Needs fewer than 0x7FFF classes and
// 2^band_shift * nx <= 0x7FFF; else the rank table stays.
constexpr size_t kRasterBandBytes = 4096;
#ifndef MGPU_RASTER_BANDS
#define MGPU_RASTER_BANDS 1
#endif
void raster_bands(Raster& R) {
  if (!MGPU_RASTER_BANDS || R.sub_n == 0 || R.rank.empty() || R.cls.size() >= 0x7FFF || R.nx > 0x7FFF) return;
  uint32_t sh = 0;
  while ((uint64_t)R.nx << (sh + 1) <= 0x7FFF && (1u << (sh + 1)) <= R.ny) sh++;
  const uint32_t nb = (R.ny + (1u << sh) - 1) >> sh;
  if ((size_t)nb * 4 > kRasterBandBytes) return;
  R.band.assign(nb, 0);
  uint32_t b = 0;
  for (uint32_t k = 0; k < nb; k++) {
    R.band[k] = b;
    const size_t p0 = (size_t)(k << sh) * R.nx, p1 = std::min<size_t>((size_t)((k + 1) << sh) * R.nx, R.cells.size());
    for (size_t p = p0; p < p1; p++)
      if ((R.rank[p >> 5].bits >> (p & 31)) & 1) R.cells[p] = (uint16_t)(0x8000u | (b++ - R.band[k]));
  }
  R.band_shift = sh;
  R.rank.clear();
}

// The second level palette-compressed (lonlat with bands): a refined mixed pixel's 256
// sub-pixels hold few distinct classes (a zone boundary: its two zones and "mixed"), so
// each block keeps <= 4 classes in one 8-byte palette word and 2 bits per sub-pixel -- 72
// bytes instead of 512, the whole level 7x smaller (C2: 68 MB -> ~10 MB); a block with more
// classes keeps its full u16 layout (pal = kPalFull | its index among those).
#ifndef MGPU_RASTER_PAL
#define MGPU_RASTER_PAL 0  // (A/B round 6, profiles/r6/ab_palette_edgepar.txt: C2 classify 0.59 -> 0.70 ms with it -- rejected)
#endif
void raster_palette(Raster& R) {
  if (!MGPU_RASTER_PAL || R.band.empty() || R.sub_n == 0 || (R.sub_n * R.sub_n) % 4) return;
  const size_t S2 = (size_t)R.sub_n * R.sub_n, nb = R.sub.size() / S2;
  R.pal.assign(nb, 0);
  R.idx2.assign(nb * S2 / 4, 0);
  std::vector<uint8_t> full(nb, 0);
  mgpu::parallel_for((int64_t)nb, 1024, [&](int64_t bb, int64_t be, int) {
    for (int64_t b = bb; b < be; b++) {
      const uint16_t* c = R.sub.data() + (size_t)b * S2;
      uint16_t p[4];
      int n = 0;
      bool ok = true;
      for (size_t i = 0; i < S2 && ok; i++) {
        int k = 0;
        while (k < n && p[k] != c[i]) k++;
        if (k == n) {
          if (n == 4) ok = false;
          else p[n++] = c[i];
        }
      }
      if (!ok) {
        full[b] = 1;
        continue;
      }
      for (int k = n; k < 4; k++) p[k] = p[0];
      // 15 bits a class (the bands need fewer than 0x7FFF classes), "mixed" as 0x7FFF: the
      // word's top bit stays kPalFull's
      auto c15 = [](uint16_t c) { return (uint64_t)(c == mgpu::kPixMixed ? 0x7FFFu : c); };
      R.pal[b] = c15(p[0]) | c15(p[1]) << 16 | c15(p[2]) << 32 | c15(p[3]) << 48;
      uint8_t* q = R.idx2.data() + (size_t)b * S2 / 4;
      for (size_t i = 0; i < S2; i++) {
        int k = 0;
        while (p[k] != c[i]) k++;
        q[i >> 2] |= (uint8_t)(k << (2 * (i & 3)));
      }
    }
  });
  // the full blocks, in order, are all the second level keeps
  uint64_t nf = 0;
  for (size_t b = 0; b < nb; b++)
    if (full[b]) {
      if (nf != b) std::memmove(R.sub.data() + nf * S2, R.sub.data() + b * S2, S2 * 2);
      R.pal[b] = mgpu::kPalFull | nf++;
    }
  R.sub.resize(nf * S2);
  R.sub.shrink_to_fit();
}

// the block table over the level-1 classes: the smallest block edge 2^s (s >= 3) whose
// table fits kRasterBlkBytes (the join kernels hold it in LDS)
#ifndef MGPU_RASTER_BLK_KB
#define MGPU_RASTER_BLK_KB 40
#endif
constexpr size_t kRasterBlkBytes = MGPU_RASTER_BLK_KB * 1024;
void raster_blocks(Raster& R) {
  for (uint32_t sh = MGPU_RASTER_BLK_KB > 64 ? 2 : 3; sh <= 8; sh++) {
    const uint32_t bnx = (R.nx + (1u << sh) - 1) >> sh, bny = (R.ny + (1u << sh) - 1) >> sh;
    if ((size_t)bnx * bny * 2 > kRasterBlkBytes) continue;
    R.bshift = sh, R.bnx = bnx, R.bny = bny;
    R.blk.assign((size_t)bnx * bny, mgpu::kPixMixed);
    for (uint32_t by = 0; by < bny; by++)
      for (uint32_t bx = 0; bx < bnx; bx++) {
        const uint32_t x0 = bx << sh, y0 = by << sh;
        const uint32_t x1 = std::min(R.nx, x0 + (1u << sh)), y1 = std::min(R.ny, y0 + (1u << sh));
        const uint16_t c = R.cells[(size_t)y0 * R.nx + x0];
        bool same = c != mgpu::kPixMixed;
        for (uint32_t y = y0; y < y1 && same; y++)
          for (uint32_t x = x0; x < x1 && same; x++) same = R.cells[(size_t)y * R.nx + x] == c;
        if (same) R.blk[(size_t)by * bnx + bx] = c;
      }
    return;
  }
}

// H3: the answer shared by every point of the rectangle [xa, xb] x [ya, yb] (degrees)
// whose corners c (projected at exactly those points, in the order (xa, ya), (xb, ya),
// (xb, yb), (xa, yb)) are given; the certificate is checked on the rectangle widened by
// (mux, muy) -- its corners lie within ~1e-6 of its size of c, a deviation the margins
// below carry -- or kAnsMixed.  (el: the four edge lengths when the caller has them --
// a grid of sub-pixels shares each edge between two of them -- else computed here; the
// side lengths enter both the diameter L and the quad's edge normals)
struct H3RasterCtx {
  const mgpu::ChipTableView& hv;
  int res;
  double k_res;
  const mgpu::DenseFace* dense;
  const std::vector<uint64_t>& grid;
};
uint64_t h3_rect_answer(const H3RasterCtx& X, double xa, double ya, double xb, double yb, const Corner* c[4],
                        double mux, double muy, std::vector<int32_t>& polys, std::vector<int32_t>& ref,
                        PixelEdges* pe = nullptr, const double* el = nullptr, HexAxisCache* hc = nullptr) {
  double q[4][2], e4[4];
  for (int p = 0; p < 4; p++) q[p][0] = c[p]->x, q[p][1] = c[p]->y;
  // (|a - b| = |b - a| exactly: the sides and the two diagonals are the six corner pairs)
  for (int e = 0; e < 4; e++)
    e4[e] = el ? el[e] : std::hypot(q[(e + 1) % 4][0] - q[e][0], q[(e + 1) % 4][1] - q[e][1]);
  double L = 0;
  for (int e = 0; e < 4; e++) L = std::max(L, e4[e]);
  L = std::max(L, std::hypot(q[0][0] - q[2][0], q[0][1] - q[2][1]));
  L = std::max(L, std::hypot(q[1][0] - q[3][0], q[1][1] - q[3][1]));
  const double ang = std::hypot(xb - xa + 2 * mux, yb - ya + 2 * muy) * kPi / 180.0;  // angular diagonal bound
  const double d_face = 1e-12 + 8.0 * ang * ang + 8e-6 * ang;
  const double d_hex = 1e-9 * (1.0 + std::fabs(q[0][0]) + std::fabs(q[0][1])) + 8.0 * L * L / X.k_res + 8e-6 * L;
  bool ok = L < 0.5;
  for (int p = 0; p < 4 && ok; p++) ok = c[p]->ok && c[p]->face == c[0]->face && c[p]->gap > d_face;
  if (!ok) return kAnsMixed;
  double mg;
  const mgpu::h3::IJK h0 = mgpu::h3::hex2d_to_ijk_fast(q[0][0], q[0][1], &mg);
  const int64_t a0 = h0.i - h0.k, b0 = h0.j - h0.k;
  // every cell a point of the rectangle can take is h0 or a neighbour (L < 1/2) whose
  // hexagon meets the quad; all must give the same polygon list
  static const int* da = kHexDa;
  static const int* db = kHexDb;
  static const int kFacing[7] = {0, 0, 0, 2, 2, 1, 1};  // (the normal toward neighbour k: 0, 120, 60 degrees)
  static const HexFrame HF;
  const QuadAxes QA(q, HF, e4);
  if (hc && (hc->a0 != a0 || hc->b0 != b0)) hex_axis_fill(*hc, a0, b0, HF);
  const mgpu::DenseFace& D = X.dense[c[0]->face];
  bool first = true;
  uint64_t cls = 0;
  for (int k = 0; k < 7; k++) {
    const int64_t a = a0 + da[k], b = b0 + db[k];
    // (k = 0, h0: the cell of corner q[0], which lies in its hexagon -- the separating
    // axis test cannot part them by the margin d_hex >= 1e-9, far above q[0]'s rounding)
    if (k > 0 && !(hc ? hex_meets_quad_cached(*hc, k, QA, HF, d_hex, kFacing[k]) : hex_meets_quad(a, b, QA, HF, d_hex, kFacing[k])))
      continue;
    const uint64_t ua = (uint64_t)(a - D.a0), ub = (uint64_t)(b - D.b0);
    const uint64_t e = (ua < D.w && ub < D.h) ? X.grid[D.base + ub * D.w + ua] : 0;
    const int64_t m = pixel_answer(X.hv, e, xa - mux, ya - muy, xb + mux, yb + muy, pe);
    if (m == kPixAnswerMixed) return kAnsMixed;
    polys.clear();
    for (uint64_t bits = (uint64_t)m; bits; bits &= bits - 1) polys.push_back(X.hv.chip_poly[(uint32_t)e + __builtin_ctzll(bits)]);
    if (first) {
      ref = polys;
      cls = m ? ((uint32_t)e | ((uint64_t)m << 32)) : 0;
      first = false;
    } else if (polys != ref) {
      return kAnsMixed;
    }
  }
  return first ? kAnsMixed : cls;
}

bool build_raster_h3(const mgpu::ChipTableView& hv, int res, double k_res, const double bbox[4],
                     const mgpu::DenseFace* dense, const std::vector<uint64_t>& grid, Raster& R,
                     const mgpu_build_opts& bo) {
  if (!bo.raster || res < 5 || !(bbox[2] - bbox[0] < 360.0) || grid.empty()) return false;
  const double W = bbox[2] - bbox[0], Hh = bbox[3] - bbox[1];
  if (!(W > 0) || !(Hh > 0)) return false;
  const double edge_deg = 1107.712591 / std::pow(mgpu::h3::kSqrt7, res) / 111.195;  // mean cell edge
  const double latc = std::max(std::fabs(bbox[1]), std::fabs(bbox[3]));
  if (latc > 80.0) return false;
  double dyp = raster_fraction(bo) * edge_deg, dxp = dyp / std::cos(latc * kPi / 180.0);
  double nxd = std::ceil(W / dxp), nyd = std::ceil(Hh / dyp);
  if (nxd * nyd > (double)kRasterMaxPixels) {
    const double s = std::sqrt(nxd * nyd / (double)kRasterMaxPixels) * 1.01;
    dxp *= s, dyp *= s;
    nxd = std::ceil(W / dxp), nyd = std::ceil(Hh / dyp);
  }
  if (dyp > 0.6 * edge_deg) return false;  // pixels as large as cells are rarely pure
  R.mode = mgpu::kRasterLonLat;
  R.nx = (uint32_t)nxd, R.ny = (uint32_t)nyd;
  R.x0 = bbox[0], R.y0 = bbox[1];
  R.inv_dx = 1.0 / dxp, R.inv_dy = 1.0 / dyp;
  const double sx = 1.0 / R.inv_dx, sy = 1.0 / R.inv_dy;  // the pixel size the kernel's index implies
  const double mag = std::max(std::max(std::fabs(bbox[0]), std::fabs(bbox[2])), std::max(std::fabs(bbox[1]), std::fabs(bbox[3])));
  const double ulp = std::nextafter(mag, INFINITY) - mag;
  // pixel / sub-pixel edge coordinates (the last ones take the clamped points up to bbox)
  auto xe = [&](uint32_t ix, double f) {
    return ix + f >= R.nx ? std::max(R.x0 + R.nx * sx, bbox[2]) : R.x0 + (ix + f) * sx;
  };
  auto ye = [&](uint32_t iy, double f) {
    return iy + f >= R.ny ? std::max(R.y0 + R.ny * sy, bbox[3]) : R.y0 + (iy + f) * sy;
  };
  const H3RasterCtx X{hv, res, k_res, dense, grid};
#ifdef MGPU_BLOB_TIMING
  const auto rl0 = std::chrono::steady_clock::now();
#endif
  // level 1: corners on the pixel grid, two rows at a time
  std::vector<uint64_t> a1((size_t)R.nx * R.ny, kAnsMixed);
  {
    const double mux = 1e-6 * sx + 64 * ulp, muy = 1e-6 * sy + 64 * ulp;
    mgpu::parallel_for((int64_t)R.ny, 8, [&](int64_t yb, int64_t ye_, int) {
      std::vector<int32_t> polys, ref;
      std::vector<Corner> lo(R.nx + 1), hi(R.nx + 1);
      std::vector<SinCos> scx(R.nx + 1);
      for (uint32_t ix = 0; ix <= R.nx; ix++) scx[ix] = deg_sincos(xe(ix, 0));
      const SinCos s0 = deg_sincos(ye((uint32_t)yb, 0));
      for (uint32_t ix = 0; ix <= R.nx; ix++) lo[ix] = h3_corner_sc(scx[ix], s0, res, k_res);
      for (int64_t iy = yb; iy < ye_; iy++) {
        const SinCos s1 = deg_sincos(ye((uint32_t)iy, 1));
        for (uint32_t ix = 0; ix <= R.nx; ix++) hi[ix] = h3_corner_sc(scx[ix], s1, res, k_res);
        for (uint32_t ix = 0; ix < R.nx; ix++) {
          const Corner* c[4] = {&lo[ix], &lo[ix + 1], &hi[ix + 1], &hi[ix]};
          a1[(size_t)iy * R.nx + ix] =
              h3_rect_answer(X, xe(ix, 0), ye((uint32_t)iy, 0), xe(ix, 1), ye((uint32_t)iy, 1), c, mux, muy, polys, ref);
        }
        std::swap(lo, hi);
      }
    });
  }
#ifdef MGPU_BLOB_TIMING
  auto rt0 = std::chrono::steady_clock::now();
  fprintf(stderr, "[raster] level 1: %u x %u pixels, %.3f s\n", R.nx, R.ny, std::chrono::duration<double>(rt0 - rl0).count());
#endif
  // level 2: the mixed pixels cut into S x S sub-pixels
  AnsVec a2;
#ifdef MGPU_BLOB_TIMING
  int64_t t_corner_ns_total = 0;
#endif
  // (S = 16 by default: on C2, 8 -> 16 took the mixed points 2.5% -> 1.3% of all and the
  // join 1.23 -> 1.11 ms per 1e8 points, its sub-pixel table 17 -> 68 MB; the largest S
  // within kRasterMaxSub entries when the mixed pixels are many)
  int S = raster_sub_wanted(bo);
  std::vector<uint32_t> mixed;
  for (size_t i = 0; i < a1.size(); i++)
    if (a1[i] == kAnsMixed) mixed.push_back((uint32_t)i);
  while (S >= 2 && (int64_t)mixed.size() * S * S > kRasterMaxSub) S--;
  if (S >= 2 && !mixed.empty()) {
    R.sub_n = (uint32_t)S;
    mixed_rank(mixed, a1.size(), R.rank);
    a2.resize(mixed.size() * S * S);  // (every answer written below)
    const double mux = 1e-6 * sx / S + 64 * ulp, muy = 1e-6 * sy / S + 64 * ulp;
    const double pmux = 1e-6 * sx + 64 * ulp, pmuy = 1e-6 * sy + 64 * ulp;  // (level 1's widening: holds every sub-pixel's)
#ifdef MGPU_BLOB_TIMING
    std::atomic<int64_t> t_corner_ns{0};
    struct Flush {
      std::atomic<int64_t>& a;
      int64_t& t;
      ~Flush() { t = a.load(); }
    } flush{t_corner_ns, t_corner_ns_total};
#endif
    mgpu::parallel_for((int64_t)mixed.size(), 64, [&](int64_t kb, int64_t ke, int) {
      std::vector<int32_t> polys, ref;
      std::vector<Corner> cg((size_t)(S + 1) * (S + 1));
      std::vector<SinCos> scx(S + 1);
      std::vector<double> hl((size_t)(S + 1) * S), vl((size_t)S * (S + 1));  // sub-pixel side lengths
      PixelEdges pe;
      HexAxisCache hc;
      for (int64_t k = kb; k < ke; k++) {
        const uint32_t ix = mixed[k] % R.nx, iy = mixed[k] / R.nx;
        pe.reset(xe(ix, 0) - pmux, ye(iy, 0) - pmuy, xe(ix, 1) + pmux, ye(iy, 1) + pmuy);
#ifdef MGPU_BLOB_TIMING
        const auto tc0 = std::chrono::steady_clock::now();
#endif
        for (int u = 0; u <= S; u++) scx[u] = deg_sincos(xe(ix, (double)u / S));
        for (int v = 0; v <= S; v++) {
          const SinCos sy_ = deg_sincos(ye(iy, (double)v / S));
          for (int u = 0; u <= S; u++) cg[v * (S + 1) + u] = h3_corner_sc(scx[u], sy_, res, k_res);
        }
#ifdef MGPU_BLOB_TIMING
        t_corner_ns += (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - tc0).count();
#endif
        for (int v = 0; v <= S; v++)
          for (int u = 0; u <= S; u++) {
            const Corner& o = cg[v * (S + 1) + u];
            if (u < S) hl[v * S + u] = std::hypot(cg[v * (S + 1) + u + 1].x - o.x, cg[v * (S + 1) + u + 1].y - o.y);
            if (v < S) vl[v * (S + 1) + u] = std::hypot(cg[(v + 1) * (S + 1) + u].x - o.x, cg[(v + 1) * (S + 1) + u].y - o.y);
          }
        for (int v = 0; v < S; v++)
          for (int u = 0; u < S; u++) {
            const Corner* c[4] = {&cg[v * (S + 1) + u], &cg[v * (S + 1) + u + 1], &cg[(v + 1) * (S + 1) + u + 1],
                                  &cg[(v + 1) * (S + 1) + u]};
            const double el[4] = {hl[v * S + u], vl[v * (S + 1) + u + 1], hl[(v + 1) * S + u], vl[v * (S + 1) + u]};
            a2[(size_t)k * S * S + v * S + u] = h3_rect_answer(X, xe(ix, (double)u / S), ye(iy, (double)v / S),
                                                               xe(ix, (double)(u + 1) / S), ye(iy, (double)(v + 1) / S), c,
                                                               mux, muy, polys, ref, &pe, el, &hc);
          }
      }
    });
  }
#ifdef MGPU_BLOB_TIMING
  fprintf(stderr, "[raster] level 2: %zu mixed pixels, S %d, %.3f s (corners: %.3f thread-s)\n", mixed.size(), S,
          std::chrono::duration<double>(std::chrono::steady_clock::now() - rt0).count(), 1e-9 * (double)t_corner_ns_total);
  rt0 = std::chrono::steady_clock::now();
#endif
  raster_classes(hv, a1, a2, R);
  raster_blocks(R);
  raster_bands(R);
  raster_palette(R);
#ifdef MGPU_BLOB_TIMING
  fprintf(stderr, "[raster] classes, blocks, bands %.3f s\n", std::chrono::duration<double>(std::chrono::steady_clock::now() - rt0).count());
#endif
  return true;
}

// (BNG: off unless raster_bng = 1 -- its cell is a few integer operations and one grid
// load already; on C4 the pixel lookups cost more than the point-in-polygon work they
// save: split 2.55 ms vs fused 2.25 ms per 1e8 points)
bool build_raster_bng(const mgpu::ChipTableView& hv, const mgpu::DenseFace& D, uint32_t edge,
                      const std::vector<uint64_t>& grid, Raster& R, const mgpu_build_opts& bo) {
  if (!bo.raster_bng || !bo.raster || edge == 0 || grid.empty()) return false;
  // pixels per cell edge: the largest k <= 1 / fraction dividing the edge, within budget
  // (default fraction 1/4 -> 2: a raster of 2 x 2 pixels per cell stays in L2 at C4's size)
  int kpc = bo.raster_milli == 250 ? 2 : (int)std::floor(1.0 / raster_fraction(bo) + 1e-9);
  for (; kpc > 1; kpc--)
    if (edge % kpc == 0 && (double)D.w * kpc * D.h * kpc <= (double)kRasterMaxPixels) break;
  if (kpc < 2) return false;
  R.mode = mgpu::kRasterBng;
  R.pix = edge / kpc;
  R.nx = D.w * kpc, R.ny = D.h * kpc;
  R.px0 = D.a0 * kpc, R.py0 = D.b0 * kpc;
  R.inv_dx = R.inv_dy = 1.0 / R.pix;
  // BNG pixels hold the match mask itself (the kernel has the cell's grid entry anyway)
  auto answer = [&](uint64_t e, double xa, double ya, double xb, double yb, double mu) -> uint16_t {
    const int64_t m = pixel_answer(hv, e, xa - mu, ya - mu, xb + mu, yb + mu);
    return (m == kPixAnswerMixed || m >= (int64_t)mgpu::kPixMixed) ? mgpu::kPixMixed : (uint16_t)m;
  };
  const double mu0 = 64 * (std::nextafter(1e7, INFINITY) - 1e7);
  R.cells.assign((size_t)R.nx * R.ny, mgpu::kPixMixed);
  R.cls.assign(1, 0);
  mgpu::parallel_for((int64_t)R.ny, 8, [&](int64_t yb, int64_t ye, int) {
    for (int64_t iy = yb; iy < ye; iy++)
      for (uint32_t ix = 0; ix < R.nx; ix++) {
        const uint64_t e = grid[D.base + (size_t)(iy / kpc) * D.w + ix / kpc];
        R.cells[(size_t)iy * R.nx + ix] =
            answer(e, (double)(R.px0 + (int64_t)ix) * R.pix, (double)(R.py0 + iy) * R.pix,
                   (double)(R.px0 + (int64_t)ix + 1) * R.pix, (double)(R.py0 + iy + 1) * R.pix, 1e-6 * R.pix + mu0);
      }
  });
  // level 2: sub-pixels of whole metres, S = the largest divisor of the pixel edge <= 8
  int S = 0;
  if (raster_sub_wanted(bo))
    for (int d = std::min<int>(raster_sub_wanted(bo), (int)R.pix); d >= 2; d--)
      if (R.pix % d == 0) {
        S = d;
        break;
      }
  std::vector<uint32_t> mixed;
  for (size_t i = 0; i < R.cells.size(); i++)
    if (R.cells[i] == mgpu::kPixMixed) mixed.push_back((uint32_t)i);
  if (S >= 2 && !mixed.empty() && (int64_t)mixed.size() * S * S <= kRasterMaxSub) {
    R.sub_n = (uint32_t)S;
    const uint32_t w = R.pix / S;
    R.sub_w = w;
    mixed_rank(mixed, R.cells.size(), R.rank);
    R.sub.assign(mixed.size() * S * S, mgpu::kPixMixed);
    mgpu::parallel_for((int64_t)mixed.size(), 256, [&](int64_t kb, int64_t ke, int) {
      for (int64_t k = kb; k < ke; k++) {
        const uint32_t ix = mixed[k] % R.nx, iy = mixed[k] / R.nx;
        const uint64_t e = grid[D.base + (size_t)(iy / kpc) * D.w + ix / kpc];
        const double x0 = (double)(R.px0 + (int64_t)ix) * R.pix, y0 = (double)(R.py0 + (int64_t)iy) * R.pix;
        for (int v = 0; v < S; v++)
          for (int u = 0; u < S; u++)
            R.sub[(size_t)k * S * S + v * S + u] =
                answer(e, x0 + (double)u * w, y0 + (double)v * w, x0 + (double)(u + 1) * w, y0 + (double)(v + 1) * w,
                       1e-6 * w + mu0);
      }
    });
  }
  R.n_pure = 0;
  for (uint16_t v : R.cells) R.n_pure += v != mgpu::kPixMixed;
  return true;
}

// BNG per-cell answer grids (ChipTableView::cell_ans): every dense cell with border chips
// (at most kCellAnsChips) is cut into g x g squares of whole metres (g = the largest
// divisor of the edge <= kCellAnsSide, at least 4), each holding the match mask of the
// cell's chips when it is certified like a pixel (pixel_answer: no chip edge meets the
// widened square, the verdicts of its centre), else kCellAnsMixed.  The fused join's
// phase 1 answers a point in a certified square with one load instead of one candidate
// (envelope, classification grid) per border chip.
struct CellAnswers {
  uint32_t g = 0, sw = 0;
  std::vector<uint32_t> row;  // answer cells before each dense row
  std::vector<uint16_t> ans;
};
// (squares per cell side: 25 -> 100 at C4 res 3, 40 m -> 10 m squares, took the join's
// candidates 25M -> 6.7M per 1e8 points and its kernel 1.85 -> 1.72 ms; 33 MB of grids,
// built in 0.5 s on 8 host threads -- profiles/r4_cell_ans_ab.txt)
#ifndef MGPU_CELL_ANS_SIDE
#define MGPU_CELL_ANS_SIDE 100
#endif
constexpr uint32_t kCellAnsSide = MGPU_CELL_ANS_SIDE;
constexpr size_t kCellAnsMaxBytes = (size_t)64 << 20;
#ifndef MGPU_CELL_ANS
#define MGPU_CELL_ANS 1
#endif
bool build_cell_answers(const mgpu::ChipTableView& hv, const mgpu::DenseFace& D, uint32_t edge,
                        std::vector<uint64_t>& grid, CellAnswers& A) {
  if (!MGPU_CELL_ANS || edge == 0 || grid.empty() || D.w > 4096) return false;
  for (uint64_t e : grid)
    if (((e >> 32) & 0xFFFF) >= 0x8000) return false;  // (bit 47 is the flag)
  std::vector<uint32_t> cells;
  for (uint32_t k = 0; k < D.w * D.h; k++) {
    const uint64_t e = grid[D.base + k];
    const uint32_t count = (uint32_t)(e >> 32) & 0xFFFF, core = (uint32_t)(e >> 48);
    if (count == 0 || count > mgpu::kCellAnsChips) continue;
    if ((core & ((1u << count) - 1)) == (1u << count) - 1) continue;  // all core: nothing to test
    cells.push_back(k);
  }
  // (only where border cells are common: at C4 res 3, 62% of the cells, the join's
  // candidates fell 130M -> 25M per 1e8 points and its kernel 2.62 -> 1.85 ms; at res 4,
  // 7.6%, candidates 13.9M -> 2.6M but the kernel 1.65 -> 1.68 ms, profiles/r4_cell_ans_ab.txt)
  size_t nonempty = 0;
  for (uint32_t k = 0; k < D.w * D.h; k++) nonempty += ((grid[D.base + k] >> 32) & 0xFFFF) != 0;
  if (cells.empty() || cells.size() * 5 < nonempty) return false;
  // the finest square side (a divisor of the edge, whole metres) within the memory bound
  uint32_t g = 0;
  for (uint32_t d = std::min(kCellAnsSide, edge); d >= 4 && !g; d--)
    if (edge % d == 0 && cells.size() * d * d * 2 <= kCellAnsMaxBytes) g = d;
  if (g == 0) return false;
  A.g = g;
  A.sw = edge / g;
  A.ans.assign(cells.size() * g * g, mgpu::kCellAnsMixed);
  const double mu0 = 64 * (std::nextafter(1e7, INFINITY) - 1e7), w = A.sw;
  mgpu::parallel_for((int64_t)cells.size(), 4, [&](int64_t kb, int64_t ke, int) {
    for (int64_t i = kb; i < ke; i++) {
      const uint32_t k = cells[i];
      const uint64_t e = grid[D.base + k];
      const double x0 = (double)(D.a0 + (int64_t)(k % D.w)) * edge, y0 = (double)(D.b0 + (int64_t)(k / D.w)) * edge;
      const double mu = 1e-6 * w + mu0;
      for (uint32_t v = 0; v < g; v++)
        for (uint32_t u = 0; u < g; u++) {
          const int64_t m = pixel_answer(hv, e, x0 + u * w - mu, y0 + v * w - mu, x0 + (u + 1) * w + mu, y0 + (v + 1) * w + mu);
          if (m != kPixAnswerMixed && m < (int64_t)mgpu::kCellAnsMixed) A.ans[(size_t)i * g * g + v * g + u] = (uint16_t)m;
        }
    }
  });
  // flag the cells (cells[] ascends: row-major), their index within the row in bits 36-47
  A.row.assign(D.h, 0);
  size_t i = 0;
  for (uint32_t r = 0; r < D.h; r++) {
    A.row[r] = (uint32_t)i;
    for (; i < cells.size() && cells[i] / D.w == r; i++) {
      uint64_t& e = grid[D.base + cells[i]];
      const uint64_t count = (e >> 32) & 0xFFFF, k = i - A.row[r];
      e = (e & ~(0xFFFFull << 32) & ~(1ull << 63)) | (count << 32) | ((k & 0x7FF) << 36) | ((k >> 11) << 63) |
          mgpu::kCellAnsFlag;
    }
  }
  return true;
}

}  // namespace

namespace mgpu {
int32_t set_error(int32_t code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}
}  // namespace mgpu

namespace {

// Workspace layout (each region 256-byte aligned):
//   [counters 16 x u64] [fast-path tie queue u64 x (1 + kTieCap)] [tile_count u32 x T]
//   [tile_where u64 x T] [group_off u64 x T/32 (T)] [group_sum u32 x T/32] [dirty tiles u32 x T]
//   [records u64 x (T * slot records + pool)]
// counters: [0] pairs [1] route near-ties [2] invalid points [3] candidates (tile_scan_kernel)
//           [5] pool records used [6] dirty tiles (u32) [8..] MGPU_STATS
// T = tiles of the largest point batch reserved; pool = overflow records (tiles with
// more pairs than points), at most the output capacity.
constexpr size_t kWsCounters = 128;  // 16 x u64

struct WsLayout {
  size_t count, where, off, gsum, dirty, ties, recs, total;
};
// mgpu_points_to_cells' queue of the points its fast projection hands to the H3 route
// (overflow: the route pass redoes every point)
constexpr int64_t kTieCap = 1 << 16;

WsLayout ws_layout(int64_t n_tiles, int64_t pool) {
  WsLayout L;
  size_t T = (size_t)std::max<int64_t>(n_tiles, 1);
  L.ties = align_up(kWsCounters, 256);
  L.count = align_up(L.ties + (size_t)(kTieCap + 1) * 8, 256);
  L.where = align_up(L.count + T * 4, 256);
  L.off = align_up(L.where + T * 8, 256);
  L.gsum = align_up(L.off + T * 8, 256);
  L.dirty = align_up(L.gsum + 2 * (T / 32 + 1) * 4, 256);  // group pair sums, group candidate sums
  L.recs = align_up(L.dirty + T * 4 * 4, 256);  // (the split pipeline's mixed tiles: 64 points)
  L.total = align_up(L.recs + (T * (size_t)mgpu::join_slot_records() + (size_t)std::max<int64_t>(pool, 0)) * 8, 256);
  return L;
}

int32_t ensure_ws(mgpu_ctx* ctx, int64_t n_tiles, int64_t pool = 0) {
  ctx->last.valid = false;  // every call that uses the workspace ends the last join's lifetime
  ctx->last.async_pending = false;
  size_t need = ws_layout(n_tiles, pool).total;
  if (need <= ctx->ws_bytes) return MGPU_OK;
  if (ctx->ws) HIP_TRY(hipFree(ctx->ws));
  ctx->ws = nullptr;
  ctx->ws_bytes = 0;
  HIP_TRY(hipMalloc(&ctx->ws, need));
  ctx->ws_bytes = need;
  return MGPU_OK;
}

// The H3 route's near-tie queue (kernels.h JoinArgs.tie_queue): 2 header words, then
// 4 words per record.  The head the synchronous calls copy back with the counters.
constexpr int64_t kTqInit = 1 << 12;
constexpr int64_t kTqHead = 64;
constexpr size_t kPinWords = 16 + 2 + 4 * kTqHead;

int32_t ensure_tq(mgpu_ctx* ctx, int64_t cap) {
  if (cap <= ctx->tq_cap) return MGPU_OK;
  if (ctx->tq) HIP_TRY(hipFree(ctx->tq));
  ctx->tq = nullptr;
  ctx->tq_cap = 0;
  HIP_TRY(hipMalloc(&ctx->tq, (size_t)(2 + 4 * cap) * 8));
  ctx->tq_cap = cap;
  return MGPU_OK;
}

int32_t ensure_ovr(mgpu_ctx* ctx, int64_t words) {
  if (words <= ctx->ovr_cap) return MGPU_OK;
  if (ctx->ovr) HIP_TRY(hipFree(ctx->ovr));
  ctx->ovr = nullptr;
  ctx->ovr_cap = 0;
  HIP_TRY(hipMalloc(&ctx->ovr, (size_t)words * 8));
  ctx->ovr_cap = words;
  return MGPU_OK;
}

// The synchronous calls' host wait (option spin_us): poll the stream, yielding the core
// between polls, for at most spin_us, then block.  The poll saves the blocking wake-up
// (1.3-1.9% of C2's 1.5 ms step, profiles/r2_spin_ab.txt); the bound keeps a long join
// (or a stuck one) from holding a host core.
hipError_t stream_wait(const mgpu_ctx* ctx, hipStream_t s) {
  const int64_t us = ctx->opt.spin_us;
  if (us > 0) {
    const auto t0 = std::chrono::steady_clock::now();
    const auto lim = std::chrono::microseconds(us);
    for (;;) {
      const hipError_t q = hipStreamQuery(s);
      if (q != hipErrorNotReady) return q;
      if (std::chrono::steady_clock::now() - t0 > lim) break;
      sched_yield();
    }
  }
  return hipStreamSynchronize(s);
}

// A near-tie record of the queue (kernels.h JoinArgs.tie_queue)
struct TieRec {
  int64_t pos;
  double x, y;
  uint64_t key;
};

// Records of the queue: the head from the pinned copy, the rest read back.
int32_t read_ties(mgpu_ctx* ctx, int64_t n, std::vector<TieRec>& out) {
  out.resize((size_t)n);
  const uint64_t* head = ctx->pin + 16;
  const int64_t nh = std::min(n, kTqHead);
  if (nh) memcpy(out.data(), head + 2, (size_t)nh * 32);
  if (n > nh) HIP_TRY(hipMemcpy(out.data() + nh, ctx->tq + 2 + 4 * nh, (size_t)(n - nh) * 32, hipMemcpyDeviceToHost));
  return MGPU_OK;
}

// The reference's lattice key of every queued point (h3_glibc.cpp), by record; and the
// (position, key) list sorted by position for the override table.
std::vector<std::pair<int64_t, uint64_t>> libm_reference_keys(std::vector<TieRec>& ties, int res) {
  std::sort(ties.begin(), ties.end(), [](const TieRec& a, const TieRec& b) { return a.pos < b.pos; });
  std::vector<std::pair<int64_t, uint64_t>> out(ties.size());
  mgpu::parallel_for((int64_t)ties.size(), 256, [&](int64_t b, int64_t e, int) {
    for (int64_t k = b; k < e; k++) out[k] = {ties[k].pos, mgpu::h3glibc::lattice_key(ties[k].x, ties[k].y, res)};
  });
  return out;
}

// The reference's libm for the near-ties (h3_glibc.cpp); cells = true: keys are cell
// ids, else lattice keys.  Returns the records whose answer differs as (pos, key),
// sorted by position.
std::vector<std::pair<int64_t, uint64_t>> libm_second_opinion(const std::vector<TieRec>& ties, int res, bool cells) {
  std::vector<uint64_t> ref(ties.size());
  mgpu::parallel_for((int64_t)ties.size(), 256, [&](int64_t b, int64_t e, int) {
    for (int64_t k = b; k < e; k++)
      ref[k] = cells ? mgpu::h3glibc::point_to_cell(ties[k].x, ties[k].y, res)
                     : mgpu::h3glibc::lattice_key(ties[k].x, ties[k].y, res);
  });
  std::vector<std::pair<int64_t, uint64_t>> diff;
  for (size_t k = 0; k < ties.size(); k++)
    if (ref[k] != ties[k].key) diff.push_back({ties[k].pos, ref[k]});
  std::sort(diff.begin(), diff.end());
  return diff;
}

int32_t check_res(int32_t is, int32_t res) {
  if (is == MGPU_H3) {
    if (res < 0 || res > 15) return fail(MGPU_E_RESOLUTION, "H3 resolution has to be between 0 and 15; found %d", res);
    return MGPU_OK;
  }
  if (is == MGPU_BNG) {
    if (res == 0 || res < -6 || res > 6) return fail(MGPU_E_RESOLUTION, "BNG resolution not supported; found %d", res);
    return MGPU_OK;
  }
  return fail(MGPU_E_INVALID_ARG, "unknown index system %d (0 = H3, 1 = BNG)", is);
}

int32_t set_device(int dev) {
  HIP_TRY(hipSetDevice(dev));
  return MGPU_OK;
}

}  // namespace

extern "C" {

const char* mgpu_last_error(void) { return g_err.c_str(); }
const char* mgpu_version(void) { return "mosaic-mi355x 0.1.0 (gfx950)"; }
int32_t mgpu_join_tile_points(void) { return (int32_t)mgpu::join_tile_points(); }

int32_t mgpu_check_resolution(int32_t index_system, int32_t res) { return check_res(index_system, res); }

int32_t mgpu_ctx_create(int32_t device_id, mgpu_ctx** out) {
  if (!out) return fail(MGPU_E_INVALID_ARG, "out is NULL");
  int n = 0;
  HIP_TRY(hipGetDeviceCount(&n));
  if (device_id < 0 || device_id >= n) return fail(MGPU_E_INVALID_ARG, "device %d not present (%d GPUs)", device_id, n);
  HIP_TRY(hipSetDevice(device_id));
  mgpu_ctx* c = new mgpu_ctx();
  c->device = device_id;
  int32_t st = MGPU_OK;
  if (hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
      hipEventCreate(&c->ev2) != hipSuccess || hipEventCreate(&c->ev3) != hipSuccess ||
      hipHostMalloc((void**)&c->pin, kPinWords * 8, hipHostMallocDefault) != hipSuccess)
    st = fail(MGPU_E_DEVICE, "mgpu_ctx_create: events / pinned page");
  if (!st) st = ensure_ws(c, 1);
  if (!st) st = ensure_tq(c, kTqInit);
  if (st) {
    mgpu_ctx_destroy(c);
    return st;
  }
  *out = c;
  return MGPU_OK;
}

int32_t mgpu_ctx_destroy(mgpu_ctx* ctx) {
  if (!ctx) return MGPU_OK;
  mgpu_comm_destroy(ctx);
  hipSetDevice(ctx->device);
  if (ctx->split_ws) hipFree(ctx->split_ws);
  if (ctx->bin_ws) hipFree(ctx->bin_ws);
  if (ctx->scratch) hipFree(ctx->scratch);
  if (ctx->redo) hipFree(ctx->redo);
  if (ctx->tq) hipFree(ctx->tq);
  if (ctx->ovr) hipFree(ctx->ovr);
  if (ctx->ws) hipFree(ctx->ws);
  if (ctx->pin) hipHostFree(ctx->pin);
  if (ctx->ev0) hipEventDestroy(ctx->ev0);
  if (ctx->ev1) hipEventDestroy(ctx->ev1);
  if (ctx->ev2) hipEventDestroy(ctx->ev2);
  if (ctx->ev3) hipEventDestroy(ctx->ev3);
  delete ctx;
  return MGPU_OK;
}

int32_t mgpu_ctx_set_option(mgpu_ctx* ctx, const char* key, int64_t v) {
  if (!ctx || !key) return fail(MGPU_E_INVALID_ARG, "ctx/key is NULL");
  mgpu_options& o = ctx->opt;
  const std::string k = key;
  auto bad = [&]() { return fail(MGPU_E_INVALID_ARG, "option %s: value %lld out of range", key, (long long)v); };
  if (k == "h3_libm") {
    if (v != MGPU_LIBM_REFERENCE && v != MGPU_LIBM_CORRECTLY_ROUNDED) return bad();
    o.h3_libm = v;
  } else if (k == "pipeline") {
    if (v < MGPU_PIPELINE_AUTO || v > MGPU_PIPELINE_BINNED) return bad();
    o.pipeline = v;
  } else if (k == "bin_count") {
    if (v < 1 || v > mgpu::bin_max()) return bad();
    o.bin_count = v;
  } else if (k == "bin_min_mb") {
    if (v < 0) return bad();
    o.bin_min_mb = v;
  } else if (k == "bin_min_points") {
    if (v < 0) return bad();
    o.bin_min_points = v;
  } else if (k == "bin_xcd") {
    if (v != 0 && v != 1) return bad();
    o.bin_xcd = v;
  } else if (k == "bin_keys") {
    if (v != 0 && v != 1) return bad();
    o.bin_keys = v;
  } else if (k == "ring_batch") {
    if (v < 1) return bad();
    o.ring_batch = v;
  } else if (k == "bng_split") {
    if (v != 0 && v != 1) return bad();
    o.bng_split = v;
  } else if (k == "spin_us") {
    if (v < 0 || v > 10000000) return bad();
    o.spin_us = v;
  } else if (k == "raster" || k == "raster_bng") {
    if (v != 0 && v != 1) return bad();
    (k == "raster" ? o.raster : o.raster_bng) = v;
  } else if (k == "raster_sub") {
    if (!(v == 0 || (v >= 2 && v <= 16))) return bad();
    o.raster_sub = v;
  } else if (k == "raster_milli") {
    if (v < 10 || v > 1000) return bad();
    o.raster_milli = v;
  } else {
    return fail(MGPU_E_INVALID_ARG, "unknown option %s", key);
  }
  return MGPU_OK;
}

int32_t mgpu_ctx_get_option(const mgpu_ctx* ctx, const char* key, int64_t* v) {
  if (!ctx || !key || !v) return fail(MGPU_E_INVALID_ARG, "NULL argument");
  const mgpu_options& o = ctx->opt;
  const std::pair<const char*, int64_t> all[] = {
      {"h3_libm", o.h3_libm},       {"pipeline", o.pipeline}, {"bin_count", o.bin_count},
      {"bin_min_mb", o.bin_min_mb}, {"bin_min_points", o.bin_min_points}, {"bin_xcd", o.bin_xcd},
      {"bin_keys", o.bin_keys},     {"spin_us", o.spin_us},   {"ring_batch", o.ring_batch},       {"raster", o.raster},     {"raster_bng", o.raster_bng},
      {"bng_split", o.bng_split},
      {"raster_sub", o.raster_sub}, {"raster_milli", o.raster_milli}};
  for (const auto& kv : all)
    if (strcmp(kv.first, key) == 0) {
      *v = kv.second;
      return MGPU_OK;
    }
  return fail(MGPU_E_INVALID_ARG, "unknown option %s", key);
}

int32_t mgpu_ctx_reserve(mgpu_ctx* ctx, int64_t max_points) {
  if (!ctx) return fail(MGPU_E_INVALID_ARG, "ctx is NULL");
  if (int32_t st = set_device(ctx->device)) return st;
  const int64_t tiles = mgpu::join_tiles(max_points);
  return ensure_ws(ctx, tiles, max_points);
}

}  // extern "C"

// IndexSystem.pointToIndex over a batch: the kernels (fast path + the H3 route for the
// points it cannot decide), then -- H3 with the reference's libm -- the route's near-ties
// recomputed on the host (h3_glibc.cpp) and the cells that moves written back.  A
// near-tie queue that overflowed is grown and the call redone.
static int32_t cells_impl(mgpu_ctx* ctx, int32_t is, int32_t res, const double* x, const double* y, int64_t n,
                          int64_t* out_cell, hipStream_t s, const uint8_t* valid, int64_t voff, mgpu_stats* stats) {
  auto* counters = (unsigned long long*)ctx->ws;
  auto* ties = (unsigned long long*)((uint8_t*)ctx->ws + ws_layout(1, 0).ties);
  int64_t n_ties = 0, n_fixed = 0;
  for (int attempt = 0;; attempt++) {
    HIP_TRY(hipMemsetAsync(counters, 0, kWsCounters, s));
    HIP_TRY(hipMemsetAsync(ties, 0, 8, s));
    HIP_TRY(hipMemsetAsync(ctx->tq, 0, 16, s));
    HIP_TRY(hipEventRecord(ctx->ev0, s));
    HIP_TRY(mgpu::launch_cells(is, res, x, y, n, out_cell, counters, ties, kTieCap, ctx->tq, ctx->tq_cap, s, valid, voff));
    HIP_TRY(hipEventRecord(ctx->ev1, s));
    // invalid coordinates must reach the caller as IllegalArgument / IllegalState, so the
    // status is read back (the cell column itself stays on the device)
    HIP_TRY(hipMemcpyAsync(ctx->pin, counters, 16 * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(ctx->pin + 16, ctx->tq, (2 + 4 * kTqHead) * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(stream_wait(ctx, s));
    if (ctx->pin[2]) {
      if (is == MGPU_BNG) return fail(MGPU_E_NAN, "NaN coordinates are not supported. (%llu points)", (unsigned long long)ctx->pin[2]);
      return fail(MGPU_E_INVALID_ARG, "Latitude or longitude were invalid. (%llu points)", (unsigned long long)ctx->pin[2]);
    }
    n_ties = (int64_t)ctx->pin[16];
    if (n_ties > ctx->tq_cap) {
      if (attempt >= 2) return fail(MGPU_E_INTERNAL, "near-tie queue overflowed twice");
      if (int32_t st = ensure_tq(ctx, n_ties + n_ties / 4 + 1024)) return st;
      continue;
    }
    break;
  }
  if (stats) {
    memset(stats, 0, sizeof *stats);
    stats->n_points = n;
    stats->n_near_ties = n_ties;
    float ms = 0;
    hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1);
    stats->kernel_ms = stats->stream_kernel_ms = ms;
  }
  if (is == MGPU_H3 && n_ties > 0 && ctx->opt.h3_libm == MGPU_LIBM_REFERENCE) {
    std::vector<TieRec> tr;
    if (int32_t st = read_ties(ctx, n_ties, tr)) return st;
    const auto diff = libm_second_opinion(tr, res, true);
    n_fixed = (int64_t)diff.size();
    if (n_fixed) {
      std::vector<int64_t> hv(2 * diff.size());
      for (size_t k = 0; k < diff.size(); k++) hv[k] = diff[k].first, hv[diff.size() + k] = (int64_t)diff[k].second;
      if (int32_t st = ensure_ovr(ctx, (int64_t)hv.size())) return st;
      HIP_TRY(hipMemcpyAsync(ctx->ovr, hv.data(), hv.size() * 8, hipMemcpyHostToDevice, s));
      HIP_TRY(mgpu::launch_scatter_i64((const int64_t*)ctx->ovr, (const int64_t*)ctx->ovr + n_fixed, n_fixed, out_cell, s));
      HIP_TRY(stream_wait(ctx, s));
    }
  }
  if (stats) stats->libm_overrides = (int32_t)n_fixed;
  return MGPU_OK;
}

extern "C" {

int32_t mgpu_points_to_cells(mgpu_ctx* ctx, int32_t is, int32_t res, const double* x, const double* y, int64_t n,
                             int64_t* out_cell, void* stream, mgpu_stats* stats) {
  if (!ctx) return fail(MGPU_E_INVALID_ARG, "ctx is NULL");
  if (int32_t r = check_res(is, res)) return r;
  if (n < 0 || (n > 0 && (!x || !y || !out_cell))) return fail(MGPU_E_INVALID_ARG, "bad point arrays");
  if (int32_t st = set_device(ctx->device)) return st;
  if (int32_t st = ensure_ws(ctx, 1)) return st;
  return cells_impl(ctx, is, res, x, y, n, out_cell, (hipStream_t)stream, nullptr, 0, stats);
}

int32_t mgpu_format_cells_device(mgpu_ctx* ctx, int32_t index_system, const int64_t* cells, int64_t n, char* out,
                                 int64_t out_bytes, int64_t* out_offsets, int64_t* out_total, void* stream) {
  if (!ctx || n < 0 || (n > 0 && (!cells || !out)) || !out_offsets || out_bytes < 0)
    return fail(MGPU_E_INVALID_ARG, "format_cells_device: bad arguments");
  if (index_system != MGPU_H3 && index_system != MGPU_BNG)
    return fail(MGPU_E_INVALID_ARG, "unknown index system %d (0 = H3, 1 = BNG)", index_system);
  if (int32_t st = set_device(ctx->device)) return st;
  hipStream_t s = (hipStream_t)stream;
  // per-chunk totals live in the workspace's tile_where region (one int64 per 256 ids
  // there, one per 4096 needed)
  if (int32_t st = ensure_ws(ctx, mgpu::join_tiles(n))) return st;
  auto* counters = (unsigned long long*)ctx->ws;
  auto* chunk = (int64_t*)((uint8_t*)ctx->ws + ws_layout(mgpu::join_tiles(n), 0).where);
  HIP_TRY(hipMemsetAsync(counters, 0, kWsCounters, s));
  HIP_TRY(mgpu::launch_format_cells(index_system, cells, n, out, out_bytes, out_offsets, chunk, counters, s));
  unsigned long long h[4] = {0};
  int64_t total = 0;
  HIP_TRY(hipMemcpyAsync(h, counters, sizeof h, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(&total, out_offsets + n, sizeof total, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (out_total) *out_total = total;
  if (h[2]) return fail(MGPU_E_INVALID_ARG, "%llu BNG cell ids have no string form", h[2]);
  if (total > out_bytes) return fail(MGPU_E_CAPACITY, "format_cells_device: %lld bytes needed, %lld given",
                                     (long long)total, (long long)out_bytes);
  return MGPU_OK;
}

int32_t mgpu_grid_kring(mgpu_ctx* ctx, int32_t index_system, const int64_t* cells, int64_t n, int32_t k,
                        int32_t loop_only, int64_t* out_cells, int64_t capacity, int64_t* out_offsets,
                        int64_t* out_total, void* stream) {
  if (!ctx || n < 0 || (n > 0 && !cells) || !out_offsets || capacity < 0 || (capacity > 0 && !out_cells))
    return fail(MGPU_E_INVALID_ARG, "grid_kring: bad arguments");
  if (index_system != MGPU_BNG && index_system != MGPU_H3)
    return fail(MGPU_E_INVALID_ARG, "grid_kring: unknown index system %d", index_system);
  if (k < 0 || k > 1024) return fail(MGPU_E_INVALID_ARG, "grid_kring: k must be in [0, 1024]");
  if (int32_t st = set_device(ctx->device)) return st;
  hipStream_t s = (hipStream_t)stream;
  if (int32_t st = ensure_ws(ctx, mgpu::join_tiles(n))) return st;
  // workspace: counters, the chunk sums (tile_where region), per-cell counts mc[n] and the
  // fallback list fb_idx[n] (the records region, >= 16 n bytes)
  const WsLayout L = ws_layout(mgpu::join_tiles(n), 0);
  auto* base = (uint8_t*)ctx->ws;
  auto* counters = (unsigned long long*)base;
  auto* chunk = (int64_t*)(base + L.where);
  auto* mc = (int64_t*)(base + L.recs);
  auto* fb_idx = (uint32_t*)(base + L.recs + (size_t)std::max<int64_t>(n, 1) * 8);
  HIP_TRY(hipMemsetAsync(counters, 0, kWsCounters, s));
  HIP_TRY(mgpu::launch_kring_count(index_system, cells, n, k, loop_only, mc, chunk, fb_idx, counters, s));
  unsigned long long h[6] = {0};
  HIP_TRY(hipMemcpyAsync(h, counters, sizeof h, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (h[2] && index_system == MGPU_H3)
    return fail(MGPU_E_INVALID_ARG, "%llu cells are not H3 cell ids", h[2]);
  if (h[2])
    return fail(MGPU_E_INVALID_ARG, "%llu cells are not BNG cells or reach ids BNGIndexSystem.isValid cannot parse "
                "(NumberFormatException in the reference)", h[2]);
  // H3 walks that met a pentagon: H3's _kRingInternal / Mosaic's kLoop fallback, in
  // batches of cells whose scratch fits 256 MB, once for the lengths, once (after the
  // offsets) for the lists
  const int64_t n_fb = (int64_t)h[3];
  uint64_t* scratch = nullptr;
  struct Free {  // the fallback scratch is freed on every return path
    uint64_t*& p;
    ~Free() {
      if (p) hipFree(p);
    }
  } free_scratch{scratch};
  int64_t batch = 0;
  if (n_fb) {
    const int64_t words = mgpu::kring_fallback_words(k);
    batch = std::max<int64_t>(1, std::min<int64_t>(n_fb, ((int64_t)256 << 20) / 8 / words));
    HIP_TRY(hipMalloc(&scratch, (size_t)batch * words * 8));
    for (int64_t j0 = 0; j0 < n_fb; j0 += batch)
      HIP_TRY(mgpu::launch_kring_fallback(cells, fb_idx, j0, std::min(n_fb, j0 + batch), k, loop_only, mc, chunk,
                                          out_offsets, out_cells, capacity, scratch, 0, counters, s));
  }
  HIP_TRY(mgpu::launch_kring_write(index_system, cells, n, k, loop_only, mc, chunk, out_offsets, out_cells, capacity,
                                   s));
  for (int64_t j0 = 0; j0 < n_fb; j0 += batch)
    HIP_TRY(mgpu::launch_kring_fallback(cells, fb_idx, j0, std::min(n_fb, j0 + batch), k, loop_only, mc, chunk,
                                        out_offsets, out_cells, capacity, scratch, 1, counters, s));
  int64_t total = 0;
  HIP_TRY(hipMemcpyAsync(h, counters, sizeof h, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(&total, out_offsets + n, sizeof total, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (out_total) *out_total = total;
  if (h[4])
    return fail(MGPU_E_INTERNAL, "grid_kring: %llu pentagon walks overflowed their hash set (inconsistent tables)", h[4]);
  if (total > capacity)
    return fail(MGPU_E_CAPACITY, "grid_kring: %lld ids, capacity %lld", (long long)total, (long long)capacity);
  return MGPU_OK;
}

int32_t mgpu_bng_format_device(mgpu_ctx* ctx, const int64_t* cells, int64_t n, char* out, int64_t out_bytes,
                               int64_t* out_offsets, int64_t* out_total, void* stream) {
  return mgpu_format_cells_device(ctx, MGPU_BNG, cells, n, out, out_bytes, out_offsets, out_total, stream);
}

int32_t mgpu_points_to_cells_host(mgpu_ctx* ctx, int32_t is, int32_t res, const double* x, const double* y, int64_t n,
                                  int64_t* out_cell) {
  if (!ctx) return fail(MGPU_E_INVALID_ARG, "ctx is NULL");
  if (n == 0) return check_res(is, res);
  if (int32_t st = set_device(ctx->device)) return st;
  double *dx = nullptr, *dy = nullptr;
  int64_t* dc = nullptr;
  HIP_TRY(hipMalloc(&dx, n * 8));
  HIP_TRY(hipMalloc(&dy, n * 8));
  HIP_TRY(hipMalloc(&dc, n * 8));
  HIP_TRY(hipMemcpy(dx, x, n * 8, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(dy, y, n * 8, hipMemcpyHostToDevice));
  int32_t st = mgpu_points_to_cells(ctx, is, res, dx, dy, n, dc, nullptr, nullptr);
  if (st == MGPU_OK) HIP_TRY(hipMemcpy(out_cell, dc, n * 8, hipMemcpyDeviceToHost));
  hipFree(dx);
  hipFree(dy);
  hipFree(dc);
  return st;
}

// ------------------------------------------------------------------ chips

}  // extern "C"

#ifdef MGPU_BLOB_TIMING
#define BLOB_T0() auto blob_t = std::chrono::steady_clock::now()
#define SIDE_T0() auto side_t = std::chrono::steady_clock::now()
#define SIDE_MARK(what)                                                                                   \
  do {                                                                                                    \
    const auto now = std::chrono::steady_clock::now();                                                    \
    fprintf(stderr, "[blob]   side:%-8s %.3f s\n", what, std::chrono::duration<double>(now - side_t).count()); \
    side_t = now;                                                                                         \
  } while (0)
#define BLOB_MARK(what)                                                                                   \
  do {                                                                                                    \
    const auto now = std::chrono::steady_clock::now();                                                    \
    fprintf(stderr, "[blob] %-10s %.3f s\n", what, std::chrono::duration<double>(now - blob_t).count()); \
    blob_t = now;                                                                                         \
  } while (0)
#else
#define BLOB_T0() \
  do {            \
  } while (0)
#define BLOB_MARK(what) \
  do {                  \
  } while (0)
#define SIDE_T0() \
  do {            \
  } while (0)
#define SIDE_MARK(what) \
  do {                  \
  } while (0)
#endif
// The host blob: malloc'd and filled without a zero pass (build_blob writes every byte)
struct HostBlob {
  uint8_t* p = nullptr;
  size_t n = 0;
  HostBlob() = default;
  HostBlob(const HostBlob&) = delete;
  HostBlob& operator=(const HostBlob&) = delete;
  ~HostBlob() { free(p); }
  bool alloc(size_t bytes) {
    free(p);
    p = (uint8_t*)malloc(bytes);
    n = p ? bytes : 0;
    return p != nullptr;
  }
  uint8_t* data() const { return p; }
  size_t size() const { return n; }
  uint8_t* release() {
    uint8_t* q = p;
    p = nullptr;
    n = 0;
    return q;
  }
};

// The blob as pieces of its byte stream: [off, off + bytes) from src, then `zero` zero
// bytes.  build_blob hands them to a sink (the upload stages them straight into pinned
// buffers: no whole host blob) or assembles the host blob from them.
struct BlobPiece {
  size_t off;
  const uint8_t* src;
  size_t bytes, zero;
};
using BlobSink = std::function<int32_t(size_t total, const std::vector<BlobPiece>& pieces)>;

// The build's multi-GB intermediates freed off the caller's thread (returning their pages
// took ~0.5 s of C3's upload on the box): moved into one heap tuple a releaser thread
// deletes.  At most one release is pending per process: the next build_blob (and process
// exit) joins it first, so back-to-back uploads never hold two tables' intermediates.
namespace {
struct PendingRelease {
  std::mutex mu;
  std::thread th;
  void join() {
    std::lock_guard<std::mutex> g(mu);
    if (th.joinable()) th.join();
  }
  ~PendingRelease() { join(); }
};
PendingRelease g_release;
}  // namespace
template <class... V>
static void release_async(V&... v) {
  auto* box = new std::tuple<std::decay_t<V>...>(std::move(v)...);
  std::lock_guard<std::mutex> g(g_release.mu);
  if (g_release.th.joinable()) g_release.th.join();
  try {
    g_release.th = std::thread([box] { delete box; });
  } catch (...) {  // (no thread: free here)
    delete box;
  }
}

// bytes [off, off + n) of the stream the (ascending, contiguous) pieces make, to dst
static void fill_from_pieces(const std::vector<BlobPiece>& pieces, uint8_t* dst, size_t off, size_t n) {
  size_t q = std::upper_bound(pieces.begin(), pieces.end(), off,
                              [](size_t o, const BlobPiece& p) { return o < p.off; }) - pieces.begin() - 1;
  const size_t end = off + n;
  for (size_t at = off; at < end; q++) {
    const BlobPiece& p = pieces[q];
    const size_t pe = p.off + p.bytes, ze = pe + p.zero;
    if (at < pe) {
      const size_t m = std::min(pe, end) - at;
      memcpy(dst + (at - off), p.src + (at - p.off), m);
      at += m;
    }
    if (at < end && at < ze) {
      const size_t m = std::min(ze, end) - at;
      memset(dst + (at - off), 0, m);
      at += m;
    }
  }
}

// chips per chunk of the parallel blob-build phases (fixed: the result never depends on
// the thread count or schedule)
constexpr int64_t kBlobChunk = 1 << 14;

// std::sort of v by cmp (a strict total order) on the host threads: chunks sorted in
// parallel, then pairwise merge rounds
template <class V, class Cmp>
static void parallel_sort(V& v, Cmp cmp) {
  const int64_t n = (int64_t)v.size();
  const int64_t P = mgpu::parallel_slots(n, 1 << 16);
  if (P <= 1) {
    std::sort(v.begin(), v.end(), cmp);
    return;
  }
  std::vector<int64_t> b(P + 1);
  for (int64_t k = 0; k <= P; k++) b[k] = n * k / P;
  mgpu::parallel_for(P, 1, [&](int64_t kb, int64_t ke, int) {
    for (int64_t k = kb; k < ke; k++) std::sort(v.begin() + b[k], v.begin() + b[k + 1], cmp);
  });
  V tmp(v.size());
  for (int64_t w = 1; w < P; w *= 2) {
    const int64_t jobs = (P + 2 * w - 1) / (2 * w);
    mgpu::parallel_for(jobs, 1, [&](int64_t jb, int64_t je, int) {
      for (int64_t j = jb; j < je; j++) {
        const int64_t lo = b[2 * w * j], mid = b[std::min(P, 2 * w * j + w)], hi = b[std::min(P, 2 * w * j + 2 * w)];
        std::merge(v.begin() + lo, v.begin() + mid, v.begin() + mid, v.begin() + hi, tmp.begin() + lo, cmp);
      }
    });
    v.swap(tmp);
  }
}

// Whole-cell chips (H3): a border chip that is its cell's own hexagon -- the reference's
// demoted border-set cells (§5 of DESIGN.md) -- contains every point of its cell but
// those next to the hexagon's edges, where H3's spherical cell and the planar lon/lat
// hexagon part.  Such a cell (the only chip of its cell, res >= 6, six boundary vertices
// -- no icosahedron edge crosses it --, not a pentagon, |lat| <= 75 deg) is
// flagged by bit 15 of its core mask (unused with one chip) in its home face's lattice
// entry only, so a point probing from another face's frame never sees the flag (its
// offset would be measured in that frame); the streaming join answers
// a point of it whose fast projection lies inside the hexagon scaled by 0.9 about the
// cell centre (h3_core.h FastHex::deep: a margin of a tenth of the apothem, against the
// planar lon/lat hexagon's deviation from the projected one -- second order in the cell's
// angular size times tan(lat) and its distance from the face centre, < 1e-3 of the cell at
// res >= 6 and |lat| <= 75) without a candidate (kernels.hip phase1_item).
// (profiles/r4_whole_cell_ab.txt: C3 candidates 68.5M -> 55.6M per 1e8 points.)
void mark_whole_cells(std::vector<mgpu::HashSlot>& cells, int res,
                      const double bbox[4], const HVec<uint8_t>& cflags, const HVec<uint32_t>& cpart,
                      const mgpu::wkb::Flat& geo) {
  if (res < 6 || !(bbox[1] >= -75.0 && bbox[3] <= 75.0)) return;
  mgpu::parallel_for((int64_t)cells.size(), 4096, [&](int64_t b, int64_t e, int) {
    for (int64_t ci = b; ci < e; ci++) {
      mgpu::HashSlot& d = cells[ci];
      if (d.count != 1 || (d.core_mask & 1)) continue;
      const uint32_t c = d.first;
      if (cflags[c] & (mgpu::kChipMulti | mgpu::kChipEmpty | mgpu::kChipNoGeom | mgpu::kChipRect)) continue;
      if (cpart[c + 1] - cpart[c] != 1) continue;
      const uint32_t r0 = geo.part_ring[cpart[c]];
      if (geo.part_ring[cpart[c] + 1] - r0 != 1) continue;
      const uint32_t v0 = geo.ring_vtx[r0], nv = geo.ring_vtx[r0 + 1] - v0;
      if (nv != 7 || mgpu::h3b::is_pentagon(d.cell)) continue;
      const auto bd = mgpu::h3b::cell_boundary(d.cell);
      if (bd.size() != 6) continue;
      bool same = true;
      for (const auto& q : bd) {
        const double qx = mgpu::h3b::to_degrees(q.lon), qy = mgpu::h3b::to_degrees(q.lat);
        bool hit = false;
        for (uint32_t k = 0; k < 6 && !hit; k++)
          hit = std::fabs(geo.vtx[2 * (v0 + k)] - qx) <= 1e-9 && std::fabs(geo.vtx[2 * (v0 + k) + 1] - qy) <= 1e-9;
        same = same && hit;
      }
      if (same) d.core_mask |= (uint16_t)mgpu::kCoreWhole;
    }
  });
}

// The whole chip table as one host blob (header + arrays, chip_table.h); uploaded as
// is by mgpu_chips_upload, evaluated in place by mgpu_test_chip_contains_host.
static int32_t build_blob(int32_t index_system, int64_t n_chips, const int64_t* cell, const int32_t* polygon_id,
                          const uint8_t* is_core, const int64_t* wkb_offsets, const uint8_t* wkb,
                          HostBlob& host, BlobHeader& hdr_out, const mgpu_build_opts& bo,
                          const BlobSink* sink = nullptr) {
  g_release.join();  // (the previous build's intermediates, before this one allocates)
  if (index_system != MGPU_H3 && index_system != MGPU_BNG)
    return fail(MGPU_E_INVALID_ARG, "unknown index system %d (0 = H3, 1 = BNG)", index_system);
  if (n_chips < 0 || n_chips > (int64_t)std::numeric_limits<int32_t>::max())
    return fail(MGPU_E_INVALID_ARG, "n_chips out of range");
  if (n_chips > 0 && (!cell || !polygon_id || !is_core || !wkb_offsets))
    return fail(MGPU_E_INVALID_ARG, "chip arrays are NULL");

  BLOB_T0();
  // chips sorted by (cell, polygon id, input row): chunks sorted in parallel, merged in
  // parallel rounds
  HVec<int64_t> order(n_chips);
  for (int64_t i = 0; i < n_chips; i++) order[i] = i;
  parallel_sort(order, [&](int64_t a, int64_t b) {
    if (cell[a] != cell[b]) return cell[a] < cell[b];
    if (polygon_id[a] != polygon_id[b]) return polygon_id[a] < polygon_id[b];
    return a < b;
  });
  BLOB_MARK("sort");

  // the chips' WKB parsed in parallel: each chunk of sorted chips into its own flat
  // geometry, then the chunks concatenated with their offsets shifted
  mgpu::wkb::Flat geo;  // parts / rings / vertices of all chips, in sorted order
  HVec<int32_t> cpoly(n_chips);
  HVec<uint8_t> cflags(n_chips);
  HVec<uint32_t> cpart(n_chips + 1);
  HVec<double> cenv(4 * (size_t)n_chips);
  HVec<int64_t> crow(n_chips);
  HVec<uint32_t> row2chip(n_chips);
  {
    const int64_t G = kBlobChunk, NC = (n_chips + G - 1) / G;
    std::vector<mgpu::wkb::Flat> cf(NC);
    std::vector<int32_t> cst(NC, MGPU_OK);
    std::vector<std::string> cmsg(NC);
    mgpu::parallel_for(NC, 1, [&](int64_t kb, int64_t ke, int) {
      for (int64_t k = kb; k < ke; k++) {
        mgpu::wkb::Flat& f = cf[k];
        for (int64_t s = k * G; s < std::min(n_chips, (k + 1) * G) && cst[k] == MGPU_OK; s++) {
          const int64_t i = order[s];
          cpoly[s] = polygon_id[i];
          crow[s] = i;
          row2chip[i] = (uint32_t)s;
          cpart[s] = (uint32_t)f.part_ring.size() - 1;  // (local: shifted below)
          uint8_t fl = is_core[i] ? mgpu::kChipCore : 0;
          const int64_t b = wkb_offsets[i], e = wkb_offsets[i + 1];
          double env[4] = {INFINITY, INFINITY, -INFINITY, -INFINITY};
          if (e < b) {
            cst[k] = MGPU_E_INVALID_ARG;
            cmsg[k] = "wkb_offsets not ascending at row " + std::to_string(i);
          } else if (e == b) {
            if (!is_core[i]) {
              cst[k] = MGPU_E_WKB;
              cmsg[k] = "border chip row " + std::to_string(i) + " has NULL geometry";
            }
            fl |= mgpu::kChipNoGeom;
          } else {
            mgpu::wkb::GeomInfo gi;
            std::string msg;
            if (!mgpu::wkb::parse(wkb + b, (size_t)(e - b), f, gi, msg)) {
              cst[k] = MGPU_E_WKB;
              cmsg[k] = "chip row " + std::to_string(i) + ": " + msg;
            }
            if (gi.multi) fl |= mgpu::kChipMulti;
            if (gi.n_points == 0) fl |= mgpu::kChipEmpty;
            if (gi.rectangle) fl |= mgpu::kChipRect;
            for (int q = 0; q < 4; q++) env[q] = gi.env[q];
          }
          cflags[s] = fl;
          for (int q = 0; q < 4; q++) cenv[4 * s + q] = env[q];
        }
      }
    });
    for (int64_t k = 0; k < NC; k++)  // the first failing row in sorted order
      if (cst[k] != MGPU_OK) return fail(cst[k], "%s", cmsg[k].c_str());
    // chunk k's parts, rings and vertices start after those of chunks < k
    std::vector<size_t> p0(NC + 1, 0), r0(NC + 1, 0), v0(NC + 1, 0);
    for (int64_t k = 0; k < NC; k++) {
      p0[k + 1] = p0[k] + cf[k].part_ring.size() - 1;
      r0[k + 1] = r0[k] + cf[k].ring_vtx.size() - 1;
      v0[k + 1] = v0[k] + cf[k].vtx.size() / 2;
    }
    geo.part_ring.assign(p0[NC] + 1, 0);
    geo.ring_vtx.assign(r0[NC] + 1, 0);
    geo.ring_env.resize(4 * r0[NC]);
    geo.vtx.resize(2 * v0[NC]);
    mgpu::parallel_for(NC, 1, [&](int64_t kb, int64_t ke, int) {
      for (int64_t k = kb; k < ke; k++) {
        const mgpu::wkb::Flat& f = cf[k];
        for (size_t q = 1; q < f.part_ring.size(); q++) geo.part_ring[p0[k] + q] = (uint32_t)(f.part_ring[q] + r0[k]);
        for (size_t q = 1; q < f.ring_vtx.size(); q++) geo.ring_vtx[r0[k] + q] = (uint32_t)(f.ring_vtx[q] + v0[k]);
        std::copy(f.ring_env.begin(), f.ring_env.end(), geo.ring_env.begin() + 4 * r0[k]);
        std::copy(f.vtx.begin(), f.vtx.end(), geo.vtx.begin() + 2 * v0[k]);
        for (int64_t s = k * G; s < std::min(n_chips, (k + 1) * G); s++) cpart[s] += (uint32_t)p0[k];
      }
    });
    if (r0[NC] > 0xFFFFFFFFull || v0[NC] > 0xFFFFFFFFull)
      return fail(MGPU_E_UNSUPPORTED, "chip table too large (%zu rings, %zu vertices)", r0[NC], v0[NC]);
  }
  cpart[n_chips] = (uint32_t)geo.part_ring.size() - 1;
  BLOB_MARK("parse");

  // cell hash over the distinct cells
  // (chunks of sorted chips, each starting at a cell's first chip, in parallel)
  std::vector<mgpu::HashSlot> distinct;
  {
    const int64_t NC = (n_chips + kBlobChunk - 1) / kBlobChunk;
    std::vector<std::vector<mgpu::HashSlot>> cd(NC);
    std::vector<int64_t> crowd(NC, -1);  // a cell of more than 65535 chips (its first sorted chip)
    mgpu::parallel_for(NC, 1, [&](int64_t kb, int64_t ke, int) {
      for (int64_t k = kb; k < ke; k++) {
        int64_t s = k * kBlobChunk;
        const int64_t lim = std::min(n_chips, (k + 1) * kBlobChunk);
        while (s > 0 && s < lim && cell[order[s]] == cell[order[s - 1]]) s++;  // (the previous chunk's cell)
        while (s < lim) {
          int64_t e = s;
          const uint64_t c = (uint64_t)cell[order[s]];
          while (e < n_chips && (uint64_t)cell[order[e]] == c) e++;
          if (e - s > 0xFFFF) {
            crowd[k] = s;
            break;
          }
          uint16_t core = 0;
          for (int64_t j = 0; j < e - s && j < 16; j++)
            if (cflags[s + j] & mgpu::kChipCore) core |= (uint16_t)(1u << j);
          cd[k].push_back(mgpu::HashSlot{c, (uint32_t)s, (uint16_t)(e - s), core});
          s = e;
        }
      }
    });
    size_t nd = 0;
    for (int64_t k = 0; k < NC; k++) {
      if (crowd[k] >= 0)
        return fail(MGPU_E_INVALID_ARG, "more than 65535 chips share cell %lld", (long long)cell[order[crowd[k]]]);
      nd += cd[k].size();
    }
    distinct.reserve(nd);
    for (int64_t k = 0; k < NC; k++) distinct.insert(distinct.end(), cd[k].begin(), cd[k].end());
  }
  BLOB_MARK("distinct");
  // The cell side (H3 lattice keys and whole cells, the dense grid, the cell hash) needs
  // only the distinct cells and the parsed geometry: it runs on its own thread while this
  // one builds the strips and chip headers (independent work; the same results)
  int32_t probe_mode = mgpu::kProbeCellId, lres = -1;
  uint32_t face_mask = (1u << 20) - 1;
  double bbox[4] = {-1e300, -1e300, 1e300, 1e300};
  std::vector<mgpu::HashSlot> entries;
  std::vector<std::pair<uint64_t, uint32_t>> keys;
  std::vector<uint64_t> grid;
  mgpu::DenseFace dense[20];
  memset(dense, 0, sizeof dense);
  uint32_t bng_edge = 0;
  uint32_t cap = 16;
  std::vector<mgpu::HashSlot> slots;
  uint32_t max_probe = 0;
  const HVec<uint8_t> cflags_pre = cflags;  // (build_strips adds kChipNoStrips to cflags meanwhile)
  auto cell_side = [&]() -> int32_t {
  SIDE_T0();
  // H3: probe by lattice key when possible (chip_table.h)
  if (index_system == MGPU_H3 && build_lattice(distinct, keys, &lres, &face_mask, bbox)) {
    probe_mode = mgpu::kProbeLattice;
    SIDE_MARK("lattice");
    mark_whole_cells(distinct, lres, bbox, cflags_pre, cpart, geo);
    SIDE_MARK("whole");
    parallel_sort(keys, [](const std::pair<uint64_t, uint32_t>& a, const std::pair<uint64_t, uint32_t>& b) { return a < b; });
    SIDE_MARK("sort");
    // (per key in parallel: duplicate / collision, the entry's core mask; then in order)
    const int64_t nk = (int64_t)keys.size();
    std::vector<uint8_t> kdup(nk);
    std::vector<uint16_t> kcore(nk);
    std::atomic<bool> collide{false};
    mgpu::parallel_for(nk, 4096, [&](int64_t kb, int64_t ke, int) {
      for (int64_t k = kb; k < ke; k++) {
        kdup[k] = k && keys[k].first == keys[k - 1].first;
        if (kdup[k]) {
          if (keys[k].second != keys[k - 1].second) collide = true;
          continue;
        }
        const mgpu::HashSlot& d = distinct[keys[k].second];
        uint16_t core = d.core_mask;
        if (core & mgpu::kCoreWhole) {  // (the whole-cell flag only where the key's face is the cell's home face)
          int hf, r_;
          mgpu::h3::IJK hijk;
          if (!mgpu::h3::h3_home_face_ijk(d.cell, &hf, &hijk, &r_) || (int)(keys[k].first >> 56) != hf)
            core = (uint16_t)(core & ~mgpu::kCoreWhole);
        }
        kcore[k] = core;
      }
    });
    if (collide) return fail(MGPU_E_INTERNAL, "lattice key collision");
    SIDE_MARK("keys");
    entries.reserve(nk);
    for (int64_t k = 0; k < nk; k++) {
      if (kdup[k]) continue;
      const mgpu::HashSlot& d = distinct[keys[k].second];
      entries.push_back(mgpu::HashSlot{keys[k].first, d.first, d.count, kcore[k]});
    }
  } else {
    entries = distinct;
    if (index_system == MGPU_H3 && !distinct.empty()) lres = (int32_t)((distinct[0].cell >> 52) & 15);
  }
  // dense lattice grid when the chip cells' (a, b) boxes are compact: one load per
  // point instead of a hash probe sequence (misses -- most points -- included)
  if (probe_mode == mgpu::kProbeLattice && !entries.empty()) {
    int64_t amin[20], amax[20], bmin[20], bmax[20];
    for (int f = 0; f < 20; f++) amin[f] = bmin[f] = INT64_MAX, amax[f] = bmax[f] = INT64_MIN;
    auto dec = [](uint64_t key, int* f, int64_t* a, int64_t* b) {
      *f = (int)(key >> 56);
      *a = (int64_t)((key >> 28) & 0xFFFFFFFULL) - (1 << 27);
      *b = (int64_t)(key & 0xFFFFFFFULL) - (1 << 27);
    };
    {
      // (per-thread extents, then combined: the same minima and maxima)
      const int64_t ne = (int64_t)entries.size();
      const int T = mgpu::parallel_slots(ne, 1 << 16);
      std::vector<std::array<int64_t, 80>> ext(T);
      for (auto& x : ext)
        for (int f = 0; f < 20; f++) x[f] = x[40 + f] = INT64_MAX, x[20 + f] = x[60 + f] = INT64_MIN;
      mgpu::parallel_for(ne, 1 << 16, [&](int64_t kb, int64_t ke, int t) {
        auto& x = ext[t];
        for (int64_t k = kb; k < ke; k++) {
          int f;
          int64_t a, b;
          dec(entries[k].cell, &f, &a, &b);
          x[f] = std::min(x[f], a), x[20 + f] = std::max(x[20 + f], a);
          x[40 + f] = std::min(x[40 + f], b), x[60 + f] = std::max(x[60 + f], b);
        }
      });
      for (auto& x : ext)
        for (int f = 0; f < 20; f++) {
          amin[f] = std::min(amin[f], x[f]), amax[f] = std::max(amax[f], x[20 + f]);
          bmin[f] = std::min(bmin[f], x[40 + f]), bmax[f] = std::max(bmax[f], x[60 + f]);
        }
    }
    int64_t total = 0;
    for (int f = 0; f < 20; f++)
      if (amax[f] >= amin[f]) total += (amax[f] - amin[f] + 1) * (bmax[f] - bmin[f] + 1);
    if (total <= std::max<int64_t>(16 * (int64_t)entries.size(), 1 << 20) && total <= (1LL << 26)) {
      uint32_t base = 0;
      for (int f = 0; f < 20; f++) {
        if (amax[f] < amin[f]) continue;
        dense[f].a0 = (int32_t)amin[f];
        dense[f].b0 = (int32_t)bmin[f];
        dense[f].w = (uint32_t)(amax[f] - amin[f] + 1);
        dense[f].h = (uint32_t)(bmax[f] - bmin[f] + 1);
        dense[f].base = base;
        base += dense[f].w * dense[f].h;
      }
      // (zeroed and filled on the host threads: each entry owns its grid position)
      grid.resize(base);
      mgpu::parallel_for((int64_t)base, 1 << 20, [&](int64_t kb, int64_t ke, int) {
        std::fill(grid.begin() + kb, grid.begin() + ke, 0ull);
      });
      mgpu::parallel_for((int64_t)entries.size(), 1 << 16, [&](int64_t kb, int64_t ke, int) {
        for (int64_t k = kb; k < ke; k++) {
          const auto& e = entries[k];
          int f;
          int64_t a, b;
          dec(e.cell, &f, &a, &b);
          grid[dense[f].base + (b - dense[f].b0) * dense[f].w + (a - dense[f].a0)] =
              (uint64_t)e.first | ((uint64_t)e.count << 32) | ((uint64_t)e.core_mask << 48);
        }
      });
      probe_mode = mgpu::kProbeDense;
    }
  }
  if (index_system == MGPU_BNG && build_bng_dense(distinct, &lres, &dense[0], &bng_edge, grid))
    probe_mode = mgpu::kProbeDense;
  SIDE_MARK("dense");
  while (cap < 2 * entries.size()) cap <<= 1;
  slots.assign(cap, mgpu::HashSlot{0, 0, 0, 0});
  for (const auto& d : entries) {
    uint32_t h = mgpu::cell_hash(d.cell) & (cap - 1), k = 0;
    while (slots[h].count) {
      h = (h + 1) & (cap - 1);
      k++;
    }
    slots[h] = d;
    max_probe = std::max(max_probe, k);
  }
  SIDE_MARK("hash");

    return MGPU_OK;
  };
  int32_t side_st = MGPU_OK;
  std::string side_msg;  // (the error text is thread-local: carried back)
  std::thread side;
  try {
    side = std::thread([&] {
      side_st = cell_side();
      if (side_st != MGPU_OK) side_msg = g_err;
    });
  } catch (...) {
    side_st = cell_side();  // (no thread: in turn)
    if (side_st != MGPU_OK) side_msg = g_err;
  }
  Strips strips;
  build_strips(n_chips, cflags, cpart, cenv, geo, strips, kBlobChunk);
  BLOB_MARK("strips");
  std::vector<mgpu::ChipHdr, NoInit<mgpu::ChipHdr>> chdr(n_chips);  // (every header written below)
  {
    // host view of the flattened geometry for the grid classification
    mgpu::ChipTableView hv{};
    hv.chip_flags = cflags.data();
    hv.chip_part = cpart.data();
    hv.chip_env = cenv.data();
    hv.part_ring = geo.part_ring.data();
    hv.ring_vtx = geo.ring_vtx.data();
    hv.ring_env = geo.ring_env.data();
    hv.vtx = geo.vtx.data();
    // chips are independent: headers and classification grids in parallel
    mgpu::parallel_for(n_chips, 1024, [&](int64_t cb, int64_t ce, int) {
    for (int64_t c = cb; c < ce; c++) {
      mgpu::ChipHdr& h = chdr[c];
      memset(&h, 0, sizeof h);
      for (int k = 0; k < 4; k++) h.env[k] = cenv[4 * c + k];
      h.inv_h = strips.chip_sy[2 * c + 1];
      h.strip_base = strips.chip_strip[c];
      h.n_strips = (uint16_t)(strips.chip_strip[c + 1] - strips.chip_strip[c]);
      h.flags = cflags[c];
      const uint32_t pb = cpart[c], pe = cpart[c + 1];
      h.single_ring = (pe - pb == 1 && geo.part_ring[pb + 1] - geo.part_ring[pb] == 1 &&
                       !(cflags[c] & mgpu::kChipMulti)) ? 1 : 0;
      if (h.n_strips) build_grid(hv, (uint32_t)c, geo, h);
    }
    });
  }
  BLOB_MARK("headers");
  if (side.joinable()) side.join();
  if (side_st != MGPU_OK) return fail(side_st, "%s", side_msg.c_str());
  BLOB_MARK("cells");
  BLOB_MARK("dense");
  // pixel index over the dense grid (chip_table.h, build_raster_*), BNG cell answer grids
  Raster raster;
  CellAnswers cell_ans;
  if (probe_mode == mgpu::kProbeDense) {
    mgpu::ChipTableView hv{};
    hv.chip_poly = cpoly.data();
    hv.chip_flags = cflags.data();
    hv.chip_part = cpart.data();
    hv.chip_env = cenv.data();
    hv.part_ring = geo.part_ring.data();
    hv.ring_vtx = geo.ring_vtx.data();
    hv.ring_env = geo.ring_env.data();
    hv.vtx = geo.vtx.data();
    bool ok = index_system == MGPU_H3
                  ? build_raster_h3(hv, lres, mgpu::h3::k_of_res(lres), bbox, dense, grid, raster, bo)
                  : build_raster_bng(hv, dense[0], bng_edge, grid, raster, bo);
    if (!ok) raster = Raster{};
    if (index_system == MGPU_BNG && !build_cell_answers(hv, dense[0], bng_edge, grid, cell_ans)) cell_ans = CellAnswers{};
  }
  BLOB_MARK("raster");
#ifdef MGPU_BLOB_TIMING
  fprintf(stderr, "[blob] raster mode %d, %u x %u pixels, %zu classes (one-match below %u)\n", raster.mode, raster.nx,
          raster.ny, raster.cls.size(), raster.pc[0]);
#endif
  BLOB_MARK("hash");
  // lonlat classes with one match -> their polygon (ChipTableView::raster_cls_poly)
  std::vector<int32_t> cls_poly;
  if (raster.mode == mgpu::kRasterLonLat) {
    cls_poly.assign(raster.cls.size(), -1);
    for (size_t c = 1; c < raster.cls.size(); c++) {
      const uint32_t m = (uint32_t)(raster.cls[c] >> 32);
      if (__builtin_popcount(m) == 1) cls_poly[c] = cpoly[(uint32_t)raster.cls[c] + __builtin_ctz(m)];
    }
  }
  // one blob
  struct Part {
    const void* src;
    size_t bytes;
    size_t off;
  };
  std::vector<Part> parts = {
      {slots.data(), slots.size() * sizeof(mgpu::HashSlot), 0},
      {cpoly.data(), cpoly.size() * 4, 0},
      {cflags.data(), cflags.size(), 0},
      {cpart.data(), cpart.size() * 4, 0},
      {cenv.data(), cenv.size() * 8, 0},
      {crow.data(), crow.size() * 8, 0},
      {geo.part_ring.data(), geo.part_ring.size() * 4, 0},
      {geo.ring_vtx.data(), geo.ring_vtx.size() * 4, 0},
      {geo.ring_env.data(), geo.ring_env.size() * 8, 0},
      {geo.vtx.data(), geo.vtx.size() * 8, 0},
      {row2chip.data(), row2chip.size() * 4, 0},
      {strips.chip_strip.data(), strips.chip_strip.size() * 4, 0},
      {strips.chip_sy.data(), strips.chip_sy.size() * 8, 0},
      {strips.strip_edge.data(), strips.strip_edge.size() * 4, 0},
      {strips.edges.data(), strips.edges.size() * 8, 0},
      {strips.edge_ring.data(), strips.edge_ring.size(), 0},
      {chdr.data(), chdr.size() * sizeof(mgpu::ChipHdr), 0},
      {grid.data(), grid.size() * 8, 0},
      {raster.cells.data(), raster.cells.size() * 2, 0},
      {raster.cls.data(), raster.cls.size() * 8, 0},
      {raster.rank.data(), raster.rank.size() * sizeof(mgpu::RankWord), 0},
      {raster.sub.data(), raster.sub.size() * 2, 0},
      {raster.blk.data(), raster.blk.size() * 2, 0},
      {cls_poly.data(), cls_poly.size() * 4, 0},
      {raster.band.data(), raster.band.size() * 4, 0},
      {cell_ans.row.data(), cell_ans.row.size() * 4, 0},
      {cell_ans.ans.data(), cell_ans.ans.size() * 2, 0},
      {raster.pal.data(), raster.pal.size() * 8, 0},
      {raster.idx2.data(), raster.idx2.size(), 0},
  };
  size_t total = kBlobHeaderBytes;
  BlobHeader hdr{};
  hdr.magic = kBlobMagic;
  hdr.version = kBlobVersion;
  hdr.hash_mask = cap - 1;
  hdr.max_probe = max_probe;
  hdr.n_chips = (uint32_t)n_chips;
  hdr.n_cells = (uint32_t)distinct.size();
  hdr.n_vertices = (int64_t)geo.vtx.size() / 2;
  hdr.probe_mode = probe_mode;
  memcpy(hdr.dense, dense, sizeof dense);
  hdr.res = lres;
  hdr.face_mask = face_mask;
  for (int k = 0; k < 4; k++) hdr.bbox[k] = bbox[k];
  hdr.k_res = index_system == MGPU_H3 && lres >= 0 ? mgpu::h3::k_of_res(lres) : 0.0;
  hdr.bng_edge = bng_edge;
  hdr.bng_inv_edge = bng_edge ? 1.0 / bng_edge : 0.0;
  hdr.index_system = index_system;
  for (const auto& d : distinct) hdr.max_cell_chips = std::max<uint32_t>(hdr.max_cell_chips, d.count);
  hdr.raster_mode = raster.mode;
  hdr.raster_nx = raster.nx;
  hdr.raster_ny = raster.ny;
  hdr.raster_pix = raster.pix;
  hdr.raster_px0 = raster.px0;
  hdr.raster_py0 = raster.py0;
  hdr.raster_x0 = raster.x0;
  hdr.raster_y0 = raster.y0;
  hdr.raster_inv_dx = raster.inv_dx;
  hdr.raster_inv_dy = raster.inv_dy;
  for (int k = 0; k < 4; k++) hdr.raster_pc[k] = raster.pc[k];
  hdr.raster_sub_n = raster.sub_n;
  hdr.raster_sub_w = raster.sub_w;
  hdr.raster_bshift = raster.bshift;
  hdr.raster_bnx = raster.bnx;
  hdr.raster_bny = raster.bny;
  hdr.raster_ncls = (uint32_t)cls_poly.size();
  hdr.raster_band_shift = raster.band_shift;
  hdr.raster_nband = (uint32_t)raster.band.size();
  hdr.cell_ans_g = cell_ans.g;
  hdr.cell_ans_sw = cell_ans.sw;
  hdr.raster_pal = raster.pal.empty() ? 0u : 1u;
  for (size_t k = 0; k < parts.size(); k++) {
    parts[k].off = total;
    hdr.off[k] = total;
    total = align_up(total + std::max<size_t>(parts[k].bytes, 1), 256);
  }
  hdr.blob_bytes = total;
  // the header, each array and the zero padding behind it, in pieces of <= 64 MiB
  std::vector<BlobPiece> pieces;
  pieces.push_back({0, (const uint8_t*)&hdr, sizeof hdr, kBlobHeaderBytes - sizeof hdr});
  for (size_t k = 0; k < parts.size(); k++) {
    const size_t end = k + 1 < parts.size() ? parts[k + 1].off : total;
    const size_t pad = end - parts[k].off - parts[k].bytes;
    for (size_t o = 0; o < parts[k].bytes; o += (64u << 20)) {
      const size_t b = std::min(parts[k].bytes - o, (size_t)64 << 20);
      pieces.push_back({parts[k].off + o, (const uint8_t*)parts[k].src + o, b, 0});
    }
    pieces.push_back({parts[k].off + parts[k].bytes, nullptr, 0, pad});
  }
  hdr_out = hdr;
  auto release = [&] {
    release_async(order, geo, cpoly, cflags, cpart, cenv, crow, row2chip, distinct, strips, chdr, keys, entries,
                  grid, raster, cell_ans, slots, cls_poly);
  };
  if (sink) {
    const int32_t st = (*sink)(total, pieces);
    BLOB_MARK("sink");
    release();
    return st;
  }
  if (!host.alloc(total)) return fail(MGPU_E_INTERNAL, "out of host memory (%zu bytes)", total);
  mgpu::parallel_for((int64_t)pieces.size(), 1, [&](int64_t qb, int64_t qe, int) {
    for (int64_t q = qb; q < qe; q++)
      fill_from_pieces(pieces, host.data() + pieces[q].off, pieces[q].off, pieces[q].bytes + pieces[q].zero);
  });
  release();
  BLOB_MARK("assemble");
  return MGPU_OK;
}

static int32_t check_build_opts(const mgpu_build_opts& o) {
  if ((o.raster != 0 && o.raster != 1) || (o.raster_bng != 0 && o.raster_bng != 1) ||
      !(o.raster_sub == 0 || (o.raster_sub >= 2 && o.raster_sub <= 16)) || o.raster_milli < 10 || o.raster_milli > 1000)
    return fail(MGPU_E_INVALID_ARG, "build options out of range (raster %d, raster_bng %d, raster_sub %d, raster_milli %d)",
                o.raster, o.raster_bng, o.raster_sub, o.raster_milli);
  return MGPU_OK;
}

static mgpu_build_opts build_opts_of(const mgpu_ctx* ctx) {
  mgpu_build_opts o;
  o.raster = (int32_t)ctx->opt.raster;
  o.raster_bng = (int32_t)ctx->opt.raster_bng;
  o.raster_sub = (int32_t)ctx->opt.raster_sub;
  o.raster_milli = (int32_t)ctx->opt.raster_milli;
  return o;
}

// A blob header read back from memory: magic, version, sizes and array offsets checked.
static int32_t check_header(const BlobHeader& hdr, int64_t bytes) {
  if (hdr.magic != kBlobMagic || hdr.version != kBlobVersion) return fail(MGPU_E_INVALID_ARG, "not a chip-table blob");
  if ((int64_t)hdr.blob_bytes != bytes) return fail(MGPU_E_INVALID_ARG, "chip-table blob of %lld bytes, header says %llu",
                                                    (long long)bytes, (unsigned long long)hdr.blob_bytes);
  for (int k = 0; k < kBlobArrays; k++)
    if (hdr.off[k] < kBlobHeaderBytes || hdr.off[k] >= (uint64_t)bytes) return fail(MGPU_E_INVALID_ARG, "corrupt chip-table blob");
  if (hdr.index_system != MGPU_H3 && hdr.index_system != MGPU_BNG) return fail(MGPU_E_INVALID_ARG, "corrupt chip-table blob");
  return MGPU_OK;
}

namespace mgpu {
int64_t blob_bytes_of_header(const void* header) {
  BlobHeader h;
  memcpy(&h, header, sizeof h);
  if (h.magic != kBlobMagic || h.version != kBlobVersion) return 0;
  return (int64_t)h.blob_bytes;
}

int32_t adopt_device_blob(mgpu_ctx* ctx, void* dev_blob, int64_t bytes, mgpu_chips** out) {
  BlobHeader hdr;
  HIP_TRY(hipMemcpy(&hdr, dev_blob, sizeof hdr, hipMemcpyDeviceToHost));
  if (int32_t st = check_header(hdr, bytes)) return st;
  mgpu_chips* ch = new mgpu_chips();
  ch->device = ctx->device;
  ch->blob = dev_blob;
  ch->bytes = (size_t)bytes;
  ch->index_system = hdr.index_system;
  ch->view = view_from_header(hdr, (uint8_t*)ch->blob);
  ch->n_vertices = hdr.n_vertices;
  *out = ch;
  return MGPU_OK;
}
}  // namespace mgpu

extern "C" {

void mgpu_build_opts_default(mgpu_build_opts* o) {
  if (!o) return;
  o->raster = 1;
  o->raster_bng = 0;
  o->raster_sub = 16;
  o->raster_milli = 250;
}

int32_t mgpu_chips_host_blob(int32_t index_system, int64_t n_chips, const int64_t* cell, const int32_t* polygon_id,
                             const uint8_t* is_core, const int64_t* wkb_offsets, const uint8_t* wkb, uint8_t** out,
                             int64_t* bytes) {
  return mgpu_chips_host_blob_ex(index_system, n_chips, cell, polygon_id, is_core, wkb_offsets, wkb, nullptr, out, bytes);
}

int32_t mgpu_chips_host_blob_ex(int32_t index_system, int64_t n_chips, const int64_t* cell, const int32_t* polygon_id,
                                const uint8_t* is_core, const int64_t* wkb_offsets, const uint8_t* wkb,
                                const mgpu_build_opts* opts, uint8_t** out, int64_t* bytes) {
  if (!out || !bytes) return fail(MGPU_E_INVALID_ARG, "out/bytes is NULL");
  mgpu_build_opts bo;
  mgpu_build_opts_default(&bo);
  if (opts) {
    if (int32_t st = check_build_opts(*opts)) return st;
    bo = *opts;
  }
  HostBlob host;
  BlobHeader hdr;
  if (int32_t st = build_blob(index_system, n_chips, cell, polygon_id, is_core, wkb_offsets, wkb, host, hdr, bo))
    return st;
  *bytes = (int64_t)host.size();
  *out = host.release();  // (malloc'd: mgpu_host_free)
  return MGPU_OK;
}

int32_t mgpu_host_free(void* p) {
  free(p);
  return MGPU_OK;
}

int32_t mgpu_host_blob_info(const void* host_blob, int64_t bytes, int32_t* index_system, int64_t* n_chips,
                            int64_t* n_cells, int64_t* n_vertices) {
  if (!host_blob || bytes < (int64_t)kBlobHeaderBytes) return fail(MGPU_E_INVALID_ARG, "blob too small");
  BlobHeader hdr;
  memcpy(&hdr, host_blob, sizeof hdr);
  if (int32_t st = check_header(hdr, bytes)) return st;
  if (index_system) *index_system = hdr.index_system;
  if (n_chips) *n_chips = hdr.n_chips;
  if (n_cells) *n_cells = hdr.n_cells;
  if (n_vertices) *n_vertices = hdr.n_vertices;
  return MGPU_OK;
}

}  // extern "C"

// Host -> device copy of `bytes` bytes that fill(dst, off, n) produces, through two pinned
// 64 MiB staging buffers: the host threads fill one piece while the DMA engine moves the
// other (a pageable hipMemcpy of C3's 5.3 GB blob ran at ~4.6 GB/s on the box).
static hipError_t stage_to_device(void* d, size_t bytes, const std::function<void(uint8_t*, size_t, size_t)>& fill) {
  constexpr size_t kPiece = (size_t)64 << 20;
  if (bytes <= 2 * kPiece) {  // (small: one pageable buffer)
    std::vector<uint8_t> tmp(bytes);
    mgpu::parallel_for((int64_t)((bytes + (1 << 20) - 1) >> 20), 1, [&](int64_t b, int64_t en, int) {
      const size_t lo = (size_t)b << 20, hi = std::min(bytes, (size_t)en << 20);
      fill(tmp.data() + lo, lo, hi - lo);
    });
    return hipMemcpy(d, tmp.data(), bytes, hipMemcpyHostToDevice);
  }
  void* stage[2] = {nullptr, nullptr};
  hipEvent_t done[2] = {nullptr, nullptr};
  hipStream_t s = nullptr;
  hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  for (int k = 0; k < 2 && e == hipSuccess; k++) {
    e = hipHostMalloc(&stage[k], kPiece, hipHostMallocDefault);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&done[k], hipEventDisableTiming);
  }
  for (size_t off = 0, k = 0; off < bytes && e == hipSuccess; off += kPiece, k ^= 1) {
    const size_t n = std::min(kPiece, bytes - off);
    if (off >= 2 * kPiece) e = hipEventSynchronize(done[k]);  // the piece this buffer held is on the device
    if (e != hipSuccess) break;
    auto* dst = (uint8_t*)stage[k];
    mgpu::parallel_for((int64_t)((n + (1 << 20) - 1) >> 20), 1, [&](int64_t b, int64_t en, int) {
      const size_t lo = (size_t)b << 20, hi = std::min(n, (size_t)en << 20);
      fill(dst + lo, off + lo, hi - lo);
    });
    e = hipMemcpyAsync((uint8_t*)d + off, stage[k], n, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipEventRecord(done[k], s);
  }
  if (s) {
    const hipError_t e2 = hipStreamSynchronize(s);
    if (e == hipSuccess) e = e2;
    hipStreamDestroy(s);
  }
  for (int k = 0; k < 2; k++) {
    if (done[k]) hipEventDestroy(done[k]);
    if (stage[k]) hipHostFree(stage[k]);
  }
  return e;
}

extern "C" {

int32_t mgpu_chips_upload_blob(mgpu_ctx* ctx, const void* host_blob, int64_t bytes, mgpu_chips** out) {
  if (!ctx || !out) return fail(MGPU_E_INVALID_ARG, "ctx/out is NULL");
  if (int32_t st = mgpu_host_blob_info(host_blob, bytes, nullptr, nullptr, nullptr, nullptr)) return st;
  if (int32_t st = set_device(ctx->device)) return st;
  void* d = nullptr;
  HIP_TRY(hipMalloc(&d, (size_t)bytes));
  hipError_t e = stage_to_device(d, (size_t)bytes, [&](uint8_t* dst, size_t off, size_t n) {
    memcpy(dst, (const uint8_t*)host_blob + off, n);
  });
  if (e != hipSuccess) {
    hipFree(d);
    return fail(MGPU_E_DEVICE, "hipMemcpy: %s", hipGetErrorString(e));
  }
  int32_t st = mgpu::adopt_device_blob(ctx, d, bytes, out);
  if (st) hipFree(d);
  return st;
}

int32_t mgpu_chips_upload(mgpu_ctx* ctx, int32_t index_system, int64_t n_chips, const int64_t* cell,
                          const int32_t* polygon_id, const uint8_t* is_core, const int64_t* wkb_offsets,
                          const uint8_t* wkb, mgpu_chips** out) {
  if (!ctx || !out) return fail(MGPU_E_INVALID_ARG, "ctx/out is NULL");
  HostBlob host;
  BlobHeader hdr;
  if (int32_t st = set_device(ctx->device)) return st;
  // the blob's pieces staged straight to the device (no whole host blob)
  void* d = nullptr;
  size_t bytes = 0;
  const BlobSink sink = [&](size_t total, const std::vector<BlobPiece>& pieces) -> int32_t {
    BLOB_T0();
    HIP_TRY(hipMalloc(&d, total));
    BLOB_MARK("sink:malloc");
    bytes = total;
    const hipError_t e = stage_to_device(d, total, [&](uint8_t* dst, size_t off, size_t n) {
      fill_from_pieces(pieces, dst, off, n);
    });
    if (e != hipSuccess) return fail(MGPU_E_DEVICE, "hipMemcpy: %s", hipGetErrorString(e));
    return MGPU_OK;
  };
  BLOB_T0();
  int32_t st = build_blob(index_system, n_chips, cell, polygon_id, is_core, wkb_offsets, wkb, host, hdr,
                          build_opts_of(ctx), &sink);
  BLOB_MARK("upl:build");
  if (st == MGPU_OK) st = mgpu::adopt_device_blob(ctx, d, (int64_t)bytes, out);
  BLOB_MARK("upl:adopt");
  if (st && d) hipFree(d);
  return st;
}

int32_t mgpu_chips_destroy(mgpu_chips* chips) {
  if (!chips) return MGPU_OK;
  hipSetDevice(chips->device);
  if (chips->blob) hipFree(chips->blob);
  delete chips;
  return MGPU_OK;
}

int32_t mgpu_chips_info(const mgpu_chips* chips, int64_t* n_chips, int64_t* n_cells, int64_t* n_vertices) {
  if (!chips) return fail(MGPU_E_INVALID_ARG, "chips is NULL");
  if (n_chips) *n_chips = chips->view.n_chips;
  if (n_cells) *n_cells = chips->view.n_cells;
  if (n_vertices) *n_vertices = chips->n_vertices;
  return MGPU_OK;
}

int32_t mgpu_chips_device_blob(const mgpu_chips* chips, void** device_ptr, int64_t* bytes) {
  if (!chips || !device_ptr || !bytes) return fail(MGPU_E_INVALID_ARG, "NULL argument");
  *device_ptr = chips->blob;
  *bytes = (int64_t)chips->bytes;
  return MGPU_OK;
}

int32_t mgpu_chips_from_device_blob(mgpu_ctx* ctx, const void* device_ptr, int64_t bytes, mgpu_chips** out) {
  if (!ctx || !device_ptr || !out || bytes <= 0) return fail(MGPU_E_INVALID_ARG, "NULL argument");
  if (int32_t st = set_device(ctx->device)) return st;
  if (bytes < (int64_t)kBlobHeaderBytes) return fail(MGPU_E_INVALID_ARG, "blob too small");
  BlobHeader hdr;
  HIP_TRY(hipMemcpy(&hdr, device_ptr, sizeof hdr, hipMemcpyDeviceToHost));
  if (int32_t st = check_header(hdr, bytes)) return st;
  void* d = nullptr;
  HIP_TRY(hipMalloc(&d, bytes));
  hipError_t e = hipMemcpy(d, device_ptr, bytes, hipMemcpyDeviceToDevice);
  if (e != hipSuccess) {
    hipFree(d);
    return fail(MGPU_E_DEVICE, "hipMemcpy: %s", hipGetErrorString(e));
  }
  int32_t st = mgpu::adopt_device_blob(ctx, d, bytes, out);
  if (st) hipFree(d);
  return st;
}

int32_t mgpu_st_contains(mgpu_ctx* ctx, const mgpu_chips* chips, const int64_t* chip_row, const double* x,
                         const double* y, int64_t n, int8_t* out, void* stream) {
  if (!ctx || !chips) return fail(MGPU_E_INVALID_ARG, "ctx/chips is NULL");
  if (n < 0 || (n > 0 && (!chip_row || !x || !y || !out))) return fail(MGPU_E_INVALID_ARG, "bad arrays");
  if (int32_t st = set_device(ctx->device)) return st;
  if (chips->device != ctx->device)
    return fail(MGPU_E_INVALID_ARG, "chip table lives on device %d, context on device %d", chips->device, ctx->device);
  hipStream_t s = (hipStream_t)stream;
  if (int32_t st = ensure_ws(ctx, 1)) return st;
  auto* counters = (unsigned long long*)ctx->ws;
  HIP_TRY(hipMemsetAsync(counters, 0, kWsCounters, s));
  HIP_TRY(mgpu::launch_st_contains(chips->view, chip_row, x, y, n, out, counters, s));
  unsigned long long h[4] = {0};
  HIP_TRY(hipMemcpyAsync(h, counters, sizeof h, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (h[2])
    return fail(MGPU_E_INVALID_ARG, "st_contains: %llu chip rows outside [0, %u)", h[2], chips->view.n_chips);
  return MGPU_OK;
}

// ------------------------------------------------------------------ join

// The binned pipeline's planner (kernels.h BinArgs): a chip table far larger than the
// caches and a large batch of points.  Option pipeline = MGPU_PIPELINE_BINNED forces it
// whenever it applies; auto takes it for tables of at least bin_min_mb (256 MB -- the
// Infinity Cache) and batches of at least bin_min_points (2^21).  The bins tile the chip
// table's extent (H3: the lon/lat box of the chip cells; BNG: the dense grid's box),
// about bin_count of them (default 64), roughly square on the ground.
static bool plan_bins(const mgpu_options& o, const mgpu_chips* chips, int32_t is, int32_t res, int64_t n,
                      const uint8_t* valid, const mgpu::JoinArgs& a, mgpu::BinArgs& b) {
  const bool forced = o.pipeline == MGPU_PIPELINE_BINNED;
  if (!(forced || o.pipeline == MGPU_PIPELINE_AUTO) || n <= 0 || valid || !a.res_match) return false;
  if (n >= (int64_t)1 << 32 || chips->view.max_cell_chips > 32) return false;
  const mgpu::ChipTableView& v = chips->view;
  double x0, y0, W, H, aspect;
  if (is == MGPU_H3) {
    if (v.probe_mode == mgpu::kProbeCellId || !(v.bbox[2] - v.bbox[0] < 360.0) || !(v.bbox[3] - v.bbox[1] < 180.0))
      return false;
    x0 = v.bbox[0], y0 = v.bbox[1], W = v.bbox[2] - v.bbox[0], H = v.bbox[3] - v.bbox[1];
    const double latc = std::min(std::max(std::fabs(v.bbox[1]), std::fabs(v.bbox[3])), 85.0);
    aspect = W * std::cos(latc * kPi / 180.0) / std::max(H, 1e-12);
  } else {
    if (v.probe_mode != mgpu::kProbeDense || res != v.res || v.bng_edge == 0) return false;
    const mgpu::DenseFace& D = v.dense[0];
    x0 = (double)D.a0 * v.bng_edge, y0 = (double)D.b0 * v.bng_edge;
    W = (double)D.w * v.bng_edge, H = (double)D.h * v.bng_edge;
    aspect = W / std::max(H, 1e-12);
  }
  if (!(W > 0) || !(H > 0)) return false;
  if (!forced && ((double)chips->bytes < (double)o.bin_min_mb * 1048576.0 || n < o.bin_min_points)) return false;
  const int nb = (int)std::min<int64_t>(std::max<int64_t>(o.bin_count, 1), mgpu::bin_max());
  int nbx = (int)std::lround(std::sqrt(nb * aspect));
  nbx = std::min(std::max(nbx, 1), nb);
  const int nby = std::max(nb / nbx, 1);
  b.x0 = x0, b.y0 = y0;
  b.nbx = nbx, b.nby = nby;
  b.inv_bx = nbx / W, b.inv_by = nby / H;
  b.xcd_runs = (int32_t)o.bin_xcd;
  return true;
}

// Launch one join on `s` (nothing waits here).  n_ovr > 0: the route's near-ties take
// the first n_ovr libm overrides of ctx->ovr (ascending input positions, lattice keys).
static int32_t join_impl(mgpu_ctx* ctx, const mgpu_chips* chips, int32_t is, int32_t res, const double* x,
                         const double* y, const int64_t* point_id, int64_t id_base, int64_t n, int64_t capacity,
                         int64_t* out_point, int32_t* out_poly, hipStream_t s, bool timed,
                         const uint8_t* valid = nullptr, int64_t valid_off = 0, int64_t n_ovr = 0,
                         int tie_host = 0) {
  if (!ctx || !chips) return fail(MGPU_E_INVALID_ARG, "ctx/chips is NULL");
  if (int32_t r = check_res(is, res)) return r;
  if (chips->index_system != is)
    return fail(MGPU_E_INVALID_ARG, "chip table built for index system %d, join asked for %d", chips->index_system, is);
  if (chips->device != ctx->device)
    return fail(MGPU_E_INVALID_ARG, "chip table lives on device %d, context on device %d", chips->device, ctx->device);
  if (n < 0 || (n > 0 && (!x || !y))) return fail(MGPU_E_INVALID_ARG, "bad point arrays");
  if (capacity < 0 || (capacity > 0 && (!out_point || !out_poly))) return fail(MGPU_E_INVALID_ARG, "bad output arrays");
  if (int32_t st = set_device(ctx->device)) return st;
  int64_t tiles = mgpu::join_tiles(n);
  // pool: the records of tiles with more pairs than points (bounded by the capacity; a
  // total beyond it is reported as MGPU_E_CAPACITY either way)
  const int64_t pool = capacity;
  if (int32_t st = ensure_ws(ctx, tiles, pool)) return st;
  auto* base = (uint8_t*)ctx->ws;
  const WsLayout L = ws_layout(tiles, pool);
  const mgpu_options& o = ctx->opt;
  mgpu::JoinArgs a;
  a.x = x;
  a.y = y;
  a.n = n;
  a.n_tiles = tiles;
  a.res = res;
  a.res_match = (is == MGPU_BNG || chips->view.res < 0 || chips->view.res == res) ? 1 : 0;
  a.chips = chips->view;
  a.counters = (unsigned long long*)base;
  a.pool_used = a.counters + 5;
  a.n_dirty = (uint32_t*)(a.counters + 6);
  a.dirty = (uint32_t*)(base + L.dirty);
  a.pool_cap = pool;
  a.tile_count = (uint32_t*)(base + L.count);
  a.tile_where = (uint64_t*)(base + L.where);
  a.recs = (uint64_t*)(base + L.recs);
  a.tie_queue = ctx->tq;
  a.tie_cap = ctx->tq_cap;
  a.ovr = ctx->ovr;
  a.n_ovr = n_ovr;
  a.tie_host = (is == MGPU_H3 && tie_host) ? 1 : 0;
  a.pos_of = nullptr;
  mgpu::EmitArgs e;
  e.tile_count = a.tile_count;
  e.group_off = (uint64_t*)(base + L.off);
  a.group_sum = (uint32_t*)(base + L.gsum);
  a.group_cand = a.group_sum + (tiles / 32 + 1);
  e.tile_where = a.tile_where;
  e.recs = a.recs;
  e.point_id = point_id;
  e.id_base = id_base;
  e.capacity = capacity;
  e.out_point = out_point;
  e.out_poly = out_poly;
  a.valid = valid;
  a.valid_off = valid_off;
  a.mixed_idx = nullptr;
  a.mixed_res = nullptr;
  a.chunk_mixed = nullptr;
  a.extra = nullptr;
  a.n_extra = nullptr;
  a.poly_answers = 0;
  HIP_TRY(hipMemsetAsync(base, 0, kWsCounters, s));
  HIP_TRY(hipMemsetAsync(ctx->tq, 0, 16, s));
  // the split pipeline (kernels.h SplitArgs) when the chip table has a pixel index for
  // this resolution and no cell holds more than 32 chips
  // (BNG dense tables without a pixel index: the grid entry is the code -- a cell whose
  // chips are all core answers its points, the rest are mixed; option bng_split)
  const bool bng_grid = is == MGPU_BNG && chips->view.raster_mode == mgpu::kRasterNone &&
                        chips->view.probe_mode == mgpu::kProbeDense && o.bng_split;
  const bool split = (o.pipeline == MGPU_PIPELINE_AUTO || o.pipeline == MGPU_PIPELINE_SPLIT) && n > 0 &&
                     (chips->view.raster_mode != mgpu::kRasterNone || bng_grid) && a.res_match &&
                     (is == MGPU_H3 || res == chips->view.res) && chips->view.max_cell_chips <= 32;
  mgpu::SplitArgs sa{};
  if (split) {
    const int64_t nc = mgpu::split_chunks(n), C = mgpu::split_chunk();
    size_t off = 0;
    auto carve = [&](size_t bytes) {
      const size_t o_ = off;
      off = align_up(off + bytes, 256);
      return o_;
    };
    const size_t o_codes = carve((size_t)nc * C * 4), o_idx = carve((size_t)nc * C * 2), o_res = carve((size_t)nc * C * 8);
    const size_t o_pairs = carve(nc * 4), o_mixed = carve(nc * 4), o_cand = carve(nc * 4), o_off = carve(nc * 8);
    const size_t o_extra = carve((size_t)nc * (C / mgpu::join_tile_points()) * 4);
    if (off > ctx->split_bytes) {
      if (ctx->split_ws) HIP_TRY(hipFree(ctx->split_ws));
      ctx->split_ws = nullptr;
      ctx->split_bytes = 0;
      HIP_TRY(hipMalloc(&ctx->split_ws, off));
      ctx->split_bytes = off;
    }
    auto* sb = (uint8_t*)ctx->split_ws;
    sa.codes = sb + o_codes;
    sa.mixed_idx = (uint16_t*)(sb + o_idx);
    sa.chunk_pairs = (uint32_t*)(sb + o_pairs);
    sa.chunk_mixed = (uint32_t*)(sb + o_mixed);
    sa.chunk_off = (uint64_t*)(sb + o_off);
    a.extra = sa.extra = (uint32_t*)(sb + o_extra);
    a.n_extra = (uint32_t*)(a.counters + 7);  // (zeroed with the counters)
    a.group_sum = sa.chunk_pairs;
    a.group_cand = (uint32_t*)(sb + o_cand);
    a.mixed_idx = sa.mixed_idx;
    a.mixed_res = (uint64_t*)(sb + o_res);
    a.chunk_mixed = sa.chunk_mixed;
    sa.point_id = point_id;
    sa.id_base = id_base;
    sa.capacity = capacity;
    sa.out_point = out_point;
    sa.out_poly = out_poly;
    sa.j = a;
    HIP_TRY(hipMemsetAsync(a.group_cand, 0, nc * 4, s));
  }
  mgpu::BinArgs ba{};
  const bool binned = !split && plan_bins(o, chips, is, res, n, valid, a, ba);
  if (binned) {
    const int64_t nc = mgpu::split_chunks(n), C = mgpu::split_chunk();
    const int64_t K = mgpu::bin_chunks(n), G = mgpu::bin_groups(n), nb = (int64_t)ba.nbx * ba.nby;
    size_t off = 0;
    auto carve = [&](size_t bytes) {
      const size_t o_ = off;
      off = align_up(off + bytes, 256);
      return o_;
    };
    const size_t o_perm = carve((size_t)n * 4), o_rorig = carve((size_t)n * 8);
    const size_t o_bx = carve((size_t)n * 8), o_by = carve((size_t)n * 8),
                 o_pre = carve((size_t)K * nb * 4), o_res = carve((size_t)nc * C * 8), o_cnt = carve((size_t)K * nb * 4),
                 o_gs = carve((size_t)G * nb * 4), o_pairs = carve(nc * 4), o_off = carve(nc * 8),
                 o_gperm = carve(nc * 4), o_gcand = carve(nc * 4);
    // H3 over a dense grid: the scatter kernel's per-slot grid keys (kernels.hip bin_key_of)
    const mgpu::ChipTableView& cv = chips->view;
    uint64_t grid_entries = 0;
    for (int f = 0; f < 20; f++) grid_entries = std::max<uint64_t>(grid_entries, (uint64_t)cv.dense[f].base + (uint64_t)cv.dense[f].w * cv.dense[f].h);
    const bool keyed = is == MGPU_H3 && cv.probe_mode == mgpu::kProbeDense && o.bin_keys && grid_entries < (1ull << 30);
    const size_t o_key = keyed ? carve((size_t)n * 4) : 0;
    if (off > ctx->bin_bytes) {
      if (ctx->bin_ws) HIP_TRY(hipFree(ctx->bin_ws));
      ctx->bin_ws = nullptr;
      ctx->bin_bytes = 0;
      HIP_TRY(hipMalloc(&ctx->bin_ws, off));
      ctx->bin_bytes = off;
    }
    auto* bb = (uint8_t*)ctx->bin_ws;
    ba.x = x;
    ba.y = y;
    ba.bx = (double*)(bb + o_bx);
    ba.by = (double*)(bb + o_by);
    ba.pre = (uint32_t*)(bb + o_pre);
    ba.perm = (uint32_t*)(bb + o_perm);
    ba.res = (uint64_t*)(bb + o_rorig);
    ba.cnt = (uint32_t*)(bb + o_cnt);
    ba.gsum = (uint32_t*)(bb + o_gs);
    ba.key = keyed ? (uint32_t*)(bb + o_key) : nullptr;
    mgpu::JoinArgs j = a;
    j.bin_key = ba.key;
    j.x = ba.bx;
    j.y = ba.by;
    j.mixed_idx = nullptr;
    j.chunk_mixed = nullptr;
    j.poly_answers = 1;
    j.pos_of = ba.perm;
    j.mixed_res = (uint64_t*)(bb + o_res);
    j.group_sum = (uint32_t*)(bb + o_gperm);
    j.group_cand = (uint32_t*)(bb + o_gcand);
    ba.s.j = j;
    ba.s.chunk_pairs = (uint32_t*)(bb + o_pairs);
    ba.s.chunk_off = (uint64_t*)(bb + o_off);
    ba.s.point_id = point_id;
    ba.s.id_base = id_base;
    ba.s.capacity = capacity;
    ba.s.out_point = out_point;
    ba.s.out_poly = out_poly;
    HIP_TRY(hipMemsetAsync(bb + o_gperm, 0, align_up(nc * 4, 256) + nc * 4, s));  // group_sum, group_cand
  } else if (!split) {
    HIP_TRY(hipMemsetAsync(base + L.gsum, 0, 2 * ((size_t)tiles / 32 + 1) * 4, s));
  }
  if (timed) HIP_TRY(hipEventRecord(ctx->ev0, s));
  if (split)
    HIP_TRY(mgpu::launch_split(is, sa, s, timed ? ctx->ev2 : nullptr, timed ? ctx->ev3 : nullptr));
  else if (binned)
    HIP_TRY(mgpu::launch_binned(is, ba, s, timed ? ctx->ev3 : nullptr, timed ? ctx->ev2 : nullptr));
  else
    HIP_TRY(mgpu::launch_join(is, a, e, s, timed ? ctx->ev2 : nullptr));
  if (timed) HIP_TRY(hipEventRecord(ctx->ev1, s));
  auto& L2 = ctx->last;
  L2.split = split;
  L2.sargs = sa;
  L2.binned = binned;
  L2.bargs = ba;
  L2.chips = chips;
  L2.is = is;
  L2.res = res;
  L2.x = x;
  L2.y = y;
  L2.point_id = point_id;
  L2.id_base = id_base;
  L2.n = n;
  L2.pts_valid = valid;
  L2.pts_valid_off = valid_off;
  L2.emit = e;
  L2.jargs = a;
  L2.n_tiles = tiles;
  L2.n_ovr = n_ovr;
  L2.tie_host = a.tie_host;
  L2.pool_ok = false;
  L2.total = -1;
  L2.valid = true;
  L2.stream = (void*)s;
  L2.capacity = capacity;
  L2.out_point = out_point;
  L2.out_poly = out_poly;
  return MGPU_OK;
}

int32_t mgpu_last_near_ties(mgpu_ctx* ctx, int64_t* out_index, int64_t cap, int64_t* out_n) {
  if (!ctx || !out_n || cap < 0 || (cap > 0 && !out_index)) return fail(MGPU_E_INVALID_ARG, "bad arguments");
  *out_n = 0;
  if (!ctx->tq) return MGPU_OK;
  if (int32_t st = set_device(ctx->device)) return st;
  if (ctx->last.valid && ctx->last.n_ovr > 0) {
    // the last join was rerun with the reference's cell of every point its first pass
    // queued: the override table (ascending positions) is the list
    const int64_t n = ctx->last.n_ovr;
    *out_n = n;
    if (n > cap) return fail(MGPU_E_CAPACITY, "%lld near-tie points, capacity %lld", (long long)n, (long long)cap);
    std::vector<uint64_t> hv((size_t)n * 2);
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(hv.data(), ctx->ovr, hv.size() * 8, hipMemcpyDeviceToHost));
    for (int64_t k = 0; k < n; k++) out_index[k] = (int64_t)hv[2 * k];
    return MGPU_OK;
  }
  uint64_t cnt = 0;
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(&cnt, ctx->tq, 8, hipMemcpyDeviceToHost));
  const int64_t n = (int64_t)cnt;
  *out_n = n;
  if (n > ctx->tq_cap)
    return fail(MGPU_E_INTERNAL, "%lld near-tie points: more than the queue of an asynchronous join holds (%lld)",
                (long long)n, (long long)ctx->tq_cap);
  if (n > cap) return fail(MGPU_E_CAPACITY, "%lld near-tie points, capacity %lld", (long long)n, (long long)cap);
  std::vector<uint64_t> rec((size_t)n * 4);
  if (n) HIP_TRY(hipMemcpy(rec.data(), ctx->tq + 2, (size_t)n * 32, hipMemcpyDeviceToHost));
  for (int64_t k = 0; k < n; k++) out_index[k] = (int64_t)rec[4 * k];
  std::sort(out_index, out_index + n);
  return MGPU_OK;
}

}  // extern "C"

// mgpu_pip_join with an optional validity bitmap of the points (the Arrow entry's nulls).
// H3 with the reference's libm: one join in which every point whose fast projection
// falls in its tie band is queued and joined with the fast cell (JoinArgs.tie_host);
// the host recomputes the queued points with the reference's arithmetic (h3_glibc.cpp:
// glibc libm + x87, as H3-Java's JNI library on this host) and, only if a cell moves
// -- the fast path's last bits, or glibc misrounding an argument that decides it --
// runs the join again with the reference's cell of EVERY queued point as an override
// (the fix kernels then take the override without computing the device route).  With
// the correctly rounded libm (option h3_libm) the fix kernels decide the ties by the
// device route.  A near-tie queue that overflowed is grown and the join redone.
// One join's arguments (the synchronous call's, or an asynchronous call's kept until
// mgpu_pip_join_finish).
struct JoinCall {
  const mgpu_chips* chips;
  int32_t is, res;
  const double *x, *y;
  const int64_t* point_id;
  int64_t id_base, n, capacity;
  int64_t* out_point;
  int32_t* out_poly;
  hipStream_t s;
  const uint8_t* valid;
  int64_t valid_off;
  int64_t* d_n_pairs;  // the asynchronous form's device count (or null)
};

static int32_t launch_call(mgpu_ctx* ctx, const JoinCall& c, bool timed, int64_t n_ovr, int tie_host) {
  int32_t st = join_impl(ctx, c.chips, c.is, c.res, c.x, c.y, c.point_id, c.id_base, c.n, c.capacity, c.out_point,
                         c.out_poly, c.s, timed, c.valid, c.valid_off, n_ovr, tie_host);
  if (st) return st;
  if (c.d_n_pairs) HIP_TRY(hipMemcpyAsync(c.d_n_pairs, ctx->ws, 8, hipMemcpyDeviceToDevice, c.s));
  return MGPU_OK;
}

// The override pass of a join whose host libm pass moved a cell: only the units holding
// the overridden points run again (the fused join's tiles; the split pipeline's chunks),
// then -- if some unit's pair count changed -- the scan and the whole emit, else only
// those units' output (kernels.hip launch_join_redo).  The binned pipeline -- its tiles
// hold binned slots -- and a fused join whose first pass used the overflow pool (a rerun
// would take more of it) run whole.
static int32_t launch_override_pass(mgpu_ctx* ctx, const JoinCall& c, bool timed, int64_t n_ovr,
                                    const std::vector<int64_t>& pos, uint64_t pool_used) {
  auto& L = ctx->last;
  if (!L.valid || L.binned || (!L.split && pool_used > 0)) return launch_call(ctx, c, timed, n_ovr, 0);
  // the units, ascending (the positions ascend)
  const int64_t unit = L.split ? mgpu::split_chunk() : mgpu::join_tile_points();
  const int64_t n_units = L.split ? mgpu::split_chunks(L.n) : L.n_tiles;
  std::vector<uint32_t> list;
  for (int64_t p : pos)
    if (list.empty() || list.back() != (uint32_t)(p / unit)) list.push_back((uint32_t)(p / unit));
  if ((int64_t)list.size() * (L.split ? mgpu::split_chunk_tiles() : 1) > L.n_tiles)
    return launch_call(ctx, c, timed, n_ovr, 0);
  const size_t o_aff = 256, o_list = align_up(o_aff + (size_t)n_units, 256), o_old = o_list + list.size() * 4;
  // [0] changed flag, [4] first changed unit (~0), [256] flags per unit, the list, the old counts
  const size_t bytes = o_old + list.size() * 4;
  if (bytes > ctx->redo_bytes) {
    if (ctx->redo) HIP_TRY(hipFree(ctx->redo));
    ctx->redo = nullptr;
    ctx->redo_bytes = 0;
    HIP_TRY(hipMalloc(&ctx->redo, bytes));
    ctx->redo_bytes = bytes;
  }
  auto* rb = (uint8_t*)ctx->redo;
  mgpu::RedoArgs R{(const uint32_t*)(rb + o_list), (uint32_t*)(rb + o_old), rb + o_aff, (uint32_t*)rb,
                   (uint32_t*)(rb + 4)};
  mgpu::JoinArgs a = L.split ? L.sargs.j : L.jargs;
  a.ovr = ctx->ovr;
  a.n_ovr = n_ovr;
  a.tie_host = 0;
  // (the first pass has finished: settle_join waited for its counters)
  HIP_TRY(hipMemsetAsync(rb, 0, o_list, c.s));
  HIP_TRY(hipMemsetAsync(rb + 4, 0xFF, 4, c.s));
  HIP_TRY(hipMemcpyAsync(rb + o_list, list.data(), list.size() * 4, hipMemcpyHostToDevice, c.s));
  const uint32_t nd = L.split ? 0u : (uint32_t)list.size();  // (split: the unpair kernel lists the tiles)
  HIP_TRY(hipMemcpyAsync(a.n_dirty, &nd, 4, hipMemcpyHostToDevice, c.s));
  HIP_TRY(hipStreamSynchronize(c.s));  // (the pageable sources above)
  if (L.split) {
    mgpu::SplitArgs sa = L.sargs;
    sa.j = a;
    HIP_TRY(mgpu::launch_split_redo(c.is, sa, R, (int64_t)list.size(), c.s));
    L.sargs = sa;
  } else {
    HIP_TRY(mgpu::launch_join_redo(c.is, a, L.emit, R, (int64_t)list.size(), c.s));
    L.jargs = a;
  }
  if (timed) HIP_TRY(hipEventRecord(ctx->ev1, c.s));
  if (c.d_n_pairs) HIP_TRY(hipMemcpyAsync(c.d_n_pairs, ctx->ws, 8, hipMemcpyDeviceToDevice, c.s));
  L.n_ovr = n_ovr;
  L.tie_host = 0;
  return MGPU_OK;
}

// After a join's first launch (near-ties queued for the host when reference_libm): read
// its counters; grow an overflowed near-tie queue and launch again; recompute the queued
// points with the reference's libm and, only if a cell moves, launch once more with the
// reference's cell of every queued point as an override.  Overflow relaunches are bounded
// separately from the one override pass, so a completed pass is never reported as a
// failure.  Fills out_n_pairs / stats and the context's record of the last join.
static int32_t settle_join(mgpu_ctx* ctx, const JoinCall& c, bool timed, bool reference_libm, int64_t* out_n_pairs,
                           mgpu_stats* stats) {
  const hipStream_t s = c.s;
  int64_t n_ovr = 0, n_ties = 0, n_moved = 0;
  int overflows = 0;
  uint64_t h[8] = {0};
  for (;;) {
    HIP_TRY(hipMemcpyAsync(ctx->pin, ctx->ws, 16 * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(ctx->pin + 16, ctx->tq, (2 + 4 * kTqHead) * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(stream_wait(ctx, s));
    memcpy(h, ctx->pin, sizeof h);
    const int64_t queued = (int64_t)ctx->pin[16];
    if (h[2]) break;  // invalid coordinates: reported below
    if (queued > ctx->tq_cap) {
      // the queue is sized from this pass's count, so one regrowth holds the next pass
      if (++overflows > 2) return fail(MGPU_E_INTERNAL, "pip_join: the near-tie queue overflowed %d times", overflows);
      if (int32_t e = ensure_tq(ctx, queued + queued / 4 + 1024)) return e;
      if (int32_t e = launch_call(ctx, c, timed, n_ovr, reference_libm && n_ovr == 0)) return e;
      continue;
    }
    if (n_ovr > 0) break;  // the pass with the reference's cells
    n_ties = queued;
    if (!reference_libm || n_ties == 0) break;
    std::vector<TieRec> tr;
    if (int32_t e = read_ties(ctx, n_ties, tr)) return e;
    // (queued once per point: the fix kernels do not queue a tile's points again)
    const auto ref = libm_reference_keys(tr, c.res);
    n_moved = 0;
    for (size_t k = 0; k < tr.size(); k++) n_moved += ref[k].second != tr[k].key;
    if (n_moved == 0) break;
    std::vector<uint64_t> hv(2 * ref.size());
    for (size_t k = 0; k < ref.size(); k++) hv[2 * k] = (uint64_t)ref[k].first, hv[2 * k + 1] = ref[k].second;
    if (int32_t e = ensure_ovr(ctx, (int64_t)hv.size())) return e;
    HIP_TRY(hipMemcpy(ctx->ovr, hv.data(), hv.size() * 8, hipMemcpyHostToDevice));
    n_ovr = (int64_t)ref.size();
    std::vector<int64_t> pos(ref.size());
    for (size_t k = 0; k < ref.size(); k++) pos[k] = (int64_t)ref[k].first;
    if (int32_t e = launch_override_pass(ctx, c, timed, n_ovr, pos, h[5])) return e;
  }
  const int32_t is = c.is;
  const int64_t n = c.n, capacity = c.capacity;
  if (out_n_pairs) *out_n_pairs = (int64_t)h[0];
  if (stats) {
    stats->n_points = n;
    stats->n_pairs = (int64_t)h[0];
    stats->n_near_ties = n_ties;
    stats->n_candidates = (int64_t)h[3];
    stats->libm_overrides = (int32_t)n_moved;
    float ms = 0, ms2 = 0;
    if (timed) {
      hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1);
      if (n > 0) hipEventElapsedTime(&ms2, ctx->ev0, ctx->ev2);
    }
    stats->kernel_ms = ms;
    stats->stream_kernel_ms = ms2;
    stats->mixed_kernel_ms = stats->emit_kernel_ms = 0;
    if (!timed) {
      // (an asynchronous join records no events)
    } else if (ctx->last.split && n > 0) {
      float m3 = 0;
      hipEventElapsedTime(&m3, ctx->ev0, ctx->ev3);
      stats->mixed_kernel_ms = m3 - ms2;
      stats->emit_kernel_ms = ms - m3;
    } else if (ctx->last.binned && n > 0) {
      // ev0 | binning | ev3 | pip_binned_kernel | ev2 | fix, count, scan, emit | ev1
      float m3 = 0;
      hipEventElapsedTime(&m3, ctx->ev0, ctx->ev3);
      stats->mixed_kernel_ms = m3;
      stats->stream_kernel_ms = ms2 - m3;
      stats->emit_kernel_ms = ms - ms2;
    }
    stats->pipeline = ctx->last.split ? MGPU_PIPELINE_SPLIT
                      : ctx->last.binned ? MGPU_PIPELINE_BINNED : MGPU_PIPELINE_FUSED;
  }
  // pool records used (counters[5]) within the pool: every record is still in the
  // workspace, so a larger output can be written by mgpu_pip_join_fetch alone (the split
  // and binned pipelines keep their answers: always)
  ctx->last.total = (int64_t)h[0];
  ctx->last.pool_ok = ctx->last.split || ctx->last.binned || (int64_t)h[5] <= capacity;
  if (h[2]) {
    ctx->last.valid = false;
    if (is == MGPU_BNG) return fail(MGPU_E_NAN, "NaN coordinates are not supported. (%llu points)", (unsigned long long)h[2]);
    return fail(MGPU_E_INVALID_ARG, "Latitude or longitude were invalid. (%llu points)", (unsigned long long)h[2]);
  }
  if ((int64_t)h[0] > capacity)
    return fail(MGPU_E_CAPACITY, "%lld pairs do not fit capacity %lld", (long long)h[0], (long long)capacity);
  return MGPU_OK;
}

static int32_t pip_join_sync(mgpu_ctx* ctx, const mgpu_chips* chips, int32_t is, int32_t res, const double* x,
                             const double* y, const int64_t* point_id, int64_t point_id_base, int64_t n,
                             int64_t capacity, int64_t* out_n_pairs, int64_t* out_point_id, int32_t* out_polygon_id,
                             void* stream, mgpu_stats* stats, const uint8_t* valid, int64_t valid_off) {
  const JoinCall c{chips, is, res, x, y, point_id, point_id_base, n, capacity, out_point_id, out_polygon_id,
                   (hipStream_t)stream, valid, valid_off, nullptr};
  const bool reference_libm = is == MGPU_H3 && ctx && ctx->opt.h3_libm == MGPU_LIBM_REFERENCE;
  if (int32_t st = launch_call(ctx, c, true, 0, reference_libm)) return st;
  return settle_join(ctx, c, true, reference_libm, out_n_pairs, stats);
}

extern "C" {

int32_t mgpu_pip_join(mgpu_ctx* ctx, const mgpu_chips* chips, int32_t is, int32_t res, const double* x,
                      const double* y, const int64_t* point_id, int64_t point_id_base, int64_t n, int64_t capacity,
                      int64_t* out_n_pairs, int64_t* out_point_id, int32_t* out_polygon_id, void* stream,
                      mgpu_stats* stats) {
  return pip_join_sync(ctx, chips, is, res, x, y, point_id, point_id_base, n, capacity, out_n_pairs, out_point_id,
                       out_polygon_id, stream, stats, nullptr, 0);
}

// The asynchronous form: the same first launch as the synchronous call (H3 near-ties
// queued with the fast cell), nothing waits; mgpu_pip_join_finish settles it.
int32_t mgpu_pip_join_async(mgpu_ctx* ctx, const mgpu_chips* chips, int32_t is, int32_t res, const double* x,
                            const double* y, const int64_t* point_id, int64_t point_id_base, int64_t n,
                            int64_t capacity, int64_t* d_n_pairs, int64_t* out_point_id, int32_t* out_polygon_id,
                            void* stream) {
  const JoinCall c{chips, is, res, x, y, point_id, point_id_base, n, capacity, out_point_id, out_polygon_id,
                   (hipStream_t)stream, nullptr, 0, d_n_pairs};
  const bool reference_libm = is == MGPU_H3 && ctx && ctx->opt.h3_libm == MGPU_LIBM_REFERENCE;
  if (int32_t st = launch_call(ctx, c, false, 0, reference_libm)) return st;
  ctx->last.async_pending = true;
  ctx->last.d_n_pairs = d_n_pairs;
  return MGPU_OK;
}

int32_t mgpu_pip_join_finish(mgpu_ctx* ctx, int64_t* out_n_pairs, mgpu_stats* stats) {
  if (!ctx) return fail(MGPU_E_INVALID_ARG, "ctx is NULL");
  auto& L = ctx->last;
  if (!L.valid || !L.async_pending)
    return fail(MGPU_E_INVALID_ARG, "pip_join_finish: no asynchronous join pending on this context");
  if (int32_t st = set_device(ctx->device)) return st;
  const JoinCall c{L.chips, L.is, L.res, L.x, L.y, L.point_id, L.id_base, L.n, L.capacity, L.out_point, L.out_poly,
                   (hipStream_t)L.stream, nullptr, 0, L.d_n_pairs};
  const bool reference_libm = L.tie_host != 0;
  L.async_pending = false;
  return settle_join(ctx, c, false, reference_libm, out_n_pairs, stats);
}

int32_t mgpu_pip_join_fetch(mgpu_ctx* ctx, int64_t capacity, int64_t* out_n_pairs, int64_t* out_point_id,
                            int32_t* out_polygon_id, void* stream) {
  if (!ctx) return fail(MGPU_E_INVALID_ARG, "ctx is NULL");
  auto& L = ctx->last;
  if (!L.valid || L.total < 0) return fail(MGPU_E_INVALID_ARG, "pip_join_fetch: no completed join on this context");
  if (out_n_pairs) *out_n_pairs = L.total;
  if (capacity < L.total)
    return fail(MGPU_E_CAPACITY, "%lld pairs do not fit capacity %lld", (long long)L.total, (long long)capacity);
  if (L.total > 0 && (!out_point_id || !out_polygon_id)) return fail(MGPU_E_INVALID_ARG, "bad output arrays");
  if (int32_t st = set_device(ctx->device)) return st;
  hipStream_t s = (hipStream_t)stream;
  if (!L.pool_ok) {
    // the overflow pool had dropped records: redo the join with a pool that holds them
    const auto c = L;
    int64_t cnt = 0;
    return pip_join_sync(ctx, c.chips, c.is, c.res, c.x, c.y, c.point_id, c.id_base, c.n, capacity,
                         out_n_pairs ? out_n_pairs : &cnt, out_point_id, out_polygon_id, stream, nullptr, c.pts_valid,
                         c.pts_valid_off);
  }
  if (L.binned) {
    mgpu::BinArgs ba = L.bargs;
    ba.s.capacity = capacity;
    ba.s.out_point = out_point_id;
    ba.s.out_poly = out_polygon_id;
    HIP_TRY(mgpu::launch_bin_emit(ba, s));
    HIP_TRY(hipStreamSynchronize(s));
    return MGPU_OK;
  }
  if (L.split) {
    mgpu::SplitArgs sa = L.sargs;
    sa.capacity = capacity;
    sa.out_point = out_point_id;
    sa.out_poly = out_polygon_id;
    HIP_TRY(mgpu::launch_split_emit(L.is, sa, s));
    HIP_TRY(hipStreamSynchronize(s));
    return MGPU_OK;
  }
  mgpu::EmitArgs e = L.emit;
  e.capacity = capacity;
  e.out_point = out_point_id;
  e.out_poly = out_polygon_id;
  HIP_TRY(mgpu::launch_emit(e, L.n_tiles, s));
  HIP_TRY(hipStreamSynchronize(s));
  return MGPU_OK;
}

int32_t mgpu_pip_join_host(mgpu_ctx* ctx, const mgpu_chips* chips, int32_t is, int32_t res, const double* x,
                           const double* y, const int64_t* point_id, int64_t n, int64_t capacity, int64_t* out_n_pairs,
                           int64_t* out_point_id, int32_t* out_polygon_id) {
  if (!ctx) return fail(MGPU_E_INVALID_ARG, "ctx is NULL");
  if (int32_t st = set_device(ctx->device)) return st;
  double *dx = nullptr, *dy = nullptr;
  int64_t *dpid = nullptr, *dop = nullptr;
  int32_t* dpo = nullptr;
  size_t nb = (size_t)std::max<int64_t>(n, 1) * 8, cb = (size_t)std::max<int64_t>(capacity, 1);
  HIP_TRY(hipMalloc(&dx, nb));
  HIP_TRY(hipMalloc(&dy, nb));
  HIP_TRY(hipMalloc(&dop, cb * 8));
  HIP_TRY(hipMalloc(&dpo, cb * 4));
  if (n) {
    HIP_TRY(hipMemcpy(dx, x, n * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(dy, y, n * 8, hipMemcpyHostToDevice));
  }
  if (point_id && n) {
    HIP_TRY(hipMalloc(&dpid, nb));
    HIP_TRY(hipMemcpy(dpid, point_id, n * 8, hipMemcpyHostToDevice));
  }
  int64_t cnt = 0;
  int32_t st = mgpu_pip_join(ctx, chips, is, res, dx, dy, dpid, 0, n, capacity, &cnt, dop, dpo, nullptr, nullptr);
  if (out_n_pairs) *out_n_pairs = cnt;
  if (st == MGPU_OK || st == MGPU_E_CAPACITY) {
    int64_t m = std::min(cnt, capacity);
    if (m > 0) {
      hipMemcpy(out_point_id, dop, m * 8, hipMemcpyDeviceToHost);
      hipMemcpy(out_polygon_id, dpo, m * 4, hipMemcpyDeviceToHost);
    }
  }
  hipFree(dx);
  hipFree(dy);
  hipFree(dop);
  hipFree(dpo);
  if (dpid) hipFree(dpid);
  return st;
}

// TEST ONLY (not part of the reference's interface): builds the chip table on the
// host and evaluates st_contains(chip row, point) for n pairs twice -- by the join's
// path (classification grid + strip index, pip::chip_contains_strips) and by the
// sequential PointLocator (pip::chip_locate) -- so the CPU test suite can check the
// grid/strip exactness claims without a GPU.  out_* = 1 / 0 (-1: NULL geometry).
int32_t mgpu_test_chip_contains_host(int32_t index_system, int64_t n_chips, const int64_t* cell,
                                     const int32_t* polygon_id, const uint8_t* is_core, const int64_t* wkb_offsets,
                                     const uint8_t* wkb, int64_t n, const int64_t* chip_row, const double* x,
                                     const double* y, int8_t* out_join_path, int8_t* out_point_locator) {
  HostBlob host;
  BlobHeader hdr;
  mgpu_build_opts bo;
  mgpu_build_opts_default(&bo);
  if (int32_t st = build_blob(index_system, n_chips, cell, polygon_id, is_core, wkb_offsets, wkb, host, hdr, bo))
    return st;
  const mgpu::ChipTableView v = view_from_header(hdr, host.data());
  for (int64_t i = 0; i < n; i++) {
    const int64_t r = chip_row[i];
    if (r < 0 || r >= n_chips) return fail(MGPU_E_INVALID_ARG, "chip row %lld out of range", (long long)r);
    const uint32_t c = v.row_to_chip[r];
    if (v.chip_flags[c] & mgpu::kChipNoGeom) {
      out_join_path[i] = out_point_locator[i] = -1;
      continue;
    }
    out_join_path[i] = mgpu::pip::chip_contains_strips(v, c, x[i], y[i]) ? 1 : 0;
    out_point_locator[i] = mgpu::pip::chip_locate(v, c, x[i], y[i]) == mgpu::pip::kInterior ? 1 : 0;
  }
  return MGPU_OK;
}

// The H3 whole-cell shortcut (mark_whole_cells + FastHex::deep), looked up as the
// streaming kernels do (dense probe tables): out_kind 1 = answered, the point matches chip
// out_first (out_mask 1); 2 = not answered (not deep, not a flagged cell); 3 = invalid
// coordinate; 4 = the table has no dense H3 probe.  Host pointers; no GPU.
int32_t mgpu_test_whole_cells_host(int32_t index_system, int32_t res, int64_t n_chips, const int64_t* cell,
                                   const int32_t* polygon_id, const uint8_t* is_core, const int64_t* wkb_offsets,
                                   const uint8_t* wkb, int64_t n, const double* x, const double* y, int8_t* out_kind,
                                   uint32_t* out_first, uint32_t* out_mask, int32_t* out_chip_poly) {
  if (index_system != MGPU_H3) return fail(MGPU_E_INVALID_ARG, "whole-cell chips are H3 only");
  HostBlob host;
  BlobHeader hdr;
  mgpu_build_opts bo;
  mgpu_build_opts_default(&bo);
  if (int32_t st = build_blob(index_system, n_chips, cell, polygon_id, is_core, wkb_offsets, wkb, host, hdr, bo))
    return st;
  const mgpu::ChipTableView v = view_from_header(hdr, host.data());
  for (int64_t c = 0; c < n_chips; c++) out_chip_poly[c] = v.chip_poly[c];
  const bool usable = v.probe_mode == mgpu::kProbeDense && v.res == res;
  for (int64_t i = 0; i < n; i++) {
    out_first[i] = out_mask[i] = 0;
    out_kind[i] = usable ? 2 : 4;
    if (!usable) continue;
    if (!std::isfinite(x[i]) || !std::isfinite(y[i])) {
      out_kind[i] = 3;
      continue;
    }
    if (!(x[i] >= v.bbox[0] && x[i] <= v.bbox[2] && y[i] >= v.bbox[1] && y[i] <= v.bbox[3])) continue;
    const mgpu::h3::FastHex f =
        mgpu::h3::fast_hex2d(mgpu::h3::to_radians_fast(y[i]), mgpu::h3::to_radians_fast(x[i]), res, v.k_res, v.face_mask);
    if (!f.deep) continue;
    const mgpu::DenseFace& D = v.dense[f.face];
    const uint32_t da = (uint32_t)(f.ijk.i - f.ijk.k - D.a0), db = (uint32_t)(f.ijk.j - f.ijk.k - D.b0);
    if (da >= D.w || db >= D.h) continue;
    const uint64_t e = v.grid[D.base + db * D.w + da];
    if (((e >> 32) & 0xFFFF) != 1 || !((e >> 48) & mgpu::kCoreWhole)) continue;
    out_kind[i] = 1;
    out_first[i] = (uint32_t)e;
    out_mask[i] = 1;
  }
  return MGPU_OK;
}

// The BNG cell answer grids (ChipTableView::cell_ans), looked up as the fused kernel's
// phase 1 does: out_kind 1 / 0 = answered (matches: chips out_first + j for the bits j of
// out_mask), 2 = not answered (no grid for the cell, a mixed square, outside the dense
// grid), 3 = invalid coordinate, 4 = the table has no answer grids.  Host pointers; no GPU.
int32_t mgpu_test_cell_answers_host(int32_t index_system, int32_t res, int64_t n_chips, const int64_t* cell,
                                    const int32_t* polygon_id, const uint8_t* is_core, const int64_t* wkb_offsets,
                                    const uint8_t* wkb, int64_t n, const double* x, const double* y, int8_t* out_kind,
                                    uint32_t* out_first, uint32_t* out_mask, int32_t* out_chip_poly) {
  if (index_system != MGPU_BNG) return fail(MGPU_E_INVALID_ARG, "cell answer grids are BNG only");
  HostBlob host;
  BlobHeader hdr;
  mgpu_build_opts bo;
  mgpu_build_opts_default(&bo);
  if (int32_t st = build_blob(index_system, n_chips, cell, polygon_id, is_core, wkb_offsets, wkb, host, hdr, bo))
    return st;
  const mgpu::ChipTableView v = view_from_header(hdr, host.data());
  for (int64_t c = 0; c < n_chips; c++) out_chip_poly[c] = v.chip_poly[c];
  const bool usable = v.cell_ans_row != nullptr && v.res == res;
  for (int64_t i = 0; i < n; i++) {
    out_first[i] = out_mask[i] = 0;
    out_kind[i] = usable ? 2 : 4;
    if (!usable) continue;
    if (!(x[i] == x[i] && y[i] == y[i])) {
      out_kind[i] = 3;
      continue;
    }
    const int32_t eI = mgpu::bng::d2i(x[i]), nI = mgpu::bng::d2i(y[i]);
    if (!((uint32_t)eI < 10000000u && (uint32_t)nI < 10000000u)) continue;
    const uint32_t ed = v.bng_edge;
    const uint32_t col = mgpu::div_fix((uint32_t)eI, ed, v.bng_inv_edge), row = mgpu::div_fix((uint32_t)nI, ed, v.bng_inv_edge);
    const mgpu::DenseFace& D = v.dense[0];
    const uint32_t da = col - (uint32_t)D.a0, db = row - (uint32_t)D.b0;
    if (da >= D.w || db >= D.h) continue;
    const uint32_t gi = D.base + db * D.w + da;
    const uint64_t e = v.grid[gi];
    if (!(e & mgpu::kCellAnsFlag)) continue;
    const uint32_t u = mgpu::div_fix((uint32_t)eI - col * ed, v.cell_ans_sw, v.cell_ans_inv_sw);
    const uint32_t w = mgpu::div_fix((uint32_t)nI - row * ed, v.cell_ans_sw, v.cell_ans_inv_sw);
    const uint64_t ai = (uint64_t)v.cell_ans_row[db] + mgpu::cell_ans_index(e);
    const uint16_t m = v.cell_ans[(ai * v.cell_ans_g + w) * v.cell_ans_g + u];
    if (m == mgpu::kCellAnsMixed) continue;
    out_kind[i] = m ? 1 : 0;
    out_first[i] = (uint32_t)v.grid[gi];
    out_mask[i] = m;
  }
  return MGPU_OK;
}

// TEST ONLY (no reference counterpart): builds the chip table on the host and looks up
// n points in its pixel index exactly as the streaming join kernel does (raster.h), so
// the CPU suite can check every pure pixel's answer against the oracle.  Per point:
// out_kind 0 = no match possible (empty pixel / outside the box), 1 = pure pixel (its
// matches are the sorted chips out_first + j for the bits j of out_mask), 2 = mixed
// (full path), 3 = invalid coordinate, 4 = the table has no pixel index.
// out_chip_poly[n_chips] = the polygon id of each sorted chip.  Host pointers; no GPU.
int32_t mgpu_test_raster_host(int32_t index_system, int32_t res, int64_t n_chips, const int64_t* cell,
                              const int32_t* polygon_id, const uint8_t* is_core, const int64_t* wkb_offsets,
                              const uint8_t* wkb, int64_t n, const double* x, const double* y, int8_t* out_kind,
                              uint32_t* out_first, uint32_t* out_mask, int32_t* out_chip_poly) {
  HostBlob host;
  BlobHeader hdr;
  mgpu_build_opts bo;  // (the BNG pixel index too: this hook tests the index itself)
  mgpu_build_opts_default(&bo);
  bo.raster_bng = 1;
  if (int32_t st = build_blob(index_system, n_chips, cell, polygon_id, is_core, wkb_offsets, wkb, host, hdr, bo))
    return st;
  const mgpu::ChipTableView v = view_from_header(hdr, host.data());
  for (int64_t c = 0; c < n_chips; c++) out_chip_poly[c] = v.chip_poly[c];
  const bool usable = v.raster_mode != mgpu::kRasterNone && (index_system == MGPU_H3 ? v.res == res : v.res == res);
  for (int64_t i = 0; i < n; i++) {
    out_first[i] = out_mask[i] = 0;
    if (!usable) {
      out_kind[i] = 4;
      continue;
    }
    bool ok = true;
    uint32_t gi = 0, sub = 0, bi = mgpu::kNoPixel;
    const uint32_t ri = index_system == MGPU_H3 ? mgpu::raster_index<MGPU_H3>(v, x[i], y[i], &ok, &gi, &sub, &bi)
                                                : mgpu::raster_index<MGPU_BNG>(v, x[i], y[i], &ok, &gi, &sub, &bi);
    if (!ok) {
      out_kind[i] = 3;
      continue;
    }
    if (ri == mgpu::kRasterFull) {
      out_kind[i] = 2;
      continue;
    }
    const uint32_t cl = ri == mgpu::kNoPixel ? mgpu::kPixEmpty : mgpu::raster_class_blk(v, v.raster_blk, ri, bi, sub);
    if (cl == mgpu::kPixMixed) {
      out_kind[i] = 2;
      continue;
    }
    uint64_t ce = 0;
    if (cl != mgpu::kPixEmpty)
      ce = index_system == MGPU_BNG ? ((uint64_t)(uint32_t)v.grid[gi] | ((uint64_t)cl << 32)) : v.raster_cls[cl];
    out_kind[i] = ce ? 1 : 0;
    out_first[i] = (uint32_t)ce;
    out_mask[i] = (uint32_t)(ce >> 32);
  }
  return MGPU_OK;
}

int32_t mgpu_test_blob_contains_host(const void* host_blob, int64_t bytes, int64_t n, const int64_t* chip_row,
                                     const double* x, const double* y, int8_t* out) {
  if (int32_t st = mgpu_host_blob_info(host_blob, bytes, nullptr, nullptr, nullptr, nullptr)) return st;
  BlobHeader hdr;
  memcpy(&hdr, host_blob, sizeof hdr);
  const mgpu::ChipTableView v = view_from_header(hdr, (uint8_t*)host_blob);
  for (int64_t i = 0; i < n; i++) {
    const int64_t r = chip_row[i];
    if (r < 0 || r >= (int64_t)v.n_chips) return fail(MGPU_E_INVALID_ARG, "chip row %lld out of range", (long long)r);
    const uint32_t c = v.row_to_chip[r];
    out[i] = (v.chip_flags[c] & mgpu::kChipNoGeom) ? -1 : (mgpu::pip::chip_contains_strips(v, c, x[i], y[i]) ? 1 : 0);
  }
  return MGPU_OK;
}

}  // extern "C"

// ------------------------------------------------------------------ geometry columns, Arrow

static int32_t ensure_scratch(mgpu_ctx* ctx, size_t bytes) {
  if (bytes <= ctx->scratch_bytes) return MGPU_OK;
  if (ctx->scratch) HIP_TRY(hipFree(ctx->scratch));
  ctx->scratch = nullptr;
  ctx->scratch_bytes = 0;
  HIP_TRY(hipMalloc(&ctx->scratch, bytes));
  ctx->scratch_bytes = bytes;
  return MGPU_OK;
}

// decode into (x, y) and check the decode counters
// the decode kernels' counters -> the reference's exception classes
static int32_t decode_status(mgpu_ctx* ctx, int32_t format, hipStream_t s) {
  static const char* names[] = {"WKB", "WKT", "hex WKB", "GeoJSON", "internal geometry"};
  unsigned long long h[8] = {0};
  HIP_TRY(hipMemcpyAsync(h, ctx->ws, sizeof h, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  const char* name = names[format >= 0 && format <= 4 ? format : 0];
  if (h[4]) return fail(MGPU_E_WKB, "%llu rows are not well-formed %s", h[4], name);
  if (h[5])
    return fail(MGPU_E_UNSUPPORTED, "%llu %s rows are of a geometry type whose centroid is not built for this format",
                h[5], name);
  if (h[6]) return fail(MGPU_E_EMPTY, "getX called on empty Point (%llu rows: empty geometries)", h[6]);
  return MGPU_OK;
}

static int32_t decode_points(mgpu_ctx* ctx, int32_t format, const uint8_t* data, const void* offsets, int off32,
                             const uint8_t* valid, int64_t voff, int64_t n, double* x, double* y, hipStream_t s) {
  if (format < MGPU_GEOM_WKB || format > MGPU_GEOM_GEOJSON) return fail(MGPU_E_INVALID_ARG, "geometry format %d", format);
  if (n < 0 || (n > 0 && (!data || !offsets || !x || !y))) return fail(MGPU_E_INVALID_ARG, "bad geometry arrays");
  if (int32_t st = ensure_ws(ctx, 1)) return st;
  auto* counters = (unsigned long long*)ctx->ws;
  HIP_TRY(hipMemsetAsync(counters, 0, kWsCounters, s));
  HIP_TRY(mgpu::launch_decode_points(format, data, offsets, off32, valid, voff, n, x, y, counters, s));
  return decode_status(ctx, format, s);
}

extern "C" {

int32_t mgpu_points_from_geometry(mgpu_ctx* ctx, int32_t format, const uint8_t* data, const int64_t* offsets,
                                  const uint8_t* valid, int64_t valid_offset, int64_t n, double* out_x, double* out_y,
                                  void* stream) {
  if (!ctx) return fail(MGPU_E_INVALID_ARG, "ctx is NULL");
  if (int32_t st = set_device(ctx->device)) return st;
  return decode_points(ctx, format, data, offsets, 0, valid, valid_offset, n, out_x, out_y, (hipStream_t)stream);
}

}  // extern "C"

static int32_t geometry_cells(mgpu_ctx* ctx, int32_t is, int32_t res, int32_t format, const uint8_t* data,
                              const void* offsets, int off32, const uint8_t* valid, int64_t voff, int64_t n,
                              int64_t* out_cell, uint8_t* out_valid, hipStream_t s, mgpu_stats* stats) {
  if (!ctx) return fail(MGPU_E_INVALID_ARG, "ctx is NULL");
  if (int32_t r = check_res(is, res)) return r;
  if (n < 0 || (n > 0 && !out_cell)) return fail(MGPU_E_INVALID_ARG, "bad output array");
  if (int32_t st = set_device(ctx->device)) return st;
  if (int32_t st = ensure_scratch(ctx, (size_t)std::max<int64_t>(n, 1) * 16)) return st;
  double* x = (double*)ctx->scratch;
  double* y = x + std::max<int64_t>(n, 1);
  if (int32_t st = decode_points(ctx, format, data, offsets, off32, valid, voff, n, x, y, s)) return st;
  if (int32_t st = cells_impl(ctx, is, res, x, y, n, out_cell, s, valid, voff, stats)) return st;
  if (out_valid) {
    HIP_TRY(mgpu::launch_valid_and(valid, voff, nullptr, 0, n, out_valid, s));
    HIP_TRY(stream_wait(ctx, s));
  }
  return MGPU_OK;
}

// an Arrow array on this context's GPU with the given format; *data = its values (offset
// applied), *valid / *voff = its validity bitmap (null: no nulls)
static int32_t arrow_column(mgpu_ctx* ctx, const ArrowDeviceArray* a, size_t elem, const void** data,
                            const uint8_t** valid, int64_t* voff, const char* what) {
  if (!a) return fail(MGPU_E_INVALID_ARG, "%s: NULL array", what);
  if (a->device_type != ARROW_DEVICE_ROCM || a->device_id != ctx->device)
    return fail(MGPU_E_INVALID_ARG, "%s: not on this context's GPU (device type %d, id %lld)", what, a->device_type,
                (long long)a->device_id);
  if (a->array.n_buffers < 2 || !a->array.buffers || a->array.length < 0 || a->array.offset < 0)
    return fail(MGPU_E_INVALID_ARG, "%s: not a primitive Arrow array", what);
  if (a->sync_event) HIP_TRY(hipEventSynchronize((hipEvent_t)a->sync_event));
  *data = (const uint8_t*)a->array.buffers[1] + (size_t)a->array.offset * elem;
  *valid = a->array.null_count != 0 ? (const uint8_t*)a->array.buffers[0] : nullptr;
  *voff = a->array.offset;
  return MGPU_OK;
}

extern "C" {

int32_t mgpu_geometry_to_cells(mgpu_ctx* ctx, int32_t index_system, int32_t res, int32_t format, const uint8_t* data,
                               const int64_t* offsets, const uint8_t* valid, int64_t valid_offset, int64_t n,
                               int64_t* out_cell, uint8_t* out_valid, void* stream, mgpu_stats* stats) {
  return geometry_cells(ctx, index_system, res, format, data, offsets, 0, valid, valid_offset, n, out_cell, out_valid,
                        (hipStream_t)stream, stats);
}

int32_t mgpu_internal_geometry_to_cells(mgpu_ctx* ctx, int32_t index_system, int32_t res, int64_t n,
                                        const int32_t* type_id, const int64_t* row_part, const int64_t* part_ring,
                                        const int64_t* ring_off, const double* xy, const uint8_t* valid,
                                        int64_t valid_offset, int64_t* out_cell, uint8_t* out_valid, void* stream,
                                        mgpu_stats* stats) {
  if (!ctx) return fail(MGPU_E_INVALID_ARG, "ctx is NULL");
  if (int32_t r = check_res(index_system, res)) return r;
  if (n < 0 || (n > 0 && (!out_cell || !type_id || !row_part || !part_ring || !ring_off || !xy)))
    return fail(MGPU_E_INVALID_ARG, "bad internal geometry arrays");
  if (int32_t st = set_device(ctx->device)) return st;
  hipStream_t s = (hipStream_t)stream;
  if (int32_t st = ensure_ws(ctx, 1)) return st;
  if (int32_t st = ensure_scratch(ctx, (size_t)std::max<int64_t>(n, 1) * 16)) return st;
  double* x = (double*)ctx->scratch;
  double* y = x + std::max<int64_t>(n, 1);
  HIP_TRY(hipMemsetAsync(ctx->ws, 0, kWsCounters, s));
  HIP_TRY(mgpu::launch_decode_internal(type_id, row_part, part_ring, ring_off, xy, valid, valid_offset, n, x, y,
                                       (unsigned long long*)ctx->ws, s));
  if (int32_t st = decode_status(ctx, 4, s)) return st;
  if (int32_t st = cells_impl(ctx, index_system, res, x, y, n, out_cell, s, valid, valid_offset, stats)) return st;
  if (out_valid) {
    HIP_TRY(mgpu::launch_valid_and(valid, valid_offset, nullptr, 0, n, out_valid, s));
    HIP_TRY(stream_wait(ctx, s));
  }
  return MGPU_OK;
}

int32_t mgpu_geometry_to_cells_arrow(mgpu_ctx* ctx, int32_t index_system, int32_t res,
                                     const struct ArrowDeviceArray* geom, const struct ArrowSchema* schema,
                                     int64_t* out_cell, uint8_t* out_valid, void* stream) {
  if (!ctx || !geom || !schema || !schema->format) return fail(MGPU_E_INVALID_ARG, "NULL argument");
  const char f = schema->format[0];
  if (!((f == 'z' || f == 'Z' || f == 'u' || f == 'U') && schema->format[1] == 0))
    return fail(MGPU_E_INVALID_ARG, "geometry column format '%s': binary (WKB) or utf8 (WKT) expected", schema->format);
  if (geom->device_type != ARROW_DEVICE_ROCM || geom->device_id != ctx->device)
    return fail(MGPU_E_INVALID_ARG, "geometry column not on this context's GPU");
  if (geom->array.n_buffers < 3 || !geom->array.buffers) return fail(MGPU_E_INVALID_ARG, "not a binary Arrow array");
  if (geom->sync_event) HIP_TRY(hipEventSynchronize((hipEvent_t)geom->sync_event));
  const bool o32 = f == 'z' || f == 'u';
  const uint8_t* offs = (const uint8_t*)geom->array.buffers[1] + (size_t)geom->array.offset * (o32 ? 4 : 8);
  const uint8_t* valid = geom->array.null_count != 0 ? (const uint8_t*)geom->array.buffers[0] : nullptr;
  return geometry_cells(ctx, index_system, res, (f == 'z' || f == 'Z') ? MGPU_GEOM_WKB : MGPU_GEOM_WKT,
                        (const uint8_t*)geom->array.buffers[2], offs, o32 ? 1 : 0, valid, geom->array.offset,
                        geom->array.length, out_cell, out_valid, (hipStream_t)stream, nullptr);
}

int32_t mgpu_pip_join_arrow(mgpu_ctx* ctx, const mgpu_chips* chips, int32_t index_system, int32_t res,
                            const struct ArrowDeviceArray* x, const struct ArrowDeviceArray* y,
                            const struct ArrowDeviceArray* point_id, int64_t capacity, int64_t* out_n_pairs,
                            int64_t* out_point_id, int32_t* out_polygon_id, void* stream, mgpu_stats* stats) {
  if (!ctx) return fail(MGPU_E_INVALID_ARG, "ctx is NULL");
  if (int32_t st = set_device(ctx->device)) return st;
  hipStream_t s = (hipStream_t)stream;
  const void *xd, *yd, *pd = nullptr;
  const uint8_t *xv, *yv, *pv = nullptr;
  int64_t xo, yo, po = 0;
  if (int32_t st = arrow_column(ctx, x, 8, &xd, &xv, &xo, "x")) return st;
  if (int32_t st = arrow_column(ctx, y, 8, &yd, &yv, &yo, "y")) return st;
  const int64_t n = x->array.length;
  if (y->array.length != n) return fail(MGPU_E_INVALID_ARG, "x and y differ in length");
  if (point_id) {
    if (int32_t st = arrow_column(ctx, point_id, 8, &pd, &pv, &po, "point_id")) return st;
    if (point_id->array.length != n) return fail(MGPU_E_INVALID_ARG, "point_id and x differ in length");
    if (pv) return fail(MGPU_E_INVALID_ARG, "point_id has nulls");
  }
  const uint8_t* valid = nullptr;
  int64_t voff = 0;
  if (xv && yv) {
    if (int32_t st = ensure_scratch(ctx, (size_t)(n + 7) / 8 + 1)) return st;
    HIP_TRY(mgpu::launch_valid_and(xv, xo, yv, yo, n, (uint8_t*)ctx->scratch, s));
    valid = (const uint8_t*)ctx->scratch;
  } else if (xv || yv) {
    valid = xv ? xv : yv;
    voff = xv ? xo : yo;
  }
  return pip_join_sync(ctx, chips, index_system, res, (const double*)xd, (const double*)yd, (const int64_t*)pd,
                       point_id ? 0 : x->array.offset, n, capacity, out_n_pairs, out_point_id, out_polygon_id, stream, stats, valid,
                       voff);
}

int32_t mgpu_test_parse_number(const char* s, int32_t len, double* out) {
  return mgpu::dec::parse_number(s, len, out);
}

int32_t mgpu_test_h3_elementary_host(int32_t fn, const double* a, const double* b, int64_t n, double* out) {
  namespace X = mgpu::exact;
  for (int64_t i = 0; i < n; ++i) {
    const double x = a[i], y = b ? b[i] : 0.0;
    double r = 0.0;
    switch (fn) {
      case 0: r = X::cr_sin(x); break;
      case 1: r = X::cr_cos(x); break;
      case 2: r = X::cr_tan(x); break;
      case 3: r = X::cr_acos(x); break;
      case 4: r = X::cr_atan2(x, y); break;
      // the integer emulation the device runs (not the host's x87 unit)
      case 5: r = X::x80_to_double(X::x80_add(X::x80_from_double(x), X::kX2Pi)); break;
      case 6: r = X::x80_to_double(X::x80_add(X::x80_from_double(x), X::x80_neg(X::kX2Pi))); break;
      case 7: r = X::x80_to_double(X::x80_mul(X::x80_from_double(x), X::kXSqrt7)); break;
      case 8: r = X::x80_to_double(X::x80_div(X::x80_from_double(x), X::kXSin60)); break;
      case 9: r = X::x80_to_double(X::x80_add(X::x80_from_double(x), X::x80_neg(X::kXAp7Rot))); break;
      case 10: r = X::x80_to_double(X::x80_div(X::x80_from_double(x), X::kXSqrt7)); break;
      case 11: r = X::x80_to_double(X::x80_add(X::x80_from_double(x), X::kXAp7Rot)); break;
      case 12: r = X::x80_cmp(X::x80_from_double(x), X::kXEpsilon) < 0 ? 1.0 : 0.0; break;
      case 13: r = X::x80_cmp(X::x80_from_double(x), X::kX2Pi) >= 0 ? 1.0 : 0.0; break;
      default: return MGPU_E_INVALID_ARG;
    }
    out[i] = r;
  }
  return MGPU_OK;
}

int32_t mgpu_test_h3_route_host(const double* lon, const double* lat, int64_t n, int32_t res, int64_t* out_cell) {
  if (res < 0 || res > 15) return MGPU_E_RESOLUTION;
  mgpu::parallel_for(n, 4096, [&](int64_t b, int64_t e, int) {
    for (int64_t i = b; i < e; ++i) {
      bool tie;
      out_cell[i] = (int64_t)mgpu::h3::point_to_cell(lon[i], lat[i], res, &tie);
    }
  });
  return MGPU_OK;
}

int32_t mgpu_test_h3_glibc_host(const double* lon, const double* lat, int64_t n, int32_t res, int64_t* out_cell) {
  if (res < 0 || res > 15) return MGPU_E_RESOLUTION;
  mgpu::parallel_for(n, 4096, [&](int64_t b, int64_t e, int) {
    for (int64_t i = b; i < e; ++i) out_cell[i] = (int64_t)mgpu::h3glibc::point_to_cell(lon[i], lat[i], res);
  });
  return MGPU_OK;
}

int32_t mgpu_test_decode_point(int32_t format, const uint8_t* data, int64_t len, double* x, double* y) {
  switch (format) {
    case MGPU_GEOM_WKB: return mgpu::geom::wkb_centroid(data, len, x, y);
    case MGPU_GEOM_WKT: return mgpu::geom::wkt_centroid((const char*)data, len, x, y);
    case MGPU_GEOM_HEX: return mgpu::geom::hex_centroid((const char*)data, len, x, y);
    case MGPU_GEOM_GEOJSON: return mgpu::geom::json_centroid((const char*)data, len, x, y);
  }
  return mgpu::geom::kDecUnsupported;
}

int32_t mgpu_test_join_counters(mgpu_ctx* ctx, uint64_t* out16) {
  if (!ctx || !out16) return fail(MGPU_E_INVALID_ARG, "bad arguments");
  memset(out16, 0, 16 * 8);
  if (!ctx->ws) return MGPU_OK;
  if (int32_t st = set_device(ctx->device)) return st;
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(out16, ctx->ws, 16 * 8, hipMemcpyDeviceToHost));
  return MGPU_OK;
}

int32_t mgpu_test_internal_centroid(int64_t n, const int32_t* type_id, const int64_t* row_part, const int64_t* part_ring,
                                    const int64_t* ring_off, const double* xy, double* x, double* y, int32_t* status) {
  for (int64_t i = 0; i < n; i++)
    status[i] = mgpu::geom::internal_centroid(type_id[i], row_part[i], row_part[i + 1], part_ring, ring_off, xy, &x[i], &y[i]);
  return MGPU_OK;
}

}  // extern "C"
