// C-ABI of the MI355X point-in-polygon join (include/mosaic_gpu.h).
//
// Host-side responsibilities: argument validation with the reference's error
// classes, chip-table construction (WKB -> SoA + cell hash, one device blob),
// workspace management and kernel launches.  No computation on the data path
// happens here; every per-point operation runs in kernels.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

#include "../../include/mosaic_gpu.h"
#include "chip_table.h"
#include "kernels.h"
#include "wkb.h"

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
constexpr int kBlobArrays = 11;
struct BlobHeader {
  uint64_t magic;
  uint32_t version, hash_mask, max_probe, n_chips, n_cells, pad;
  int64_t n_vertices;
  uint64_t off[kBlobArrays];
};
constexpr size_t kBlobHeaderBytes = 256;
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
  return v;
}

}  // namespace

struct mgpu_ctx {
  int device = 0;
  // workspace: tile status words + ticket + counters
  void* ws = nullptr;
  size_t ws_bytes = 0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
};

struct mgpu_chips {
  int device = 0;
  void* blob = nullptr;
  size_t bytes = 0;
  mgpu::ChipTableView view{};
  int64_t n_vertices = 0;
};

namespace {

// Workspace layout: [counters 8 x u64][ticket u32 + pad to 64 B][tile status n_tiles x u64]
constexpr size_t kWsCounters = 64;
constexpr size_t kWsTicket = 64;

int32_t ensure_ws(mgpu_ctx* ctx, int64_t n_tiles) {
  size_t need = kWsCounters + kWsTicket + align_up((size_t)std::max<int64_t>(n_tiles, 1) * 8, 256);
  if (need <= ctx->ws_bytes) return MGPU_OK;
  if (ctx->ws) HIP_TRY(hipFree(ctx->ws));
  ctx->ws = nullptr;
  HIP_TRY(hipMalloc(&ctx->ws, need));
  ctx->ws_bytes = need;
  return MGPU_OK;
}

int32_t check_res(int32_t is, int32_t res) {
  if (is == MGPU_H3) {
    if (res < 0 || res > 15) return fail(MGPU_E_RESOLUTION, "H3 resolution has to be between 0 and 15; found %d", res);
    return res;
  }
  if (is == MGPU_BNG) {
    if (res == 0 || res < -6 || res > 6) return fail(MGPU_E_RESOLUTION, "BNG resolution not supported; found %d", res);
    return res;
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

int32_t mgpu_check_resolution(int32_t index_system, int32_t res) { return check_res(index_system, res); }

int32_t mgpu_ctx_create(int32_t device_id, mgpu_ctx** out) {
  if (!out) return fail(MGPU_E_INVALID_ARG, "out is NULL");
  int n = 0;
  HIP_TRY(hipGetDeviceCount(&n));
  if (device_id < 0 || device_id >= n) return fail(MGPU_E_INVALID_ARG, "device %d not present (%d GPUs)", device_id, n);
  HIP_TRY(hipSetDevice(device_id));
  mgpu_ctx* c = new mgpu_ctx();
  c->device = device_id;
  HIP_TRY(hipEventCreate(&c->ev0));
  HIP_TRY(hipEventCreate(&c->ev1));
  int32_t st = ensure_ws(c, 1 << 16);
  if (st) {
    delete c;
    return st;
  }
  *out = c;
  return MGPU_OK;
}

int32_t mgpu_ctx_destroy(mgpu_ctx* ctx) {
  if (!ctx) return MGPU_OK;
  hipSetDevice(ctx->device);
  if (ctx->ws) hipFree(ctx->ws);
  if (ctx->ev0) hipEventDestroy(ctx->ev0);
  if (ctx->ev1) hipEventDestroy(ctx->ev1);
  delete ctx;
  return MGPU_OK;
}

int32_t mgpu_ctx_reserve(mgpu_ctx* ctx, int64_t max_points) {
  if (!ctx) return fail(MGPU_E_INVALID_ARG, "ctx is NULL");
  if (int32_t st = set_device(ctx->device)) return st;
  return ensure_ws(ctx, mgpu::join_tiles(max_points));
}

int32_t mgpu_points_to_cells(mgpu_ctx* ctx, int32_t is, int32_t res, const double* x, const double* y, int64_t n,
                             int64_t* out_cell, void* stream, mgpu_stats* stats) {
  if (!ctx) return fail(MGPU_E_INVALID_ARG, "ctx is NULL");
  int32_t r = check_res(is, res);
  if (r < 0) return r;
  if (n < 0 || (n > 0 && (!x || !y || !out_cell))) return fail(MGPU_E_INVALID_ARG, "bad point arrays");
  if (int32_t st = set_device(ctx->device)) return st;
  hipStream_t s = (hipStream_t)stream;
  auto* counters = (unsigned long long*)ctx->ws;
  HIP_TRY(hipMemsetAsync(counters, 0, kWsCounters, s));
  HIP_TRY(hipEventRecord(ctx->ev0, s));
  HIP_TRY(mgpu::launch_cells(is, res, x, y, n, out_cell, counters, s));
  HIP_TRY(hipEventRecord(ctx->ev1, s));
  unsigned long long h[8] = {0};
  bool need_sync = stats != nullptr;
  if (need_sync || true) {
    // invalid-coordinate detection must reach the caller (IllegalArgument/IllegalState)
    HIP_TRY(hipMemcpyAsync(h, counters, sizeof h, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
  }
  if (stats) {
    stats->n_points = n;
    stats->n_pairs = 0;
    stats->n_near_ties = (int64_t)h[1];
    stats->n_candidates = 0;
    float ms = 0;
    hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1);
    stats->kernel_ms = ms;
  }
  if (h[2]) {
    if (is == MGPU_BNG) return fail(MGPU_E_NAN, "NaN coordinates are not supported. (%llu points)", h[2]);
    return fail(MGPU_E_INVALID_ARG, "Latitude or longitude were invalid. (%llu points)", h[2]);
  }
  return MGPU_OK;
}

int32_t mgpu_points_to_cells_host(mgpu_ctx* ctx, int32_t is, int32_t res, const double* x, const double* y, int64_t n,
                                  int64_t* out_cell) {
  if (!ctx) return fail(MGPU_E_INVALID_ARG, "ctx is NULL");
  if (n == 0) return check_res(is, res) < 0 ? MGPU_E_RESOLUTION : MGPU_OK;
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

int32_t mgpu_chips_upload(mgpu_ctx* ctx, int64_t n_chips, const int64_t* cell, const int32_t* polygon_id,
                          const uint8_t* is_core, const int64_t* wkb_offsets, const uint8_t* wkb, mgpu_chips** out) {
  if (!ctx || !out) return fail(MGPU_E_INVALID_ARG, "ctx/out is NULL");
  if (n_chips < 0 || n_chips > (int64_t)std::numeric_limits<int32_t>::max())
    return fail(MGPU_E_INVALID_ARG, "n_chips out of range");
  if (n_chips > 0 && (!cell || !polygon_id || !is_core || !wkb_offsets))
    return fail(MGPU_E_INVALID_ARG, "chip arrays are NULL");
  if (int32_t st = set_device(ctx->device)) return st;

  std::vector<int64_t> order(n_chips);
  for (int64_t i = 0; i < n_chips; i++) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
    if (cell[a] != cell[b]) return cell[a] < cell[b];
    return polygon_id[a] < polygon_id[b];
  });

  mgpu::wkb::Flat geo;  // parts / rings / vertices of all chips, in sorted order
  std::vector<int32_t> cpoly(n_chips);
  std::vector<uint8_t> cflags(n_chips);
  std::vector<uint32_t> cpart(n_chips + 1);
  std::vector<double> cenv(4 * (size_t)n_chips);
  std::vector<int64_t> crow(n_chips);
  std::vector<uint32_t> row2chip(n_chips);
  for (int64_t s = 0; s < n_chips; s++) {
    int64_t i = order[s];
    cpoly[s] = polygon_id[i];
    crow[s] = i;
    row2chip[i] = (uint32_t)s;
    cpart[s] = (uint32_t)geo.part_ring.size() - 1;
    uint8_t fl = is_core[i] ? mgpu::kChipCore : 0;
    int64_t b = wkb_offsets[i], e = wkb_offsets[i + 1];
    if (e < b) return fail(MGPU_E_INVALID_ARG, "wkb_offsets not ascending at row %lld", (long long)i);
    double env[4] = {INFINITY, INFINITY, -INFINITY, -INFINITY};
    if (e == b) {
      if (!is_core[i]) return fail(MGPU_E_WKB, "border chip row %lld has NULL geometry", (long long)i);
      fl |= mgpu::kChipNoGeom;
    } else {
      mgpu::wkb::GeomInfo gi;
      std::string msg;
      if (!mgpu::wkb::parse(wkb + b, (size_t)(e - b), geo, gi, msg))
        return fail(MGPU_E_WKB, "chip row %lld: %s", (long long)i, msg.c_str());
      if (gi.multi) fl |= mgpu::kChipMulti;
      if (gi.n_points == 0) fl |= mgpu::kChipEmpty;
      if (gi.rectangle) fl |= mgpu::kChipRect;
      env[0] = gi.env[0];
      env[1] = gi.env[1];
      env[2] = gi.env[2];
      env[3] = gi.env[3];
    }
    cflags[s] = fl;
    for (int k = 0; k < 4; k++) cenv[4 * s + k] = env[k];
  }
  cpart[n_chips] = (uint32_t)geo.part_ring.size() - 1;

  // cell hash over the distinct cells
  std::vector<mgpu::HashSlot> distinct;
  for (int64_t s = 0; s < n_chips;) {
    int64_t e = s;
    uint64_t c = (uint64_t)cell[order[s]];
    while (e < n_chips && (uint64_t)cell[order[e]] == c) e++;
    distinct.push_back(mgpu::HashSlot{c, (uint32_t)s, (uint32_t)(e - s)});
    s = e;
  }
  uint32_t cap = 16;
  while (cap < 2 * distinct.size()) cap <<= 1;
  std::vector<mgpu::HashSlot> slots(cap, mgpu::HashSlot{0, 0, 0});
  uint32_t max_probe = 0;
  for (const auto& d : distinct) {
    uint32_t h = mgpu::cell_hash(d.cell) & (cap - 1), k = 0;
    while (slots[h].count) {
      h = (h + 1) & (cap - 1);
      k++;
    }
    slots[h] = d;
    max_probe = std::max(max_probe, k);
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
  };
  size_t total = kBlobHeaderBytes;
  BlobHeader hdr{};
  hdr.magic = kBlobMagic;
  hdr.version = 1;
  hdr.hash_mask = cap - 1;
  hdr.max_probe = max_probe;
  hdr.n_chips = (uint32_t)n_chips;
  hdr.n_cells = (uint32_t)distinct.size();
  hdr.n_vertices = (int64_t)geo.vtx.size() / 2;
  for (size_t k = 0; k < parts.size(); k++) {
    parts[k].off = total;
    hdr.off[k] = total;
    total = align_up(total + std::max<size_t>(parts[k].bytes, 1), 256);
  }
  std::vector<uint8_t> host(total, 0);
  memcpy(host.data(), &hdr, sizeof hdr);
  for (auto& p : parts)
    if (p.bytes) memcpy(host.data() + p.off, p.src, p.bytes);
  mgpu_chips* ch = new mgpu_chips();
  ch->device = ctx->device;
  hipError_t e1 = hipMalloc(&ch->blob, total);
  if (e1 != hipSuccess) {
    delete ch;
    return fail(MGPU_E_DEVICE, "hipMalloc(%zu): %s", total, hipGetErrorString(e1));
  }
  hipError_t e2 = hipMemcpy(ch->blob, host.data(), total, hipMemcpyHostToDevice);
  if (e2 != hipSuccess) {
    hipFree(ch->blob);
    delete ch;
    return fail(MGPU_E_DEVICE, "hipMemcpy: %s", hipGetErrorString(e2));
  }
  ch->bytes = total;
  ch->view = view_from_header(hdr, (uint8_t*)ch->blob);
  ch->n_vertices = hdr.n_vertices;
  *out = ch;
  return MGPU_OK;
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
  if (hdr.magic != kBlobMagic || hdr.version != 1) return fail(MGPU_E_INVALID_ARG, "not a chip-table blob");
  for (int k = 0; k < kBlobArrays; k++)
    if (hdr.off[k] >= (uint64_t)bytes) return fail(MGPU_E_INVALID_ARG, "corrupt chip-table blob");
  mgpu_chips* ch = new mgpu_chips();
  ch->device = ctx->device;
  HIP_TRY(hipMalloc(&ch->blob, bytes));
  HIP_TRY(hipMemcpy(ch->blob, device_ptr, bytes, hipMemcpyDeviceToDevice));
  ch->bytes = bytes;
  ch->view = view_from_header(hdr, (uint8_t*)ch->blob);
  ch->n_vertices = hdr.n_vertices;
  *out = ch;
  return MGPU_OK;
}

int32_t mgpu_st_contains(mgpu_ctx* ctx, const mgpu_chips* chips, const int64_t* chip_row, const double* x,
                         const double* y, int64_t n, int8_t* out, void* stream) {
  if (!ctx || !chips) return fail(MGPU_E_INVALID_ARG, "ctx/chips is NULL");
  if (n < 0 || (n > 0 && (!chip_row || !x || !y || !out))) return fail(MGPU_E_INVALID_ARG, "bad arrays");
  if (int32_t st = set_device(ctx->device)) return st;
  HIP_TRY(mgpu::launch_st_contains(chips->view, chip_row, x, y, n, out, (hipStream_t)stream));
  return MGPU_OK;
}

// ------------------------------------------------------------------ join

static int32_t join_impl(mgpu_ctx* ctx, const mgpu_chips* chips, int32_t is, int32_t res, const double* x,
                         const double* y, const int64_t* point_id, int64_t id_base, int64_t n, int64_t capacity,
                         int64_t* out_point, int32_t* out_poly, hipStream_t s, bool timed) {
  if (!ctx || !chips) return fail(MGPU_E_INVALID_ARG, "ctx/chips is NULL");
  int32_t r = check_res(is, res);
  if (r < 0) return r;
  if (n < 0 || (n > 0 && (!x || !y))) return fail(MGPU_E_INVALID_ARG, "bad point arrays");
  if (capacity < 0 || (capacity > 0 && (!out_point || !out_poly))) return fail(MGPU_E_INVALID_ARG, "bad output arrays");
  if (int32_t st = set_device(ctx->device)) return st;
  int64_t tiles = mgpu::join_tiles(n);
  if (int32_t st = ensure_ws(ctx, tiles)) return st;
  auto* base = (uint8_t*)ctx->ws;
  mgpu::JoinArgs a;
  a.x = x;
  a.y = y;
  a.point_id = point_id;
  a.id_base = id_base;
  a.n = n;
  a.n_tiles = tiles;
  a.res = res;
  a.chips = chips->view;
  a.capacity = capacity;
  a.out_point = out_point;
  a.out_poly = out_poly;
  a.counters = (unsigned long long*)base;
  a.tile_ticket = (uint32_t*)(base + kWsCounters);
  a.tile_status = (uint64_t*)(base + kWsCounters + kWsTicket);
  HIP_TRY(hipMemsetAsync(base, 0, kWsCounters + kWsTicket + align_up((size_t)std::max<int64_t>(tiles, 1) * 8, 256), s));
  if (timed) HIP_TRY(hipEventRecord(ctx->ev0, s));
  HIP_TRY(mgpu::launch_join(is, a, s));
  if (timed) HIP_TRY(hipEventRecord(ctx->ev1, s));
  return MGPU_OK;
}

int32_t mgpu_pip_join_async(mgpu_ctx* ctx, const mgpu_chips* chips, int32_t is, int32_t res, const double* x,
                            const double* y, const int64_t* point_id, int64_t point_id_base, int64_t n,
                            int64_t capacity, int64_t* d_n_pairs, int64_t* out_point_id, int32_t* out_polygon_id,
                            void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int32_t st = join_impl(ctx, chips, is, res, x, y, point_id, point_id_base, n, capacity, out_point_id, out_polygon_id,
                         s, false);
  if (st) return st;
  if (d_n_pairs) HIP_TRY(hipMemcpyAsync(d_n_pairs, ctx->ws, 8, hipMemcpyDeviceToDevice, s));
  return MGPU_OK;
}

int32_t mgpu_pip_join(mgpu_ctx* ctx, const mgpu_chips* chips, int32_t is, int32_t res, const double* x,
                      const double* y, const int64_t* point_id, int64_t point_id_base, int64_t n, int64_t capacity,
                      int64_t* out_n_pairs, int64_t* out_point_id, int32_t* out_polygon_id, void* stream,
                      mgpu_stats* stats) {
  hipStream_t s = (hipStream_t)stream;
  int32_t st = join_impl(ctx, chips, is, res, x, y, point_id, point_id_base, n, capacity, out_point_id, out_polygon_id,
                         s, true);
  if (st) return st;
  unsigned long long h[8] = {0};
  HIP_TRY(hipMemcpyAsync(h, ctx->ws, sizeof h, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (out_n_pairs) *out_n_pairs = (int64_t)h[0];
  if (stats) {
    stats->n_points = n;
    stats->n_pairs = (int64_t)h[0];
    stats->n_near_ties = (int64_t)h[1];
    stats->n_candidates = (int64_t)h[3];
    float ms = 0;
    hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1);
    stats->kernel_ms = ms;
  }
  if (h[4]) return fail(MGPU_E_INTERNAL, "look-back scan timed out in %llu tiles", h[4]);
  if (h[2]) {
    if (is == MGPU_BNG) return fail(MGPU_E_NAN, "NaN coordinates are not supported. (%llu points)", h[2]);
    return fail(MGPU_E_INVALID_ARG, "Latitude or longitude were invalid. (%llu points)", h[2]);
  }
  if ((int64_t)h[0] > capacity)
    return fail(MGPU_E_CAPACITY, "%lld pairs do not fit capacity %lld", (long long)h[0], (long long)capacity);
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

}  // extern "C"
