// Internal: the C-ABI handle types and the helpers capi.cpp shares with comm.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mosaic_gpu.h"
#include "chip_table.h"
#include "kernels.h"

// Per-context options (mgpu_ctx_set_option; include/mosaic_gpu.h lists the keys).  They
// replace process environment variables: a JVM host sets them per context.
struct mgpu_options {
  int64_t h3_libm = MGPU_LIBM_REFERENCE;  // near-tie cells: the reference's libm or correctly rounded
  int64_t pipeline = MGPU_PIPELINE_AUTO;  // the join's planner (or a forced pipeline)
  int64_t bin_count = 64;                 // binned pipeline: bins over the chip table's extent
  int64_t bin_min_mb = 256;               // ... for chip tables of at least this size
  int64_t bin_min_points = 1 << 21;       // ... and batches of at least this many points
  int64_t bin_xcd = 1;                    // ... tiles dealt to the XCDs in contiguous runs
  int64_t bin_keys = 0;                   // ... H3: grid keys computed by the scatter kernel (A/B r5: slower)
  int64_t spin_us = 2000;                 // synchronous calls: poll (yielding) this long, then block
  int64_t ring_batch = (int64_t)1 << 26;   // ring joins: candidate pairs held in scratch at a time
  int64_t bng_split = 0;                  // BNG dense tables: the split pipeline, the grid entry as the code (A/B r6: C4 2.43 vs 2.17 ms fused -- off)
  // the chip-table builder of mgpu_chips_upload on this context (mgpu_build_opts)
  int64_t raster = 1, raster_bng = 0, raster_sub = 16, raster_milli = 250;
};

struct mgpu_ctx {
  int device = 0;
  mgpu_options opt;
  // workspace: tile status words + ticket + counters
  void* ws = nullptr;
  size_t ws_bytes = 0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr, ev3 = nullptr;
  void* comm = nullptr;  // comm.cpp CommState: the RCCL communicator (mgpu_comm_init)
  // the split pipeline's per-point buffers (codes, mixed lists and answers), grown on demand
  void* split_ws = nullptr;
  size_t split_bytes = 0;
  // the binned pipeline's per-point buffers (binned copies, slots, answers), grown on demand
  void* bin_ws = nullptr;
  size_t bin_bytes = 0;
  // the H3 route's near-tie queue (kernels.h JoinArgs.tie_queue; grown when a call
  // overflows it, then the call is redone), the libm overrides of the join being run,
  // and a pinned host page for the counters and the queue's head
  uint64_t* tq = nullptr;
  int64_t tq_cap = 0;
  uint64_t* ovr = nullptr;
  int64_t ovr_cap = 0;
  uint64_t* pin = nullptr;
  // scratch of the geometry / Arrow entries (decoded points, validity bitmaps), grown on demand
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  // the override pass's scratch (kernels.h RedoArgs), grown on demand
  void* redo = nullptr;
  size_t redo_bytes = 0;
  // the last mgpu_pip_join on this context, whose pair records stay in the workspace
  // until the next call (mgpu_pip_join_fetch)
  struct {
    bool valid = false, pool_ok = false;
    const mgpu_chips* chips = nullptr;
    int32_t is = 0, res = 0;
    const double *x = nullptr, *y = nullptr;
    const int64_t* point_id = nullptr;
    int64_t id_base = 0, n = 0, total = 0;
    const uint8_t* pts_valid = nullptr;
    int64_t pts_valid_off = 0;
    mgpu::EmitArgs emit{};
    mgpu::JoinArgs jargs{};  // (the fused pipeline's, for a rerun of some tiles)
    int64_t n_tiles = 0;
    int64_t n_ovr = 0;  // libm overrides the join ran with
    int tie_host = 0;   // near-ties queued for the host (JoinArgs.tie_host)
    bool split = false;
    mgpu::SplitArgs sargs{};
    bool binned = false;
    mgpu::BinArgs bargs{};
    // an mgpu_pip_join_async call waiting for mgpu_pip_join_finish (its H3 near-ties
    // are queued for the host's libm pass); any other call on the context ends it
    bool async_pending = false;
    int64_t* d_n_pairs = nullptr;
    void* stream = nullptr;
    int64_t capacity = 0;
    int64_t* out_point = nullptr;
    int32_t* out_poly = nullptr;
  } last;
};

struct mgpu_chips {
  int device = 0;
  int32_t index_system = MGPU_H3;
  void* blob = nullptr;
  size_t bytes = 0;
  mgpu::ChipTableView view{};
  int64_t n_vertices = 0;
};

namespace mgpu {
int32_t set_error(int32_t code, const char* fmt, ...);
// Size of the whole chip-table blob from its 1 KiB header (host copy); 0 if not a blob.
int64_t blob_bytes_of_header(const void* header);
constexpr int64_t kBlobHeaderSize = 1024;
// Take ownership of a device allocation holding a complete blob (no copy).
int32_t adopt_device_blob(mgpu_ctx* ctx, void* dev_blob, int64_t bytes, mgpu_chips** out);
}  // namespace mgpu
