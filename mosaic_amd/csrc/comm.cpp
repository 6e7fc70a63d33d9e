// Multi-GPU data path of the join behind the C ABI (include/mosaic_gpu.h "Multi-GPU"):
// one process per GPU, points sharded by contiguous id range, the chip table replicated.
//
// The reference scales the join with Spark: the chip side is broadcast to every
// executor (the BroadcastHashJoin of notebooks/examples/python/Quickstart/
// QuickstartNotebook.ipynb:1835's plan) and each task joins its partition of points.
// Here the executor is a GPU: ONE RCCL broadcast over xGMI replicates the self-describing
// chip-table blob straight into the receiving allocation (header first, to size it), and
// ONE all-gather of the per-rank pair counts gives each rank its slice of the globally
// ordered output.  The unique id travels out of band (the JVM host's driver broadcast,
// or torch.distributed's store in this repository's Python host).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <vector>

#include "capi_internal.h"

namespace {

struct CommState {
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1;
  void* scratch = nullptr;  // device: the broadcast header, the gathered counts
  // pinned host staging of the values copied to / from `scratch` (a status word, a count):
  // an asynchronous copy never reads a stack local that dies before the copy runs
  int64_t* host = nullptr;
};
constexpr size_t kScratch = 4096;  // >= the blob header + a status word; the counts

CommState* state(mgpu_ctx* ctx) { return (CommState*)ctx->comm; }

#define NCCL_TRY(expr)                                                                                  \
  do {                                                                                                  \
    ncclResult_t _r = (expr);                                                                           \
    if (_r != ncclSuccess) return mgpu::set_error(MGPU_E_DEVICE, "%s: %s", #expr, ncclGetErrorString(_r)); \
  } while (0)
#define HIP_TRY(expr)                                                                                    \
  do {                                                                                                   \
    hipError_t _e = (expr);                                                                              \
    if (_e != hipSuccess) return mgpu::set_error(MGPU_E_DEVICE, "%s: %s", #expr, hipGetErrorString(_e)); \
  } while (0)

}  // namespace

extern "C" {

int32_t mgpu_comm_unique_id(uint8_t* out_id) {
  if (!out_id) return mgpu::set_error(MGPU_E_INVALID_ARG, "out_id is NULL");
  ncclUniqueId id;
  NCCL_TRY(ncclGetUniqueId(&id));
  static_assert(sizeof id == MGPU_COMM_ID_BYTES, "unique id size");
  memcpy(out_id, &id, sizeof id);
  return MGPU_OK;
}

int32_t mgpu_comm_init(mgpu_ctx* ctx, const uint8_t* unique_id, int32_t rank, int32_t world) {
  if (!ctx || !unique_id) return mgpu::set_error(MGPU_E_INVALID_ARG, "ctx/unique_id is NULL");
  if (world < 1 || rank < 0 || rank >= world) return mgpu::set_error(MGPU_E_INVALID_ARG, "rank %d of %d", rank, world);
  if (ctx->comm) return mgpu::set_error(MGPU_E_INVALID_ARG, "context already has a communicator");
  HIP_TRY(hipSetDevice(ctx->device));
  ncclUniqueId id;
  memcpy(&id, unique_id, sizeof id);
  CommState* c = new CommState();
  c->rank = rank;
  c->world = world;
  hipError_t e = hipMalloc(&c->scratch, kScratch);
  if (e == hipSuccess) {
    e = hipHostMalloc((void**)&c->host, 64, hipHostMallocDefault);
    if (e != hipSuccess) hipFree(c->scratch);
  }
  if (e != hipSuccess) {
    delete c;
    return mgpu::set_error(MGPU_E_DEVICE, "hipMalloc: %s", hipGetErrorString(e));
  }
  ncclResult_t r = ncclCommInitRank(&c->comm, world, id, rank);
  if (r != ncclSuccess) {
    hipFree(c->scratch);
    hipHostFree(c->host);
    delete c;
    return mgpu::set_error(MGPU_E_DEVICE, "ncclCommInitRank(rank %d of %d): %s", rank, world, ncclGetErrorString(r));
  }
  ctx->comm = c;
  return MGPU_OK;
}

int32_t mgpu_comm_destroy(mgpu_ctx* ctx) {
  if (!ctx || !ctx->comm) return MGPU_OK;
  CommState* c = state(ctx);
  hipSetDevice(ctx->device);
  if (c->comm) ncclCommDestroy(c->comm);
  if (c->scratch) hipFree(c->scratch);
  if (c->host) hipHostFree(c->host);
  delete c;
  ctx->comm = nullptr;
  return MGPU_OK;
}

int32_t mgpu_comm_info(mgpu_ctx* ctx, int32_t* rank, int32_t* world) {
  if (!ctx || !ctx->comm) return mgpu::set_error(MGPU_E_INVALID_ARG, "context has no communicator");
  if (rank) *rank = state(ctx)->rank;
  if (world) *world = state(ctx)->world;
  return MGPU_OK;
}

// Every rank issues the same collectives in the same order whatever fails locally: (1) the
// 1 KiB header broadcast, (2) an all-reduce(min) of a status word -- each rank's "ready"
// (root: a valid table; receivers: a valid header and the receiving allocation), and only
// if every rank is ready (3) the bulk broadcast.  A local failure therefore never leaves
// the other ranks blocked in a broadcast this rank skipped: all ranks see the failed
// agreement and return an error.  A failed RCCL call aborts the communicator
// (ncclCommAbort): later calls on the context fail instead of hanging.
namespace {
// (the stream is drained first: copies staged through c->host may still be pending)
int32_t comm_failed(mgpu_ctx* ctx, const char* what, ncclResult_t r, hipStream_t s) {
  CommState* c = state(ctx);
  int32_t st = mgpu::set_error(MGPU_E_DEVICE, "%s: %s (communicator aborted)", what, ncclGetErrorString(r));
  if (c->comm) ncclCommAbort(c->comm);
  (void)hipStreamSynchronize(s);
  if (c->scratch) hipFree(c->scratch);
  if (c->host) hipHostFree(c->host);
  delete c;
  ctx->comm = nullptr;
  return st;
}

// A receiving rank's side of step 1: read the broadcast header, size and allocate the
// receiving table.  Returns its status (MGPU_OK or the error class, *why the reason);
// fail_alloc (test hook only) makes the allocation fail.
int32_t receiver_prepare(const void* hdr_dev, hipStream_t s, bool fail_alloc, int64_t* bytes, void** dst,
                         const char** why) {
  *bytes = 0;
  *dst = nullptr;
  std::vector<uint8_t> h((size_t)mgpu::kBlobHeaderSize);
  if (hipMemcpyAsync(h.data(), hdr_dev, h.size(), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) {
    *why = "reading the broadcast header";
    return MGPU_E_DEVICE;
  }
  *bytes = mgpu::blob_bytes_of_header(h.data());
  if (*bytes < mgpu::kBlobHeaderSize) {
    *why = "the root sent no chip-table blob";
    return MGPU_E_INVALID_ARG;
  }
  if (fail_alloc || hipMalloc(dst, (size_t)*bytes) != hipSuccess) {
    *dst = nullptr;
    *why = "hipMalloc of the receiving table";
    return MGPU_E_DEVICE;
  }
  return MGPU_OK;
}
}  // namespace

// TEST ONLY: the receiving rank's path without RCCL -- header read, allocation (forced to
// fail with fail_alloc), the blob's bytes copied in as the bulk broadcast would, adoption.
int32_t mgpu_test_receive_blob(mgpu_ctx* ctx, const void* dev_blob, int32_t fail_alloc, mgpu_chips** out) {
  if (!ctx || !dev_blob || !out) return mgpu::set_error(MGPU_E_INVALID_ARG, "receive_blob: NULL argument");
  *out = nullptr;
  HIP_TRY(hipSetDevice(ctx->device));
  int64_t bytes = 0;
  void* dst = nullptr;
  const char* why = "";
  if (int32_t st = receiver_prepare(dev_blob, nullptr, fail_alloc != 0, &bytes, &dst, &why))
    return mgpu::set_error(st, "chips_broadcast: %s", why);
  if (hipMemcpy(dst, dev_blob, (size_t)bytes, hipMemcpyDeviceToDevice) != hipSuccess) {
    hipFree(dst);
    return mgpu::set_error(MGPU_E_DEVICE, "receive_blob: copy");
  }
  int32_t st = mgpu::adopt_device_blob(ctx, dst, bytes, out);
  if (st) hipFree(dst);
  return st;
}

int32_t mgpu_chips_broadcast(mgpu_ctx* ctx, const mgpu_chips* chips, int32_t root, mgpu_chips** out, void* stream) {
  if (!ctx || !ctx->comm || !out) return mgpu::set_error(MGPU_E_INVALID_ARG, "chips_broadcast: no communicator / out");
  CommState* c = state(ctx);
  // (every rank sees the same root and world: an argument error here is the same on all)
  if (root < 0 || root >= c->world) return mgpu::set_error(MGPU_E_INVALID_ARG, "root %d of %d", root, c->world);
  const bool is_root = c->rank == root;
  *out = nullptr;
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  int32_t* status = (int32_t*)((uint8_t*)c->scratch + mgpu::kBlobHeaderSize);
  const bool root_ok = !is_root || (chips && chips->device == ctx->device && chips->blob);
  // 1. the header (a root without a table sends zeros: no receiver accepts them)
  void* hdr_dev = (is_root && root_ok) ? chips->blob : c->scratch;
  if (is_root && !root_ok) (void)hipMemsetAsync(c->scratch, 0, (size_t)mgpu::kBlobHeaderSize, s);
  ncclResult_t r = ncclBroadcast(hdr_dev, hdr_dev, (size_t)mgpu::kBlobHeaderSize, ncclUint8, root, c->comm, s);
  if (r != ncclSuccess) return comm_failed(ctx, "ncclBroadcast(header)", r, s);
  int64_t bytes = 0;
  void* dst = nullptr;
  int32_t mine = MGPU_OK;
  const char* why = "";
  if (is_root) {
    if (root_ok) bytes = (int64_t)chips->bytes;
    else mine = MGPU_E_INVALID_ARG, why = "the root needs its chip table on the context's GPU";
  } else {
    mine = receiver_prepare(c->scratch, s, false, &bytes, &dst, &why);
  }
  // 2. agreement: the smallest status (errors are negative) over all ranks.  The status
  // word is first set negative on the stream, so a failed copy of `mine` still
  // contributes a failure (never a stale OK from an earlier call)
  int32_t agreed = mine;
  // (both steps are tried whatever the first gave: a failed memset makes the copied value
  // a failure itself, so no stale OK from an earlier call can reach the all-reduce)
  // (staged through the pinned c->host, read by the copy whenever it runs; the stream is
  // synchronised below before the word is reused or any return)
  const bool set_ok = hipMemsetAsync(status, 0x80, 4, s) == hipSuccess;
  int32_t* contrib = (int32_t*)c->host;
  *contrib = set_ok ? mine : (int32_t)MGPU_E_DEVICE;
  const bool copy_ok = hipMemcpyAsync(status, contrib, 4, hipMemcpyHostToDevice, s) == hipSuccess;
  if (!set_ok || !copy_ok) agreed = MGPU_E_DEVICE;
  r = ncclAllReduce(status, status, 1, ncclInt32, ncclMin, c->comm, s);
  if (r != ncclSuccess) {
    if (dst) hipFree(dst);
    return comm_failed(ctx, "ncclAllReduce(status)", r, s);
  }
  int32_t* back = (int32_t*)(c->host + 1);
  *back = MGPU_OK;
  int32_t all = MGPU_OK;
  const bool back_ok = hipMemcpyAsync(back, status, 4, hipMemcpyDeviceToHost, s) == hipSuccess;
  if (hipStreamSynchronize(s) != hipSuccess || !back_ok) all = MGPU_E_DEVICE;
  else all = *back;
  if (agreed != MGPU_OK && all == MGPU_OK) all = agreed;
  if (all != MGPU_OK) {
    // every rank skips the bulk broadcast
    if (dst) hipFree(dst);
    if (mine != MGPU_OK) return mgpu::set_error(mine, "chips_broadcast: %s", why);
    return mgpu::set_error(all, "chips_broadcast: another rank could not take part (status %d)", all);
  }
  // 3. the whole blob, straight into the receiving ranks' new allocation
  void* buf = is_root ? chips->blob : dst;
  r = ncclBroadcast(buf, buf, (size_t)bytes, ncclUint8, root, c->comm, s);
  if (r != ncclSuccess) {
    if (dst) hipFree(dst);
    return comm_failed(ctx, "ncclBroadcast(blob)", r, s);
  }
  if (hipStreamSynchronize(s) != hipSuccess) {
    if (dst) hipFree(dst);
    return mgpu::set_error(MGPU_E_DEVICE, "chips_broadcast: stream synchronize failed");
  }
  if (is_root) return MGPU_OK;
  int32_t st = mgpu::adopt_device_blob(ctx, dst, bytes, out);
  if (st) hipFree(dst);
  return st;
}

int32_t mgpu_pair_offsets(mgpu_ctx* ctx, int64_t local_pairs, int64_t* out_offset, int64_t* out_total,
                          int64_t* out_counts, void* stream) {
  if (!ctx || !ctx->comm) return mgpu::set_error(MGPU_E_INVALID_ARG, "pair_offsets: no communicator");
  CommState* c = state(ctx);
  if ((size_t)(c->world + 1) * 8 > kScratch) return mgpu::set_error(MGPU_E_INVALID_ARG, "world too large");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  int64_t* mine = (int64_t*)c->scratch;
  int64_t* all = mine + 1;
  // a negative count still takes part in the all-gather (as -1): every rank then fails.
  // The slot is set to -1 on the stream first, so a failed copy also contributes -1
  // instead of returning before the collective the other ranks wait in
  // (the copy is tried even when the memset failed -- then carrying -1 itself -- and a
  // local failure is reported after the collective, so this rank never relies on the
  // slot holding the previous call's count)
  // (the count is staged through the pinned c->host; every return after the copy has
  // synchronised the stream)
  const int64_t v = local_pairs < 0 ? -1 : local_pairs;
  const bool set_ok = hipMemsetAsync(mine, 0xFF, 8, s) == hipSuccess;
  c->host[0] = set_ok ? v : -1;
  const bool copy_ok = hipMemcpyAsync(mine, c->host, 8, hipMemcpyHostToDevice, s) == hipSuccess;
  ncclResult_t r = ncclAllGather(mine, all, 1, ncclInt64, c->comm, s);
  if (r != ncclSuccess) return comm_failed(ctx, "ncclAllGather(pair counts)", r, s);
  std::vector<int64_t> counts((size_t)c->world);
  const bool back_ok = hipMemcpyAsync(counts.data(), all, counts.size() * 8, hipMemcpyDeviceToHost, s) == hipSuccess;
  const bool sync_ok = hipStreamSynchronize(s) == hipSuccess;
  if (!set_ok || !copy_ok) return mgpu::set_error(MGPU_E_DEVICE, "pair_offsets: staging this rank's count failed");
  if (!back_ok || !sync_ok) return mgpu::set_error(MGPU_E_DEVICE, "pair_offsets: reading the gathered counts failed");
  int64_t off = 0, tot = 0;
  for (int k = 0; k < c->world; k++) {
    if (counts[k] < 0) return mgpu::set_error(MGPU_E_INVALID_ARG, "pair_offsets: negative count on rank %d", k);
    if (k < c->rank) off += counts[k];
    tot += counts[k];
    if (out_counts) out_counts[k] = counts[k];
  }
  if (out_offset) *out_offset = off;
  if (out_total) *out_total = tot;
  return MGPU_OK;
}

}  // extern "C"
