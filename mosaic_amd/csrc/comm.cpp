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
};
constexpr size_t kScratch = 4096;

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
  if (e != hipSuccess) {
    delete c;
    return mgpu::set_error(MGPU_E_DEVICE, "hipMalloc: %s", hipGetErrorString(e));
  }
  ncclResult_t r = ncclCommInitRank(&c->comm, world, id, rank);
  if (r != ncclSuccess) {
    hipFree(c->scratch);
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

int32_t mgpu_chips_broadcast(mgpu_ctx* ctx, const mgpu_chips* chips, int32_t root, mgpu_chips** out, void* stream) {
  if (!ctx || !ctx->comm || !out) return mgpu::set_error(MGPU_E_INVALID_ARG, "chips_broadcast: no communicator / out");
  CommState* c = state(ctx);
  if (root < 0 || root >= c->world) return mgpu::set_error(MGPU_E_INVALID_ARG, "root %d of %d", root, c->world);
  const bool is_root = c->rank == root;
  if (is_root && (!chips || chips->device != ctx->device))
    return mgpu::set_error(MGPU_E_INVALID_ARG, "chips_broadcast: the root needs its chip table on the context's GPU");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  *out = nullptr;
  // 1. the 1 KiB header, to size the receiving allocation
  void* hdr_dev = is_root ? chips->blob : c->scratch;
  NCCL_TRY(ncclBroadcast(hdr_dev, hdr_dev, (size_t)mgpu::kBlobHeaderSize, ncclUint8, root, c->comm, s));
  int64_t bytes = 0;
  if (is_root) {
    bytes = (int64_t)chips->bytes;
  } else {
    std::vector<uint8_t> h((size_t)mgpu::kBlobHeaderSize);
    HIP_TRY(hipMemcpyAsync(h.data(), c->scratch, h.size(), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    bytes = mgpu::blob_bytes_of_header(h.data());
    if (bytes < mgpu::kBlobHeaderSize) return mgpu::set_error(MGPU_E_INVALID_ARG, "chips_broadcast: not a chip-table blob");
  }
  // 2. the whole blob, straight into the receiving ranks' new allocation
  void* dst = nullptr;
  if (!is_root) HIP_TRY(hipMalloc(&dst, (size_t)bytes));
  void* buf = is_root ? chips->blob : dst;
  ncclResult_t r = ncclBroadcast(buf, buf, (size_t)bytes, ncclUint8, root, c->comm, s);
  if (r != ncclSuccess) {
    if (dst) hipFree(dst);
    return mgpu::set_error(MGPU_E_DEVICE, "ncclBroadcast(%lld bytes): %s", (long long)bytes, ncclGetErrorString(r));
  }
  HIP_TRY(hipStreamSynchronize(s));
  if (is_root) return MGPU_OK;
  int32_t st = mgpu::adopt_device_blob(ctx, dst, bytes, out);
  if (st) hipFree(dst);
  return st;
}

int32_t mgpu_pair_offsets(mgpu_ctx* ctx, int64_t local_pairs, int64_t* out_offset, int64_t* out_total,
                          int64_t* out_counts, void* stream) {
  if (!ctx || !ctx->comm) return mgpu::set_error(MGPU_E_INVALID_ARG, "pair_offsets: no communicator");
  if (local_pairs < 0) return mgpu::set_error(MGPU_E_INVALID_ARG, "pair_offsets: negative count");
  CommState* c = state(ctx);
  if ((size_t)(c->world + 1) * 8 > kScratch) return mgpu::set_error(MGPU_E_INVALID_ARG, "world too large");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  int64_t* mine = (int64_t*)c->scratch;
  int64_t* all = mine + 1;
  HIP_TRY(hipMemcpyAsync(mine, &local_pairs, 8, hipMemcpyHostToDevice, s));
  NCCL_TRY(ncclAllGather(mine, all, 1, ncclInt64, c->comm, s));
  std::vector<int64_t> counts((size_t)c->world);
  HIP_TRY(hipMemcpyAsync(counts.data(), all, counts.size() * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  int64_t off = 0, tot = 0;
  for (int r = 0; r < c->world; r++) {
    if (r < c->rank) off += counts[r];
    tot += counts[r];
    if (out_counts) out_counts[r] = counts[r];
  }
  if (out_offset) *out_offset = off;
  if (out_total) *out_total = tot;
  return MGPU_OK;
}

}  // extern "C"
