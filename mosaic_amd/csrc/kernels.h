// Launch interface between the C-ABI layer (capi.cpp) and the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mosaic_gpu.h"
#include "chip_table.h"

namespace mgpu {

struct JoinArgs {
  const double* x;
  const double* y;
  int64_t n;
  int64_t n_tiles;
  int res;
  int res_match;                    // H3: the chips' resolution equals `res` (else nothing can match)
  ChipTableView chips;
  uint32_t* tile_count;             // [n_tiles] pairs of each tile
  uint32_t* group_sum;              // [n_tiles / 32] pairs per group of 32 tiles, zeroed before launch
  uint32_t* group_cand;             // [n_tiles / 32] border-chip candidates per group (statistics), zeroed
  uint64_t* tile_where;             // [n_tiles] first record of the tile in `recs` (~0: dropped)
  uint64_t* recs;                   // [n_tiles * tile points] slots, then [pool_cap] overflow pool
  int64_t pool_cap;
  unsigned long long* pool_used;    // zeroed before launch
  uint32_t* dirty;                  // [n_tiles] tiles with a near-tie point (for pip_fix_kernel)
  uint32_t* n_dirty;                // zeroed before launch
  unsigned long long* counters;     // [0] pairs [1] near-ties [2] invalid [3] candidates
  // The H3 route's near-ties (the points it resolved inside its tie band): tie_queue[0] =
  // count (zeroed before launch), record q = tie_queue[2 + 4q ..] {input position, x bits,
  // y bits, lattice key of the route's (face, ijk)} while q < tie_cap.  The host resolves
  // them with the reference's libm (h3_glibc.h) and, where that moves a cell, reruns the
  // join with the overrides: ovr[2k] = input position (ascending), ovr[2k + 1] = the
  // lattice key to use instead of the route's.
  uint64_t* tie_queue;
  int64_t tie_cap;
  const uint64_t* ovr;
  int64_t n_ovr;
  // tie_host = 1 (H3 with the reference's libm, first pass): a point whose FAST projection
  // is in its tie band is queued as above with the fast path's lattice key and joined with
  // that cell -- no tile goes to a fix kernel for it, no device route runs; the host then
  // recomputes every queued point with the reference's libm and, only if some cell moves,
  // reruns the join (tie_host = 0) with an override for every queued point.
  int tie_host;
  const uint32_t* pos_of;           // binned pipeline: input position of binned slot s (else null)
  // split pipeline (launch_split): the mixed points of chunk c are the chunk's listed
  // points c * split_chunk() + mixed_idx[c * split_chunk() + m], m < chunk_mixed[c]; their
  // answers (first chip | match mask << 32) go to mixed_res at the same list position;
  // group_sum / group_cand are then per chunk
  const uint16_t* mixed_idx;
  uint64_t* mixed_res;
  const uint32_t* chunk_mixed;
  // a chunk with more than one tile of mixed points queues its further tiles here (for
  // pip_mixed_more_kernel): extra[0 .. *n_extra), capacity chunks * (tiles per chunk - 1)
  uint32_t* extra;
  uint32_t* n_extra;

  const uint8_t* valid;             // null points (Arrow validity bitmap at bit offset valid_off), or null
  int64_t valid_off;
  int poly_answers;                 // binned pipeline: a one-match answer is (polygon id | 1 << 32)
  // binned H3 pipeline over a dense lattice grid: per binned slot, the point's grid entry
  // index (| kKeyDeep) or a kKey* code, written by bin_scatter_kernel (else null)
  const uint32_t* bin_key = nullptr;
  // binned pipeline (MGPU_BIN_JOIN_COUNTS): the join adds each slot's match count to its
  // INPUT chunk's pair count here (pos_of[slot] / bin_chunk()), zeroed before launch --
  // the emit's offsets without a separate gather pass (else null)
  uint32_t* in_chunk_pairs = nullptr;
};

// The override pass's scratch (launch_join_redo / launch_split_redo): the units (fused
// tiles / split chunks) to rerun, their counts before, a flag per unit, and whether any
// count changed.
struct RedoArgs {
  const uint32_t* list;
  uint32_t* old;
  uint8_t* affected;  // [units], zeroed
  uint32_t* changed;  // zeroed: 1 when some unit's count changed
  uint32_t* first;    // ~0 before: the first unit whose count changed
};

// The split pipeline (a chip table with a pixel index and at most 32 chips per cell):
//   classify_kernel   per point: pixel class -> code (pure answer or "mixed"); per chunk of
//                     split_chunk() points the pure pairs and the ordered list of mixed points
//   pip_mixed_kernel  the mixed points, tiles of join_tile_points() gathered from the lists
//                     (+ pip_mixed_fix_kernel for tiles holding an H3 near-tie)
//   tile_scan_kernel  chunk pair counts -> output offsets
//   split_emit_kernel codes + mixed answers -> ordered (point_id, polygon_id) pairs
struct SplitArgs {
  JoinArgs j;                       // points, chips, counters, dirty list, mixed lists
  void* codes;                      // [n] u16 (H3: pixel class) / u32 (BNG: first << 8 | mask)
  uint32_t* chunk_pairs;            // [chunks] (= j.group_sum)
  uint32_t* chunk_mixed;            // [chunks]
  uint16_t* mixed_idx;              // [chunks * split_chunk()]
  uint32_t* extra;                  // [chunks * split_chunk() / join_tile_points()] (j.extra)
  uint64_t* chunk_off;              // [chunks] written by the scan
  const int64_t* point_id;
  int64_t id_base;
  int64_t capacity;
  int64_t* out_point;
  int32_t* out_poly;
  // an override rerun (launch_split_redo): as EmitArgs.redo_*, per chunk
  const uint32_t* redo_first = nullptr;
  const uint8_t* redo_affected = nullptr;
};
int64_t split_chunk();
int64_t split_chunk_tiles();
int64_t split_chunks(int64_t n);
hipError_t launch_split(int is, const SplitArgs& a, hipStream_t s, hipEvent_t after_classify, hipEvent_t after_mixed);
hipError_t launch_split_emit(int is, const SplitArgs& a, hipStream_t s);
// the override passes (kernels.hip launch_join_redo): the split pipeline's over R.list's n chunks
hipError_t launch_split_redo(int is, const SplitArgs& sa, const RedoArgs& R, int64_t n, hipStream_t s);

// The binned pipeline (a chip table far larger than the caches): the points
// are counting-sorted by a coarse spatial bin so that the join walks the chip table bin
// by bin instead of at random, then the answers are gathered back into input order.
//   bin_hist_kernel     per chunk of bin_chunk() points: the chunk's bin counts
//   bin_colscan_kernel  + bin_base_kernel: counts -> run offsets (bin-major, chunk-minor)
//   bin_scatter_kernel  x, y -> their binned slots (sorted by bin in LDS, written as runs),
//                       perm[slot] = the input position
//   pip_binned_kernel   join_tile's phases over the binned points, tiles dealt to the XCDs
//                       in contiguous runs (one bin's chips stay in one L2); answers
//                       (first chip | match mask << 32) per slot in j.mixed_res
//                       (+ pip_mixed_fix_kernel for the tiles holding an H3 near-tie)
//   bin_gather_kernel   the answers back in input order (bin runs read whole, placed via
//                       perm[] in LDS); pairs per input chunk of split_chunk() points
//   tile_scan_kernel    -> output offsets;  bin_emit_kernel: ordered pairs
struct BinArgs {
  SplitArgs s;                      // s.j: the BINNED points (x, y = the binned copies),
                                    // mixed_idx = chunk_mixed = null; s.chunk_pairs / chunk_off:
                                    // per INPUT chunk; s.j.group_sum / group_cand: per binned chunk
  const double* x;                  // the input points
  const double* y;
  double* bx;                       // [n] binned copies
  double* by;
  uint32_t* perm;                   // [n] input point of binned slot s
  uint64_t* res;                    // [n] the answers (first chip | match mask << 32) in input order
  uint32_t* cnt;                    // [bin chunks * nb] bin counts per chunk of bin_chunk() points
  uint32_t* pre;                    // [bin chunks * nb] their prefixes within the chunk's group
  uint32_t* gsum;                   // [bin groups * nb] group sums, then group bases
  double x0, y0, inv_bx, inv_by;    // the bin grid over the chip table's extent
  int32_t nbx, nby;                 // nbx * nby <= bin_max()
  int32_t xcd_runs;                 // deal each XCD a contiguous run of binned tiles (option bin_xcd)
  uint32_t* key;                    // [n] H3, dense grid: the binned slot's grid key (JoinArgs.bin_key), or null
};
int64_t bin_chunk();
int64_t bin_chunks(int64_t n);
int64_t bin_groups(int64_t n);
int32_t bin_max();
hipError_t launch_binned(int is, const BinArgs& a, hipStream_t s, hipEvent_t after_bin, hipEvent_t after_join);
hipError_t launch_bin_emit(const BinArgs& a, hipStream_t s);

// pair_emit_kernel: tile records -> ordered (point_id, polygon_id) output
struct EmitArgs {
  const uint32_t* tile_count;       // records of each tile
  uint64_t* group_off;              // [n_tiles / 32] written by the tile scan
  const uint64_t* tile_where;
  const uint64_t* recs;
  const int64_t* point_id;
  int64_t id_base;
  int64_t capacity;
  int64_t* out_point;
  int32_t* out_poly;
  // an override rerun (launch_join_redo): a tile before *redo_first (the first whose count
  // changed, ~0: none) and not flagged in redo_affected keeps its output (null: every tile
  // is emitted)
  const uint32_t* redo_first = nullptr;
  const uint8_t* redo_affected = nullptr;
};


// ties: [0] count, [1 .. tie_cap] positions of the points the fast projection hands to the
// H3 route (zero ties[0] before launch; on overflow the route pass redoes every point);
// tie_queue / tq_cap: the route's own near-ties as JoinArgs.tie_queue, the key being the
// route's cell id (zero tie_queue[0] before launch).  `valid` (optional Arrow bitmap at bit
// offset voff): null points get cell 0
hipError_t launch_cells(int is, int res, const double* x, const double* y, int64_t n, int64_t* out,
                        unsigned long long* counters, unsigned long long* ties, int64_t tie_cap,
                        uint64_t* tie_queue, int64_t tq_cap, hipStream_t s, const uint8_t* valid = nullptr,
                        int64_t voff = 0);
// out[pos[k]] = val[k], k < n (the host's libm corrections of near-tie cells)
hipError_t launch_scatter_i64(const int64_t* pos, const int64_t* val, int64_t n, int64_t* out, hipStream_t s);
// x[pos[k]], y[pos[k]] -> xy[2k], xy[2k + 1] (coordinates of a few points, for the host)
hipError_t launch_gather_xy(const double* x, const double* y, const int64_t* pos, int64_t n, double* xy,
                            hipStream_t s);
// the point (centroid) of each POINT / MULTIPOINT geometry, WKB (format 0) or WKT (1),
// rows data[offsets[i] .. offsets[i + 1]); null rows (valid bitmap) -> NaN.  counters[4..6]
// += malformed / unsupported type / empty rows
hipError_t launch_decode_internal(const int32_t* type_id, const int64_t* row_part, const int64_t* part_ring,
                                  const int64_t* ring_off, const double* xy, const uint8_t* valid, int64_t voff,
                                  int64_t n, double* x, double* y, unsigned long long* counters, hipStream_t s);
hipError_t launch_decode_points(int format, const uint8_t* data, const void* offsets, int off32, const uint8_t* valid,
                                int64_t voff, int64_t n, double* x, double* y, unsigned long long* counters,
                                hipStream_t s);
// AND of two validity bitmaps (either may be null) into out (bit offset 0), n bits
hipError_t launch_valid_and(const uint8_t* a, int64_t aoff, const uint8_t* b, int64_t boff, int64_t n, uint8_t* out,
                            hipStream_t s);
int64_t join_tiles(int64_t n);
int64_t join_tile_points();
int64_t join_slot_records();   // records reserved per tile (pairs beyond go to the overflow pool)
// `after_stream` (optional) is recorded right after pip_join_kernel
hipError_t launch_join(int is, const JoinArgs& a, const EmitArgs& e, hipStream_t s, hipEvent_t after_stream);
// ... and the fused join's over R.list's n tiles
hipError_t launch_join_redo(int is, const JoinArgs& a, const EmitArgs& e, const RedoArgs& R, int64_t n, hipStream_t s);
// pair_emit_kernel alone, over the records a join left in the workspace
hipError_t launch_emit(const EmitArgs& e, int64_t n_tiles, hipStream_t s);
// StringType cell ids: offsets[n + 1] (device); chunk: scratch of format_chunks(n) int64;
// counters[2] += ids without a string form (BNG)
int64_t format_chunks(int64_t n);
hipError_t launch_format_cells(int is, const int64_t* cells, int64_t n, char* out, int64_t out_bytes,
                               int64_t* offsets, int64_t* chunk, unsigned long long* counters, hipStream_t s);
// kRing / kLoop lists (BNG; H3 with the pentagon fallbacks), in three steps:
//   launch_kring_count     mc[i] = list length, -1 (invalid cell) or -2 (an H3 walk met a
//                          pentagon; fb_idx lists those, counters[3] = their number),
//                          chunk[] = the direct lists' sums per chunk
//   launch_kring_fallback  those cells fb_idx[j0 .. j1) with H3's _kRingInternal / Mosaic's
//                          kLoop set difference, kring_fallback_words(k) u64 of scratch per
//                          cell (k <= kring_fallback_max_k()); write = 0: their lengths into
//                          mc and chunk; write = 1 (after launch_kring_write): their lists
//   launch_kring_write     chunk scan, offsets[n + 1], the direct lists at out[offsets[i]]
//                          (written when within capacity)
int64_t format_chunks(int64_t n);
hipError_t launch_kring_count(int is, const int64_t* cells, int64_t n, int k, int loop_only, int64_t* mc,
                              int64_t* chunk, uint32_t* fb_idx, unsigned long long* counters, hipStream_t s);
int64_t kring_fallback_words(int k);
int32_t kring_fallback_max_k();
hipError_t launch_kring_fallback(const int64_t* cells, const uint32_t* fb_idx, int64_t j0, int64_t j1, int k,
                                 int loop_only, int64_t* mc, int64_t* chunk, const int64_t* offsets, int64_t* out,
                                 int64_t capacity, uint64_t* scratch, int write, unsigned long long* counters,
                                 hipStream_t s);
hipError_t launch_kring_write(int is, const int64_t* cells, int64_t n, int k, int loop_only, const int64_t* mc,
                              int64_t* chunk, int64_t* offsets, int64_t* out, int64_t capacity, hipStream_t s);
// counters[2] += chip rows outside [0, n_chips) (their out is -2)
hipError_t launch_st_contains(const ChipTableView& t, const int64_t* row, const double* x, const double* y, int64_t n,
                              int8_t* out, unsigned long long* counters, hipStream_t s);

}  // namespace mgpu
