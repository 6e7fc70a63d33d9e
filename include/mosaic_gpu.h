/*
 * mosaic_gpu.h -- C ABI of the MI355X grid-indexed point-in-polygon join.
 *
 * The drop-in boundary for the reference's hot path (tiems90/mosaic 0.4.3):
 *   points -> cell id        grid_pointascellid / grid_longlatascellid
 *   polygons -> chips        grid_tessellateexplode rows (is_core, index_id, wkb)
 *   join + filter            cell == index_id AND (is_core OR st_contains(wkb, pt))
 * behind the reference's IndexSystem plugin interface
 *   src/main/scala/com/databricks/labs/mosaic/core/index/IndexSystem.scala:15-318
 * Each entry point below names the reference interface it replaces.  A JVM host
 * binds them through a thin JNI shim; this repository's Python
 * host (mosaic_amd/) binds them with ctypes.
 *
 * Conventions
 *  - Plain C types only.  Status codes: 0 = ok, negative = error class; the
 *    message of the calling thread's last error is mgpu_last_error().
 *  - "device" pointers are HBM allocations on the context's GPU (hipMalloc /
 *    torch tensors); "host" pointers are ordinary memory.  `stream` is a
 *    hipStream_t (NULL = the legacy default stream).
 *  - Functions are thread-safe for distinct contexts; one context must not be used
 *    concurrently from several threads (one context per executor thread/GPU).
 *  - index_system: MGPU_H3 (H3IndexSystem) or MGPU_BNG (BNGIndexSystem);
 *    resolutions are validated like IndexSystem.getResolution
 *    (H3IndexSystem.scala:45-60: 0..15; BNGIndexSystem.scala:349-360: +-1..+-6).
 */
#ifndef MOSAIC_GPU_H
#define MOSAIC_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MGPU_OK 0
#define MGPU_E_INVALID_ARG -1       /* IllegalArgumentException (bad argument, NaN H3 coordinate) */
#define MGPU_E_RESOLUTION -2        /* IllegalStateException (resolution not supported) */
#define MGPU_E_NAN -3               /* IllegalStateException (BNG: "NaN coordinates are not supported.") */
#define MGPU_E_WKB -4               /* JTS ParseException / unsupported chip geometry */
#define MGPU_E_CAPACITY -5          /* output arrays too small; the required count is returned */
#define MGPU_E_DEVICE -6            /* HIP runtime error */
#define MGPU_E_INTERNAL -7          /* kernel protocol failure (look-back timeout) */
#define MGPU_E_UNSUPPORTED -8       /* input outside what the device path builds (geometry types, huge polygons) */
#define MGPU_E_EMPTY -9             /* IllegalStateException (JTS: getX / getY of an empty Point) */

#define MGPU_H3 0
#define MGPU_BNG 1

typedef struct mgpu_ctx mgpu_ctx;
typedef struct mgpu_chips mgpu_chips;

/* Per-call statistics (optional out-parameter). */
typedef struct mgpu_stats {
    int64_t n_points;       /* points processed */
    int64_t n_pairs;        /* (point, polygon) pairs produced */
    int64_t n_near_ties;    /* H3 points whose hex2d coordinate is within 2^-40 (relative)
                               of a cell edge: the only points where an ulp-level libm
                               difference could change the cell */
    int64_t n_candidates;   /* (point, border chip) PIP evaluations */
    float kernel_ms;        /* device time of the whole call's launches (HIP events) */
    float stream_kernel_ms; /* of which the streaming kernel over all points (pip_join_kernel,
                               classify_kernel in the split pipeline, pip_binned_kernel in
                               the binned one) */
    float mixed_kernel_ms;  /* split pipeline: pip_mixed_kernel + pip_mixed_fix_kernel;
                               binned pipeline: the binning (rank, scan, scatter) */
    float emit_kernel_ms;   /* split pipeline: tile_scan_kernel + split_emit_kernel;
                               binned pipeline: fix, count, scan and emit */
    int32_t pipeline;       /* MGPU_PIPELINE_FUSED, _SPLIT or _BINNED */
    int32_t libm_overrides; /* near-tie cells the reference's libm placed differently from the
                               device's correctly rounded route (the call was then completed
                               with the reference's cells; h3_libm option) */
} mgpu_stats;
/* the join's three pipelines: one fused kernel per tile of points; for a chip
 * table with a pixel index, classify all points, resolve the mixed ones, emit; for a chip
 * table far larger than the caches, bin the points spatially (counting sort), join the
 * binned points, gather the answers back in input order */
#define MGPU_PIPELINE_AUTO (-1)
#define MGPU_PIPELINE_FUSED 0
#define MGPU_PIPELINE_SPLIT 1
#define MGPU_PIPELINE_BINNED 2

/* H3 near-tie points (the few whose cell an ulp of libm can move): the reference's
 * arithmetic -- H3-Java's JNI library on the host: platform glibc sin/cos/tan/acos/atan2,
 * x87 long double -- or the device's correctly rounded route. */
#define MGPU_LIBM_REFERENCE 0
#define MGPU_LIBM_CORRECTLY_ROUNDED 1

const char* mgpu_last_error(void);
const char* mgpu_version(void);
/* Points per tile of mgpu_pip_join (its per-tile workspace and statistics; no
 * reference counterpart). */
int32_t mgpu_join_tile_points(void);

/* One context per GPU/executor: owns the stream-ordered workspace (and, after
 * mgpu_comm_init, the RCCL communicator; destroyed with the context). */
int32_t mgpu_ctx_create(int32_t device_id, mgpu_ctx** out);
int32_t mgpu_ctx_destroy(mgpu_ctx* ctx);

/* Per-context options (no reference counterpart: the reference's planner is Spark's).
 * Nothing is read from the process environment; a JVM host sets these per context.
 *   "h3_libm"         MGPU_LIBM_REFERENCE (default) / MGPU_LIBM_CORRECTLY_ROUNDED
 *   "pipeline"        MGPU_PIPELINE_AUTO (default), or force _FUSED, _SPLIT (tables with a
 *                     pixel index), _BINNED (whenever it applies, at any size)
 *   "bin_count"       bins of the binned pipeline, 1..512 (default 64)
 *   "bin_min_mb"      the planner bins for chip tables of at least this size (256)
 *   "bin_min_points"  ... and batches of at least this many points (2^21)
 *   "bin_xcd"         1 (default): binned tiles dealt to the 8 XCDs in contiguous runs
 *   "bin_keys"        1: H3 binned joins over a dense grid take each point's grid entry from
 *                     the binning pass (which projects the point); 0 (default): the join
 *                     projects (C3: binning +1.4 ms, join -0.16 ms per 1.25e8 points)
 *   "ring_batch"      ring joins hold at most this many candidate pairs in scratch at a time
 *                     (landmarks in batches; default 2^26)
 *   "spin_us"         synchronous calls poll their stream (yielding the core between polls)
 *                     at most this long, then block in hipStreamSynchronize (default 2000;
 *                     0 = block at once)
 *   "bng_split"       1 / 0 (default): a BNG table on a dense grid without a pixel index
 *                     joins through the split pipeline with the grid entry as the code (a
 *                     cell of core chips, or an answer-grid square, answers its points; the
 *                     rest go to the mixed tiles) / through the fused pipeline
 *   "raster", "raster_bng", "raster_sub", "raster_milli"
 *                     the chip-table builder of mgpu_chips_upload on this context
 *                     (mgpu_build_opts below)
 * MGPU_E_INVALID_ARG for an unknown key or a value out of range. */
int32_t mgpu_ctx_set_option(mgpu_ctx* ctx, const char* key, int64_t value);
int32_t mgpu_ctx_get_option(const mgpu_ctx* ctx, const char* key, int64_t* value);

/* Chip-table builder options (mgpu_chips_host_blob_ex; mgpu_chips_upload takes its
 * context's).  raster: 1 = build the pixel index where it pays (H3 res >= 5), 0 = never;
 * raster_bng: 1 = build it for BNG tables too (default 0: measured slower on C4);
 * raster_sub: sub-pixels per mixed pixel edge (2..16, 0 = no second level; default 16);
 * raster_milli: pixel edge / mean cell edge x 1000 (10..1000, default 250). */
typedef struct mgpu_build_opts {
    int32_t raster, raster_bng, raster_sub, raster_milli;
} mgpu_build_opts;
void mgpu_build_opts_default(mgpu_build_opts* opts);

/* IndexSystem.getResolution for an integer resolution (H3IndexSystem.scala:45-60,
 * BNGIndexSystem.scala:349-360).  Returns MGPU_OK or MGPU_E_RESOLUTION. */
int32_t mgpu_check_resolution(int32_t index_system, int32_t res);

/* IndexSystem.pointToIndex(x, y, res) over a batch (IndexSystem.scala:237;
 * H3IndexSystem.scala:168-170 = H3Core.geoToH3(lat, lon, res);
 * BNGIndexSystem.scala:284-298).  x = lon / eastings, y = lat / northings.
 * Device pointers, asynchronous on `stream`; `stats` (optional) is filled after
 * a stream synchronisation. */
int32_t mgpu_points_to_cells(mgpu_ctx* ctx, int32_t index_system, int32_t res,
                             const double* x, const double* y, int64_t n,
                             int64_t* out_cell, void* stream, mgpu_stats* stats);

/* grid_pointascellid on a geometry column (PointIndexGeom.scala:33-47: GeometryAPI.geometry
 * (GeometryAPI.scala:81-89) decodes BinaryType as WKB, StringType as WKT, HexType as
 * hex WKB, JSONType as GeoJSON, then getCentroid -- JTS Centroid: area-weighted for
 * polygons, length-weighted for lines, the mean of points -- then pointToIndex).  Rows
 * are data[offsets[i] .. offsets[i + 1]) (the Arrow binary / utf8 layout).  WKB / HEX:
 * every geometry type (big- or little-endian, EWKB / ISO Z, M, nested collections; the
 * rings and one-point lines JTS's non-strict WKBReader repairs are repaired); WKT (Java
 * Double.parseDouble rounding; WKTReader) and GeoJSON (GeoJsonReader): every type, Z / M
 * ignored, collections nested up to 8 deep, strict rings.  Malformed rows MGPU_E_WKB (JTS
 * ParseException / IllegalArgumentException), empty
 * geometries MGPU_E_EMPTY.  `valid` (optional Arrow bitmap, bit offset valid_offset): null rows are
 * null out -- out_cell 0 and a 0 bit in out_valid ((n + 7) / 8 bytes, optional).
 * mgpu_points_from_geometry stops at the point (x, y; NaN for null rows).  Device
 * pointers; synchronises `stream`. */
#define MGPU_GEOM_WKB 0
#define MGPU_GEOM_WKT 1
#define MGPU_GEOM_HEX 2     /* HexType: WKB as hex text (WKBReader.hexToBytes) */
#define MGPU_GEOM_GEOJSON 3 /* JSONType: GeoJSON text (GeoJsonReader) */
int32_t mgpu_points_from_geometry(mgpu_ctx* ctx, int32_t format, const uint8_t* data, const int64_t* offsets,
                                  const uint8_t* valid, int64_t valid_offset, int64_t n, double* out_x, double* out_y,
                                  void* stream);
int32_t mgpu_geometry_to_cells(mgpu_ctx* ctx, int32_t index_system, int32_t res, int32_t format, const uint8_t* data,
                               const int64_t* offsets, const uint8_t* valid, int64_t valid_offset, int64_t n,
                               int64_t* out_cell, uint8_t* out_valid, void* stream, mgpu_stats* stats);

/* grid_pointascellid on Mosaic's InternalGeometryType column (InternalGeometry.scala:
 * typeId, boundaries, holes; MosaicGeometryJTS.fromInternal, MosaicGeometryJTS.scala:343-357)
 * flattened as nested lists: row i's parts [row_part[i], row_part[i + 1]), part q's
 * rings [part_ring[q], part_ring[q + 1]) (the boundary, then its holes), ring k's points
 * xy[2 ring_off[k] .. 2 ring_off[k + 1]) -- the Arrow layout of list<list<list<x, y>>>.
 * type_id: POINT 1, MULTIPOINT 2, LINESTRING 3, MULTILINESTRING 4, POLYGON 5,
 * MULTIPOLYGON 6 (GeometryTypeEnum); others MGPU_E_UNSUPPORTED.  Centroid, validity and
 * errors as mgpu_geometry_to_cells.  Device pointers; synchronises `stream`. */
int32_t mgpu_internal_geometry_to_cells(mgpu_ctx* ctx, int32_t index_system, int32_t res, int64_t n,
                                        const int32_t* type_id, const int64_t* row_part, const int64_t* part_ring,
                                        const int64_t* ring_off, const double* xy, const uint8_t* valid,
                                        int64_t valid_offset, int64_t* out_cell, uint8_t* out_valid, void* stream,
                                        mgpu_stats* stats);

/* Host-pointer convenience form (copies over PCIe). */
int32_t mgpu_points_to_cells_host(mgpu_ctx* ctx, int32_t index_system, int32_t res,
                                  const double* x, const double* y, int64_t n, int64_t* out_cell);

/* BNGIndexSystem.format / parse (BNGIndexSystem.scala:119-134, 440-442; parse at
 * the `parse` method) -- the StringType cell id (default for BNG).  `out` receives
 * concatenated ASCII ids, out_offsets[n + 1] their boundaries; out_bytes is the
 * capacity of `out` (ids are at most 16 chars). Host pointers. */
int32_t mgpu_bng_format(const int64_t* cells, int64_t n, char* out, int64_t out_bytes, int64_t* out_offsets);
int32_t mgpu_bng_parse(const char* ids, const int64_t* offsets, int64_t n, int64_t* out_cells);
/* StringType cell ids on the device (IndexSystem.serializeCellId, IndexSystem.scala:61-70):
 * BNG = BNGIndexSystem.format as above, H3 = h3ToString (lowercase hex, H3IndexSystem
 * format).  Device pointers, out_offsets[n + 1] device int64.  Synchronises `stream`;
 * *out_total = bytes the ids need.  MGPU_E_INVALID_ARG if an id has no string form
 * (the reference throws), MGPU_E_CAPACITY if out_bytes is too small (only the ids
 * that fit are written).  mgpu_bng_format_device = index_system MGPU_BNG. */
int32_t mgpu_format_cells_device(mgpu_ctx* ctx, int32_t index_system, const int64_t* cells, int64_t n, char* out,
                                 int64_t out_bytes, int64_t* out_offsets, int64_t* out_total, void* stream);
int32_t mgpu_bng_format_device(mgpu_ctx* ctx, const int64_t* cells, int64_t n, char* out, int64_t out_bytes,
                               int64_t* out_offsets, int64_t* out_total, void* stream);

/* IndexSystem.kRing / kLoop over a device column of cells (grid_cellkring /
 * grid_cellkloop: expressions/index/CellKRing.scala:68, CellKLoop.scala:63) --
 * BNGIndexSystem.kRing / kLoop, BNGIndexSystem.scala:221-252 (the cell, then loops
 * 1..k; a loop = pointToIndex of the 8k corners around the cell, kept when isValid),
 * in the reference's order.  H3: H3IndexSystem.kRing / kLoop, H3IndexSystem.scala:
 * 182-205 (H3 v3.7 kRing spiral / hexRing order; a walk that meets a pentagon takes H3's
 * _kRingInternal hash-set order, and kLoop Mosaic's kRing(k) diff kRing(k - 1) in Scala
 * HashSet order, any k).  Cell i's list
 * is out_cells[out_offsets[i] .. out_offsets[i + 1]); device pointers; *out_total =
 * entries needed (MGPU_E_CAPACITY when above `capacity`).  0 <= k <= 1024. */
int32_t mgpu_grid_kring(mgpu_ctx* ctx, int32_t index_system, const int64_t* cells, int64_t n, int32_t k,
                        int32_t loop_only, int64_t* out_cells, int64_t capacity, int64_t* out_offsets,
                        int64_t* out_total, void* stream);

/* Upload a chip table (the rows of grid_tessellateexplode, MosaicExplode.scala:70-83,
 * ChipType.scala:17-29): cell id, owning polygon id, is_core, and the chip WKB
 * (big- or little-endian, Polygon / MultiPolygon / GeometryCollection of those;
 * a NULL geometry is wkb_offsets[i] == wkb_offsets[i+1]).  Host pointers.  The WKB
 * is parsed once here (the reference re-parses it per candidate row).  For H3 the
 * cell hash is keyed by lattice position (see mosaic_amd/csrc/chip_table.h). */
int32_t mgpu_chips_upload(mgpu_ctx* ctx, int32_t index_system, int64_t n_chips, const int64_t* cell,
                          const int32_t* polygon_id, const uint8_t* is_core, const int64_t* wkb_offsets,
                          const uint8_t* wkb, mgpu_chips** out);
int32_t mgpu_chips_destroy(mgpu_chips* chips);
/* The chip table is one device allocation: expose it for replication (RCCL
 * broadcast of `bytes` at `device_ptr`), and rebuild a handle on another GPU from
 * a received copy (the received buffer is copied into a new allocation). */
int32_t mgpu_chips_device_blob(const mgpu_chips* chips, void** device_ptr, int64_t* bytes);
int32_t mgpu_chips_from_device_blob(mgpu_ctx* ctx, const void* device_ptr, int64_t bytes, mgpu_chips** out);
int32_t mgpu_chips_info(const mgpu_chips* chips, int64_t* n_chips, int64_t* n_cells, int64_t* n_vertices);

/* The chip table as one self-describing host blob (what mgpu_chips_upload uploads): a
 * JVM driver can build it once and ship the bytes to its executors, which upload them
 * with mgpu_chips_upload_blob.  Free with mgpu_host_free.  mgpu_host_blob_info checks a
 * received blob (magic, version, size, offsets) and reports its contents.  Host only. */
int32_t mgpu_chips_host_blob(int32_t index_system, int64_t n_chips, const int64_t* cell, const int32_t* polygon_id,
                             const uint8_t* is_core, const int64_t* wkb_offsets, const uint8_t* wkb, uint8_t** out,
                             int64_t* bytes);
int32_t mgpu_chips_host_blob_ex(int32_t index_system, int64_t n_chips, const int64_t* cell, const int32_t* polygon_id,
                                const uint8_t* is_core, const int64_t* wkb_offsets, const uint8_t* wkb,
                                const mgpu_build_opts* opts, uint8_t** out, int64_t* bytes);
int32_t mgpu_host_free(void* p);
int32_t mgpu_host_blob_info(const void* host_blob, int64_t bytes, int32_t* index_system, int64_t* n_chips,
                            int64_t* n_cells, int64_t* n_vertices);
int32_t mgpu_chips_upload_blob(mgpu_ctx* ctx, const void* host_blob, int64_t bytes, mgpu_chips** out);

/* Multi-GPU (one process per GPU): points are sharded by contiguous id range,
 * the chip table is replicated.  The reference's scale-out is Spark's broadcast of the
 * chip side to every executor (BroadcastHashJoin in the plan of notebooks/examples/python/
 * Quickstart/QuickstartNotebook.ipynb:1835); here each GPU's context owns an RCCL
 * communicator:
 *   mgpu_comm_unique_id  one rank creates the id (ncclGetUniqueId) and ships its
 *                        MGPU_COMM_ID_BYTES to every rank out of band (the JVM driver's
 *                        broadcast; torch.distributed's store in mosaic_amd/dist.py);
 *   mgpu_comm_init       every rank joins (ncclCommInitRank; blocks until all have);
 *   mgpu_chips_broadcast the root's chip table is replicated into a new allocation on
 *                        every other rank by one RCCL broadcast of the blob (plus one of
 *                        its 1 KiB header to size it); *out = the replica (NULL on root);
 *   mgpu_pair_offsets    RCCL all-gather of the per-rank pair counts: this rank's offset
 *                        in the globally ordered output, the total, and (optionally)
 *                        out_counts[world].
 * The collectives are enqueued on `stream` and complete before the calls return. */
#define MGPU_COMM_ID_BYTES 128
int32_t mgpu_comm_unique_id(uint8_t* out_id);
int32_t mgpu_comm_init(mgpu_ctx* ctx, const uint8_t* unique_id, int32_t rank, int32_t world);
int32_t mgpu_comm_info(mgpu_ctx* ctx, int32_t* rank, int32_t* world);
int32_t mgpu_comm_destroy(mgpu_ctx* ctx);
int32_t mgpu_chips_broadcast(mgpu_ctx* ctx, const mgpu_chips* chips, int32_t root, mgpu_chips** out, void* stream);
int32_t mgpu_pair_offsets(mgpu_ctx* ctx, int64_t local_pairs, int64_t* out_offset, int64_t* out_total,
                          int64_t* out_counts, void* stream);
/* TEST ONLY: a receiving rank's side of mgpu_chips_broadcast without RCCL -- the header
 * read from the device buffer dev_blob, the receiving allocation (fail_alloc != 0 forces
 * it to fail), the blob copied in, the table adopted -- so a corrupt header or a failed
 * allocation can be shown to return an error (it does not wait on anything). */
int32_t mgpu_test_receive_blob(mgpu_ctx* ctx, const void* dev_blob, int32_t fail_alloc, mgpu_chips** out);

/* The grid-ring neighbour join of SpatialKNN for point landmarks and point candidates, one
 * iteration (models/knn/GridRingNeighbours.scala: transform :121 and resultTransform;
 * SpatialKNN.scala's per-iteration filter): each landmark's cells -- kRing(cell, k)
 * (loop_only = 0: iteration 1's grid_geometrykringexplode) or kLoop(cell, k) (loop_only =
 * 1: iteration k's grid_geometrykloopexplode) of pointToIndex(landmark) -- joined with the
 * candidates' cells (grid_tessellateexplode of a point: its one chip); every (landmark,
 * candidate) sharing a cell is a pair once, self matches (identical coordinates) dropped,
 * distance = st_distance (JTS Coordinate.distance: Math.hypot), pairs with distance <=
 * max_distance (< 0: no threshold), per landmark ordered by (distance, candidate index)
 * and cut to the first max_per_left (0: all; SpatialKNN's neighbour_number <= k).  Output:
 * out_left = left_id_base + landmark index, out_right = candidate index, out_dist; landmarks
 * in order.  Device pointers; synchronises `stream`; MGPU_E_CAPACITY with *out_n when the
 * pairs exceed `capacity`. */
int32_t mgpu_ring_join(mgpu_ctx* ctx, int32_t index_system, int32_t res, int32_t k, int32_t loop_only,
                       const double* left_x, const double* left_y, int64_t n_left, const double* right_x,
                       const double* right_y, int64_t n_right, int64_t left_id_base, int32_t max_per_left,
                       double max_distance, int64_t capacity, int64_t* out_n, int64_t* out_left, int64_t* out_right,
                       double* out_dist, void* stream);
/* mgpu_ring_join with flags.  MGPU_RING_LEFT_OUTER: the join is left_outer
 * (GridRingNeighbours.scala:128) and resultTransform keeps the null group
 * (coalesce(intersects, true), :151): a landmark with a ring cell that holds no candidate
 * gets one row (left, -1, NaN) before its pairs -- Spark orders the null distance first in
 * the ascending window -- not counted by max_per_left nor filtered by max_distance.
 * Self matches: dropped when the coordinates are bit-identical; the reference compares
 * hash() of the geometry column (:154), so two rows holding the same point in different
 * text or WKB (or -0.0 vs 0.0) are distinct there but one here. */
#define MGPU_RING_LEFT_OUTER 1
int32_t mgpu_ring_join_ex(mgpu_ctx* ctx, int32_t index_system, int32_t res, int32_t k, int32_t loop_only,
                          const double* left_x, const double* left_y, int64_t n_left, const double* right_x,
                          const double* right_y, int64_t n_right, int64_t left_id_base, int32_t max_per_left,
                          double max_distance, int32_t flags, int64_t capacity, int64_t* out_n, int64_t* out_left,
                          int64_t* out_right, double* out_dist, void* stream);
/* SpatialKNN's exactness iteration (GridRingNeighbours.leftTransform, iterationID = -1,
 * GridRingNeighbours.scala:82-90; SpatialKNN.resultTransform): per landmark i, the cells of
 * grid_tessellate(st_buffer(landmark, radius[i]), res) -- JTS's 32-gon circle, mosaicFill's
 * cells (mgpu_tessellate) -- minus grid_geometrykring(landmark, res, k_iterated[i])
 * (array_except), joined with the candidates as mgpu_ring_join_ex does.  radius[i] (the
 * landmark's k-th match distance) NaN or <= 0 gives the landmark no cells.  radius and
 * k_iterated are HOST arrays; the points are device pointers.  Synchronises `stream`. */
int32_t mgpu_ring_join_final(mgpu_ctx* ctx, int32_t index_system, int32_t res, const double* left_x,
                             const double* left_y, const double* radius, const int32_t* k_iterated, int64_t n_left,
                             const double* right_x, const double* right_y, int64_t n_right, int64_t left_id_base,
                             int32_t max_per_left, double max_distance, int32_t flags, int64_t capacity,
                             int64_t* out_n, int64_t* out_left, int64_t* out_right, double* out_dist, void* stream);

/* st_contains(chip.wkb, point) for explicit (chip row, point) pairs
 * (ST_Contains.scala:21-44 -> MosaicGeometryJTS.contains, MosaicGeometryJTS.scala:197).
 * out[i] = 1 / 0, or -1 when the chip's geometry is NULL.  Device pointers.
 * Synchronises `stream`: a chip row outside [0, n_chips) fails the call with
 * MGPU_E_INVALID_ARG (its out[i] is -2). */
int32_t mgpu_st_contains(mgpu_ctx* ctx, const mgpu_chips* chips, const int64_t* chip_row,
                         const double* x, const double* y, int64_t n, int8_t* out, void* stream);

/* The hot path: cell id per point, equi-join against the chip table's
 * cell ids, `is_core OR st_contains` filter (one of three pipelines, chosen per call:
 * split for pixel-indexed tables, binned for tables beyond the caches, else fused --
 * mgpu_stats.pipeline); emits (point_id, polygon_id) pairs
 * ordered by input position then polygon id (sorted by point_id when point ids
 * ascend, e.g. contiguous id shards).  point_id may be NULL: ids are
 * point_id_base + index.  Device pointers.  Synchronises `stream` to return the
 * pair count in *out_n_pairs; if it exceeds `capacity` only the first `capacity`
 * pairs are written and MGPU_E_CAPACITY is returned.
 * H3 cells are the reference's bit for bit: the device decides every point outside a
 * 2^-40 tie band around the cell boundaries; the few inside it (mgpu_stats.n_near_ties)
 * are recomputed on the host with the reference's libm (option h3_libm), and when that
 * moves a cell the join is rerun with the corrected cells (mgpu_stats.libm_overrides). */
int32_t mgpu_pip_join(mgpu_ctx* ctx, const mgpu_chips* chips, int32_t index_system, int32_t res,
                      const double* x, const double* y, const int64_t* point_id, int64_t point_id_base,
                      int64_t n, int64_t capacity, int64_t* out_n_pairs, int64_t* out_point_id,
                      int32_t* out_polygon_id, void* stream, mgpu_stats* stats);

/* After mgpu_pip_join returned MGPU_E_CAPACITY (*out_n_pairs = the count): write all
 * pairs of that join into larger output arrays without redoing it -- the join's pair
 * records stay in the context until its next call.  (Only when the workspace's overflow
 * pool had to drop records -- tiles with more pairs than points beyond the capacity --
 * is the join redone, from the same, unchanged, input arrays.)  Synchronises `stream`;
 * MGPU_E_INVALID_ARG if no join was kept, MGPU_E_CAPACITY if capacity is still short. */
int32_t mgpu_pip_join_fetch(mgpu_ctx* ctx, int64_t capacity, int64_t* out_n_pairs, int64_t* out_point_id,
                            int32_t* out_polygon_id, void* stream);

/* Asynchronous form, in two calls.  mgpu_pip_join_async enqueues the join on `stream`
 * and returns at once: the pair count is left in device memory (*d_n_pairs, one int64)
 * -- graph-capturable once mgpu_ctx_reserve has sized the workspace and one call of the
 * same size has grown the split / binned pipeline's buffers.  As in the synchronous
 * call, H3 points inside the fast path's tie band are joined with the fast cell and
 * queued; mgpu_pip_join_finish (same context, no other call on it in between) waits
 * for the stream, recomputes the queued points with the reference's libm (option
 * h3_libm; H3IndexSystem.scala:168-170 -> H3-Java's glibc) and, only when that moves a
 * cell, reruns the join into the same output arrays and *d_n_pairs.  The pairs equal
 * mgpu_pip_join's once mgpu_pip_join_finish has returned MGPU_OK (or MGPU_E_CAPACITY,
 * with *out_n_pairs the count: mgpu_pip_join_fetch then writes them all); before it, a
 * batch with near-ties may hold the fast cell at those points.  BNG joins and the
 * correctly rounded mode have no host step, but the call is still required.
 * mgpu_pip_join_finish: MGPU_E_INVALID_ARG when no asynchronous join is pending (another
 * call on the context ended it).
 * Graph replays are NOT settled: finish pairs with the host-side mgpu_pip_join_async call
 * that queued the work, so a captured join replayed from a graph keeps the fast cell at
 * the points of its tie band (H3, reference libm) and finish after a replay returns
 * MGPU_E_INVALID_ARG.  A caller replaying graphs either sets h3_libm to
 * MGPU_LIBM_CORRECTLY_ROUNDED (the device decides every point, no host step) or reads the
 * replay's queued positions with mgpu_last_near_ties and reruns those batches with
 * mgpu_pip_join. */
int32_t mgpu_pip_join_async(mgpu_ctx* ctx, const mgpu_chips* chips, int32_t index_system, int32_t res,
                            const double* x, const double* y, const int64_t* point_id, int64_t point_id_base,
                            int64_t n, int64_t capacity, int64_t* d_n_pairs, int64_t* out_point_id,
                            int32_t* out_polygon_id, void* stream);
int32_t mgpu_pip_join_finish(mgpu_ctx* ctx, int64_t* out_n_pairs, mgpu_stats* stats);
int32_t mgpu_ctx_reserve(mgpu_ctx* ctx, int64_t max_points);

/* Parity audit (no reference counterpart): the input positions of the H3 near-tie
 * points of the last call on `ctx` (mgpu_pip_join, mgpu_points_to_cells, the geometry
 * entries) -- the points the device's route resolved inside its tie band
 * (mgpu_stats.n_near_ties), the only ones whose cell an ulp of libm can move; the
 * synchronous calls gave each of them the reference's cell.  Ascending.  Synchronises
 * the device.  MGPU_E_CAPACITY (with *out_n set) if cap is too small; MGPU_E_INTERNAL
 * if an asynchronous join found more than the queue holds. */
int32_t mgpu_last_near_ties(mgpu_ctx* ctx, int64_t* out_index, int64_t cap, int64_t* out_n);

/* Host-pointer convenience form of mgpu_pip_join (copies points in, pairs out). */
int32_t mgpu_pip_join_host(mgpu_ctx* ctx, const mgpu_chips* chips, int32_t index_system, int32_t res,
                           const double* x, const double* y, const int64_t* point_id, int64_t n,
                           int64_t capacity, int64_t* out_n_pairs, int64_t* out_point_id,
                           int32_t* out_polygon_id);

/* grid_tessellateexplode for a polygon set (Mosaic.getChips / mosaicFill,
 * core/Mosaic.scala:22-99; IndexSystem.getCoreChips/getBorderChips,
 * IndexSystem.scala:178-213).  Polygons are given as flat rings:
 *   polygon p has parts [poly_part_off[p], poly_part_off[p+1]),
 *   part q has rings [part_ring_off[q], part_ring_off[q+1]) (first = shell),
 *   ring r has vertices xy[2*ring_off[r] .. 2*ring_off[r+1]) (closed rings).
 * Output rows are returned through an opaque result read with
 * mgpu_tess_result_*; chip WKB is big-endian (JTS WKBWriter).  Host only. */
typedef struct mgpu_tess mgpu_tess;
int32_t mgpu_tessellate(int32_t index_system, int32_t res, int64_t n_polys, const int32_t* polygon_id,
                        const int64_t* poly_part_off, const int64_t* part_ring_off, const int64_t* ring_off,
                        const double* xy, int32_t keep_core_geometries, mgpu_tess** out);
/* The is_core rule (mgpu_tessellate uses MGPU_CORE_MOSAICFILL):
 *   MGPU_CORE_MOSAICFILL  the reference's: core iff the cell is in polyfill(buffer(-r))
 *                         (Mosaic.scala:71-93, getCoreChips IndexSystem.scala:208-213: its
 *                         centre inside the polygon at distance >= r = getBufferRadius from
 *                         the boundary); a border-set cell is never core -- getBorderChips'
 *                         equalsExact (IndexSystem.scala:186-188) compares JTS overlay's
 *                         clockwise shell with indexToGeometry's counter-clockwise cell --
 *                         so a cell the polygon holds whole but outside the core set is a
 *                         border chip whose geometry is the whole cell; chip cells beyond
 *                         the border band are dropped (never visited by the reference);
 *                         Near r the sets are decided as JTS 1.20's BufferOp builds them
 *                         (8 quadrant segments: fillets of chords, input simplification,
 *                         depth >= 1 of the raw offset curves -- mosaic_amd/csrc/jts_buffer.h);
 *   MGPU_CORE_CLIP        every cell the polygon holds whole is core;
 *   MGPU_CORE_DISTANCE    round 4's form of MOSAICFILL: the sets decided by the centre's
 *                         exact distance to the boundary (arcs, no simplification).
 * mgpu_tess_result_stats: out6 = {rows, core rows, whole cells flagged border (demoted),
 * partly covered cells flagged core (promoted), dropped, rows the restatement leaves
 * undecided (ambiguous: a centre within 1e-9 r of a buffer curve, or band membership
 * within the band simplification's 0.01 r; MGPU_CORE_DISTANCE: rows within the JTS
 * tolerance bands)}. */
#define MGPU_CORE_MOSAICFILL 0
#define MGPU_CORE_CLIP 1
#define MGPU_CORE_DISTANCE 2
int32_t mgpu_tessellate_ex(int32_t index_system, int32_t res, int64_t n_polys, const int32_t* polygon_id,
                           const int64_t* poly_part_off, const int64_t* part_ring_off, const int64_t* ring_off,
                           const double* xy, int32_t keep_core_geometries, int32_t core_rule, mgpu_tess** out);
/* mgpu_tessellate_geom: mgpu_tessellate_ex with the input geometries' types and the way
 * border chips are cut.  poly_type[n_polys] (NULL: MULTIPOLYGON iff several parts) holds
 * each geometry's WKB type, 3 = POLYGON or 6 = MULTIPOLYGON: coerceChipGeometry
 * (IndexSystem.scala:293-303) re-nodes a chip whose type differs from its polygon's.
 * chip_geometry: MGPU_CHIPS_OVERLAY (default) -- `polygon INTERSECTION cell` as JTS
 * OverlayNG computes it (RobustLineIntersector nodes, minimal result rings, separate pieces;
 * mosaic_amd/csrc/jts_overlay.h); MGPU_CHIPS_SUTHERLAND_HODGMAN -- rounds 1-5's ring clip
 * (its own crossing arithmetic, pieces bridged along the cell boundary), kept to count what
 * the overlay changes. */
#define MGPU_CHIPS_OVERLAY 0
#define MGPU_CHIPS_SUTHERLAND_HODGMAN 1
int32_t mgpu_tessellate_geom(int32_t index_system, int32_t res, int64_t n_polys, const int32_t* polygon_id,
                             const int64_t* poly_part_off, const int64_t* part_ring_off, const int64_t* ring_off,
                             const double* xy, const uint8_t* poly_type, int32_t keep_core_geometries,
                             int32_t core_rule, int32_t chip_geometry, mgpu_tess** out);
int32_t mgpu_tess_result_stats(const mgpu_tess* t, int64_t* out6);
/* mgpu_tess_result_core_stats: the first n of {rows, core rows, demoted, promoted,
 * dropped, ambiguous, carved tests, band tests, core rows whose centre is < r deep,
 * border rows whose centre is >= r deep, chip cells outside the band (dropped),
 * DP-sensitive rows, unresolved rows, polygons with an empty buffer(-r), border chips cut
 * by the overlay, ... of several pieces, ... re-noded by coerceChipGeometry, nodes that
 * re-noding added, ... whose overlay also gave lines / points}. */
int32_t mgpu_tess_result_core_stats(const mgpu_tess* t, int64_t* out, int32_t n);
int32_t mgpu_tess_result_sizes(const mgpu_tess* t, int64_t* n_chips, int64_t* wkb_bytes);
int32_t mgpu_tess_result_copy(const mgpu_tess* t, int64_t* cell, int32_t* polygon_id, uint8_t* is_core,
                              int64_t* wkb_offsets, uint8_t* wkb);
/* The rows the core rule left undecided (core_stats' ambiguous): n, their WKB bytes, and
 * when cell != NULL per row its cell, polygon, {kind (1 DP-sensitive band membership, 2 a
 * centre on a buffer curve), kept (the table holds the row), core}, and its chip -- the
 * one the table holds, or the one a dropped row would carry -- to count the pairs at stake. */
int32_t mgpu_tess_result_undecided(const mgpu_tess* t, int64_t* n, int64_t* wkb_bytes, int64_t* cell, int32_t* poly,
                                   uint8_t* kind_kept_core, int64_t* wkb_offsets, uint8_t* wkb);
/* frees the result (its memory returns on a helper thread, joined by the next
 * mgpu_tessellate* call and at unload: at most one result is in release at a time) */
int32_t mgpu_tess_destroy(mgpu_tess* t);

/* TEST ONLY -- not an interface of the reference.  Builds the chip table on the host
 * and evaluates st_contains(chip row, point) for n pairs by the join's path (the
 * classification grid + strip index of the device chip table) and by the sequential
 * JTS PointLocator; out_* = 1 / 0, -1 for a NULL geometry.  Host pointers; no GPU. */
int32_t mgpu_test_chip_contains_host(int32_t index_system, int64_t n_chips, const int64_t* cell,
                                     const int32_t* polygon_id, const uint8_t* is_core, const int64_t* wkb_offsets,
                                     const uint8_t* wkb, int64_t n, const int64_t* chip_row, const double* x,
                                     const double* y, int8_t* out_join_path, int8_t* out_point_locator);

/* TEST ONLY -- while on, every border chip the overlay's one-crossing-chain shortcut cuts
 * (jts_overlay.h Clipper::one_crossing_chain) is cut again by the general noded graph and
 * the two compared; out2 = {cells so checked, cells that differed} since it was turned on
 * (on = 1 resets the counts; on = 0 reads them and stops). */
int32_t mgpu_test_overlay_verify(int32_t on, int64_t* out2);

/* TEST ONLY -- the decimal parser of the WKT path (Double.parseDouble semantics) on one
 * string: characters consumed (0: not a number) and the value.  Host only. */
int32_t mgpu_test_parse_number(const char* s, int32_t len, double* out);
/* TEST ONLY -- the WKB / WKT point decoder on one host row: status 0 ok, 1 malformed,
 * 2 unsupported type, 3 empty. */
/* Test hooks of the exact H3 route (h3_exact.h), host-side: the route's elementary
 * operations (fn codes as oracle/oracle.h orc_h3_elementary: correctly rounded libm and
 * emulated x87 long-double expressions), and point -> cell by the route alone. */
int32_t mgpu_test_h3_elementary_host(int32_t fn, const double* a, const double* b, int64_t n, double* out);
int32_t mgpu_test_h3_route_host(const double* lon, const double* lat, int64_t n, int32_t res, int64_t* out_cell);
/* The near-tie resolver of the synchronous calls (h3_glibc.cpp: the reference's libm and
 * x87 arithmetic) on n host points. */
int32_t mgpu_test_h3_glibc_host(const double* lon, const double* lat, int64_t n, int32_t res, int64_t* out_cell);
/* H3 cell geometry as the builder computes it (h3ToGeoBoundary / h3ToGeo, degrees):
 * out_lonlat[20 n] (up to 10 vertices per cell), out_nverts[n], out_center[2 n]. */
int32_t mgpu_test_h3_boundary_host(const int64_t* cells, int64_t n, double* out_lonlat, int32_t* out_nverts,
                                   double* out_center);
/* TEST ONLY: an H3 cell's geometry as a core chip of it carries it (indexToGeometry,
 * H3IndexSystem.scala:103-112: the polar caps of makePoleGeometry, antimeridian cells
 * cut) as WKB into out[cap]; *out_len = its size (MGPU_E_CAPACITY when it exceeds cap). */
int32_t mgpu_test_h3_cell_wkb_host(int64_t cell, uint8_t* out, int64_t cap, int64_t* out_len);
int32_t mgpu_test_decode_point(int32_t format, const uint8_t* data, int64_t len, double* x, double* y);
/* TEST ONLY (profiling): the last join's 16 workspace counters (pairs, near-ties, invalid
 * points, candidates, ...; builds with -DMGPU_STAMPS add per-phase clock ticks of the
 * join tiles at [10..14]).  Waits for the device. */
int32_t mgpu_test_join_counters(mgpu_ctx* ctx, uint64_t* out16);

/* TEST ONLY: the centroids of n InternalGeometryType rows (layout of
 * mgpu_internal_geometry_to_cells) on the host; status[i] 0 ok, 1 malformed, 2 unsupported,
 * 3 empty. */
int32_t mgpu_test_internal_centroid(int64_t n, const int32_t* type_id, const int64_t* row_part, const int64_t* part_ring,
                                    const int64_t* ring_off, const double* xy, double* x, double* y, int32_t* status);

/* TEST ONLY -- st_contains(chip row, point) evaluated on a HOST blob (the join's
 * classification grid + strip path), to check on the CPU that a shipped blob is a
 * complete chip table.  out = 1 / 0, -1 NULL geometry.  Host pointers; no GPU. */
int32_t mgpu_test_blob_contains_host(const void* host_blob, int64_t bytes, int64_t n, const int64_t* chip_row,
                                     const double* x, const double* y, int8_t* out);

/* TEST ONLY -- not an interface of the reference.  Builds the chip table on the host and
 * looks n points up in its pixel index (the pre-resolved answers of the streaming join,
 * chip_table.h): out_kind 0 = no match, 1 = pure pixel (matches = sorted chips
 * out_first + j for the bits j of out_mask), 2 = full path, 3 = invalid coordinate,
 * 4 = no pixel index for this table/resolution; out_chip_poly[n_chips] = polygon id of
 * each sorted chip.  Host pointers; no GPU. */
int32_t mgpu_test_raster_host(int32_t index_system, int32_t res, int64_t n_chips, const int64_t* cell,
                              const int32_t* polygon_id, const uint8_t* is_core, const int64_t* wkb_offsets,
                              const uint8_t* wkb, int64_t n, const double* x, const double* y, int8_t* out_kind,
                              uint32_t* out_first, uint32_t* out_mask, int32_t* out_chip_poly);

/* TEST ONLY -- as mgpu_test_raster_host, for the BNG per-cell answer grids the fused
 * join's phase 1 reads (chip_table.h cell_ans): out_kind 0 / 1 = answered, 2 = not
 * answered (candidates' path), 3 = invalid coordinate, 4 = the table has none.
 * MGPU_E_INVALID_ARG for H3.  Host pointers; no GPU. */
int32_t mgpu_test_cell_answers_host(int32_t index_system, int32_t res, int64_t n_chips, const int64_t* cell,
                                    const int32_t* polygon_id, const uint8_t* is_core, const int64_t* wkb_offsets,
                                    const uint8_t* wkb, int64_t n, const double* x, const double* y, int8_t* out_kind,
                                    uint32_t* out_first, uint32_t* out_mask, int32_t* out_chip_poly);

/* TEST ONLY -- as mgpu_test_raster_host, for the H3 whole-cell shortcut of the streaming
 * joins (a one-chip cell whose chip is its own hexagon, a point deep inside the cell):
 * out_kind 1 = answered (chip out_first), 2 = not answered, 3 = invalid coordinate,
 * 4 = no dense H3 probe.  MGPU_E_INVALID_ARG for BNG.  Host pointers; no GPU. */
int32_t mgpu_test_whole_cells_host(int32_t index_system, int32_t res, int64_t n_chips, const int64_t* cell,
                                   const int32_t* polygon_id, const uint8_t* is_core, const int64_t* wkb_offsets,
                                   const uint8_t* wkb, int64_t n, const double* x, const double* y, int8_t* out_kind,
                                   uint32_t* out_first, uint32_t* out_mask, int32_t* out_chip_poly);

#ifdef __cplusplus
}
#endif

#endif /* MOSAIC_GPU_H */
