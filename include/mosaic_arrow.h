/*
 * mosaic_arrow.h -- the columnar entry of the join: Arrow C (Device) Data Interface.
 *
 * The reference evaluates its hot expressions row by row (`CodegenFallback`:
 * expressions/index/PointIndexGeom.scala:10-13, PointIndexLonLat.scala:8-12); a Spark
 * host with columnar batches hands the point columns over as Arrow arrays instead --
 * in Arrow's own ABI, so no Arrow library is needed on either side.  The structs below
 * are the Arrow C Data Interface and C Device Data Interface definitions (the standard
 * layout; guarded so an Arrow header included first takes precedence).
 */
#ifndef MOSAIC_ARROW_H
#define MOSAIC_ARROW_H

#include <stdint.h>

#include "mosaic_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

#ifndef ARROW_C_DATA_INTERFACE
#define ARROW_C_DATA_INTERFACE
#define ARROW_FLAG_DICTIONARY_ORDERED 1
#define ARROW_FLAG_NULLABLE 2
#define ARROW_FLAG_MAP_KEYS_SORTED 4
struct ArrowSchema {
    const char* format;
    const char* name;
    const char* metadata;
    int64_t flags;
    int64_t n_children;
    struct ArrowSchema** children;
    struct ArrowSchema* dictionary;
    void (*release)(struct ArrowSchema*);
    void* private_data;
};
struct ArrowArray {
    int64_t length;
    int64_t null_count;
    int64_t offset;
    int64_t n_buffers;
    int64_t n_children;
    const void** buffers;
    struct ArrowArray** children;
    struct ArrowArray* dictionary;
    void (*release)(struct ArrowArray*);
    void* private_data;
};
#endif

#ifndef ARROW_C_DEVICE_DATA_INTERFACE
#define ARROW_C_DEVICE_DATA_INTERFACE
typedef int32_t ArrowDeviceType;
#define ARROW_DEVICE_CPU 1
#define ARROW_DEVICE_CUDA 2
#define ARROW_DEVICE_CUDA_HOST 3
#define ARROW_DEVICE_ROCM 10
#define ARROW_DEVICE_ROCM_HOST 11
struct ArrowDeviceArray {
    struct ArrowArray array;
    int64_t device_id;
    ArrowDeviceType device_type;
    void* sync_event;
    int64_t reserved[3];
};
#endif

/* The join over Arrow columns on the context's GPU (ARROW_DEVICE_ROCM arrays, device_id =
 * the context's device): x, y float64 (format "g"), optional point_id int64 ("l", no
 * nulls; NULL = offset + row index).  Array offsets are honoured; a null x or y (validity
 * bitmaps) is a null point, which matches nothing (NullIntolerant: no pair), as in the
 * reference.  If an array carries a sync_event (a hipEvent_t) the work waits on it.
 * Otherwise as mgpu_pip_join. */
int32_t mgpu_pip_join_arrow(mgpu_ctx* ctx, const mgpu_chips* chips, int32_t index_system, int32_t res,
                            const struct ArrowDeviceArray* x, const struct ArrowDeviceArray* y,
                            const struct ArrowDeviceArray* point_id, int64_t capacity, int64_t* out_n_pairs,
                            int64_t* out_point_id, int32_t* out_polygon_id, void* stream, mgpu_stats* stats);

/* grid_pointascellid over an Arrow geometry column on the GPU: binary ("z" / "Z",
 * WKB) or utf8 ("u" / "U", WKT) with int32 / int64 offsets.  out_cell[i] (device int64);
 * null rows give cell 0 and a 0 bit in out_valid (device, (length + 7) / 8 bytes,
 * optional).  Errors as mgpu_geometry_to_cells. */
int32_t mgpu_geometry_to_cells_arrow(mgpu_ctx* ctx, int32_t index_system, int32_t res,
                                     const struct ArrowDeviceArray* geom, const struct ArrowSchema* schema,
                                     int64_t* out_cell, uint8_t* out_valid, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* MOSAIC_ARROW_H */
