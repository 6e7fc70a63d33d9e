/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's JVM hot path for the grid-indexed
 * point-in-polygon join, used as the parity checker for the MI355X HIP path.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library; the product (mosaic_amd/) never links or calls it.
 *
 * What it restates (reference file:line, all under /root/reference):
 *   - H3IndexSystem.pointToIndex -> H3Core.geoToH3(lat, lon, res)
 *       src/main/scala/com/databricks/labs/mosaic/core/index/H3IndexSystem.scala:168-170
 *     H3 itself (com.uber:h3:3.7.0, pom.xml:91-97 -> H3 C core v3.7.x) is NOT in
 *     the reference; its published geoToH3 algorithm is restated in h3_oracle.c
 *     with the same x87 long-double constants and glibc libm calls.
 *   - BNGIndexSystem.pointToIndex / getQuadrant / encode
 *       .../core/index/BNGIndexSystem.scala:284-334, 540-553
 *   - ST_Contains -> MosaicGeometryJTS.contains -> JTS Geometry.contains
 *       .../expressions/geometry/ST_Contains.scala:34-36,
 *       .../core/geometry/MosaicGeometryJTS.scala:197
 *     JTS (org.locationtech.jts:jts-core:1.20.0, pom.xml:98-102) is not in the
 *     reference; PointLocator / RayCrossingCounter / CGAlgorithmsDD are restated.
 *   - WKB reading of chip geometry (MosaicGeometryIOCodeGenJTS.scala:23-29), both
 *     byte orders.
 *   - the user-level join `cell == index_id AND (is_core OR st_contains(wkb, pt))`
 *       notebooks/examples/python/Quickstart/QuickstartNotebook.ipynb:1835
 *
 * Pinning: see tests/golden/README.md (H3 / BNG / ST_Contains known-answer
 * vectors mined from the reference's tests, docs and notebook outputs).
 */
#ifndef MOSAIC_ORACLE_H
#define MOSAIC_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* The H3 route's elementary operations as the native library evaluates them (glibc
 * libm, x87 long-double constants): fn 0 sin, 1 cos, 2 tan, 3 acos, 4 atan2(a, b),
 * 5 a + M_2PI, 6 a - M_2PI, 7 a * M_SQRT7, 8 a / M_SIN60, 9 a - M_AP7_ROT_RADS,
 * 10 a / M_SQRT7, 11 a + M_AP7_ROT_RADS, 12 a < EPSILON, 13 a >= M_2PI; 20..24 the
 * correctly rounded sin, cos, tan, acos, atan2 (libquadmath, rounded once). */
/* The geoToH3 route's libm: 0 = glibc (the reference's, default), 1 = correctly rounded. */
void orc_h3_set_libm(int correctly_rounded);
void orc_h3_elementary(int fn, const double* a, const double* b, int64_t n, double* out);
/* H3 v3.7 geoToH3 on radians (C-API semantics: 0 on bad input). */
uint64_t orc_h3_geo_to_h3(double lat_rad, double lon_rad, int res);
/* H3IndexSystem.pointToIndex(lon, lat, res) in degrees.  jdk = 8 uses JDK 8's
 * Math.toRadians (deg / 180.0 * PI), jdk = 9 JDK 9+ (deg * (PI/180)). */
uint64_t orc_h3_point_to_index(double lon_deg, double lat_deg, int res, int jdk);
void orc_h3_points_to_cells(const double* lon, const double* lat, int64_t n, int res, int jdk,
                            uint64_t* out, int nthreads);
/* Diagnostics: hex2d coordinates and face that geoToH3 computes. */
void orc_h3_geo_to_hex2d(double lat_rad, double lon_rad, int res, int* face, double* x, double* y);

/* BNGIndexSystem.pointToIndex; returns 0 and sets *err=1 on NaN input. */
int64_t orc_bng_point_to_index(double e, double n, int res, int* err);
void orc_bng_points_to_cells(const double* e, const double* n, int64_t cnt, int res,
                             int64_t* out, int nthreads);

/* JTS-semantics point location against a parsed chip.  Returns 0 EXTERIOR,
 * 1 BOUNDARY, 2 INTERIOR (JTS Location codes differ; this is internal). */
int orc_wkb_contains(const uint8_t* wkb, int64_t len, double px, double py, int* err);

/* The join.  Chips are the ChipType rows: cell id, polygon id, is_core, WKB blob
 * (offsets[i]..offsets[i+1]).  index_system 0 = H3, 1 = BNG.  Produces pairs
 * sorted by (point index, polygon id); returns the pair count, or -1 on error.
 * If out arrays are NULL only counts. */
int64_t orc_pip_join(int index_system, int res, int jdk,
                     const double* x, const double* y, int64_t n,
                     int64_t n_chips, const int64_t* chip_cell, const int32_t* chip_poly,
                     const uint8_t* chip_core, const int64_t* wkb_off, const uint8_t* wkb,
                     int64_t* out_point, int32_t* out_poly, int64_t capacity, int nthreads);

#ifdef __cplusplus
}
#endif
#endif

/* H3 kRing / hexRing (H3IndexSystem.scala:182-205 -> H3-Java 3.7.0 -> H3 C v3.7 algos.c) */
uint64_t orc_h3_neighbor_rotations(uint64_t origin, int dir, int* rotations);
int64_t orc_h3_max_kring_size(int k);
int orc_h3_kring_raw(uint64_t origin, int k, uint64_t* out);
int orc_h3_hex_ring(uint64_t origin, int k, uint64_t* out);
