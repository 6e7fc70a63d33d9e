/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Restatement of H3 v3.7.x geoToH3 (the arithmetic behind H3-Java 3.7.0, the
 * un-vendored dependency of the reference: pom.xml:91-97).  Reference call site:
 *   H3IndexSystem.pointToIndex(lon, lat, res) = h3.geoToH3(lat, lon, res)
 *     src/main/scala/com/databricks/labs/mosaic/core/index/H3IndexSystem.scala:168-170
 *
 * Faithfulness notes (bit-exactness with the JVM path):
 *  - H3's constants.h declares M_2PI, M_SQRT7, M_SQRT3_2, M_AP7_ROT_RADS and
 *    EPSILON as long-double literals, so on x86-64 the expressions that use them
 *    are evaluated in 80-bit x87 precision and rounded to double on assignment.
 *    This file keeps exactly those literals and expression shapes; compile with
 *    gcc on x86-64 and -ffp-contract=off (no FMA) like the H3 native library.
 *  - sin/cos/tan/acos/atan2 are glibc libm, as for the JNI library on the
 *    reference's Ubuntu 22.04 / glibc 2.35 toolchain.
 *  - Degree conversion is JDK Math.toRadians: JDK 8 computes deg / 180.0 * PI.
 */
#include <math.h>
#include <quadmath.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <pthread.h>

#include "oracle.h"
#include "h3_tables.inc"

#define M_2PI_L 6.28318530717958647692528676655900576839433L
#define EPSILON_L 0.0000000000000001L
#define M_SQRT3_2_L 0.8660254037844386467637231707529361834714L
#define M_SIN60_L M_SQRT3_2_L
#define M_AP7_ROT_RADS_L 0.333473172251832115336090755351601070065900389L
#define RES0_U_GNOMONIC 0.38196601125010500003
#define M_SQRT7_L 2.6457513110645905905016157536392604257102L

#define MAX_H3_RES 15
#define H3_INIT 35184372088831ULL
#define MAX_FACE_COORD 2

typedef struct { int i, j, k; } CoordIJK;

static double posAngleRads(double rads) {
    double tmp = ((rads < 0.0L) ? rads + M_2PI_L : rads);
    if (rads >= M_2PI_L) tmp -= M_2PI_L;
    return tmp;
}

static double square(double x) { return x * x; }

static void ijkNormalize(CoordIJK* c) {
    if (c->i < 0) { c->j -= c->i; c->k -= c->i; c->i = 0; }
    if (c->j < 0) { c->i -= c->j; c->k -= c->j; c->j = 0; }
    if (c->k < 0) { c->i -= c->k; c->j -= c->k; c->k = 0; }
    int min = c->i;
    if (c->j < min) min = c->j;
    if (c->k < min) min = c->k;
    if (min > 0) { c->i -= min; c->j -= min; c->k -= min; }
}

static void hex2dToCoordIJK(double vx, double vy, CoordIJK* h) {
    double a1, a2, x1, x2, r1, r2;
    int m1, m2;
    h->k = 0;
    a1 = fabsl(vx);
    a2 = fabsl(vy);
    x2 = a2 / M_SIN60_L;
    x1 = a1 + x2 / 2.0;
    m1 = x1;
    m2 = x2;
    r1 = x1 - m1;
    r2 = x2 - m2;
    if (r1 < 0.5) {
        if (r1 < 1.0 / 3.0) {
            if (r2 < (1.0 + r1) / 2.0) { h->i = m1; h->j = m2; }
            else { h->i = m1; h->j = m2 + 1; }
        } else {
            if (r2 < (1.0 - r1)) h->j = m2; else h->j = m2 + 1;
            if ((1.0 - r1) <= r2 && r2 < (2.0 * r1)) h->i = m1 + 1; else h->i = m1;
        }
    } else {
        if (r1 < 2.0 / 3.0) {
            if (r2 < (1.0 - r1)) h->j = m2; else h->j = m2 + 1;
            if ((2.0 * r1 - 1.0) < r2 && r2 < (1.0 - r1)) h->i = m1; else h->i = m1 + 1;
        } else {
            if (r2 < (r1 / 2.0)) { h->i = m1 + 1; h->j = m2; }
            else { h->i = m1 + 1; h->j = m2 + 1; }
        }
    }
    if (vx < 0.0) {
        if ((h->j % 2) == 0) {
            long long axisi = h->j / 2;
            long long diff = h->i - axisi;
            h->i = h->i - 2.0 * diff;
        } else {
            long long axisi = (h->j + 1) / 2;
            long long diff = h->i - axisi;
            h->i = h->i - (2.0 * diff + 1);
        }
    }
    if (vy < 0.0) {
        h->i = h->i - (2 * h->j + 1) / 2;
        h->j = -1 * h->j;
    }
    ijkNormalize(h);
}

/* The route's libm: glibc (the reference's, default) or correctly rounded (quadmath's
 * 113-bit functions rounded once to double) -- the independent restatement the device's
 * correctly rounded route (mosaic_amd/csrc/h3_exact.h) is checked against bit for bit;
 * the difference between the two modes is exactly glibc's misrounding. */
static int g_cr_libm = 0;
void orc_h3_set_libm(int correctly_rounded) { g_cr_libm = correctly_rounded; }
static double L_sin(double x) { return g_cr_libm ? (double)sinq((__float128)x) : sin(x); }
static double L_cos(double x) { return g_cr_libm ? (double)cosq((__float128)x) : cos(x); }
static double L_tan(double x) { return g_cr_libm ? (double)tanq((__float128)x) : tan(x); }
static double L_acos(double x) { return g_cr_libm ? (double)acosq((__float128)x) : acos(x); }
static double L_atan2(double y, double x) {
    return g_cr_libm ? (double)atan2q((__float128)y, (__float128)x) : atan2(y, x);
}

static double geoAzimuthRads(double lat1, double lon1, double lat2, double lon2) {
    return L_atan2(L_cos(lat2) * L_sin(lon2 - lon1),
                   L_cos(lat1) * L_sin(lat2) - L_sin(lat1) * L_cos(lat2) * L_cos(lon2 - lon1));
}

static void geoToHex2d(double lat, double lon, int res, int* face, double* vx, double* vy) {
    /* _geoToVec3d */
    double r0 = L_cos(lat);
    double z = L_sin(lat);
    double x = L_cos(lon) * r0;
    double y = L_sin(lon) * r0;
    /* _geoToClosestFace */
    *face = 0;
    double sqd = 5.0;
    for (int f = 0; f < H3T_NUM_FACES; ++f) {
        double sqdT = square(H3T_FACE_CENTER_POINT[f][0] - x) + square(H3T_FACE_CENTER_POINT[f][1] - y) +
                      square(H3T_FACE_CENTER_POINT[f][2] - z);
        if (sqdT < sqd) { *face = f; sqd = sqdT; }
    }
    double r = L_acos(1 - sqd / 2);
    if (r < EPSILON_L) { *vx = *vy = 0.0L; return; }
    double theta = posAngleRads(H3T_FACE_AXES_AZ_CII[*face][0] -
                                posAngleRads(geoAzimuthRads(H3T_FACE_CENTER_GEO[*face][0],
                                                            H3T_FACE_CENTER_GEO[*face][1], lat, lon)));
    if (res % 2) theta = posAngleRads(theta - M_AP7_ROT_RADS_L);
    r = L_tan(r);
    r /= RES0_U_GNOMONIC;
    for (int i = 0; i < res; i++) r *= M_SQRT7_L;
    *vx = r * L_cos(theta);
    *vy = r * L_sin(theta);
}

/* nearest integer of n / 7 (lround((n) / 7.0) in H3; never a tie) */
static int lround7(int n) { return (int)lround(n / 7.0); }

static void upAp7(CoordIJK* ijk) {
    int i = ijk->i - ijk->k, j = ijk->j - ijk->k;
    ijk->i = lround7(3 * i - j);
    ijk->j = lround7(i + 2 * j);
    ijk->k = 0;
    ijkNormalize(ijk);
}
static void upAp7r(CoordIJK* ijk) {
    int i = ijk->i - ijk->k, j = ijk->j - ijk->k;
    ijk->i = lround7(2 * i + j);
    ijk->j = lround7(3 * j - i);
    ijk->k = 0;
    ijkNormalize(ijk);
}
static void downAp7(CoordIJK* c) {
    int i = c->i, j = c->j, k = c->k;
    /* iVec {3,0,1}, jVec {1,3,0}, kVec {0,1,3} */
    c->i = 3 * i + j;
    c->j = 3 * j + k;
    c->k = i + 3 * k;
    ijkNormalize(c);
}
static void downAp7r(CoordIJK* c) {
    int i = c->i, j = c->j, k = c->k;
    /* iVec {3,1,0}, jVec {0,3,1}, kVec {1,0,3} */
    c->i = 3 * i + k;
    c->j = i + 3 * j;
    c->k = j + 3 * k;
    ijkNormalize(c);
}

static int unitIjkToDigit(CoordIJK c) {
    ijkNormalize(&c);
    if (c.i <= 1 && c.j <= 1 && c.k <= 1 && c.i >= 0 && c.j >= 0 && c.k >= 0)
        return c.i * 4 + c.j * 2 + c.k; /* UNIT_VECS[d] has bits (i j k) */
    return 7;
}

static int rotate60ccw(int d) {
    switch (d) { case 1: return 5; case 5: return 4; case 4: return 6; case 6: return 2; case 2: return 3; case 3: return 1; default: return d; }
}
static int rotate60cw(int d) {
    switch (d) { case 1: return 3; case 3: return 2; case 2: return 6; case 6: return 4; case 4: return 5; case 5: return 1; default: return d; }
}

#define GET_DIGIT(h, r) ((int)(((h) >> ((MAX_H3_RES - (r)) * 3)) & 7))
#define SET_DIGIT(h, r, d) ((h) = ((h) & ~(7ULL << ((MAX_H3_RES - (r)) * 3))) | ((uint64_t)(d) << ((MAX_H3_RES - (r)) * 3)))

static int leadingNonZeroDigit(uint64_t h, int res) {
    for (int r = 1; r <= res; r++) if (GET_DIGIT(h, r)) return GET_DIGIT(h, r);
    return 0;
}
static uint64_t h3Rotate60ccw(uint64_t h, int res) {
    for (int r = 1; r <= res; r++) SET_DIGIT(h, r, rotate60ccw(GET_DIGIT(h, r)));
    return h;
}
static uint64_t h3Rotate60cw(uint64_t h, int res) {
    for (int r = 1; r <= res; r++) SET_DIGIT(h, r, rotate60cw(GET_DIGIT(h, r)));
    return h;
}
static uint64_t h3RotatePent60ccw(uint64_t h, int res) {
    int found = 0;
    for (int r = 1; r <= res; r++) {
        SET_DIGIT(h, r, rotate60ccw(GET_DIGIT(h, r)));
        if (!found && GET_DIGIT(h, r) != 0) {
            found = 1;
            if (leadingNonZeroDigit(h, res) == 1) h = h3Rotate60ccw(h, res);
        }
    }
    return h;
}

static uint64_t faceIjkToH3(int face, CoordIJK ijk, int res) {
    uint64_t h = H3_INIT;
    h = (h & ~(15ULL << 59)) | (1ULL << 59);
    h = (h & ~(15ULL << 52)) | ((uint64_t)res << 52);
    if (res == 0) {
        if (ijk.i > MAX_FACE_COORD || ijk.j > MAX_FACE_COORD || ijk.k > MAX_FACE_COORD) return 0;
        int bc = H3T_FACE_IJK_BASE_CELLS[face][ijk.i][ijk.j][ijk.k] & 0xff;
        return (h & ~(127ULL << 45)) | ((uint64_t)bc << 45);
    }
    for (int r = res - 1; r >= 0; r--) {
        CoordIJK last = ijk, center;
        if ((r + 1) % 2) { upAp7(&ijk); center = ijk; downAp7(&center); }
        else { upAp7r(&ijk); center = ijk; downAp7r(&center); }
        CoordIJK diff = {last.i - center.i, last.j - center.j, last.k - center.k};
        ijkNormalize(&diff);
        SET_DIGIT(h, r + 1, unitIjkToDigit(diff));
    }
    if (ijk.i > MAX_FACE_COORD || ijk.j > MAX_FACE_COORD || ijk.k > MAX_FACE_COORD) return 0;
    unsigned short e = H3T_FACE_IJK_BASE_CELLS[face][ijk.i][ijk.j][ijk.k];
    int bc = e & 0xff, numRots = e >> 8;
    h = (h & ~(127ULL << 45)) | ((uint64_t)bc << 45);
    if (H3T_BASE_CELL_DATA[bc][4]) {
        if (leadingNonZeroDigit(h, res) == 1) {
            if (H3T_BASE_CELL_DATA[bc][5] == face || H3T_BASE_CELL_DATA[bc][6] == face)
                h = h3Rotate60cw(h, res);
            else
                h = h3Rotate60ccw(h, res);
        }
        for (int i = 0; i < numRots; i++) h = h3RotatePent60ccw(h, res);
    } else {
        for (int i = 0; i < numRots; i++) h = h3Rotate60ccw(h, res);
    }
    return h;
}

uint64_t orc_h3_geo_to_h3(double lat, double lon, int res) {
    if (res < 0 || res > MAX_H3_RES) return 0;
    if (!isfinite(lat) || !isfinite(lon)) return 0;
    int face;
    double vx, vy;
    geoToHex2d(lat, lon, res, &face, &vx, &vy);
    CoordIJK ijk;
    hex2dToCoordIJK(vx, vy, &ijk);
    return faceIjkToH3(face, ijk, res);
}

void orc_h3_geo_to_hex2d(double lat, double lon, int res, int* face, double* x, double* y) {
    geoToHex2d(lat, lon, res, face, x, y);
}

static double to_radians(double deg, int jdk) {
    /* java.lang.Math.toRadians: JDK 8 `angdeg / 180.0 * PI`; JDK 9+
     * `angdeg * DEGREES_TO_RADIANS` with DEGREES_TO_RADIANS = 0.017453292519943295 */
    if (jdk >= 9) return deg * 0.017453292519943295;
    return deg / 180.0 * 3.14159265358979323846;
}

uint64_t orc_h3_point_to_index(double lon_deg, double lat_deg, int res, int jdk) {
    return orc_h3_geo_to_h3(to_radians(lat_deg, jdk), to_radians(lon_deg, jdk), res);
}

typedef struct {
    const double *lon, *lat;
    int64_t begin, end;
    int res, jdk;
    uint64_t* out;
} h3_job;

static void* h3_worker(void* p) {
    h3_job* j = (h3_job*)p;
    for (int64_t i = j->begin; i < j->end; i++)
        j->out[i] = orc_h3_point_to_index(j->lon[i], j->lat[i], j->res, j->jdk);
    return 0;
}

void orc_h3_points_to_cells(const double* lon, const double* lat, int64_t n, int res, int jdk,
                            uint64_t* out, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    h3_job jobs[256];
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (h3_job){lon, lat, n * t / nthreads, n * (t + 1) / nthreads, res, jdk, out};
        pthread_create(&th[t], 0, h3_worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], 0);
}

/* ------------------------------------------------------------------ kRing / hexRing
 * H3IndexSystem.kRing / kLoop (H3IndexSystem.scala:182-205) call H3-Java 3.7.0
 * kRing(h, k) = nonzero entries, in array order, of H3 C kRing's maxKringSize(k)
 * array, and hexRing(h, k), which throws PentagonEncounteredException when the C call
 * reports failure.  Restated from H3 v3.7 algos.c: h3NeighborRotations,
 * hexRangeDistances (spiral; fails on pentagons), the _kRingInternal fallback (the
 * output array is an open-addressing hash set keyed by h % maxIdx), hexRing.
 * Tables: h3_neighbors.inc (tools/gen_h3_neighbors.py). */
#include "h3_neighbors.inc"

#define H3_RES(h) ((int)(((h) >> 52) & 15))
#define H3_BASE(h) ((int)(((h) >> 45) & 127))
#define H3_SET_BASE(h, b) ((h) = ((h) & ~(127ULL << 45)) | ((uint64_t)(b) << 45))

static const int DIRECTIONS[6] = {2, 3, 1, 5, 4, 6}; /* J, JK, K, IK, I, IJ */
#define NEXT_RING_DIRECTION 4                      /* I */

static int isBaseCellPentagon(int b) { return H3T_BASE_CELL_DATA[b][4]; }
static int isBaseCellPolarPentagon(int b) { return b == 4 || b == 117; }
static int baseCellIsCwOffset(int b, int face) {
    return H3T_BASE_CELL_DATA[b][5] == face || H3T_BASE_CELL_DATA[b][6] == face;
}
static int isResClassIII(int r) { return r % 2; }

static int h3IsPentagon(uint64_t h) {
    return isBaseCellPentagon(H3_BASE(h)) && leadingNonZeroDigit(h, H3_RES(h)) == 0;
}

uint64_t orc_h3_neighbor_rotations(uint64_t origin, int dir, int* rotations) {
    uint64_t out = origin;
    const int res = H3_RES(out);
    for (int i = 0; i < *rotations; i++) dir = rotate60ccw(dir);
    int newRotations = 0;
    const int oldBaseCell = H3_BASE(out);
    const int oldLeadingDigit = leadingNonZeroDigit(out, res);
    int r = res - 1;
    for (;;) {
        if (r == -1) {
            H3_SET_BASE(out, H3T_BASE_CELL_NEIGHBORS[oldBaseCell][dir]);
            newRotations = H3T_BASE_CELL_NEIGHBOR_ROTS[oldBaseCell][dir];
            if (H3_BASE(out) == H3T_INVALID_BASE_CELL) {
                /* the deleted K vertex at the base-cell level: this edge borders a
                   different neighbour */
                H3_SET_BASE(out, H3T_BASE_CELL_NEIGHBORS[oldBaseCell][5]);
                newRotations = H3T_BASE_CELL_NEIGHBOR_ROTS[oldBaseCell][5];
                out = h3Rotate60ccw(out, res);
                *rotations = *rotations + 1;
            }
            break;
        } else {
            const int oldDigit = GET_DIGIT(out, r + 1);
            int nextDir;
            if (isResClassIII(r + 1)) {
                SET_DIGIT(out, r + 1, H3T_NEW_DIGIT_II[oldDigit][dir]);
                nextDir = H3T_NEW_ADJUSTMENT_II[oldDigit][dir];
            } else {
                SET_DIGIT(out, r + 1, H3T_NEW_DIGIT_III[oldDigit][dir]);
                nextDir = H3T_NEW_ADJUSTMENT_III[oldDigit][dir];
            }
            if (nextDir != 0) {
                dir = nextDir;
                r--;
            } else {
                break;
            }
        }
    }
    const int newBaseCell = H3_BASE(out);
    if (isBaseCellPentagon(newBaseCell)) {
        int alreadyAdjustedKSubsequence = 0;
        if (leadingNonZeroDigit(out, res) == 1) {
            if (oldBaseCell != newBaseCell) {
                /* traversed into the deleted K subsequence of a pentagon base cell */
                if (baseCellIsCwOffset(newBaseCell, H3T_BASE_CELL_DATA[oldBaseCell][0]))
                    out = h3Rotate60cw(out, res);
                else
                    out = h3Rotate60ccw(out, res);
                alreadyAdjustedKSubsequence = 1;
            } else {
                /* into the deleted K subsequence from within the same pentagon */
                if (oldLeadingDigit == 0) {
                    return 0; /* undefined: the K direction is deleted from here */
                } else if (oldLeadingDigit == 3) {
                    out = h3Rotate60ccw(out, res);
                    *rotations = *rotations + 1;
                } else if (oldLeadingDigit == 5) {
                    out = h3Rotate60cw(out, res);
                    *rotations = *rotations + 5;
                } else {
                    return 0;
                }
            }
        }
        for (int i = 0; i < newRotations; i++) out = h3RotatePent60ccw(out, res);
        if (oldBaseCell != newBaseCell) {
            if (isBaseCellPolarPentagon(newBaseCell)) {
                if (oldBaseCell != 118 && oldBaseCell != 8 && leadingNonZeroDigit(out, res) != 3)
                    *rotations = *rotations + 1;
            } else if (leadingNonZeroDigit(out, res) == 5 && !alreadyAdjustedKSubsequence) {
                *rotations = *rotations + 1;
            }
        }
    } else {
        for (int i = 0; i < newRotations; i++) out = h3Rotate60ccw(out, res);
    }
    *rotations = (*rotations + newRotations) % 6;
    return out;
}

int64_t orc_h3_max_kring_size(int k) { return 3 * (int64_t)k * (k + 1) + 1; }

/* hexRangeDistances: 0 = success, 1 = pentagon encountered, 2 = pentagon distortion */
static int hexRange(uint64_t origin, int k, uint64_t* out) {
    int64_t idx = 0;
    int currentK = 0, direction = 0, i = 0, rotations = 0;
    out[idx++] = origin;
    if (h3IsPentagon(origin)) return 1;
    while (currentK < k) {
        if (direction == 0 && i == 0) {
            origin = orc_h3_neighbor_rotations(origin, NEXT_RING_DIRECTION, &rotations);
            if (origin == 0) return 2;
            if (h3IsPentagon(origin)) return 1;
        }
        origin = orc_h3_neighbor_rotations(origin, DIRECTIONS[direction], &rotations);
        if (origin == 0) return 2;
        out[idx++] = origin;
        i++;
        if (i == currentK + 1) {
            i = 0;
            direction++;
            if (direction == 6) {
                direction = 0;
                currentK++;
            }
        }
        if (h3IsPentagon(origin)) return 1;
    }
    return 0;
}

static void kRingInternal(uint64_t origin, int k, uint64_t* out, int* distances, int64_t maxIdx, int curK) {
    if (origin == 0) return;
    int64_t off = (int64_t)(origin % (uint64_t)maxIdx), probes = 0;
    while (out[off] != 0 && out[off] != origin) {
        off = (off + 1) % maxIdx;
        if (++probes >= maxIdx) return; /* full (H3 would spin): only reachable with bad tables */
    }
    if (out[off] == origin && distances[off] <= curK) return;
    out[off] = origin;
    distances[off] = curK;
    if (curK >= k) return;
    for (int i = 0; i < 6; i++) {
        int rotations = 0;
        kRingInternal(orc_h3_neighbor_rotations(origin, DIRECTIONS[i], &rotations), k, out, distances, maxIdx,
                      curK + 1);
    }
}

/* H3 C kRing into out[maxKringSize(k)] (zeros = empty slots); returns 1 when the
   hexRange spiral failed and the hash-set fallback produced the array */
int orc_h3_kring_raw(uint64_t origin, int k, uint64_t* out) {
    const int64_t maxIdx = orc_h3_max_kring_size(k);
    memset(out, 0, (size_t)maxIdx * sizeof(uint64_t));
    if (hexRange(origin, k, out) == 0) return 0;
    memset(out, 0, (size_t)maxIdx * sizeof(uint64_t));
    int* distances = (int*)calloc((size_t)maxIdx, sizeof(int));
    kRingInternal(origin, k, out, distances, maxIdx, 0);
    free(distances);
    return 1;
}

/* H3 C hexRing: 0 = success (6k entries, 1 for k = 0), 1 = pentagon / distortion */
int orc_h3_hex_ring(uint64_t origin, int k, uint64_t* out) {
    if (k == 0) {
        out[0] = origin;
        return 0;
    }
    int64_t idx = 0;
    int rotations = 0;
    if (h3IsPentagon(origin)) return 1;
    for (int ring = 0; ring < k; ring++) {
        origin = orc_h3_neighbor_rotations(origin, NEXT_RING_DIRECTION, &rotations);
        if (origin == 0) return 1;
        if (h3IsPentagon(origin)) return 1;
    }
    const uint64_t lastIndex = origin;
    out[idx++] = origin;
    for (int direction = 0; direction < 6; direction++) {
        for (int pos = 0; pos < k; pos++) {
            origin = orc_h3_neighbor_rotations(origin, DIRECTIONS[direction], &rotations);
            if (origin == 0) return 1;
            if (pos != k - 1 || direction != 5) {
                out[idx++] = origin;
                if (h3IsPentagon(origin)) return 1;
            }
        }
    }
    return lastIndex != origin;
}

/* ------------------------------------------------------------------ libm / x87 probe
 * The reference route's elementary operations as the native H3 library evaluates them
 * on x86-64 (glibc libm; long-double constants on the x87 unit), for
 * tests/test_h3_exact_host.py: out[i] = op(a[i], b[i]). */
void orc_h3_elementary(int fn, const double* a, const double* b, int64_t n, double* out) {
    for (int64_t i = 0; i < n; i++) {
        double x = a[i], y = b ? b[i] : 0.0, r;
        switch (fn) {
            case 0: r = sin(x); break;
            case 1: r = cos(x); break;
            case 2: r = tan(x); break;
            case 3: r = acos(x); break;
            case 4: r = atan2(x, y); break;
            case 5: r = x + M_2PI_L; break;
            case 6: r = x - M_2PI_L; break;
            case 7: r = x * M_SQRT7_L; break;
            case 8: r = x / M_SIN60_L; break;
            case 9: r = x - M_AP7_ROT_RADS_L; break;
            case 10: r = x / M_SQRT7_L; break;
            case 11: r = x + M_AP7_ROT_RADS_L; break;
            case 12: r = (x < EPSILON_L) ? 1.0 : 0.0; break;
            case 13: r = (x >= M_2PI_L) ? 1.0 : 0.0; break;
            case 20: r = (double)sinq((__float128)x); break;
            case 21: r = (double)cosq((__float128)x); break;
            case 22: r = (double)tanq((__float128)x); break;
            case 23: r = (double)acosq((__float128)x); break;
            case 24: r = (double)atan2q((__float128)x, (__float128)y); break;
            default: r = 0.0; break;
        }
        out[i] = r;
    }
}
