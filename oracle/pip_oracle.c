/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * `st_contains(chip.wkb, point)` as the reference evaluates it:
 *   ST_Contains.scala:34-42 -> MosaicGeometryIOCodeGenJTS.fromWKB (:23-29, a fresh
 *   WKBReader per row) -> MosaicGeometryJTS.contains (MosaicGeometryJTS.scala:197)
 *   -> JTS 1.20 Geometry.contains(Point).
 * JTS is not part of the reference tree; its published semantics are restated:
 *   Geometry.contains: empty -> false; envelope must contain the point (inclusive);
 *     Polygon.isRectangle() -> RectangleContains (strictly inside);
 *     otherwise relate(...).isContains() == PointLocator.locate(p) == INTERIOR.
 *   PointLocator (Mod-2 boundary rule): Polygon -> shell then holes, each ring
 *     skipped when its envelope misses p; multi/collection -> isIn / numBoundaries.
 *   RayCrossingCounter.locatePointInRing (p1 = ring[i], p2 = ring[i-1]) with
 *     CGAlgorithmsDD.orientationIndex (1e-15 filter, then DoubleDouble).
 * Compiled with -ffp-contract=off so every product and sum rounds exactly as on
 * the JVM (no FMA).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#include "oracle.h"

/* ---------------- CGAlgorithmsDD.orientationIndex ---------------- */

typedef struct { double hi, lo; } DD;

static DD dd_add(DD a, double yhi, double ylo) {
    double H, h, T, t, S, s, e, f;
    S = a.hi + yhi;
    T = a.lo + ylo;
    e = S - a.hi;
    f = T - a.lo;
    s = S - e;
    t = T - f;
    s = (yhi - e) + (a.hi - s);
    t = (ylo - f) + (a.lo - t);
    e = s + T;
    H = S + e;
    h = e + (S - H);
    e = t + h;
    DD z;
    z.hi = H + e;
    z.lo = e + (H - z.hi);
    return z;
}

static DD dd_mul(DD a, double yhi, double ylo) {
    const double SPLIT = 134217729.0;
    double hx, tx, hy, ty, C, c;
    C = SPLIT * a.hi;
    hx = C - a.hi;
    c = SPLIT * yhi;
    hx = C - hx;
    tx = a.hi - hx;
    hy = c - yhi;
    C = a.hi * yhi;
    hy = c - hy;
    ty = yhi - hy;
    c = ((((hx * hy - C) + hx * ty) + tx * hy) + tx * ty) + (a.hi * ylo + a.lo * yhi);
    DD z;
    z.hi = C + c;
    hx = C - z.hi;
    z.lo = c + hx;
    return z;
}

static int signum_d(double x) { return x > 0 ? 1 : (x < 0 ? -1 : 0); }

static int orientation_filter(double pax, double pay, double pbx, double pby, double pcx, double pcy) {
    double detsum;
    double detleft = (pax - pcx) * (pby - pcy);
    double detright = (pay - pcy) * (pbx - pcx);
    double det = detleft - detright;
    if (detleft > 0.0) {
        if (detright <= 0.0) return signum_d(det);
        detsum = detleft + detright;
    } else if (detleft < 0.0) {
        if (detright >= 0.0) return signum_d(det);
        detsum = -detleft - detright;
    } else {
        return signum_d(det);
    }
    double errbound = 1e-15 * detsum;
    if ((det >= errbound) || (-det >= errbound)) return signum_d(det);
    return 2;
}

static int orientation_index(double p1x, double p1y, double p2x, double p2y, double qx, double qy) {
    int index = orientation_filter(p1x, p1y, p2x, p2y, qx, qy);
    if (index <= 1) return index;
    DD dx1 = dd_add((DD){p2x, 0.0}, -p1x, 0.0);
    DD dy1 = dd_add((DD){p2y, 0.0}, -p1y, 0.0);
    DD dx2 = dd_add((DD){qx, 0.0}, -p2x, 0.0);
    DD dy2 = dd_add((DD){qy, 0.0}, -p2y, 0.0);
    DD a = dd_mul(dx1, dy2.hi, dy2.lo);
    DD b = dd_mul(dy1, dx2.hi, dx2.lo);
    DD d = dd_add(a, -b.hi, -b.lo);
    if (d.hi > 0) return 1;
    if (d.hi < 0) return -1;
    if (d.lo > 0) return 1;
    if (d.lo < 0) return -1;
    return 0;
}

/* ---------------- WKB reader ---------------- */

enum { LOC_EXTERIOR = 0, LOC_BOUNDARY = 1, LOC_INTERIOR = 2 };

typedef struct {
    const uint8_t* p;
    const uint8_t* end;
    int err;
} rd;

static uint32_t rd_u32(rd* r, int le) {
    if (r->end - r->p < 4) { r->err = 1; return 0; }
    uint32_t v = le ? (uint32_t)r->p[0] | ((uint32_t)r->p[1] << 8) | ((uint32_t)r->p[2] << 16) | ((uint32_t)r->p[3] << 24)
                    : (uint32_t)r->p[3] | ((uint32_t)r->p[2] << 8) | ((uint32_t)r->p[1] << 16) | ((uint32_t)r->p[0] << 24);
    r->p += 4;
    return v;
}
static double rd_f64(rd* r, int le) {
    if (r->end - r->p < 8) { r->err = 1; return 0; }
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v |= (uint64_t)r->p[le ? i : 7 - i] << (8 * i);
    r->p += 8;
    double d;
    memcpy(&d, &v, 8);
    return d;
}

/* accumulated PointLocator state over a geometry tree */
typedef struct {
    int isIn;
    int numBoundaries;
} locstate;

/* locate p in one ring read from the stream (JTS RayCrossingCounter); consumes the ring */
static int ring_locate(rd* r, int le, int dims, double px, double py, int* npts_out) {
    uint32_t n = rd_u32(r, le);
    if (r->err) return LOC_EXTERIOR;
    if ((uint64_t)(r->end - r->p) < (uint64_t)n * 8 * dims) { r->err = 1; return LOC_EXTERIOR; }
    *npts_out = (int)n;
    const uint8_t* base = r->p;
    r->p += (size_t)n * 8 * dims;
    if (n == 0) return LOC_EXTERIOR;
    rd v = {base, r->p, 0};
    /* ring envelope check (Envelope.intersects(p), inclusive) */
    double minx = INFINITY, maxx = -INFINITY, miny = INFINITY, maxy = -INFINITY;
    for (uint32_t i = 0; i < n; i++) {
        double x = rd_f64(&v, le), y = rd_f64(&v, le);
        for (int d = 2; d < dims; d++) rd_f64(&v, le);
        if (x < minx) minx = x;
        if (x > maxx) maxx = x;
        if (y < miny) miny = y;
        if (y > maxy) maxy = y;
    }
    if (!(px >= minx && px <= maxx && py >= miny && py <= maxy)) return LOC_EXTERIOR;
    v.p = base;
    double prevx = rd_f64(&v, le), prevy = rd_f64(&v, le);
    for (int d = 2; d < dims; d++) rd_f64(&v, le);
    int crossings = 0;
    for (uint32_t i = 1; i < n; i++) {
        double x = rd_f64(&v, le), y = rd_f64(&v, le);
        for (int d = 2; d < dims; d++) rd_f64(&v, le);
        /* countSegment(p1 = ring[i], p2 = ring[i-1]) */
        double p1x = x, p1y = y, p2x = prevx, p2y = prevy;
        prevx = x;
        prevy = y;
        if (p1x < px && p2x < px) continue;
        if (px == p2x && py == p2y) return LOC_BOUNDARY;
        if (p1y == py && p2y == py) {
            double mn = p1x, mx = p2x;
            if (mn > mx) { mn = p2x; mx = p1x; }
            if (px >= mn && px <= mx) return LOC_BOUNDARY;
            continue;
        }
        if (((p1y > py) && (p2y <= py)) || ((p2y > py) && (p1y <= py))) {
            int orient = orientation_index(p1x, p1y, p2x, p2y, px, py);
            if (orient == 0) return LOC_BOUNDARY;
            if (p2y < p1y) orient = -orient;
            if (orient == 1) crossings++;
        }
    }
    return (crossings % 2) == 1 ? LOC_INTERIOR : LOC_EXTERIOR;
}

static int header(rd* r, int* le, uint32_t* type, int* dims) {
    if (r->end - r->p < 1) { r->err = 1; return 0; }
    uint8_t bo = *r->p++;
    if (bo > 1) { r->err = 1; return 0; }
    *le = bo == 1;
    uint32_t t = rd_u32(r, *le);
    int hasZ = (t & 0x80000000u) != 0, hasM = (t & 0x40000000u) != 0, hasSrid = (t & 0x20000000u) != 0;
    t &= 0x0fffffffu;
    uint32_t iso = t / 1000;
    t = t % 1000;
    if (iso == 1 || iso == 3) hasZ = 1;
    if (iso == 2 || iso == 3) hasM = 1;
    if (hasSrid) rd_u32(r, *le);
    *type = t;
    *dims = 2 + hasZ + hasM;
    return !r->err;
}

/* Polygon body after the header: shell then holes (PointLocator.locateInPolygon) */
static int polygon_locate(rd* r, int le, int dims, double px, double py) {
    uint32_t nrings = rd_u32(r, le);
    if (r->err) return LOC_EXTERIOR;
    int result = LOC_INTERIOR, decided = 0;
    if (nrings == 0) { result = LOC_EXTERIOR; decided = 1; }
    for (uint32_t k = 0; k < nrings; k++) {
        int np = 0;
        int loc = ring_locate(r, le, dims, px, py, &np);
        if (r->err) return LOC_EXTERIOR;
        if (decided) continue; /* keep consuming the stream */
        if (k == 0) {
            if (np == 0) { result = LOC_EXTERIOR; decided = 1; }
            else if (loc == LOC_EXTERIOR) { result = LOC_EXTERIOR; decided = 1; }
            else if (loc == LOC_BOUNDARY) { result = LOC_BOUNDARY; decided = 1; }
        } else {
            if (loc == LOC_INTERIOR) { result = LOC_EXTERIOR; decided = 1; }
            else if (loc == LOC_BOUNDARY) { result = LOC_BOUNDARY; decided = 1; }
        }
    }
    return result;
}

static void geom_locate(rd* r, double px, double py, locstate* st, int depth) {
    int le, dims;
    uint32_t type;
    if (depth > 32) { r->err = 1; return; }
    if (!header(r, &le, &type, &dims)) return;
    if (type == 3) {
        int loc = polygon_locate(r, le, dims, px, py);
        if (loc == LOC_INTERIOR) st->isIn = 1;
        if (loc == LOC_BOUNDARY) st->numBoundaries++;
    } else if (type == 6 || type == 7) {
        uint32_t n = rd_u32(r, le);
        for (uint32_t i = 0; i < n && !r->err; i++) geom_locate(r, px, py, st, depth + 1);
    } else {
        r->err = 2; /* non-areal chip member: unsupported */
    }
}

/* envelope / emptiness / rectangle information of a geometry, for Geometry.contains */
typedef struct {
    double minx, maxx, miny, maxy;
    int64_t npts;
    int top_type, nrings_top;
    int rect_ok;
} geominfo;

static void scan_info(rd* r, geominfo* gi, int depth) {
    int le, dims;
    uint32_t type;
    if (depth > 32) { r->err = 1; return; }
    if (!header(r, &le, &type, &dims)) return;
    if (depth == 0) gi->top_type = (int)type;
    if (type == 3) {
        uint32_t nr = rd_u32(r, le);
        if (depth == 0) gi->nrings_top = (int)nr;
        for (uint32_t k = 0; k < nr && !r->err; k++) {
            uint32_t n = rd_u32(r, le);
            if ((uint64_t)(r->end - r->p) < (uint64_t)n * 8 * dims) { r->err = 1; return; }
            for (uint32_t i = 0; i < n; i++) {
                double x = rd_f64(r, le), y = rd_f64(r, le);
                for (int d = 2; d < dims; d++) rd_f64(r, le);
                if (x < gi->minx) gi->minx = x;
                if (x > gi->maxx) gi->maxx = x;
                if (y < gi->miny) gi->miny = y;
                if (y > gi->maxy) gi->maxy = y;
                gi->npts++;
            }
        }
    } else if (type == 6 || type == 7) {
        uint32_t n = rd_u32(r, le);
        for (uint32_t i = 0; i < n && !r->err; i++) scan_info(r, gi, depth + 1);
    } else {
        r->err = 2;
    }
}

/* Polygon.isRectangle() on a top-level single-ring polygon */
static int is_rectangle(const uint8_t* wkb, int64_t len, const geominfo* gi) {
    if (gi->top_type != 3 || gi->nrings_top != 1) return 0;
    rd r = {wkb, wkb + len, 0};
    int le, dims;
    uint32_t type;
    header(&r, &le, &type, &dims);
    rd_u32(&r, le);
    uint32_t n = rd_u32(&r, le);
    if (r.err || n != 5) return 0;
    double xs[5], ys[5];
    for (int i = 0; i < 5; i++) {
        xs[i] = rd_f64(&r, le);
        ys[i] = rd_f64(&r, le);
        for (int d = 2; d < dims; d++) rd_f64(&r, le);
    }
    for (int i = 0; i < 5; i++) {
        if (!(xs[i] == gi->minx || xs[i] == gi->maxx)) return 0;
        if (!(ys[i] == gi->miny || ys[i] == gi->maxy)) return 0;
    }
    for (int i = 1; i <= 4; i++) {
        int xc = xs[i] != xs[i - 1], yc = ys[i] != ys[i - 1];
        if (xc == yc) return 0;
    }
    return 1;
}

int orc_wkb_contains(const uint8_t* wkb, int64_t len, double px, double py, int* err) {
    if (err) *err = 0;
    geominfo gi = {INFINITY, -INFINITY, INFINITY, -INFINITY, 0, -1, 0, 0};
    rd r = {wkb, wkb + len, 0};
    scan_info(&r, &gi, 0);
    if (r.err) { if (err) *err = r.err; return LOC_EXTERIOR; }
    if (gi.npts == 0) return LOC_EXTERIOR; /* empty geometry contains nothing */
    if (!(px >= gi.minx && px <= gi.maxx && py >= gi.miny && py <= gi.maxy)) return LOC_EXTERIOR;
    if (is_rectangle(wkb, len, &gi)) {
        if (px == gi.minx || px == gi.maxx || py == gi.miny || py == gi.maxy) return LOC_BOUNDARY;
        return LOC_INTERIOR;
    }
    locstate st = {0, 0};
    rd r2 = {wkb, wkb + len, 0};
    if (gi.top_type == 3) {
        int le, dims;
        uint32_t type;
        header(&r2, &le, &type, &dims);
        return polygon_locate(&r2, le, dims, px, py);
    }
    geom_locate(&r2, px, py, &st, 0);
    if (r2.err) { if (err) *err = r2.err; return LOC_EXTERIOR; }
    if (st.numBoundaries % 2 == 1) return LOC_BOUNDARY;
    if (st.numBoundaries > 0 || st.isIn) return LOC_INTERIOR;
    return LOC_EXTERIOR;
}

/* ---------------- the join ---------------- */

typedef struct {
    int64_t cell;
    int32_t poly;
    int64_t idx;
} chipkey;

static int chipkey_cmp(const void* a, const void* b) {
    const chipkey *x = (const chipkey*)a, *y = (const chipkey*)b;
    if (x->cell != y->cell) return x->cell < y->cell ? -1 : 1;
    if (x->poly != y->poly) return x->poly < y->poly ? -1 : 1;
    return x->idx < y->idx ? -1 : (x->idx > y->idx);
}

typedef struct {
    int index_system, res, jdk;
    const double *x, *y;
    int64_t begin, end;
    const chipkey* keys;
    int64_t n_chips;
    const uint8_t* core;
    const int64_t* off;
    const uint8_t* wkb;
    int64_t count, cap;
    int64_t* pt;
    int32_t* poly;
    int err;
} join_job;

static void* join_worker(void* p) {
    join_job* j = (join_job*)p;
    for (int64_t i = j->begin; i < j->end; i++) {
        int64_t cell;
        if (j->index_system == 0) {
            cell = (int64_t)orc_h3_point_to_index(j->x[i], j->y[i], j->res, j->jdk);
        } else {
            int e = 0;
            cell = orc_bng_point_to_index(j->x[i], j->y[i], j->res, &e);
            if (e) { j->err = 1; continue; }
        }
        /* lower bound on cell */
        int64_t lo = 0, hi = j->n_chips;
        while (lo < hi) {
            int64_t mid = (lo + hi) / 2;
            if (j->keys[mid].cell < cell) lo = mid + 1; else hi = mid;
        }
        for (int64_t c = lo; c < j->n_chips && j->keys[c].cell == cell; c++) {
            int64_t ci = j->keys[c].idx;
            int match = j->core[ci];
            if (!match) {
                int e = 0;
                int loc = orc_wkb_contains(j->wkb + j->off[ci], j->off[ci + 1] - j->off[ci], j->x[i], j->y[i], &e);
                if (e) j->err = 2;
                match = loc == LOC_INTERIOR;
            }
            if (match) {
                if (j->count >= j->cap) {
                    j->cap = j->cap ? j->cap * 2 : 1024;
                    j->pt = (int64_t*)realloc(j->pt, j->cap * sizeof(int64_t));
                    j->poly = (int32_t*)realloc(j->poly, j->cap * sizeof(int32_t));
                }
                j->pt[j->count] = i;
                j->poly[j->count] = j->keys[c].poly;
                j->count++;
            }
        }
    }
    return 0;
}

int64_t orc_pip_join(int index_system, int res, int jdk, const double* x, const double* y, int64_t n,
                     int64_t n_chips, const int64_t* chip_cell, const int32_t* chip_poly, const uint8_t* chip_core,
                     const int64_t* wkb_off, const uint8_t* wkb, int64_t* out_point, int32_t* out_poly,
                     int64_t capacity, int nthreads) {
    chipkey* keys = (chipkey*)malloc(sizeof(chipkey) * (n_chips > 0 ? n_chips : 1));
    for (int64_t c = 0; c < n_chips; c++) keys[c] = (chipkey){chip_cell[c], chip_poly[c], c};
    qsort(keys, n_chips, sizeof(chipkey), chipkey_cmp);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    join_job jobs[256];
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (join_job){index_system, res, jdk, x, y, n * t / nthreads, n * (t + 1) / nthreads, keys, n_chips,
                             chip_core, wkb_off, wkb, 0, 0, 0, 0, 0};
        pthread_create(&th[t], 0, join_worker, &jobs[t]);
    }
    int64_t total = 0;
    int err = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], 0);
        err |= jobs[t].err;
    }
    for (int t = 0; t < nthreads; t++) {
        if (out_point && out_poly) {
            for (int64_t k = 0; k < jobs[t].count && total + k < capacity; k++) {
                out_point[total + k] = jobs[t].pt[k];
                out_poly[total + k] = jobs[t].poly[k];
            }
        }
        total += jobs[t].count;
        free(jobs[t].pt);
        free(jobs[t].poly);
    }
    free(keys);
    return err ? -1 : total;
}
