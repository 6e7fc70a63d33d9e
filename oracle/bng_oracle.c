/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Restatement of BNGIndexSystem.pointToIndex
 *   src/main/scala/com/databricks/labs/mosaic/core/index/BNGIndexSystem.scala:284-298
 * with getQuadrant (:316-334) and encode (:540-553).  The Scala arithmetic is kept
 * operation for operation: Int truncation (`toInt`, JVM d2i saturating), Int `/`
 * and `%` (truncating, sign of dividend), Double division/floor for the bins and
 * quadrant, and the Double sum of `encode` followed by `toLong` (d2l).
 */
#include <math.h>
#include <stdint.h>
#include <pthread.h>

#include "oracle.h"

/* JVM d2i: NaN -> 0, saturate to [INT_MIN, INT_MAX], otherwise truncate */
static int32_t d2i(double v) {
    if (v != v) return 0;
    if (v >= 2147483647.0) return 2147483647;
    if (v <= -2147483648.0) return (int32_t)-2147483648LL;
    return (int32_t)v;
}
/* JVM d2l */
static int64_t d2l(double v) {
    if (v != v) return 0;
    if (v >= 9223372036854775807.0) return INT64_MAX;
    if (v <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)v;
}

static const double POW10[] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10,
                               1e11, 1e12, 1e13, 1e14, 1e15, 1e16, 1e17};

static double pow10i(int k) { return k >= 0 ? POW10[k] : 1.0 / POW10[-k]; }

int64_t orc_bng_point_to_index(double eastings, double northings, int resolution, int* err) {
    if (err) *err = 0;
    if (eastings != eastings || northings != northings) { if (err) *err = 1; return 0; }
    int32_t eI = d2i(eastings), nI = d2i(northings);
    int32_t eLetter = d2i(floor((double)(eI / 100000)));
    int32_t nLetter = d2i(floor((double)(nI / 100000)));
    int ar = resolution < 0 ? -resolution : resolution;
    double divisor = resolution < 0 ? pow10i(6 - ar + 1) : pow10i(6 - resolution);
    int quadrant = 0;
    if (resolution < -1) {
        double eQ = (double)eI / divisor, nQ = (double)nI / divisor;
        double eD = eQ - floor(eQ), nD = nQ - floor(nQ);
        if (eD < 0.5 && nD < 0.5) quadrant = 1;
        else if (eD < 0.5) quadrant = 2;
        else if (nD < 0.5) quadrant = 4;
        else quadrant = 3;
    }
    int nPositions = resolution >= -1 ? ar : ar - 1;
    int32_t eBin = d2i(floor((double)(eI % 100000) / divisor));
    int32_t nBin = d2i(floor((double)(nI % 100000) / divisor));
    /* encode */
    double idPlaceholder = pow10i(5 + 2 * nPositions - 2);
    double eLetterShift = pow10i(3 + 2 * nPositions - 2);
    double nLetterShift = pow10i(1 + 2 * nPositions - 2);
    double eShift = pow10i(nPositions);
    double nShift = 10;
    double id;
    if (resolution == -1)
        id = (idPlaceholder + eLetter * eLetterShift) / 100 + quadrant;
    else
        id = idPlaceholder + eLetter * eLetterShift + nLetter * nLetterShift + eBin * eShift + nBin * nShift +
             quadrant;
    return d2l(id);
}

typedef struct {
    const double *e, *n;
    int64_t begin, end;
    int res;
    int64_t* out;
} bng_job;

static void* bng_worker(void* p) {
    bng_job* j = (bng_job*)p;
    for (int64_t i = j->begin; i < j->end; i++) j->out[i] = orc_bng_point_to_index(j->e[i], j->n[i], j->res, 0);
    return 0;
}

void orc_bng_points_to_cells(const double* e, const double* n, int64_t cnt, int res, int64_t* out, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    bng_job jobs[256];
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (bng_job){e, n, cnt * t / nthreads, cnt * (t + 1) / nthreads, res, out};
        pthread_create(&th[t], 0, bng_worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], 0);
}
