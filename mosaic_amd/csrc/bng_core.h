// British National Grid point -> cell id.
//
// Replaces BNGIndexSystem.pointToIndex / getQuadrant / encode
//   /root/reference/src/main/scala/com/databricks/labs/mosaic/core/index/BNGIndexSystem.scala:284-334, 540-553
// Operation-for-operation with the Scala code: JVM d2i truncation of the
// coordinates, Int `/` and `%`, Double division + floor for bins and quadrant,
// and the Double sum of `encode` converted with d2l.  Pure IEEE arithmetic, so
// the device result is bit-identical to the JVM's.
#pragma once
#include <math.h>
#include <stdint.h>

#ifdef __HIPCC__
#define MGPU_HDB __host__ __device__ __forceinline__
#else
#define MGPU_HDB inline
#endif

namespace mgpu {
namespace bng {

MGPU_HDB int32_t d2i(double v) {
  if (v != v) return 0;
  if (v >= 2147483647.0) return 2147483647;
  if (v <= -2147483648.0) return (int32_t)(-2147483647 - 1);
  return (int32_t)v;
}
MGPU_HDB int64_t d2l(double v) {
  if (v != v) return 0;
  if (v >= 9223372036854775807.0) return (int64_t)0x7fffffffffffffffLL;
  if (v <= -9223372036854775808.0) return (int64_t)(-0x7fffffffffffffffLL - 1);
  return (int64_t)v;
}
// exact powers of ten 10^0 .. 10^17 (Math.pow(10, k) is exact for these)
MGPU_HDB double pow10i(int k) {
  double r = 1.0;
  for (int i = 0; i < k; i++) r *= 10.0;
  return r;
}

// returns false for NaN input (IllegalStateException in the reference)
MGPU_HDB bool point_to_cell(double eastings, double northings, int resolution, int64_t* out) {
  if (eastings != eastings || northings != northings) return false;
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
  double idPlaceholder = pow10i(5 + 2 * nPositions - 2);
  double eLetterShift = pow10i(3 + 2 * nPositions - 2);
  double nLetterShift = pow10i(1 + 2 * nPositions - 2);
  double eShift = pow10i(nPositions);
  double nShift = 10;
  double id;
  if (resolution == -1)
    id = (idPlaceholder + eLetter * eLetterShift) / 100 + quadrant;
  else
    id = idPlaceholder + eLetter * eLetterShift + nLetter * nLetterShift + eBin * eShift + nBin * nShift + quadrant;
  *out = d2l(id);
  return true;
}

}  // namespace bng
}  // namespace mgpu
