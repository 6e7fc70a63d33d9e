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
#define MGPU_UNROLL _Pragma("unroll")
#else
#define MGPU_HDB inline
#define MGPU_UNROLL
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

// BNGIndexSystem.format (BNGIndexSystem.scala:119-134) with indexDigits = Long.toString
// (:440-442): the decimal digits d of the id -> letters letterMap(d(3..4))(d(1..2)) (one
// letter for the 500 km ids of fewer than 6 digits), then the eastings and northings
// bins (the digits between position 5 and the last, split in halves), then the
// quadrant suffix of the last digit.  The string comes back packed little-endian in
// (lo, hi) (char k = byte k; at most 16 chars); returns the length, or -1 when the id
// has no string form (non-positive, or a lookup that throws in the reference: fewer
// than 4 digits, letter indices beyond the map, a quadrant digit above 4).
// Digit arithmetic in doubles: every id below 2^53 (all BNG ids) is exact, and so is
// floor(x / 10^k) of a correctly rounded division of two exact integers below 2^53.
// No per-digit loop and no indexed local arrays (which become register waterfalls on
// the GPU).  Shared by the host formatter and the device kernels.
MGPU_HDB void put_char(uint64_t* lo, uint64_t* hi, int pos, uint32_t c) {
  if (pos < 8) *lo |= (uint64_t)c << (8 * pos);
  else *hi |= (uint64_t)c << (8 * (pos - 8));
}

// the digit arithmetic of format_cell_packed, in T = double (exact below 2^53) or
// uint64_t (ids from 2^53: slower divisions, never a BNG id in practice)
template <class T>
MGPU_HDB T fl_div(T a, T b) { return a / b; }
template <>
MGPU_HDB double fl_div<double>(double a, double b) { return floor(a / b); }

template <class T>
MGPU_HDB int format_digits(T x, int max_digits, uint64_t* lo, uint64_t* hi) {
  T p10[20];
  p10[0] = (T)1;
MGPU_UNROLL
  for (int k = 1; k < 20; k++) p10[k] = p10[k - 1] * (T)10;
  int n = 1;
MGPU_UNROLL
  for (int k = 1; k < 20; k++) n += (k < max_digits && x >= p10[k]) ? 1 : 0;
  if (n < 4) return -1;  // digits.slice(3, 5) empty: "".toInt throws
  // 10^j for a data-dependent j without indexing a local array (a register waterfall
  // on the GPU): an unrolled select
  auto pow_sel = [&](int j) {
    T r = (T)1;
MGPU_UNROLL
    for (int k = 0; k < 20; k++) r = (k == j) ? p10[k] : r;
    return r;
  };
  const T l5 = n == 4 ? x * (T)10 : fl_div(x, pow_sel(n - 5));  // digits 0..4 (n == 4: d0..d3 then 0)
  const T t = fl_div(l5, (T)100);
  const int col = (int)(t - fl_div(t, (T)100) * (T)100);
  const int row = n == 4 ? (int)((l5 - t * (T)100) / (T)10) : (int)(l5 - t * (T)100);
  if (row >= 14 || col >= 8) return -1;  // letterMap lookup out of bounds
  // letterMap (BNGIndexSystem.scala:88-104): rows 0..13 south to north, columns 0..7
  // west to east; first letter from the 500 km square, second from the 100 km one
  const uint32_t first = (row < 5) ? (col < 5 ? 'S' : 'T') : (row < 10 ? (col < 5 ? 'N' : 'O') : (col < 5 ? 'H' : 'J'));
  const uint32_t second = (uint32_t)"VWXYZQRSTULMNOPFGHJKABCDE"[(row % 5) * 5 + (col % 5)];
  if (n < 6) {
    *lo = first;
    return 1;
  }
  const T x10 = fl_div(x, (T)10);
  const int q = (int)(x - x10 * (T)10);
  if (q > 4) return -1;  // quadrants(q) out of bounds
  const int clen = n - 6, k = clen / 2;  // digits.drop(5).dropRight(1), split in halves
  const T pc = pow_sel(clen), pk = pow_sel(k);
  const T coords = x10 - fl_div(x10, pc) * pc;
  const uint32_t E = (uint32_t)fl_div(coords, pow_sel(clen - k));
  const T nn = fl_div(coords, pow_sel(clen - 2 * k));
  const uint32_t Nb = (uint32_t)(nn - fl_div(nn, pk) * pk);
  *lo = first | (second << 8);
  // k <= 6: k digits of E then of N, most significant first
  uint32_t e = E, m = Nb;
MGPU_UNROLL
  for (int i = 5; i >= 0; i--) {
    if (i < k) {
      put_char(lo, hi, 2 + i, '0' + e % 10u);
      put_char(lo, hi, 2 + k + i, '0' + m % 10u);
      e /= 10u;
      m /= 10u;
    }
  }
  int len = 2 + 2 * k;
  if (q) {
    put_char(lo, hi, len, (q == 1 || q == 4) ? 'S' : 'N');
    put_char(lo, hi, len + 1, (q == 1 || q == 2) ? 'W' : 'E');
    len += 2;
  }
  return len;
}

MGPU_HDB int format_cell_packed(int64_t id, uint64_t* lo, uint64_t* hi) {
  *lo = *hi = 0;
  if (id <= 0) return -1;
  if (id < ((int64_t)1 << 53)) return format_digits<double>((double)id, 16, lo, hi);
  return format_digits<uint64_t>((uint64_t)id, 20, lo, hi);
}

// the same into chars (host formatter)
MGPU_HDB int format_cell(int64_t id, char* out) {
  uint64_t lo, hi;
  const int len = format_cell_packed(id, &lo, &hi);
  for (int i = 0; i < len; i++) out[i] = (char)((i < 8 ? lo >> (8 * i) : hi >> (8 * (i - 8))) & 0xFF);
  return len;
}

// BNGIndexSystem.getEdgeSize(resolution) (BNGIndexSystem.scala:163-170, sizeMap :64-79)
MGPU_HDB int32_t edge_of_res(int r) {
  switch (r) {
    case 1: return 100000;
    case -1: return 500000;
    case 2: return 10000;
    case -2: return 50000;
    case 3: return 1000;
    case -3: return 5000;
    case 4: return 100;
    case -4: return 500;
    case 5: return 10;
    case -5: return 50;
    case 6: return 1;
    case -6: return 5;
    default: return 0;
  }
}

// getResolution(digits), getX / getY (the cell's south-west corner) and the letter
// indices isValid checks (BNGIndexSystem.scala:261-270, 451-506), for an id below 2^53
// (doubles exact).  Returns false where the Scala code would throw ("".toInt on an id
// of fewer than 4 digits) or for a non-positive id.  The Int arithmetic wraps as on
// the JVM.
MGPU_HDB bool cell_corner(int64_t id, int* res, int32_t* edge, int32_t* x, int32_t* y, int* x_letter, int* y_letter) {
  if (id <= 0 || id >= ((int64_t)1 << 53)) return false;
  const double v = (double)id;
  double p10[17];
  p10[0] = 1.0;
MGPU_UNROLL
  for (int k = 1; k < 17; k++) p10[k] = p10[k - 1] * 10.0;
  int n = 1;
MGPU_UNROLL
  for (int k = 1; k < 16; k++) n += v >= p10[k] ? 1 : 0;
  if (n < 4) return false;
  auto pw = [&](int j) {
    double r = 1.0;
MGPU_UNROLL
    for (int k = 0; k < 17; k++) r = (k == j) ? p10[k] : r;
    return r;
  };
  // digits [a, b) of the id as a number (b <= n)
  auto slice = [&](int a, int b) {
    const double hi = floor(v / pw(n - b));
    const double m = pw(b - a);
    return hi - floor(hi / m) * m;
  };
  const int q = (int)slice(n - 1, n);
  const int r = n < 6 ? -1 : (q > 0 ? -((n - 6) / 2 + 2) : (n - 6) / 2 + 1);
  const int32_t e = edge_of_res(r);
  if (!e) return false;
  const int k = (n - 6) / 2;  // JVM Int division (n = 4: -1, the bin slices are empty)
  const int kk = k > 0 ? k : 0;
  const int b_end = n < 5 ? n : 5;
  const double A = slice(1, 3), B = slice(3, b_end);
  const double xv = A * pw(kk) + (kk ? slice(5, 5 + kk) : 0.0);
  const double yv = B * pw(kk) + (kk ? slice(5 + kk, 5 + 2 * kk) : 0.0);
  const uint32_t adj = (uint32_t)(q > 0 ? 2 * e : e);
  *x = (int32_t)((uint32_t)(int32_t)xv * adj + (uint32_t)((q == 3 || q == 4) ? e : 0));
  *y = (int32_t)((uint32_t)(int32_t)yv * adj + (uint32_t)((q == 2 || q == 3) ? e : 0));
  *res = r;
  *edge = e;
  *x_letter = (int)B;  // isValid's xLetterIndex = digits.slice(3, 5)
  *y_letter = (int)A;  // yLetterIndex = digits.slice(1, 3)
  return true;
}

// BNGIndexSystem.isValid (BNGIndexSystem.scala:261-270): 1 / 0, or -1 where the Scala
// code throws (NumberFormatException from "".toInt on an id of fewer than 4 digits;
// a non-positive id, whose digits are not digits, is treated the same)
MGPU_HDB int valid_state(int64_t id) {
  int r, xl, yl;
  int32_t e, x, y;
  if (!cell_corner(id, &r, &e, &x, &y, &xl, &yl)) return -1;
  return (x >= 0 && x <= 700000 && y >= 0 && y <= 1300000 && xl < 14 && yl < 8) ? 1 : 0;
}

// Position c of kLoop(index, k)'s candidate list (BNGIndexSystem.scala:233-246): the
// bottom, right, top and left sides, 2k corners each, as (x, y) in metres.
MGPU_HDB void kloop_xy(int32_t x, int32_t y, int32_t e, int k, int c, int32_t* px, int32_t* py) {
  const int side = c / (2 * k), t = c % (2 * k);
  if (side == 0) {
    *px = x + (t - k) * e;
    *py = y - k * e;
  } else if (side == 1) {
    *px = x + k * e;
    *py = y + (t - k) * e;
  } else if (side == 2) {
    *px = x + (k - t) * e;
    *py = y + k * e;
  } else {
    *px = x - k * e;
    *py = y + (k - t) * e;
  }
}

}  // namespace bng
}  // namespace mgpu
