// Decimal text -> double, correctly rounded (round half to even), host and device.
//
// The reference decodes WKT geometry with JTS WKTReader, whose numbers go through
// java.lang.Double.parseDouble (JTS io/WKTReader.getNextNumber), which rounds the
// decimal value exactly.  Here: Clinger's fast path when the significand fits a double
// and |exponent| <= 22 (one IEEE multiply / divide of exact operands -- the common case
// for coordinates such as "-73.956758"), otherwise a close double approximation moved
// to the correctly rounded one by exact big-integer comparisons of the decimal value
// with the midpoints between neighbouring doubles.
#pragma once
#include <math.h>
#include <stdint.h>

#ifdef __HIPCC__
#define MGPU_DEC __host__ __device__ inline
#else
#define MGPU_DEC inline
#endif

namespace mgpu {
namespace dec {

constexpr int kMaxDigits = 64;    // significant digits kept (more: not parsed)
constexpr int kLimbs = 64;        // 2048-bit big integers
constexpr int kMaxExp10 = 400;    // |decimal exponent| handled (beyond: 0 / infinity)

struct Big {
  uint32_t d[kLimbs];
  int n;  // limbs in use
};

MGPU_DEC void big_set(Big& b, uint64_t v) {
  b.d[0] = (uint32_t)v;
  b.d[1] = (uint32_t)(v >> 32);
  b.n = b.d[1] ? 2 : (b.d[0] ? 1 : 0);
}
MGPU_DEC bool big_mul_small(Big& b, uint32_t m) {
  uint64_t c = 0;
  for (int i = 0; i < b.n; i++) {
    const uint64_t t = (uint64_t)b.d[i] * m + c;
    b.d[i] = (uint32_t)t;
    c = t >> 32;
  }
  if (c) {
    if (b.n >= kLimbs) return false;
    b.d[b.n++] = (uint32_t)c;
  }
  return true;
}
MGPU_DEC bool big_add_small(Big& b, uint32_t a) {
  uint64_t c = a;
  for (int i = 0; i < b.n && c; i++) {
    const uint64_t t = (uint64_t)b.d[i] + c;
    b.d[i] = (uint32_t)t;
    c = t >> 32;
  }
  if (c) {
    if (b.n >= kLimbs) return false;
    b.d[b.n++] = (uint32_t)c;
  }
  return true;
}
MGPU_DEC bool big_mul_pow10(Big& b, int e) {
  for (; e >= 9; e -= 9)
    if (!big_mul_small(b, 1000000000u)) return false;
  uint32_t m = 1;
  for (; e > 0; e--) m *= 10;
  return big_mul_small(b, m);
}
MGPU_DEC bool big_shl(Big& b, int s) {
  if (b.n == 0) return true;
  const int w = s / 32, r = s % 32;
  if (b.n + w + 1 > kLimbs) return false;
  if (r) {
    b.d[b.n] = 0;
    for (int i = b.n; i > 0; i--) b.d[i] = (b.d[i] << r) | (b.d[i - 1] >> (32 - r));
    b.d[0] <<= r;
    b.n++;
  }
  if (w) {
    for (int i = b.n - 1; i >= 0; i--) b.d[i + w] = b.d[i];
    for (int i = 0; i < w; i++) b.d[i] = 0;
    b.n += w;
  }
  while (b.n && b.d[b.n - 1] == 0) b.n--;
  return true;
}
MGPU_DEC int big_cmp(const Big& a, const Big& b) {
  if (a.n != b.n) return a.n < b.n ? -1 : 1;
  for (int i = a.n - 1; i >= 0; i--)
    if (a.d[i] != b.d[i]) return a.d[i] < b.d[i] ? -1 : 1;
  return 0;
}

// decimal digits (most significant first, no leading zeros) as a big integer
MGPU_DEC bool big_from_digits(Big& b, const uint8_t* dg, int nd) {
  b.n = 0;
  for (int i = 0; i < nd; i++) {
    if (!big_mul_small(b, 10)) return false;
    if (b.n == 0) b.n = 1, b.d[0] = 0;
    if (!big_add_small(b, dg[i])) return false;
    while (b.n && b.d[b.n - 1] == 0) b.n--;
  }
  return true;
}

// sign of (digits x 10^e) - (k x 2^f), exactly; *ok = false if out of range
MGPU_DEC int cmp_dec_bin(const uint8_t* dg, int nd, int e, uint64_t k, int f, bool* ok) {
  Big L, R;
  if (!big_from_digits(L, dg, nd)) return *ok = false, 0;
  big_set(R, k);
  bool g = true;
  if (e >= 0) g = g && big_mul_pow10(L, e);
  else g = g && big_mul_pow10(R, -e);
  if (f >= 0) g = g && big_shl(R, f);
  else g = g && big_shl(L, -f);
  if (!g) return *ok = false, 0;
  return big_cmp(L, R);
}

MGPU_DEC double exact_pow10(int e) {  // 10^e for 0 <= e <= 22 (exact doubles)
  double p = 1.0;
  for (int i = 0; i < e; i++) p *= 10.0;
  return p;
}

// value of nd digits (sig. digits, no leading zeros) x 10^e, positive, correctly rounded.
// *ok = false when the value is outside what this parser handles.
MGPU_DEC double digits_to_double(const uint8_t* dg, int nd, int e, bool* ok) {
  *ok = true;
  if (nd == 0) return 0.0;
  // Clinger: an exact significand below 2^53 and an exact power of ten
  uint64_t m = 0;
  const int nm = nd < 19 ? nd : 19;
  for (int i = 0; i < nm; i++) m = m * 10 + dg[i];
  if (nd <= 19 && m < (1ULL << 53) && e >= -22 && e <= 22) {
    const double dm = (double)m;
    return e >= 0 ? dm * exact_pow10(e) : dm / exact_pow10(-e);
  }
  const int e10 = e + nd;  // value in [10^(e10-1), 10^e10)
  if (e10 > 310) return INFINITY;
  if (e10 < -326) return 0.0;
  if (e < -kMaxExp10 - kMaxDigits || e > kMaxExp10) return *ok = false, 0.0;
  // approximation: leading 19 digits x 10^(e + nd - nm), a few ulps off at most
  // (scaled by 10^-+300 around the loop so no intermediate overflows or goes subnormal)
  int r = e + (nd - nm);
  double post = 1.0;
  if (r < -280) {
    post = 1e-300;
    r += 300;
  } else if (r > 280) {
    post = 1e300;
    r -= 300;
  }
  double a = (double)m;
  while (r > 0) {
    const int s = r > 22 ? 22 : r;
    a *= exact_pow10(s);
    r -= s;
  }
  while (r < 0) {
    const int s = -r > 22 ? 22 : -r;
    a /= exact_pow10(s);
    r += s;
  }
  a *= post;
  if (!(a > 0.0)) a = 4.9406564584124654e-324;
  if (isinf(a)) a = 1.7976931348623157e308;
  // walk to the nearest double: compare with the midpoints to the neighbours
  for (int it = 0; it < 4096; it++) {
    union {
      double f;
      uint64_t u;
    } c;
    c.f = a;
    const int be = (int)((c.u >> 52) & 0x7FF);
    const uint64_t frac = c.u & ((1ULL << 52) - 1);
    const uint64_t mm = be ? (frac | (1ULL << 52)) : frac;   // a = mm x 2^E
    const int E = (be ? be : 1) - 1075;
    // upper midpoint (2 mm + 1) 2^(E-1)
    const int up = cmp_dec_bin(dg, nd, e, 2 * mm + 1, E - 1, ok);
    if (!*ok) return 0.0;
    if (up > 0 || (up == 0 && (mm & 1))) {
      if (be == 0x7FE && mm == (1ULL << 53) - 1) return INFINITY;
      c.u += 1;
      a = c.f;
      if (up > 0) continue;
      return a;  // tie: to even
    }
    // lower midpoint
    int lo;
    if (be > 1 && frac == 0)
      lo = cmp_dec_bin(dg, nd, e, 4 * mm - 1, E - 2, ok);
    else
      lo = mm ? cmp_dec_bin(dg, nd, e, 2 * mm - 1, E - 1, ok) : 1;
    if (!*ok) return 0.0;
    if (lo < 0 || (lo == 0 && (mm & 1))) {
      c.u -= 1;
      a = c.f;
      if (lo < 0) continue;
      return a;
    }
    return a;
  }
  *ok = false;
  return 0.0;
}

// A decimal number as java.lang.Double.parseDouble reads it (the forms a WKT
// tokenizer hands over): [+-]digits[.digits][(e|E)[+-]digits], ".5", "5.", "NaN".
// Returns the number of characters consumed (0: not a number) and the value.
MGPU_DEC int parse_number(const char* s, int len, double* out) {
  int i = 0;
  bool neg = false;
  if (i < len && (s[i] == '+' || s[i] == '-')) neg = s[i++] == '-';
  if (i + 3 <= len && (s[i] | 32) == 'n' && (s[i + 1] | 32) == 'a' && (s[i + 2] | 32) == 'n') {
    *out = NAN;
    return i + 3;
  }
  uint8_t dg[kMaxDigits];
  int nd = 0, e = 0, nseen = 0;
  bool dot = false, over = false;
  for (; i < len; i++) {
    const char ch = s[i];
    if (ch == '.') {
      if (dot) break;
      dot = true;
      continue;
    }
    if (ch < '0' || ch > '9') break;
    nseen++;
    if (nd == 0 && ch == '0') {  // leading zeros
      if (dot) e--;
      continue;
    }
    if (nd < kMaxDigits) {
      dg[nd++] = (uint8_t)(ch - '0');
      if (dot) e--;
    } else {
      if (ch != '0') over = true;
      if (!dot) e++;
    }
  }
  if (nseen == 0) return 0;
  if (i < len && (s[i] == 'e' || s[i] == 'E')) {
    int j = i + 1;
    bool en = false;
    if (j < len && (s[j] == '+' || s[j] == '-')) en = s[j++] == '-';
    int x = 0, nx = 0;
    for (; j < len && s[j] >= '0' && s[j] <= '9'; j++, nx++)
      if (x < 100000) x = x * 10 + (s[j] - '0');
    if (nx == 0) return 0;
    e += en ? -x : x;
    i = j;
  }
  if (over) return 0;  // more significant digits than kept: not handled
  // trailing zeros of the significand into the exponent
  while (nd > 0 && dg[nd - 1] == 0) nd--, e++;
  bool ok;
  const double v = digits_to_double(dg, nd, e, &ok);
  if (!ok) return 0;
  *out = neg ? -v : v;
  return i;
}

}  // namespace dec
}  // namespace mgpu
