// Decimal text -> double, shared by the host parsers (csrc/host/csv.cpp, records.cpp) and the K1
// device kernels (csrc/kernels/csv.hip, records.hip) so that every path yields the same bits.
//
// Grammar: [+-]digits[.digits][(e|E)[+-]digits] (at least one digit), NaN otherwise; the caller
// trims white space.  Correct rounding (what Java's Double.parseDouble and Python's float() give)
// by Clinger's fast path: the significant digits accumulate EXACTLY into a 64-bit integer mantissa
// with a decimal exponent; when the mantissa is <= 2^53 and |exponent| <= 22 a single IEEE
// multiply or divide by an exact power of ten is the correctly rounded result.  That covers every
// field of up to 15 significant digits with a modest exponent, i.e. all the reference's data.
// Beyond it ``*slow`` is set: the host parsers then call strtod (correctly rounded), the device
// keeps the approximate m * 10^e (the summing loop this replaces rounded on every fractional digit:
// "0.3" came out as 0.30000000000000004).
//
// Include with AVNUM_HD defined as ``__device__`` in a HIP translation unit; empty on the host.
#pragma once
#include <cmath>
#include <cstdint>

#ifndef AVNUM_HD
#define AVNUM_HD
#endif

namespace avnum {

// 10^k for 0 <= k <= 22 by binary powering: every partial product is a power of ten <= 10^22, exactly
// representable, so each multiply is exact (no table: a dynamically indexed local array would live
// in scratch memory on the device)
AVNUM_HD inline double pow10_exact(int k) {
  double r = 1.0, b = 10.0;
  for (; k; k >>= 1, b *= b)
    if (k & 1) r *= b;
  return r;
}

// [p, e) already trimmed.  Returns the value (NaN on garbage); *slow = true when the fast path
// does not apply (the result is then only approximately rounded).
AVNUM_HD inline double parse_decimal(const char* p, const char* e, bool* slow) {
  *slow = false;
  const double nan = __builtin_nan("");
  if (p >= e) return nan;
  bool neg = false;
  if (*p == '+' || *p == '-') {
    neg = *p == '-';
    ++p;
  }
  uint64_t m = 0;
  int nd = 0, digits = 0, ex10 = 0;
  bool inexact = false;
  for (; p < e && *p >= '0' && *p <= '9'; ++p) {
    ++digits;
    const int d = *p - '0';
    if (m == 0 && d == 0) continue;  // leading zeros
    if (nd < 19) {
      m = m * 10 + (uint64_t)d;
      ++nd;
    } else {
      ++ex10;
      inexact |= d != 0;
    }
  }
  if (p < e && *p == '.') {
    ++p;
    for (; p < e && *p >= '0' && *p <= '9'; ++p) {
      ++digits;
      const int d = *p - '0';
      if (m == 0 && d == 0) {
        --ex10;
        continue;
      }
      if (nd < 19) {
        m = m * 10 + (uint64_t)d;
        ++nd;
        --ex10;
      } else {
        inexact |= d != 0;
      }
    }
  }
  if (digits == 0) return nan;
  if (p < e && (*p == 'e' || *p == 'E')) {
    ++p;
    bool eneg = false;
    if (p < e && (*p == '+' || *p == '-')) {
      eneg = *p == '-';
      ++p;
    }
    int ex = 0, ed = 0;
    for (; p < e && *p >= '0' && *p <= '9'; ++p, ++ed)
      if (ex < 100000) ex = ex * 10 + (*p - '0');
    if (ed == 0) return nan;
    ex10 += eneg ? -ex : ex;
  }
  if (p != e) return nan;
  double v;
  if (m == 0) {
    v = 0.0;
  } else if (!inexact && m <= (1ull << 53) && ex10 >= -22 && ex10 <= 22) {
    v = ex10 >= 0 ? (double)m * pow10_exact(ex10) : (double)m / pow10_exact(-ex10);
  } else {
    *slow = true;
    v = (double)m * pow(10.0, (double)ex10);
  }
  return neg ? -v : v;
}

}  // namespace avnum
