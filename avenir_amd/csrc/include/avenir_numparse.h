// Decimal text -> double, shared by the host parsers (csrc/host/csv.cpp, records.cpp) and the K1
// device kernels (csrc/kernels/csv.hip, records.hip) so that every path yields the same bits.
//
// Grammar: [+-]digits[.digits][(e|E)[+-]digits] (at least one digit), NaN otherwise; the caller
// trims white space.  Correctly rounded (what Java's Double.parseDouble, Python's float() and
// strtod give), in three tiers:
//  1. Clinger's fast path: the significant digits accumulate EXACTLY into a 64-bit integer
//     mantissa w with a decimal exponent q; when w <= 2^53 and |q| <= 22 a single IEEE multiply or
//     divide by an exact power of ten is the correctly rounded result (every field of up to 15
//     significant digits with a modest exponent: all the reference's data);
//  2. Eisel-Lemire (Lemire 2021, "Number Parsing at a Gigabyte per Second" §5-6): w times a 128-bit
//     approximation of 5^q (avenir_pow5_table.h), the top 55 bits of the 128-bit product rounded
//     to nearest-even, subnormals and overflow included.  Exact for every w of up to 19 digits,
//     i.e. every full-precision double (Java Double.toString / repr print <= 17 digits);
//  3. more than 19 significant digits (w truncated): Eisel-Lemire of w and of w + 1 agree -> that
//     is the answer; otherwise ``*slow`` is set — the host parsers call strtod, the device kernels
//     count the token in a slow counter and the host re-parses that batch (never seen in practice).
//
// Include with AVNUM_HD defined as ``__device__`` in a HIP translation unit; empty on the host.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>

#ifndef AVNUM_HD
#define AVNUM_HD
#endif
#ifndef AVNUM_TABLE
#ifdef __HIPCC__
#define AVNUM_TABLE static __device__ const
#else
#define AVNUM_TABLE static const
#endif
#endif

#include "avenir_pow5_table.h"

namespace avnum {

AVNUM_HD inline uint64_t mulhi64(uint64_t a, uint64_t b) {
#ifdef __HIP_DEVICE_COMPILE__
  return __umul64hi(a, b);
#else
  return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

AVNUM_HD inline double bits_to_double(uint64_t u) {
#ifdef __HIP_DEVICE_COMPILE__
  return __longlong_as_double((long long)u);
#else
  double d;
  std::memcpy(&d, &u, sizeof d);
  return d;
#endif
}

AVNUM_HD inline int clz64(uint64_t x) {
#ifdef __HIP_DEVICE_COMPILE__
  return __clzll((long long)x);
#else
  return __builtin_clzll(x);
#endif
}

// Eisel-Lemire: w != 0 (exact), returns the binary64 bits of w * 10^q correctly rounded (positive).
AVNUM_HD inline uint64_t eisel_lemire(uint64_t w, int q) {
  if (q < POW5_MIN_Q) return 0;                      // below the smallest subnormal
  if (q > POW5_MAX_Q) return 0x7FF0000000000000ull;  // overflow
  const int lz = clz64(w);
  w <<= lz;
  const int idx = 2 * (q - POW5_MIN_Q);
  uint64_t hi = mulhi64(w, POW5_128[idx]);
  uint64_t lo = w * POW5_128[idx];
  if ((hi & 0x1FFull) == 0x1FFull) {  // the truncated 5^q may matter: add the second 64 bits
    const uint64_t hi2 = mulhi64(w, POW5_128[idx + 1]);
    lo += hi2;
    if (hi2 > lo) ++hi;
  }
  const int upper = (int)(hi >> 63);
  const int shift = upper + 9;
  uint64_t mant = hi >> shift;
  int p2 = (int)((((152170 + 65536) * (long long)q) >> 16) + 63) + upper - lz + 1023;
  if (p2 <= 0) {  // subnormal
    if (-p2 + 1 >= 64) return 0;
    mant >>= -p2 + 1;
    mant += mant & 1;
    mant >>= 1;
    p2 = mant < (1ull << 52) ? 0 : 1;
    return ((uint64_t)p2 << 52) | (mant & ((1ull << 52) - 1));
  }
  // exactly halfway between two doubles (possible only where 5^q fits one word): round to even
  if (lo <= 1 && q >= -4 && q <= 23 && (mant & 3) == 1 && (mant << shift) == hi) mant &= ~1ull;
  mant += mant & 1;
  mant >>= 1;
  if (mant >= (2ull << 52)) {
    mant = 1ull << 52;
    ++p2;
  }
  mant &= ~(1ull << 52);
  if (p2 >= 0x7FF) return 0x7FF0000000000000ull;
  return ((uint64_t)p2 << 52) | mant;
}

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
    const uint64_t b = eisel_lemire(m, ex10);
    if (inexact && eisel_lemire(m + 1, ex10) != b) *slow = true;  // truncated digits decide it
    v = bits_to_double(b);
  }
  return neg ? -v : v;
}

}  // namespace avnum
