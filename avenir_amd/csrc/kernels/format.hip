// Output text on the GPU (CDNA4, gfx950): the rows of a job's output assembled by one thread per
// row from device columns — string-table lookups, CSR string lists, integers, fixed-precision
// doubles, literals and the input line bytes the device tokenizer / CSV parser already uploaded.
//
// The reference's mappers / reducers emit one Text record per input record through Hadoop's
// TextOutputFormat (e.g. J/markov/ViterbiStatePredictor.java:114-142, J/bayesian/
// BayesianPredictor.java:271-285).  At 10^7+ records per rank the host formatter's per-row work
// is the largest part of such a job; here the rows are formatted where the data already is:
//   pass 1  row lengths (and an "unsupported value" flag: doubles outside the exact fast path),
//   scan    row offsets (torch cumsum on the device),
//   pass 2  every row written at its offset.
// The bytes then go to the host once (pinned) and are written by the host threads.  Doubles use an
// exact fixed-point conversion (mantissa x 10^p in 128-bit, round half to even on the exact binary
// value) — the same digits as printf("%.*f") / std::to_chars / Python's format for precision p.
#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

constexpr int FT = 256;

__device__ __forceinline__ bool is_sep(const uint32_t* sep, uint8_t c) { return (sep[c >> 5] >> (c & 31)) & 1u; }

// decimal digits of v (< 2^64) into buf from the right; returns the count
__device__ __forceinline__ int u64_digits(uint64_t v, char* buf) {
  int n = 0;
  do {
    buf[n++] = (char)('0' + (int)(v % 10ull));
    v /= 10ull;
  } while (v);
  return n;  // reversed
}

struct Sink {
  char* out;      // nullptr in the length pass
  int64_t pos;
  __device__ __forceinline__ void put(char c) {
    if (out) out[pos] = c;
    ++pos;
  }
  __device__ __forceinline__ void put(const uint8_t* p, int64_t n) {
    if (out)
      for (int64_t i = 0; i < n; ++i) out[pos + i] = (char)p[i];
    pos += n;
  }
  __device__ __forceinline__ void put(const char* p, int64_t n) { put(reinterpret_cast<const uint8_t*>(p), n); }
};

__device__ __forceinline__ void put_i64(Sink& s, long long v) {
  char b[24];
  uint64_t u = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
  if (v < 0) s.put('-');
  const int n = u64_digits(u, b);
  for (int i = n - 1; i >= 0; --i) s.put(b[i]);
}

__device__ __constant__ uint64_t kPow10[10] = {1ull, 10ull, 100ull, 1000ull, 10000ull, 100000ull, 1000000ull,
                                               10000000ull, 100000000ull, 1000000000ull};

// fixed notation with p (0..9) fraction digits, exact; false when |v| * 10^p >= 2^64
__device__ __forceinline__ bool put_fixed(Sink& s, double v, int p) {
  if (v != v) {
    s.put("NaN", 3);
    return true;
  }
  const uint64_t bits = (uint64_t)__double_as_longlong(v);
  const bool neg = bits >> 63;
  const int be = (int)((bits >> 52) & 0x7ff);
  uint64_t m = bits & ((1ull << 52) - 1);
  if (be == 0x7ff) {  // inf
    if (neg) s.put('-');
    s.put("inf", 3);
    return true;
  }
  int e;
  if (be == 0) e = -1074;  // subnormal (or zero)
  else {
    m |= 1ull << 52;
    e = be - 1075;
  }
  const unsigned __int128 N = (unsigned __int128)m * kPow10[p];
  uint64_t q;
  if (e >= 0) {
    if (e > 63) return false;
    const unsigned __int128 t = N << e;
    if ((t >> 64) != 0 || (e > 0 && (t >> e) != N)) return false;
    q = (uint64_t)t;
  } else {
    const int sh = -e;
    if (sh >= 127) {
      q = 0;  // below 2^-44 * 10^9: rounds to zero
    } else {
      const unsigned __int128 qq = N >> sh;
      const unsigned __int128 r = N - (qq << sh);
      const unsigned __int128 half = (unsigned __int128)1 << (sh - 1);
      if ((qq >> 64) != 0) return false;
      q = (uint64_t)qq;
      if (r > half || (r == half && (q & 1ull))) ++q;
    }
  }
  if (neg) s.put('-');
  const uint64_t ip = q / kPow10[p], fp = q % kPow10[p];
  put_i64(s, (long long)ip);
  if (p > 0) {
    s.put('.');
    char b[24];
    const int n = u64_digits(fp, b);
    for (int i = 0; i < p - n; ++i) s.put('0');
    for (int i = n - 1; i >= 0; --i) s.put(b[i]);
  }
  return true;
}

// Python's repr(float) — the fewest significant digits that parse back to v, the nearest such
// decimal, fixed notation for decimal exponents -4 <= x < 16 and d.ddde[+-]XX otherwise (the host
// formatter's put_pyrepr, std::to_chars shortest) — by exact 128-bit integer arithmetic.
// v = m 2^e (e <= -1); for k = 0, 1, .. 31 fraction digits, with 10^k = 5^k 2^k and s = -e - k:
//   D = round(m 5^k / 2^s) (half to even), and D 10^-k round-trips iff it lies inside v's
//   rounding interval:  (4m - 2) 5^k <= D 2^(s+2) <= (4m + 2) 5^k
// (bounds included only for even m; the lower bound is (4m - 1) 5^k when m = 2^52 — the gap below
// a power of two is half the gap above — and then D + 1 is tried too).  Every product stays below
// 2^128 (m 5^31 < 2^125); k = -e fraction digits are exact, so the loop ends by then.  False
// outside that range (|v| >= 2^53, subnormals, values needing more
// than 31 fraction digits): the host formatter takes over.
__device__ __forceinline__ bool put_repr(Sink& s, double v) {
  if (v != v) {
    s.put("nan", 3);
    return true;
  }
  const uint64_t bits = (uint64_t)__double_as_longlong(v);
  const bool neg = bits >> 63;
  const int be = (int)((bits >> 52) & 0x7ff);
  const uint64_t frac = bits & ((1ull << 52) - 1);
  if (be == 0x7ff) {
    if (neg) s.put('-');
    s.put("inf", 3);
    return true;
  }
  if (be == 0 && frac == 0) {
    if (neg) s.put('-');
    s.put("0.0", 3);
    return true;
  }
  if (be == 0) return false;  // subnormal
  const uint64_t m = frac | (1ull << 52);
  const int sh = 1075 - be;   // -e
  if (sh < 0) return false;   // |v| >= 2^53
  const bool even = (m & 1ull) == 0, pow2 = frac == 0 && be > 1;
  const unsigned __int128 one = 1;
  unsigned __int128 p5 = 1;
  uint64_t D = 0;
  int k = 0;
  bool found = false;
  for (; k <= 31; ++k, p5 *= 5u) {
    const int s2 = sh - k;
    if (s2 > 125) continue;  // D would be 0
    if (s2 < 0) return false;  // unreachable: k = -e digits are exact (s2 = 0)
    const unsigned __int128 N = (unsigned __int128)m * p5;
    unsigned __int128 q = N >> s2;
    if (s2 > 0) {
      const unsigned __int128 r = N - (q << s2), half = one << (s2 - 1);
      if (r > half || (r == half && (q & 1u))) ++q;
    }
    const unsigned __int128 hi = ((unsigned __int128)(4 * m + 2)) * p5;
    const unsigned __int128 lo = ((unsigned __int128)(pow2 ? 4 * m - 1 : 4 * m - 2)) * p5;
    for (int t = 0; t < (pow2 ? 2 : 1) && !found; ++t) {
      const unsigned __int128 c = q + (unsigned)t;
      if ((c >> 64) != 0) return false;
      const unsigned __int128 L = c << (s2 + 2);
      if (even ? (L >= lo && L <= hi) : (L > lo && L < hi)) {
        D = (uint64_t)c;
        found = true;
      }
    }
    if (found) break;
  }
  if (!found || D == 0) return false;
  // digits of D, trailing zeros dropped (k fraction digits: decimal exponent x = nd - 1 - k)
  char b[24];
  int nd = u64_digits(D, b);  // reversed: b[0] is the last digit
  const int x = nd - 1 - k;
  int z = 0;
  while (z < nd - 1 && b[z] == '0') ++z;  // trailing zeros
  const int sig = nd - z;                  // significant digits b[nd-1] .. b[z]
  if (neg) s.put('-');
  if (x >= -4 && x < 16) {
    if (x >= 0) {
      for (int i = 0; i <= x; ++i) s.put(i < sig ? b[nd - 1 - i] : '0');
      s.put('.');
      if (sig > x + 1)
        for (int i = x + 1; i < sig; ++i) s.put(b[nd - 1 - i]);
      else
        s.put('0');
    } else {
      s.put("0.", 2);
      for (int i = 0; i < -x - 1; ++i) s.put('0');
      for (int i = 0; i < sig; ++i) s.put(b[nd - 1 - i]);
    }
    return true;
  }
  s.put(b[nd - 1]);
  if (sig > 1) {
    s.put('.');
    for (int i = 1; i < sig; ++i) s.put(b[nd - 1 - i]);
  }
  s.put('e');
  s.put(x < 0 ? '-' : '+');
  const int ax = x < 0 ? -x : x;
  if (ax < 10) s.put('0');
  put_i64(s, ax);
  return true;
}

// [a, e) of field f of the line (negative: from the end); false when the line is shorter
__device__ __forceinline__ bool field_span(const uint8_t* p, int64_t n, int f, const uint32_t* sep, int64_t* a,
                                           int64_t* e) {
  if (f >= 0) {
    int64_t s0 = 0;
    for (int k = 0; k < f; ++k) {
      while (s0 < n && !is_sep(sep, p[s0])) ++s0;
      if (s0 >= n) return false;
      ++s0;
    }
    int64_t t = s0;
    while (t < n && !is_sep(sep, p[t])) ++t;
    *a = s0;
    *e = t;
    return true;
  }
  int64_t t = n;
  for (int k = -1; k > f; --k) {
    while (t > 0 && !is_sep(sep, p[t - 1])) --t;
    if (t <= 0) return false;
    --t;
  }
  int64_t s0 = t;
  while (s0 > 0 && !is_sep(sep, p[s0 - 1])) --s0;
  *a = s0;
  *e = t;
  return true;
}

__device__ __forceinline__ void put_rejoined(Sink& s, const uint8_t* p, int64_t n, const uint32_t* sep, bool same,
                                             const uint8_t* delim, int dl) {
  if (same) {
    s.put(p, n);
    return;
  }
  for (int64_t i = 0; i < n; ++i) {
    if (is_sep(sep, p[i])) s.put(delim, dl);
    else s.put((char)p[i]);
  }
}

__device__ __forceinline__ void put_tab(Sink& s, const avk::DevFmtCol& c, int32_t k) {
  if (k >= 0 && (int64_t)k < c.tV) s.put(c.tbytes + c.toff[k], c.toff[k + 1] - c.toff[k]);
}

// one row; returns false when a value needs the host formatter
__device__ bool fmt_row(int64_t r, const avk::DevFmtCol* cols, int ncols, const uint8_t* delim, int dl, Sink& s) {
  bool first = true, ok = true;
  for (int ci = 0; ci < ncols; ++ci) {
    const avk::DevFmtCol& c = cols[ci];
    if (c.kind == avk::DevFmtCol::GLUE) {
      s.put(c.lit, c.litlen);
      continue;
    }
    if (c.kind == avk::DevFmtCol::LIST || c.kind == avk::DevFmtCol::PAIRS) {
      for (int64_t j = c.off[r]; j < c.off[r + 1]; ++j) {
        if (!first) s.put(delim, dl);
        first = false;
        put_tab(s, c, c.idx[j]);
        if (c.kind == avk::DevFmtCol::PAIRS) {
          s.put(delim, dl);
          put_i64(s, c.iv[j]);
        }
      }
      continue;
    }
    if (!first) s.put(delim, dl);
    first = false;
    switch (c.kind) {
      case avk::DevFmtCol::STR: put_tab(s, c, c.idx[r]); break;
      case avk::DevFmtCol::F64: ok &= c.prec == -2 ? put_repr(s, c.dv[r]) : put_fixed(s, c.dv[r], c.prec); break;
      case avk::DevFmtCol::I64: put_i64(s, c.iv[r]); break;
      case avk::DevFmtCol::LIT: s.put(c.lit, c.litlen); break;
      case avk::DevFmtCol::RAW:
        put_rejoined(s, c.lbytes + c.lstart[r], c.llen[r], c.sep, c.same != 0, delim, dl);
        break;
      case avk::DevFmtCol::FIELD: {
        int64_t a, e;
        const uint8_t* p = c.lbytes + c.lstart[r];
        if (field_span(p, c.llen[r], c.field, c.sep, &a, &e)) s.put(p + a, e - a);
        break;
      }
      case avk::DevFmtCol::TAIL: {
        int64_t a, e;
        const uint8_t* p = c.lbytes + c.lstart[r];
        if (field_span(p, c.llen[r], c.field, c.sep, &a, &e)) put_rejoined(s, p + a, c.llen[r] - a, c.sep, false, delim, dl);
        break;
      }
      default: break;
    }
  }
  s.put('\n');
  return ok;
}

__global__ __launch_bounds__(FT) void fmt_len_kernel(const avk::DevFmtCol* __restrict__ cols, int ncols, int64_t n,
                                                     const uint8_t* __restrict__ delim, int dl,
                                                     int64_t* __restrict__ len, int* __restrict__ bad) {
  const int64_t r = (int64_t)blockIdx.x * FT + threadIdx.x;
  if (r >= n) return;
  Sink s{nullptr, 0};
  const bool ok = fmt_row(r, cols, ncols, delim, dl, s);
  len[r] = s.pos;
  if (!ok) bad[0] = 1;  // plain vector store: any writer sets it
}

__global__ __launch_bounds__(FT) void fmt_write_kernel(const avk::DevFmtCol* __restrict__ cols, int ncols, int64_t n,
                                                       const uint8_t* __restrict__ delim, int dl,
                                                       const int64_t* __restrict__ start, char* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * FT + threadIdx.x;
  if (r >= n) return;
  Sink s{out, start[r]};
  fmt_row(r, cols, ncols, delim, dl, s);
}

}  // namespace

namespace avk {

void format_rows_len(const DevFmtCol* cols, int ncols, int64_t n, const uint8_t* delim, int dl, int64_t* len, int* bad,
                     hipStream_t stream) {
  if (n <= 0) return;
  fmt_len_kernel<<<(unsigned)((n + FT - 1) / FT), FT, 0, stream>>>(cols, ncols, n, delim, dl, len, bad);
  AV_HIP_CHECK(hipGetLastError());
}

void format_rows_write(const DevFmtCol* cols, int ncols, int64_t n, const uint8_t* delim, int dl, const int64_t* start,
                       char* out, hipStream_t stream) {
  if (n <= 0) return;
  fmt_write_kernel<<<(unsigned)((n + FT - 1) / FT), FT, 0, stream>>>(cols, ncols, n, delim, dl, start, out);
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
