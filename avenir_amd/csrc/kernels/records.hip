// K1 on the device for the non-schema record layouts (host twin:
// csrc/host/records.cpp TextShard, whose output this reproduces exactly).
//
// The reference splits every line with String.split and looks each token up in a HashMap inside
// its mappers (J/markov/MarkovStateTransitionModel.java:116-133, J/association/
// FrequentItemsApriori.java:133-196, J/markov/HiddenMarkovModelBuilder.java:136-260,
// J/explore/TopMatchesByClass.java:133-211, J/knn/NearestNeighbor.java:130-183,
// S/markov/StateTransitionRate.scala:91-167).  Here a rank's byte range is uploaded once and
// turned into a CSR token table on the GPU:
//   1. newline index (csv.hip kernels);
//   2. rec_lines_kernel  : one thread per raw line: CR strip, blank test, token count;
//   3. (exclusive scan of the counts -> token offsets);
//   4. rec_tokens_kernel : one thread per line walks its fields once: dictionary fields are hashed
//      (the host tokenizer's 64-bit hash) and inserted into an open-addressing table of 64-bit
//      keys (device-scope CAS; a plain load first, so hot keys cost one cached read), the
//      first-occurrence key 2*token + is_sub is kept per slot with a 64-bit atomicMin (values only
//      decrease, so a stale cached read can only cause a redundant atomic, never a missed one);
//      numeric fields are parsed to double;
//   5. (slots ordered by first occurrence -> dense codes: the host dictionary's order);
//   6. rec_codes_kernel  : token codes by gather, and an exactness check: every token carries a
//      second, independent 32-bit hash that must equal its slot's (written by the inserting
//      thread) — a 64-bit collision is detected instead of silently merging two strings;
//   7. rec_vocab_kernel  : the bytes of each dictionary entry's first occurrence, packed.
// Index safety: line walks stay inside [lstart, lend) of the uploaded buffer; table probes are
// masked by the power-of-two capacity and bounded by it (overflow flag -> the caller retries
// with a larger table); token indices are < off[L] by construction.
#include "avenir_common.h"
#include "avenir_kernels.h"
#define AVNUM_HD __device__
#include "avenir_numparse.h"

namespace {

constexpr int RT = 256;
constexpr unsigned long long EMPTY_FIRST = ~0ull;

struct TokArgs {
  unsigned sep[8];         // 256-bit separator set
  unsigned char modes[64];  // per field index: 'd' / 'n' / 'x'
  int nmodes;
  unsigned char tail_mode, sub_delim, trim, last_mode;  // last_mode: mode of every line's last field (0: none)
};

__device__ __forceinline__ bool is_sep(const TokArgs& a, uint8_t c) { return (a.sep[c >> 5] >> (c & 31)) & 1u; }
__device__ __forceinline__ bool is_ws(uint8_t c) { return c == ' ' || c == '\t' || c == '\r' || c == '\v' || c == '\f'; }

// csrc/host/records.cpp hash_bytes: 8-byte little-endian words, a partial last word zero-padded
__device__ __forceinline__ unsigned long long hash64(const uint8_t* p, int n) {
  unsigned long long h = 0x9E3779B97F4A7C15ull ^ ((unsigned long long)n * 0xC2B2AE3D27D4EB4Full);
  while (n > 0) {
    unsigned long long w = 0;
    const int k = n < 8 ? n : 8;
    for (int i = 0; i < k; ++i) w |= (unsigned long long)p[i] << (8 * i);
    h = (h ^ w) * 0xFF51AFD7ED558CCDull;
    h ^= h >> 32;
    p += k;
    n -= k;
  }
  h *= 0xC4CEB9FE1A85EC53ull;
  return h ^ (h >> 29);
}

// independent check hash (FNV-1a 32 over the bytes, length folded in)
__device__ __forceinline__ unsigned hash32(const uint8_t* p, int n) {
  unsigned h = 2166136261u ^ (unsigned)n;
  for (int i = 0; i < n; ++i) h = (h ^ p[i]) * 16777619u;
  return h ^ (h >> 13);
}

// host parse_num semantics (records.cpp, avenir_numparse.h): trim, [+-]digits[.digits][e[+-]digits],
// correctly rounded on the fast path, NaN otherwise
// tokens whose rounding the device cannot settle (> 19 significant digits, avenir_numparse.h tier
// 3): counted, read and reset by avk::rec_slow_tokens_take; the host then tokenizes the shard itself
__device__ unsigned long long g_rec_slow_tokens;

__device__ double parse_num(const uint8_t* p, const uint8_t* e) {
  while (p < e && is_ws(*p)) ++p;
  while (e > p && is_ws(e[-1])) --e;
  bool slow;
  const double v = avnum::parse_decimal(reinterpret_cast<const char*>(p), reinterpret_cast<const char*>(e), &slow);
  if (slow) atomicAdd(&g_rec_slow_tokens, 1ull);
  return v;
}

__global__ __launch_bounds__(RT) void rec_lines_kernel(const uint8_t* __restrict__ bytes,
                                                       const long long* __restrict__ nlpos, long long nraw,
                                                       TokArgs a, long long* __restrict__ lstart,
                                                       long long* __restrict__ lend, int* __restrict__ ntok) {
  const long long stride = (long long)gridDim.x * RT;
  for (long long i = (long long)blockIdx.x * RT + threadIdx.x; i < nraw; i += stride) {
    const long long s = i == 0 ? 0 : nlpos[i - 1] + 1;
    long long e = nlpos[i];
    if (e > s && bytes[e - 1] == '\r') --e;
    bool blank = true;
    int n = 1;
    for (long long k = s; k < e; ++k) {
      const uint8_t c = bytes[k];
      blank = blank && is_ws(c);
      n += is_sep(a, c) ? 1 : 0;
    }
    lstart[i] = s;
    lend[i] = e;
    ntok[i] = blank ? 0 : n;
  }
}

__device__ __forceinline__ int insert_key(unsigned long long* __restrict__ keys, unsigned* __restrict__ h2tab,
                                          unsigned long long mask, unsigned long long h, unsigned h2,
                                          unsigned* __restrict__ inserted, unsigned* __restrict__ overflow) {
  if (h == 0) h = 1;  // 0 marks an empty slot
  unsigned long long s = h & mask;
  for (unsigned long long probe = 0; probe <= mask; ++probe) {
    const unsigned long long k = keys[s];
    if (k == h) return (int)s;
    if (k == 0) {
      const unsigned long long old = atomicCAS(keys + s, 0ull, h);
      if (old == 0) {
        h2tab[s] = h2;
        const unsigned c = atomicAdd(inserted, 1u);
        if ((unsigned long long)c + 1 > (mask + 1) / 2) atomicOr(overflow, 1u);  // keep the load <= 1/2
        return (int)s;
      }
      if (old == h) return (int)s;
    }
    s = (s + 1) & mask;
  }
  atomicOr(overflow, 1u);
  return -1;
}

__global__ __launch_bounds__(RT) void rec_tokens_kernel(
    const uint8_t* __restrict__ bytes, const long long* __restrict__ lstart, const long long* __restrict__ lend,
    const long long* __restrict__ off, long long L, TokArgs a, unsigned long long* __restrict__ keys,
    unsigned* __restrict__ h2tab, unsigned long long* __restrict__ first, unsigned long long mask,
    int* __restrict__ tslot, unsigned* __restrict__ th2, int* __restrict__ tsub, unsigned* __restrict__ th2sub,
    double* __restrict__ nums, unsigned* __restrict__ inserted, unsigned* __restrict__ overflow) {
  const long long stride = (long long)gridDim.x * RT;
  for (long long l = (long long)blockIdx.x * RT + threadIdx.x; l < L; l += stride) {
    const uint8_t* p = bytes + lstart[l];
    const uint8_t* e = bytes + lend[l];
    long long k = off[l];
    int f = 0;
    while (true) {
      const uint8_t* q = p;
      while (q < e && !is_sep(a, *q)) ++q;
      const unsigned char m = (q >= e && a.last_mode) ? a.last_mode : (f < a.nmodes ? a.modes[f] : a.tail_mode);
      const uint8_t* s0 = p;
      const uint8_t* s1 = q;
      if (a.trim) {
        while (s0 < s1 && is_ws(*s0)) ++s0;
        while (s1 > s0 && is_ws(s1[-1])) --s1;
      }
      int slot = -1, sslot = -1;
      unsigned c2 = 0, c2s = 0;
      double v = __longlong_as_double(0x7ff8000000000000LL);
      if (m == 'd') {
        const uint8_t* mid = s1;
        if (a.sub_delim)
          for (const uint8_t* c = s0; c < s1; ++c)
            if (*c == a.sub_delim) { mid = c; break; }
        const int n0 = (int)(mid - s0);
        c2 = hash32(s0, n0);
        slot = insert_key(keys, h2tab, mask, hash64(s0, n0), c2, inserted, overflow);
        if (slot >= 0) {
          const unsigned long long occ = 2ull * (unsigned long long)k;
          if (first[slot] > occ) atomicMin(first + slot, occ);
        }
        if (mid < s1) {
          const int n1 = (int)(s1 - mid - 1);
          c2s = hash32(mid + 1, n1);
          sslot = insert_key(keys, h2tab, mask, hash64(mid + 1, n1), c2s, inserted, overflow);
          if (sslot >= 0) {
            const unsigned long long occ = 2ull * (unsigned long long)k + 1ull;
            if (first[sslot] > occ) atomicMin(first + sslot, occ);
          }
        }
      } else if (m == 'n') {
        v = parse_num(s0, s1);
      }
      tslot[k] = slot;
      th2[k] = c2;
      if (tsub) {
        tsub[k] = sslot;
        th2sub[k] = c2s;
      }
      if (nums) nums[k] = v;
      ++k;
      ++f;
      if (q >= e) break;
      p = q + 1;
    }
  }
}

__global__ __launch_bounds__(RT) void rec_codes_kernel(const int* __restrict__ tslot, const unsigned* __restrict__ th2,
                                                       long long T, const int* __restrict__ slot_code,
                                                       const unsigned* __restrict__ h2tab, int* __restrict__ codes,
                                                       unsigned* __restrict__ mismatch) {
  unsigned bad = 0;
  const long long stride = (long long)gridDim.x * RT;
  for (long long k = (long long)blockIdx.x * RT + threadIdx.x; k < T; k += stride) {
    const int s = tslot[k];
    int c = -1;
    if (s >= 0) {
      c = slot_code[s];
      bad += (h2tab[s] != th2[k]) ? 1u : 0u;
    }
    codes[k] = c;
  }
  bad = av::wave_sum(bad);
  if (av::lane_id() == 0 && bad) atomicAdd(mismatch, bad);
}

// byte span of dictionary entry r (its first occurrence occ[r] = 2 * token + is_sub)
__global__ __launch_bounds__(RT) void rec_span_kernel(const uint8_t* __restrict__ bytes,
                                                      const long long* __restrict__ lstart,
                                                      const long long* __restrict__ lend,
                                                      const long long* __restrict__ off, long long L,
                                                      const unsigned long long* __restrict__ occ, long long D,
                                                      TokArgs a, long long* __restrict__ vstart,
                                                      int* __restrict__ vlen) {
  const long long stride = (long long)gridDim.x * RT;
  for (long long r = (long long)blockIdx.x * RT + threadIdx.x; r < D; r += stride) {
    const long long k = (long long)(occ[r] >> 1);
    const bool sub = occ[r] & 1ull;
    long long lo = 0, hi = L;  // last line with off[line] <= k
    while (hi - lo > 1) {
      const long long m = (lo + hi) >> 1;
      if (off[m] <= k) lo = m; else hi = m;
    }
    const uint8_t* p = bytes + lstart[lo];
    const uint8_t* e = bytes + lend[lo];
    for (long long f = off[lo]; f < k; ++f) {
      while (p < e && !is_sep(a, *p)) ++p;
      ++p;
    }
    const uint8_t* q = p;
    while (q < e && !is_sep(a, *q)) ++q;
    if (a.trim) {
      while (p < q && is_ws(*p)) ++p;
      while (q > p && is_ws(q[-1])) --q;
    }
    const uint8_t* mid = q;
    if (a.sub_delim)
      for (const uint8_t* c = p; c < q; ++c)
        if (*c == a.sub_delim) { mid = c; break; }
    if (sub) {
      vstart[r] = (long long)(mid + 1 - bytes);
      vlen[r] = (int)(q - mid - 1);
    } else {
      vstart[r] = (long long)(p - bytes);
      vlen[r] = (int)(mid - p);
    }
  }
}

__global__ __launch_bounds__(RT) void rec_gather_kernel(const uint8_t* __restrict__ bytes,
                                                        const long long* __restrict__ vstart,
                                                        const int* __restrict__ vlen,
                                                        const long long* __restrict__ vout, long long D,
                                                        uint8_t* __restrict__ out) {
  const long long stride = (long long)gridDim.x * RT;
  for (long long r = (long long)blockIdx.x * RT + threadIdx.x; r < D; r += stride) {
    const uint8_t* s = bytes + vstart[r];
    uint8_t* d = out + vout[r];
    for (int i = 0; i < vlen[r]; ++i) d[i] = s[i];
  }
}

TokArgs make_args(const char* delims, int ndelims, const char* modes, int nmodes, char tail_mode, char sub_delim,
                  bool trim, char last_mode = 0) {
  TokArgs a{};
  if (nmodes > 64) throw std::runtime_error("device tokenizer: at most 64 per-field modes");
  for (int i = 0; i < ndelims; ++i) {
    const uint8_t c = (uint8_t)delims[i];
    a.sep[c >> 5] |= 1u << (c & 31);
  }
  for (int i = 0; i < nmodes; ++i) a.modes[i] = (unsigned char)modes[i];
  a.nmodes = nmodes;
  a.tail_mode = (unsigned char)tail_mode;
  a.sub_delim = (unsigned char)sub_delim;
  a.trim = trim ? 1 : 0;
  a.last_mode = (unsigned char)last_mode;
  return a;
}

}  // namespace

namespace avk {

unsigned long long rec_slow_tokens_take(hipStream_t stream) {
  unsigned long long v = 0, zero = 0;
  AV_HIP_CHECK(hipMemcpyFromSymbolAsync(&v, HIP_SYMBOL(g_rec_slow_tokens), sizeof(v), 0, hipMemcpyDeviceToHost, stream));
  AV_HIP_CHECK(hipStreamSynchronize(stream));
  if (v) {
    AV_HIP_CHECK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_rec_slow_tokens), &zero, sizeof(zero), 0, hipMemcpyHostToDevice, stream));
    AV_HIP_CHECK(hipStreamSynchronize(stream));
  }
  return v;
}


void rec_lines(const uint8_t* bytes, const long long* nlpos, long long nraw, const char* delims, int ndelims,
               long long* lstart, long long* lend, int* ntok, hipStream_t stream) {
  if (nraw <= 0) return;
  const TokArgs a = make_args(delims, ndelims, "", 0, 'd', 0, false);
  rec_lines_kernel<<<av::stream_grid(nraw, RT, 1, 8192), RT, 0, stream>>>(bytes, nlpos, nraw, a, lstart, lend, ntok);
  AV_HIP_CHECK(hipGetLastError());
}

void rec_tokens(const uint8_t* bytes, const long long* lstart, const long long* lend, const long long* off, long long L,
                const char* delims, int ndelims, const char* modes, int nmodes, char tail_mode, char sub_delim,
                bool trim, char last_mode, unsigned long long* keys, unsigned* h2tab, unsigned long long* first,
                unsigned long long mask, int* tslot, unsigned* th2, int* tsub, unsigned* th2sub, double* nums,
                unsigned* inserted, unsigned* overflow, hipStream_t stream) {
  if (L <= 0) return;
  const TokArgs a = make_args(delims, ndelims, modes, nmodes, tail_mode, sub_delim, trim, last_mode);
  rec_tokens_kernel<<<av::stream_grid(L, RT, 1, 8192), RT, 0, stream>>>(bytes, lstart, lend, off, L, a, keys, h2tab,
                                                                         first, mask, tslot, th2, tsub, th2sub, nums,
                                                                         inserted, overflow);
  AV_HIP_CHECK(hipGetLastError());
}

void rec_codes(const int* tslot, const unsigned* th2, long long T, const int* slot_code, const unsigned* h2tab,
               int* codes, unsigned* mismatch, hipStream_t stream) {
  if (T <= 0) return;
  rec_codes_kernel<<<av::stream_grid(T, RT, 1, 8192), RT, 0, stream>>>(tslot, th2, T, slot_code, h2tab, codes,
                                                                        mismatch);
  AV_HIP_CHECK(hipGetLastError());
}

void rec_vocab(const uint8_t* bytes, const long long* lstart, const long long* lend, const long long* off, long long L,
               const unsigned long long* occ, long long D, const char* delims, int ndelims, char sub_delim, bool trim,
               long long* vstart, int* vlen, hipStream_t stream) {
  if (D <= 0) return;
  const TokArgs a = make_args(delims, ndelims, "", 0, 'd', sub_delim, trim);
  rec_span_kernel<<<av::stream_grid(D, RT, 1, 8192), RT, 0, stream>>>(bytes, lstart, lend, off, L, occ, D, a, vstart,
                                                                       vlen);
  AV_HIP_CHECK(hipGetLastError());
}

void rec_gather(const uint8_t* bytes, const long long* vstart, const int* vlen, const long long* vout, long long D,
                uint8_t* out, hipStream_t stream) {
  if (D <= 0) return;
  rec_gather_kernel<<<av::stream_grid(D, RT, 1, 8192), RT, 0, stream>>>(bytes, vstart, vlen, vout, D, out);
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
