// K1 on the device: schema-driven CSV -> columnar encode.
//
// The reference parses every record with String.split + schema lookups inside each mapper
// (e.g. J/bayesian/BayesianDistribution.java mapper); the host path here is the multi-threaded
// mmap parser (csrc/host/csv.cpp).  For large files bound for the GPU the raw bytes are uploaded
// once and parsed where they will be used:
//   1. csv_nl_count_kernel   : newlines per 64 KiB chunk (16-byte loads, SWAR byte compare);
//   2. (device exclusive scan of the chunk counts);
//   3. csv_nl_pos_kernel     : every newline's byte offset, in order (block scan of per-thread
//                              counts inside each chunk);
//   4. csv_parse_kernel      : tiles of 256 consecutive records; the tile's bytes are staged in
//                              LDS by 16-byte loads (and dictionaries up to 16 KB copied to LDS), then one thread per record walks its fields
//                              once and writes every schema column: dictionary codes (FNV-1a
//                              open-addressing table per field, verified against the vocabulary
//                              bytes), bucket codes, floats.
// Field semantics match the host parser exactly (trim of spaces / tabs / CR, the same decimal
// accumulation in double, integer-division buckets, 'missing' for unknown values / short rows).
#include "avenir_common.h"
#include "avenir_kernels.h"
#define AVNUM_HD __device__
#include "avenir_numparse.h"

namespace {

constexpr int CT = 256;              // threads per block
constexpr long long CHUNK = 1 << 16;  // bytes per counting chunk (one block each)

__device__ __forceinline__ unsigned zero_bytes(unsigned x) {  // high bit of each zero byte of x
  return (x - 0x01010101u) & ~x & 0x80808080u;
}

__global__ __launch_bounds__(CT) void csv_nl_count_kernel(const uint8_t* __restrict__ bytes, long long size,
                                                          unsigned* __restrict__ counts) {
  const long long c0 = (long long)blockIdx.x * CHUNK;
  const long long c1 = min(size, c0 + CHUNK);
  unsigned cnt = 0;
  // 16-byte vectors (the buffer is padded to a multiple of 16 and 16-byte aligned)
  for (long long v = c0 + 16LL * threadIdx.x; v < c1; v += 16LL * CT) {
    const uint4 q = *reinterpret_cast<const uint4*>(bytes + v);
    const unsigned w[4] = {q.x, q.y, q.z, q.w};
    const int valid = (int)min(16LL, c1 - v);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      unsigned m = zero_bytes(w[i] ^ 0x0A0A0A0Au);
      const int lim = valid - 4 * i;  // bytes of this word inside the file
      if (lim < 4) m &= lim <= 0 ? 0u : (0xFFFFFFFFu >> (8 * (4 - lim)));
      cnt += __popc(m);
    }
  }
  cnt = av::wave_sum(cnt);
  __shared__ unsigned part[CT / 64];
  if (av::lane_id() == 0) part[av::wave_id()] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned t = 0;
    for (int w = 0; w < CT / 64; ++w) t += part[w];
    counts[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(CT) void csv_nl_pos_kernel(const uint8_t* __restrict__ bytes, long long size,
                                                        const long long* __restrict__ offsets,
                                                        long long* __restrict__ pos) {
  __shared__ unsigned s_wtot[CT / 64];
  const long long c0 = (long long)blockIdx.x * CHUNK;
  const long long c1 = min(size, c0 + CHUNK);
  long long out = offsets[blockIdx.x];
  const int lane = av::lane_id(), wave = av::wave_id();
  for (long long base = c0; base < c1; base += 16LL * CT) {
    const long long v = base + 16LL * threadIdx.x;
    unsigned bits = 0;  // bit i: byte v + i is a newline
    if (v < c1) {
      const uint4 q = *reinterpret_cast<const uint4*>(bytes + v);
      const unsigned w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const unsigned m = zero_bytes(w[i] ^ 0x0A0A0A0Au);
#pragma unroll
        for (int b = 0; b < 4; ++b)
          if ((m >> (8 * b + 7)) & 1u) bits |= 1u << (4 * i + b);
      }
      const int valid = (int)min(16LL, c1 - v);
      if (valid < 16) bits &= (1u << valid) - 1u;
    }
    const unsigned mine = __popc(bits);
    unsigned inc = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned y = __shfl_up(inc, o, 64);
      if (lane >= o) inc += y;
    }
    if (lane == 63) s_wtot[wave] = inc;
    __syncthreads();
    unsigned before = 0, tot = 0;
    for (int w = 0; w < CT / 64; ++w) {
      if (w < wave) before += s_wtot[w];
      tot += s_wtot[w];
    }
    long long o = out + before + inc - mine;
    while (bits) {
      const int b = __ffs(bits) - 1;
      pos[o++] = v + b;
      bits &= bits - 1u;
    }
    out += tot;
    __syncthreads();  // s_wtot is rewritten by the next step
  }
}

// line i = bytes [i ? pos[i-1] + 1 : 0, pos[i]); blank lines (empty after a trailing CR) flagged
// 0 in keep and counted in *blank — one pass instead of ~10 tensor ops over the line index
__global__ __launch_bounds__(CT) void csv_bounds_kernel(const uint8_t* __restrict__ bytes,
                                                        const long long* __restrict__ pos, long long nl,
                                                        long long* __restrict__ starts, long long* __restrict__ ends,
                                                        uint8_t* __restrict__ keep,
                                                        unsigned long long* __restrict__ blank) {
  unsigned nb = 0;
  const long long stride = (long long)gridDim.x * CT;
  for (long long i = (long long)blockIdx.x * CT + threadIdx.x; i < nl; i += stride) {
    const long long b = i ? pos[i - 1] + 1 : 0, e = pos[i];
    const long long eff = e - b - ((e > b && bytes[e - 1] == '\r') ? 1 : 0);
    starts[i] = b;
    ends[i] = e;
    const bool k = eff > 0;
    keep[i] = k ? 1 : 0;
    nb += k ? 0u : 1u;
  }
  nb = av::wave_sum(nb);
  if (av::lane_id() == 0 && nb) atomicAdd(blank, (unsigned long long)nb);
}

struct DevSpec {
  int ordinal, kind, wide, max_code;
  int bucket_offset, tab_off, tab_mask, vbase;  // vbase: global index of the field's first vocab entry
  double bucket_width;
  unsigned long long out;  // device address of the output column
};

__device__ __forceinline__ bool is_space(uint8_t c) { return c == ' ' || c == '\t' || c == '\r'; }

// the host parser's decimal conversion (csrc/host/csv.cpp parse_double, avenir_numparse.h), NaN on
// garbage / empty; [p, e) is trimmed by the caller
// tokens of more than 19 significant digits whose rounding the device cannot settle (see
// avenir_numparse.h tier 3): counted here, read and reset by avk::csv_slow_tokens_take; the host
// then re-parses the file with the host parser (strtod for those tokens)
__device__ unsigned long long g_csv_slow_tokens;

__device__ double dev_parse_double(const uint8_t* p, const uint8_t* e) {
  bool slow;
  const double v = avnum::parse_decimal(reinterpret_cast<const char*>(p), reinterpret_cast<const char*>(e), &slow);
  if (slow) atomicAdd(&g_csv_slow_tokens, 1ull);
  return v;
}

constexpr int CSV_MAX_SPECS = 64;  // columns per parse pass (the host splits wider schemas)
constexpr int PT_BYTES = 32 * 1024;  // LDS tile of the block's line bytes
constexpr int PD_BYTES = 16 * 1024;  // LDS copy of the dictionaries (probe table, lengths, offsets, bytes)

// one record: p..e its bytes (LDS tile or global), r its output row
__device__ __forceinline__ bool parse_record(const uint8_t* p, const uint8_t* e, long long r, char delim,
                                             const DevSpec* s_spec, int nspecs, int max_ord,
                                             const int* __restrict__ tabs, const int* __restrict__ voff,
                                             const int* __restrict__ vlen, const uint8_t* __restrict__ vbytes) {
  int o = 0, si = 0;  // specs are sorted by ordinal
  const uint8_t* a = p;
  while (o <= max_ord && si < nspecs) {
    const uint8_t* q = a;
    while (q < e && *q != (uint8_t)delim) ++q;
    while (si < nspecs && s_spec[si].ordinal == o) {
      const DevSpec& sp = s_spec[si];
      const uint8_t* f0 = a;
      const uint8_t* f1 = q;
      while (f0 < f1 && is_space(*f0)) ++f0;
      while (f1 > f0 && is_space(f1[-1])) --f1;
      unsigned code = 65535u;
      if (sp.kind == 0) {  // CAT
        unsigned h = 2166136261u;
        for (const uint8_t* c = f0; c < f1; ++c) h = (h ^ *c) * 16777619u;
        h ^= h >> 15;
        unsigned slot = h & (unsigned)sp.tab_mask;
        const int len = (int)(f1 - f0);
        while (true) {
          const int ci = tabs[sp.tab_off + slot];  // the field's code, -1 = empty slot
          if (ci < 0) break;
          const int gi = sp.vbase + ci;
          if (vlen[gi] == len) {
            const uint8_t* vb = vbytes + voff[gi];
            int k = 0;
            while (k < len && vb[k] == f0[k]) ++k;
            if (k == len) { code = (unsigned)ci; break; }
          }
          slot = (slot + 1) & (unsigned)sp.tab_mask;
        }
      } else if (sp.kind == 1) {  // BUCKET: the reference's integer division
        const double v = dev_parse_double(f0, f1);
        if (!isnan(v)) {
          const long long b = (long long)floor(v / sp.bucket_width) - sp.bucket_offset;
          if (b >= 0 && b <= sp.max_code) code = (unsigned)b;
        }
      } else {  // FLOAT
        reinterpret_cast<float*>(sp.out)[r] = (float)dev_parse_double(f0, f1);
      }
      if (sp.kind != 2) {
        if (sp.wide) reinterpret_cast<uint16_t*>(sp.out)[r] = (uint16_t)min(code, 65535u);
        else reinterpret_cast<uint8_t*>(sp.out)[r] = (uint8_t)min(code, 255u);
      }
      ++si;
    }
    ++o;
    if (q >= e) break;
    a = q + 1;
  }
  const bool short_row = si < nspecs;
  for (; si < nspecs; ++si) {  // fields beyond the end of the row: missing
    const DevSpec& sp = s_spec[si];
    if (sp.kind == 2) reinterpret_cast<float*>(sp.out)[r] = __int_as_float(0x7fc00000);
    else if (sp.wide) reinterpret_cast<uint16_t*>(sp.out)[r] = 65535;
    else reinterpret_cast<uint8_t*>(sp.out)[r] = 255;
  }
  return short_row;
}

// A tile of CT consecutive records per step: their byte span (rows are in file order) is staged
// into LDS with 16-byte coalesced loads, then every thread walks its own record in LDS (the
// per-thread byte walk was a stream of uncoalesced global byte loads); spans above the tile size
// are walked in global memory.  The byte buffer is padded to a multiple of 16.
__global__ __launch_bounds__(CT) void csv_parse_kernel(const uint8_t* __restrict__ bytes, long long size_padded,
                                                       const long long* __restrict__ starts,
                                                       const long long* __restrict__ ends, long long n, char delim,
                                                       const DevSpec* __restrict__ specs, int nspecs, int max_ord,
                                                       const int* __restrict__ tabs, const int* __restrict__ voff,
                                                       const int* __restrict__ vlen, const uint8_t* __restrict__ vbytes,
                                                       int ntab, int nvoc, int nvb,
                                                       unsigned long long* __restrict__ short_rows) {
  __shared__ DevSpec s_spec[CSV_MAX_SPECS];
  __shared__ __attribute__((aligned(16))) uint8_t tile[PT_BYTES];
  __shared__ __attribute__((aligned(16))) int dict[PD_BYTES / 4];
  for (int i = threadIdx.x; i < nspecs; i += CT) s_spec[i] = specs[i];
  // small dictionaries (every schema of the reference's examples) are probed in LDS: the probe
  // chain tabs -> vlen -> voff -> vbytes was four dependent global loads per categorical field
  const bool dict_lds = 4LL * ntab + 8LL * nvoc + nvb <= PD_BYTES;
  int* l_tabs = dict;
  int* l_vlen = dict + ntab;
  int* l_voff = l_vlen + nvoc;
  uint8_t* l_vb = reinterpret_cast<uint8_t*>(l_voff + nvoc);
  if (dict_lds) {
    for (int i = threadIdx.x; i < ntab; i += CT) l_tabs[i] = tabs[i];
    for (int i = threadIdx.x; i < nvoc; i += CT) { l_vlen[i] = vlen[i]; l_voff[i] = voff[i]; }
    for (int i = threadIdx.x; i < nvb; i += CT) l_vb[i] = vbytes[i];
  }
  unsigned bad = 0;
  for (long long r0 = (long long)blockIdx.x * CT; r0 < n; r0 += (long long)gridDim.x * CT) {
    const long long r1 = min(n, r0 + CT);
    const long long lo = starts[r0] & ~15LL;
    const long long hi = min(size_padded, (ends[r1 - 1] + 15) & ~15LL);
    const bool staged = hi - lo <= PT_BYTES;
    __syncthreads();  // s_spec written / the previous tile fully parsed
    if (staged) {
      for (long long v = lo + 16LL * threadIdx.x; v < hi; v += 16LL * CT)
        *reinterpret_cast<uint4*>(tile + (v - lo)) = *reinterpret_cast<const uint4*>(bytes + v);
    }
    __syncthreads();
    const long long r = r0 + threadIdx.x;
    if (r < r1) {
      const long long b = starts[r], e = ends[r];
      bool sr;
      if (staged && b >= lo && e <= hi && dict_lds)
        sr = parse_record(tile + (b - lo), tile + (e - lo), r, delim, s_spec, nspecs, max_ord, l_tabs, l_voff, l_vlen,
                          l_vb);
      else
        sr = parse_record(bytes + b, bytes + e, r, delim, s_spec, nspecs, max_ord, tabs, voff, vlen, vbytes);
      bad += sr ? 1u : 0u;
    }
  }
  bad = av::wave_sum(bad);
  if (av::lane_id() == 0 && bad) atomicAdd(short_rows, (unsigned long long)bad);
}

}  // namespace

namespace avk {

unsigned long long csv_slow_tokens_take(hipStream_t stream) {
  unsigned long long v = 0, zero = 0;
  AV_HIP_CHECK(hipMemcpyFromSymbolAsync(&v, HIP_SYMBOL(g_csv_slow_tokens), sizeof(v), 0, hipMemcpyDeviceToHost, stream));
  AV_HIP_CHECK(hipStreamSynchronize(stream));
  if (v) {
    AV_HIP_CHECK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_csv_slow_tokens), &zero, sizeof(zero), 0, hipMemcpyHostToDevice, stream));
    AV_HIP_CHECK(hipStreamSynchronize(stream));
  }
  return v;
}


long long csv_chunks(long long size) { return (size + CHUNK - 1) / CHUNK; }

void csv_newline_counts(const uint8_t* bytes, long long size, unsigned* counts, hipStream_t stream) {
  if (size <= 0) return;
  csv_nl_count_kernel<<<(unsigned)csv_chunks(size), CT, 0, stream>>>(bytes, size, counts);
  AV_HIP_CHECK(hipGetLastError());
}

void csv_newline_positions(const uint8_t* bytes, long long size, const long long* offsets, long long* pos,
                           hipStream_t stream) {
  if (size <= 0) return;
  csv_nl_pos_kernel<<<(unsigned)csv_chunks(size), CT, 0, stream>>>(bytes, size, offsets, pos);
  AV_HIP_CHECK(hipGetLastError());
}

void csv_line_bounds(const uint8_t* bytes, const long long* pos, long long nl, long long* starts, long long* ends,
                     uint8_t* keep, unsigned long long* blank, hipStream_t stream) {
  if (nl <= 0) return;
  csv_bounds_kernel<<<av::stream_grid(nl, CT, 4, 8192), CT, 0, stream>>>(bytes, pos, nl, starts, ends, keep, blank);
  AV_HIP_CHECK(hipGetLastError());
}

void csv_parse_rows(const uint8_t* bytes, long long size_padded, const long long* starts, const long long* ends,
                    long long n, char delim, const void* specs, int nspecs, int max_ord, const int* tabs,
                    const int* voff, const int* vlen, const uint8_t* vbytes, int ntab, int nvoc, int nvb,
                    unsigned long long* short_rows, hipStream_t stream) {
  if (n <= 0 || nspecs <= 0) return;
  if (nspecs > CSV_MAX_SPECS) throw std::runtime_error("csv_parse_rows: at most 64 parsed columns per pass");
  if (size_padded % 16) throw std::runtime_error("csv_parse_rows: the byte buffer must be padded to 16");
  csv_parse_kernel<<<av::stream_grid(n, CT, 1, 8192), CT, 0, stream>>>(
      bytes, size_padded, starts, ends, n, delim, reinterpret_cast<const DevSpec*>(specs), nspecs, max_ord, tabs, voff, vlen,
      vbytes, ntab, nvoc, nvb, short_rows);
  AV_HIP_CHECK(hipGetLastError());
}

int csv_devspec_bytes() { return (int)sizeof(DevSpec); }

}  // namespace avk
