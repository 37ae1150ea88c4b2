// K2 / K3 / K4 counting kernels for CDNA4 (gfx950).
//
// K2  class-conditional categorical histogram  out[c][off_f + b]  (Naive Bayes training,
//     categorical encodings, class affinity, Fisher/KS stats, event-time distributions ...).
//     Replaces the per-record emit + shuffle of BayesianDistribution's mapper/reducer
//     (reference: src/main/java/org/avenir/bayesian/BayesianDistribution.java:137-178, :263-327).
// K3  pair / contingency histogram  out[p][c][b1][b2]   (MutualInformation, CramerCorrelation,
//     HeterogeneityReductionCorrelation: J/explore/MutualInformation.java:138-216,
//     J/explore/CramerCorrelation.java:162-182).
// K4  Markov bigram histogram  out[c][s][s']  (J/markov/MarkovStateTransitionModel.java:116-133).
//
// Row-packed records (all codes + one-hot class of a record in <= 15 bits): hist_joint_dense_kernel
// counts each record with ONE LDS atomic into the block's joint table (dense B-bit record stream,
// 1.63 B/record for churn) and takes the class-conditional marginals once per block — the NB
// training headline; hist_joint_kernel / hist_rowpack_kernel are the 16-bit-word variants.
//
// Data layout (SoA, feature-major): codes are uint8 [F][ld] with ld % 16 == 0, so every lane
// streams 16 rows per 128-bit load.  A code is either < bins[f] or the missing sentinel 255.
//
// Fast path (every C*bins[f] <= 16): each lane keeps 16 one-hot BYTE counters packed in two
// u64 registers; incrementing bin i is `acc += 1 << 8*(i&7)` — no LDS, no atomics in the hot
// loop.  Every 15 tiles (<= 240 increments/byte) the wave widens bytes to 16-bit lanes,
// reduces them with 64-lane shuffles (64*240 < 2^16) and lane 0 adds into an LDS table.
// This keeps the kernel at the HBM roofline even with 2 classes (where a plain atomic
// histogram would serialise on a handful of hot addresses).
#include <cstdlib>
#include <string>

#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

constexpr int HB = 256;          // threads per block for the histogram kernels
constexpr int FLUSH_EVERY = 15;  // tiles between byte-counter flushes (16 rows/lane/tile)

__device__ __forceinline__ void flush_packed(unsigned long long& lo, unsigned long long& hi,
                                             unsigned int* s_bins /*16*/) {
  const unsigned long long M = 0x00FF00FF00FF00FFull;
  unsigned long long w[4] = {lo & M, (lo >> 8) & M, hi & M, (hi >> 8) & M};
#pragma unroll
  for (int q = 0; q < 4; ++q) w[q] = av::wave_sum_u64(w[q]);
  if (av::lane_id() == 0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int base = (q >> 1) * 8 + (q & 1);  // even bytes / odd bytes of lo / hi
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        unsigned v = (unsigned)((w[q] >> (16 * k)) & 0xFFFFu);
        if (v) atomicAdd(&s_bins[base + 2 * k], v);
      }
    }
  }
  lo = 0;
  hi = 0;
}

__device__ __forceinline__ void acc_byte(unsigned idx, unsigned long long& lo,
                                         unsigned long long& hi) {
  const unsigned long long b = 1ull << ((idx & 7u) << 3);
  const bool in = idx < 16u;
  const bool h = idx >= 8u;
  lo += (in && !h) ? b : 0ull;
  hi += (in && h) ? b : 0ull;
}

__device__ __forceinline__ void acc_word(unsigned cw, unsigned vw, unsigned B,
                                         unsigned long long& lo, unsigned long long& hi) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const unsigned c = (cw >> (8 * j)) & 0xFFu;
    const unsigned v = (vw >> (8 * j)) & 0xFFu;
    acc_byte(c * B + v, lo, hi);
  }
}

template <int NF>
__global__ __launch_bounds__(HB) void hist_packed_kernel(
    const uint8_t* __restrict__ codes, long long ld, long long n, const uint8_t* __restrict__ labels,
    const int* __restrict__ bins, const int* __restrict__ offs, int f0, int nfeat, int total_bins,
    int n_classes, int count_labels, unsigned long long* __restrict__ out) {
  // s_bins[NF*16 .. NF*16+15]: per-class record counts (count_labels), stored in column TB-1
  __shared__ unsigned int s_bins[NF * 16 + 16];
  for (int i = threadIdx.x; i < NF * 16 + 16; i += HB) s_bins[i] = 0;
  __syncthreads();

  unsigned B[NF];
  const uint4* col[NF];
#pragma unroll
  for (int k = 0; k < NF; ++k) {
    const int f = f0 + (k < nfeat ? k : 0);
    B[k] = (unsigned)bins[f];
    col[k] = reinterpret_cast<const uint4*>(codes + (long long)f * ld);
  }
  const uint4* lab = reinterpret_cast<const uint4*>(labels);

  unsigned long long lo[NF], hi[NF], clo = 0, chi = 0;
#pragma unroll
  for (int k = 0; k < NF; ++k) { lo[k] = 0; hi[k] = 0; }
  const bool cl_cnt = count_labels && f0 == 0;

  const long long nvec = n >> 4;  // full 16-row vectors
  const long long ntiles = (nvec + AV_WAVE - 1) / AV_WAVE;
  const int waves_per_block = HB / AV_WAVE;
  const long long gw = (long long)blockIdx.x * waves_per_block + av::wave_id();
  const long long nw = (long long)gridDim.x * waves_per_block;
  int since_flush = 0;
  for (long long t = gw; t < ntiles; t += nw) {
    const long long v = t * AV_WAVE + av::lane_id();
    if (v < nvec) {
      uint4 cl = lab ? lab[v] : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int k = 0; k < NF; ++k) {
        if (k < nfeat) {
          const uint4 x = col[k][v];
          acc_word(cl.x, x.x, B[k], lo[k], hi[k]);
          acc_word(cl.y, x.y, B[k], lo[k], hi[k]);
          acc_word(cl.z, x.z, B[k], lo[k], hi[k]);
          acc_word(cl.w, x.w, B[k], lo[k], hi[k]);
        }
      }
      if (cl_cnt) {  // class-only counter: bin index = class code
        acc_word(cl.x, 0u, 1u, clo, chi);
        acc_word(cl.y, 0u, 1u, clo, chi);
        acc_word(cl.z, 0u, 1u, clo, chi);
        acc_word(cl.w, 0u, 1u, clo, chi);
      }
    }
    if (++since_flush == FLUSH_EVERY) {  // wave-uniform
#pragma unroll
      for (int k = 0; k < NF; ++k)
        if (k < nfeat) flush_packed(lo[k], hi[k], &s_bins[k * 16]);
      if (cl_cnt) flush_packed(clo, chi, &s_bins[NF * 16]);
      since_flush = 0;
    }
  }
#pragma unroll
  for (int k = 0; k < NF; ++k)
    if (k < nfeat) flush_packed(lo[k], hi[k], &s_bins[k * 16]);
  if (cl_cnt) flush_packed(clo, chi, &s_bins[NF * 16]);

  // tail rows (n % 16) — block 0 only, scalar
  if (blockIdx.x == 0) {
    __syncthreads();  // slice 0 is final before the tail's atomics land in it
    for (long long r = nvec * 16 + threadIdx.x; r < n; r += HB) {
      const unsigned c = labels ? labels[r] : 0u;
#pragma unroll
      for (int k = 0; k < NF; ++k) {
        if (k < nfeat) {
          const unsigned v = codes[(long long)(f0 + k) * ld + r];
          if (c < (unsigned)n_classes && v < B[k]) atomicAdd(&s_bins[k * 16 + c * B[k] + v], 1u);
        }
      }
      if (cl_cnt && c < (unsigned)n_classes) atomicAdd(&s_bins[NF * 16 + c], 1u);
    }
  }
  __syncthreads();
  if (cl_cnt && threadIdx.x < n_classes && s_bins[NF * 16 + threadIdx.x])
    atomicAdd(&out[(long long)threadIdx.x * total_bins + total_bins - 1],
              (unsigned long long)s_bins[NF * 16 + threadIdx.x]);
  for (int i = threadIdx.x; i < NF * 16; i += HB) {
    const int k = i >> 4, idx = i & 15;
    if (k >= nfeat) continue;
    const unsigned v = s_bins[i];
    const int Bk = bins[f0 + k];
    if (v && idx < n_classes * Bk) {
      const int c = idx / Bk, b = idx - c * Bk;
      atomicAdd(&out[(long long)c * total_bins + offs[f0 + k] + b], (unsigned long long)v);
    }
  }
}


// ---------------------------------------------------------------------------------------------
// Class-split byte counters (fastest path: every bins[f] <= 7 and C <= 4).
//
// Per lane and per (class, feature) one u64 holds 8 byte counters indexed by the feature code.
// The class of a row is turned into C 0/1 masks ONCE per row and shared by all features; a
// feature byte then costs one bfe (shift amount 8*(code&7) precomputed SWAR for 4 rows) plus C
// fused `v_lshl_add_u64` (acc += x_c << s).  A missing code (255) lands in byte 7, which is never a
// valid bin (bins <= 7), so no validity test is needed in the hot loop — and byte 0..7 of the
// first feature sum to the class's record count for free.
// Every 15 tiles the byte counters are widened into per-lane 16-bit counters (no cross-lane
// traffic); the 64-lane reduction (widened to 32-bit fields first) happens once at the end (or
// every 256 flushes).
// ---------------------------------------------------------------------------------------------
template <int NF, int C>
__global__ __launch_bounds__(HB) void hist_split_kernel(
    const uint8_t* __restrict__ codes, long long ld, long long n, const uint8_t* __restrict__ labels,
    const int* __restrict__ bins, const int* __restrict__ offs, int f0, int nfeat, int total_bins,
    int count_labels, unsigned long long* __restrict__ out) {
  constexpr int TAB = NF * C * 8;
  constexpr int WPB = HB / AV_WAVE;
  __shared__ unsigned int s_tab[WPB * TAB];  // one private slice per wave: plain stores, no atomics
  for (int i = threadIdx.x; i < WPB * TAB; i += HB) s_tab[i] = 0;
  __syncthreads();
  unsigned int* my_tab = s_tab + av::wave_id() * TAB;

  const uint4* col[NF];
#pragma unroll
  for (int k = 0; k < NF; ++k)
    col[k] = reinterpret_cast<const uint4*>(codes + (long long)(f0 + k) * ld);
  const uint4* lab = reinterpret_cast<const uint4*>(labels);

  unsigned long long a8[C][NF], ae[C][NF], ao[C][NF];
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int k = 0; k < NF; ++k) { a8[c][k] = 0; ae[c][k] = 0; ao[c][k] = 0; }

  const unsigned long long M = 0x00FF00FF00FF00FFull;
  auto widen = [&]() {
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int k = 0; k < NF; ++k) {
        ae[c][k] += a8[c][k] & M;
        ao[c][k] += (a8[c][k] >> 8) & M;
        a8[c][k] = 0;
      }
  };
  auto reduce_to_lds = [&]() {
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int k = 0; k < NF; ++k) {
        {
          // widen the 16-bit per-lane fields to 32 bits BEFORE the cross-lane sum: a lane field
          // holds up to 256 * 240 counts, 64 of them overflow 16 bits (skewed bins, long runs)
          const unsigned long long W = 0x0000FFFF0000FFFFull;
          const unsigned long long e0 = av::wave_sum_u64(ae[c][k] & W);          // bytes 0, 4
          const unsigned long long e1 = av::wave_sum_u64((ae[c][k] >> 16) & W);  // bytes 2, 6
          const unsigned long long o0 = av::wave_sum_u64(ao[c][k] & W);          // bytes 1, 5
          const unsigned long long o1 = av::wave_sum_u64((ao[c][k] >> 16) & W);  // bytes 3, 7
          // lane l < 8 owns byte counter l
          const int l = av::lane_id();
          const unsigned long long src = (l & 1) ? ((l & 2) ? o1 : o0) : ((l & 2) ? e1 : e0);
          const unsigned val = (unsigned)(src >> (32 * (l >> 2)));
          if (l < 8) my_tab[(k * C + c) * 8 + l] += val;
        }
        ae[c][k] = 0;
        ao[c][k] = 0;
      }
  };

  const long long nvec = n >> 4;
  const long long ntiles = (nvec + AV_WAVE - 1) / AV_WAVE;
  const int wpb = HB / AV_WAVE;
  const long long gw = (long long)blockIdx.x * wpb + av::wave_id();
  const long long nw = (long long)gridDim.x * wpb;
  int since_flush = 0, flushes = 0;
  for (long long t = gw; t < ntiles; t += nw) {
    const long long v = t * AV_WAVE + av::lane_id();
    if (v < nvec) {
      const uint4 cl4 = (C > 1) ? lab[v] : make_uint4(0, 0, 0, 0);
      uint4 x4[NF];
#pragma unroll
      for (int k = 0; k < NF; ++k)
        x4[k] = col[k][v];
      const unsigned cw[4] = {cl4.x, cl4.y, cl4.z, cl4.w};
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        // shift amounts 8*(code & 7) for 4 rows at once (SWAR, no carries)
        unsigned sw[NF];
#pragma unroll
        for (int k = 0; k < NF; ++k) {
          const unsigned xw = (w == 0) ? x4[k].x : (w == 1) ? x4[k].y : (w == 2) ? x4[k].z : x4[k].w;
          sw[k] = (xw & 0x07070707u) << 3;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          unsigned long long xc[C];
          if (C == 1) {
            xc[0] = 1ull;
          } else {
            const unsigned cb = (cw[w] >> (8 * j)) & 0xFFu;
#pragma unroll
            for (int c = 0; c < C; ++c) xc[c] = (cb == (unsigned)c) ? 1ull : 0ull;
          }
#pragma unroll
          for (int k = 0; k < NF; ++k) {
            const unsigned sh = (sw[k] >> (8 * j)) & 0xFFu;
#pragma unroll
            for (int c = 0; c < C; ++c) a8[c][k] += xc[c] << sh;
          }
        }
      }
    }
    if (++since_flush == FLUSH_EVERY) {  // wave-uniform
      widen();
      since_flush = 0;
      if (++flushes == 256) {  // 16-bit per-lane counters: 256 * 240 < 65536
        reduce_to_lds();
        flushes = 0;
      }
    }
  }
  widen();
  reduce_to_lds();

  // tail rows (n % 16): block 0, scalar LDS atomics
  if (blockIdx.x == 0) {
    __syncthreads();  // slice 0 is final before the tail's atomics land in it
    for (long long r = nvec * 16 + threadIdx.x; r < n; r += HB) {
      const unsigned c = (C > 1) ? labels[r] : 0u;
      if (c >= (unsigned)C) continue;
#pragma unroll
      for (int k = 0; k < NF; ++k) {
        const unsigned v = codes[(long long)(f0 + k) * ld + r];
        atomicAdd(&s_tab[(k * C + c) * 8 + (v & 7u)], 1u);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < TAB; i += HB) {
    unsigned long long tot = 0;
#pragma unroll
    for (int w = 0; w < WPB; ++w) tot += s_tab[w * TAB + i];
    s_tab[i] = (unsigned)tot;  // slice 0 now holds the block total (each i owned by one thread)
  }
  __syncthreads();
  for (int i = threadIdx.x; i < TAB; i += HB) {
    const int k = i / (C * 8), c = (i / 8) % C, b = i % 8;
    const unsigned v = s_tab[i];
    if (v && b < bins[f0 + k])
      atomicAdd(&out[(long long)c * total_bins + offs[f0 + k] + b], (unsigned long long)v);
  }
  if (count_labels && f0 == 0 && threadIdx.x < C) {
    unsigned long long s = 0;
#pragma unroll
    for (int b = 0; b < 8; ++b) s += s_tab[(0 * C + threadIdx.x) * 8 + b];
    if (s) atomicAdd(&out[(long long)threadIdx.x * total_bins + total_bins - 1], s);
  }
}

template <int C, int NF>
void launch_split_nf(int grid, const uint8_t* codes, long long ld, long long n, const uint8_t* labels,
                     const int* d_bins, const int* d_offs, int f0, int total_bins, int count_labels,
                     unsigned long long* out, hipStream_t stream) {
  // never more workgroups than are resident at once: a second partial round of blocks would run
  // at lower occupancy (measured: 1.20 vs 1.28-1.32 ms per 1.07 G-row NB step)
  static const int res = av::resident_blocks((const void*)hist_split_kernel<NF, C>, HB, 0);
  hist_split_kernel<NF, C><<<std::min(grid, res), HB, 0, stream>>>(codes, ld, n, labels, d_bins, d_offs, f0, NF,
                                                                 total_bins, count_labels, out);
  AV_HIP_CHECK(hipGetLastError());
}

template <int C>
void launch_split(const uint8_t* codes, long long ld, long long n, const uint8_t* labels,
                  const int* d_bins, const int* d_offs, int nfeat, int total_bins, int count_labels,
                  unsigned long long* out, hipStream_t stream) {
  const long long nvec = n >> 4;
  const int grid = av::stream_grid(std::max(1LL, nvec), HB, 4, 2048);
  constexpr int MAXF = (C <= 2) ? 8 : 4;
  for (int f0 = 0; f0 < nfeat; f0 += MAXF) {
    const int nf = std::min(MAXF, nfeat - f0);
#define AV_SPLIT(K) launch_split_nf<C, K>(grid, codes, ld, n, labels, d_bins, d_offs, f0, total_bins, count_labels, out, stream)
    switch (nf) {
      case 1: AV_SPLIT(1); break;
      case 2: AV_SPLIT(2); break;
      case 3: AV_SPLIT(3); break;
      case 4: AV_SPLIT(4); break;
      default:
        if constexpr (MAXF == 8) {
          switch (nf) {
            case 5: AV_SPLIT(5); break;
            case 6: AV_SPLIT(6); break;
            case 7: AV_SPLIT(7); break;
            default: AV_SPLIT(8); break;
          }
        }
    }
#undef AV_SPLIT
  }
}

// ---------------------------------------------------------------------------------------------
// K2, row-packed layout: every record is ONE 16-bit word holding all of its categorical codes
// and its class (field k at bit sh[k], width w[k] <= 3 bits; a field that has missing values
// keeps its all-ones value as the missing code, never a valid bin; for C = 2 the class is two
// one-hot bits 0-1, both clear for an unknown class, and the fields follow from bit 2).  For low-cardinality schemas such as
// R/churn.json (5 features of 3-5 values + a binary class = 13 bits) this is 2 bytes per record
// instead of F + 1 = 6 bytes of byte-per-code columns.
//
// At 2 B/record the pass is ALU-bound unless a record costs < ~15 VALU ops (one wave64 VALU op
// per ~4 cycles per SIMD measured), so the counting uses only full-rate 32-bit ops (the byte-
// counter-in-u64 scheme, one 64-bit variable shift per (record, feature, class), measured
// 1.48 ms per 2^30 records — slower than the 6 B/record columns):
//  * per lane, one u32 of eight 4-bit counters per accumulator, incremented with ONE
//    v_lshl_add_u32 (acc += valid << 4*slot);
//  * the NM leading features (C = 2, width <= 2: at most 4 codes) merge class and code into one
//    slot 4c + code, so they cost one increment per record instead of one per class; the other
//    features keep one accumulator per class (acc_c += is_class_c << 4*code);
//  * after every tile (8 records per lane, <= 8 per nibble) the nibbles are spread into two u32
//    of byte counters (even / odd slots); every 31 tiles (<= 248 per byte) those are widened into
//    16-bit lane fields; after 256 widenings (<= 63488) or at the end the fields are summed
//    across the wave into the wave's private LDS slice [feature][class][code];
//  * the next tile's 16-byte load is issued before the current tile is counted.
// ---------------------------------------------------------------------------------------------
struct RowPackSpec {
  int sh[8];  // bit offset of feature k (kernel order: class-merged features first)
  int w[8];   // bit width of feature k (1..3)
  int lsh;    // first of the C one-hot class bits (C >= 2)
};

// acc += x << s as ONE v_lshl_add_u32: left to itself the compiler turns the chain of 8 record
// increments into v_lshlrev_b32 + v_add3_u32 trees (1.5 ops per increment instead of 1)
__device__ __forceinline__ void lshl_add_u32(unsigned& acc, unsigned x, unsigned s) {
  asm("v_lshl_add_u32 %0, %1, %2, %0" : "+v"(acc) : "v"(x), "v"(s));
}

template <int NF, int C, int NM>
__global__ __launch_bounds__(HB) void hist_rowpack_kernel(const uint16_t* __restrict__ words, long long n,
                                                          RowPackSpec spec, const int* __restrict__ bins,
                                                          const int* __restrict__ offs, int total_bins,
                                                          int count_labels, unsigned long long* __restrict__ out) {
  static_assert(NM == 0 || C == 2, "class-merged slots need C == 2");
  constexpr int NA = NM + C * (NF - NM);  // accumulators per lane; separate (k, c) -> NM + (k - NM) * C + c
  constexpr int TAB = NF * C * 8;
  constexpr int WPB = HB / AV_WAVE;
  constexpr int FLUSH = 31;  // 31 tiles x 8 records = 248 increments per byte counter at most
  __shared__ unsigned int s_tab[WPB * TAB];
  for (int i = threadIdx.x; i < WPB * TAB; i += HB) s_tab[i] = 0;
  __syncthreads();
  unsigned int* my_tab = s_tab + av::wave_id() * TAB;
  const uint4* w4 = reinterpret_cast<const uint4*>(words);

  unsigned a4[NA], be[NA], bo[NA], w16[NA][4];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    a4[j] = 0;
    be[j] = 0;
    bo[j] = 0;
#pragma unroll
    for (int m = 0; m < 4; ++m) w16[j][m] = 0;
  }
  unsigned m4[NF];  // C = 2: (4 * code) field mask of both records of a dword
#pragma unroll
  for (int k = 0; k < NF; ++k) m4[k] = (((1u << spec.w[k]) - 1u) << 2) * 0x00010001u;
  const unsigned N4 = 0x0F0F0F0Fu, B8 = 0x00FF00FFu;
  auto spread = [&]() __attribute__((always_inline)) {  // nibbles -> bytes: be byte i = slot 2i, bo = 2i + 1
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      be[j] += a4[j] & N4;
      bo[j] += (a4[j] >> 4) & N4;
      a4[j] = 0;
    }
  };
  auto widen = [&]() __attribute__((always_inline)) {  // -> 16-bit: [0] slots {0,4}, [1] {2,6}, [2] {1,5}, [3] {3,7}
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      w16[j][0] += be[j] & B8;
      w16[j][1] += (be[j] >> 8) & B8;
      w16[j][2] += bo[j] & B8;
      w16[j][3] += (bo[j] >> 8) & B8;
      be[j] = 0;
      bo[j] = 0;
    }
  };
  auto reduce_to_lds = [&]() __attribute__((always_inline)) {  // lane l < 8 owns slot l
    const int l = av::lane_id();
    const int r = l & 3, mi = ((r & 1) << 1) | (r >> 1), half = (l >> 2) & 1;
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      unsigned sel = 0;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const unsigned lo = av::wave_sum(w16[j][m] & 0xFFFFu);
        const unsigned hi = av::wave_sum(w16[j][m] >> 16);
        if (m == mi) sel = half ? hi : lo;
        w16[j][m] = 0;
      }
      int dst;
      if (j < NM) {
        dst = (j * C + (l >> 2)) * 8 + (l & 3);  // slot 4c + code
      } else {
        const int k = NM + (j - NM) / C, c = (j - NM) % C;
        dst = (k * C + c) * 8 + l;
      }
      if (l < 8) my_tab[dst] += sel;
    }
  };

  const long long nvec = n >> 3;  // 8 records per 16-byte load
  const long long ntiles = (nvec + AV_WAVE - 1) / AV_WAVE;
  const long long gw = (long long)blockIdx.x * WPB + av::wave_id();
  const long long nw = (long long)gridDim.x * WPB;
  int since_flush = 0, flushes = 0;
  // two tiles per iteration, and the next iteration's two 16-byte loads in flight while these
  // are counted (counting costs ~22 VALU ops per record, so loads must run well ahead)
  auto count = [&](const uint4 q) __attribute__((always_inline)) {
    const unsigned dw[4] = {q.x, q.y, q.z, q.w};
    if (C == 1) {
#pragma unroll
      for (int h = 0; h < 8; ++h) {
        const unsigned d = dw[h >> 1];
        const int o = 16 * (h & 1);  // record h sits in bits [o, o + 16) of its dword
#pragma unroll
        for (int k = 0; k < NF; ++k)
          lshl_add_u32(a4[k], 1u, __builtin_amdgcn_ubfe(d, (unsigned)(spec.sh[k] + o), (unsigned)spec.w[k]) << 2);
      }
    } else {
      // two records per dword: class one-hot bits at 0-1 / 16-17 and every field at bit >= 2,
      // so (d >> (sh - 2)) & mask puts 4 * code of both records at bits 2-4 / 18-20 in two ops
      // (v_lshl_add_u32 reads only bits [4:0] of its shift operand)
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const unsigned d = dw[h];
        const unsigned x0a = d & 1u, x1a = __builtin_amdgcn_ubfe(d, 1u, 1u);
        const unsigned x0b = __builtin_amdgcn_ubfe(d, 16u, 1u), x1b = __builtin_amdgcn_ubfe(d, 17u, 1u);
        const unsigned va = x0a | x1a, vb = x0b | x1b;  // known class
        const unsigned c16 = (d << 3) & 0x00100010u;    // class 1: slot + 4 = nibble shift + 16
#pragma unroll
        for (int k = 0; k < NF; ++k) {
          const unsigned t = (d >> (unsigned)(spec.sh[k] - 2)) & m4[k];
          if (k < NM) {
            const unsigned sm = t | c16;
            lshl_add_u32(a4[k], va, sm);
            lshl_add_u32(a4[k], vb, sm >> 16);
          } else {
            const int j = NM + (k - NM) * C;
            const unsigned tb = t >> 16;
            lshl_add_u32(a4[j], x0a, t);
            lshl_add_u32(a4[j + 1], x1a, t);
            lshl_add_u32(a4[j], x0b, tb);
            lshl_add_u32(a4[j + 1], x1b, tb);
          }
        }
      }
    }
    };
  const long long vstride = nw * AV_WAVE;
  long long v = gw * AV_WAVE + av::lane_id();
  const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
  uint4 qa = (gw < ntiles && v < nvec) ? w4[v] : z4;
  uint4 qb = (gw + nw < ntiles && v + vstride < nvec) ? w4[v + vstride] : z4;
  for (long long t = gw; t < ntiles; t += 2 * nw) {
    const uint4 q0 = qa, q1 = qb;
    const bool h0 = v < nvec, h1 = t + nw < ntiles && v + vstride < nvec;
    v += 2 * vstride;
    if (t + 2 * nw < ntiles && v < nvec) qa = w4[v];
    if (t + 3 * nw < ntiles && v + vstride < nvec) qb = w4[v + vstride];
    if (h0) count(q0);
    spread();
    if (h1) count(q1);
    spread();
    since_flush += 2;
    if (since_flush >= FLUSH - 1) {  // wave-uniform; <= 30 tiles x 8 records per byte counter
      widen();
      since_flush = 0;
      if (++flushes == 256) {
        reduce_to_lds();
        flushes = 0;
      }
    }
  }
  widen();
  reduce_to_lds();

  if (blockIdx.x == 0) {  // tail records (n % 8), once every wave's slice is final
    __syncthreads();
    for (long long r = nvec * 8 + threadIdx.x; r < n; r += HB) {
      const unsigned w = words[r];
#pragma unroll
      for (int c = 0; c < C; ++c) {
        if (C > 1 && !__builtin_amdgcn_ubfe(w, (unsigned)(spec.lsh + c), 1u)) continue;
#pragma unroll
        for (int k = 0; k < NF; ++k)
          atomicAdd(&s_tab[(k * C + c) * 8 + __builtin_amdgcn_ubfe(w, (unsigned)spec.sh[k], (unsigned)spec.w[k])], 1u);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < TAB; i += HB) {
    unsigned long long tot = 0;
#pragma unroll
    for (int w = 0; w < WPB; ++w) tot += s_tab[w * TAB + i];
    s_tab[i] = (unsigned)tot;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < TAB; i += HB) {
    const int k = i / (C * 8), c = (i / 8) % C, b = i % 8;
    const unsigned cnt = s_tab[i];
    if (cnt && b < bins[k]) atomicAdd(&out[(long long)c * total_bins + offs[k] + b], (unsigned long long)cnt);
  }
  if (count_labels && threadIdx.x < C) {  // every record of a class has exactly one feature-0 code
    unsigned long long sum = 0;
#pragma unroll
    for (int b = 0; b < 8; ++b) sum += s_tab[(0 * C + threadIdx.x) * 8 + b];
    if (sum) atomicAdd(&out[(long long)threadIdx.x * total_bins + total_bins - 1], sum);
  }
}


// ---------------------------------------------------------------------------------------------
// K2 joint variant for row-packed records of at most 15 bits: every record is ONE LDS atomic into
// the block's 2^bits joint table (record value -> count); the class-conditional marginals are
// taken from that table once per block (2^bits entries x F fields, LDS atomics into a [C][TB]
// table) and flushed with one global atomic per non-zero count.  Per record this is one
// ds_add_u32 instead of ~22 VALU ops (hist_rowpack_kernel), so the pass is no longer VALU-issue
// bound.  The record words are the same as pack_rows'.
// ---------------------------------------------------------------------------------------------
// Record value -> LDS slot: the low 6 bits (the LDS bank) XOR-folded with bits 6-11 and 12-17, so
// the bank depends on every field, not only on the class bits and the first fields (which take few
// distinct values); bits >= 6 are unchanged, so the map is a bijection and its own inverse.
__device__ __forceinline__ unsigned joint_slot(unsigned j) {
  return j ^ __builtin_amdgcn_ubfe(j, 6u, 6u) ^ __builtin_amdgcn_ubfe(j, 12u, 6u);  // 2 v_bfe + v_xor3
}

__global__ __launch_bounds__(HB) void hist_joint_kernel(const uint16_t* __restrict__ words, long long n, int nbits,
                                                        RowPackSpec spec, int nfeat, int n_classes,
                                                        const int* __restrict__ bins, const int* __restrict__ offs,
                                                        int total_bins, int count_labels,
                                                        unsigned long long* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned int s_joint[];
  unsigned int* s_small = s_joint + (1 << nbits);  // [C][total_bins]
  const int J = 1 << nbits;
  const unsigned mask = (unsigned)J - 1u;
  for (int i = threadIdx.x; i < J + n_classes * total_bins; i += HB) s_joint[i] = 0;
  __syncthreads();
  const uint4* w4 = reinterpret_cast<const uint4*>(words);
  const long long nvec = n >> 3;
  const long long stride = (long long)gridDim.x * HB;
  long long v = (long long)blockIdx.x * HB + threadIdx.x;
  uint4 q = v < nvec ? w4[v] : make_uint4(0u, 0u, 0u, 0u);
  for (; v < nvec; v += stride) {
    const uint4 cur = q;
    if (v + stride < nvec) q = w4[v + stride];  // next vector in flight while this one is counted
    const unsigned dw[4] = {cur.x, cur.y, cur.z, cur.w};
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      atomicAdd(&s_joint[joint_slot(dw[h] & mask)], 1u);
      atomicAdd(&s_joint[joint_slot((dw[h] >> 16) & mask)], 1u);
    }
  }
  if (blockIdx.x == 0)
    for (long long r = nvec * 8 + threadIdx.x; r < n; r += HB) atomicAdd(&s_joint[joint_slot(words[r] & mask)], 1u);
  __syncthreads();
  for (int p = threadIdx.x; p < J; p += HB) {
    const unsigned cnt = s_joint[p];
    if (!cnt) continue;
    const int j = (int)joint_slot((unsigned)p);  // the slot map is its own inverse
    int c = 0;
    if (n_classes > 1) {
      const unsigned lb = __builtin_amdgcn_ubfe((unsigned)j, (unsigned)spec.lsh, (unsigned)n_classes);
      if (lb == 1u) c = 0;
      else if (lb == 2u) c = 1;
      else continue;  // unknown class: not counted (as in the column histogram)
    }
    unsigned int* row = s_small + c * total_bins;
    for (int k = 0; k < nfeat; ++k) {
      const int code = (int)__builtin_amdgcn_ubfe((unsigned)j, (unsigned)spec.sh[k], (unsigned)spec.w[k]);
      if (code < bins[k]) atomicAdd(&row[offs[k] + code], cnt);
    }
    if (count_labels) atomicAdd(&row[total_bins - 1], cnt);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n_classes * total_bins; i += HB) {
    const unsigned cnt = s_small[i];
    if (cnt) atomicAdd(&out[i], (unsigned long long)cnt);
  }
}


// Dense variant: records of B bits packed back to back, 32 records per B dwords (a lane's group),
// so a 2^30-record churn table (B = 13) streams 1.63 B/record instead of 2.  Each lane loads its
// group's B dwords (consecutive lanes read consecutive groups) and extracts the 32 records at
// compile-time bit offsets (one v_bfe, or v_alignbit across a dword boundary).  Records at index
// >= n (the last group's padding) are skipped.
// R replicas of the joint table, interleaved (slot * R + lane % R): lanes of different residues
// never share a bank, which divides the LDS atomic conflicts of random records by about R; NT
// threads per block keep enough waves per CU when the replicated table limits blocks per CU.
template <int B, int R, int NT>
__global__ __launch_bounds__(NT) void hist_joint_dense_kernel(const uint32_t* __restrict__ dense, long long n,
                                                              RowPackSpec spec, int nfeat, int n_classes,
                                                              const int* __restrict__ bins,
                                                              const int* __restrict__ offs, int total_bins,
                                                              int count_labels, unsigned long long* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned int s_joint[];
  constexpr int J = 1 << B;
  constexpr unsigned M = (unsigned)J - 1u;
  unsigned int* s_small = s_joint + J * R;
  for (int i = threadIdx.x; i < J * R + n_classes * total_bins; i += NT) s_joint[i] = 0;
  const unsigned rep = threadIdx.x & (R - 1);
  // xorshift slot map j ^ (j >> S), S = the bank bits left to the record (5 - log2 R): the bank then
  // depends on two groups of fields; a bijection, inverted below by xor-ing all shifts of S
  constexpr int S = R == 4 ? 3 : (R == 2 ? 4 : 5);
  __syncthreads();
  const long long groups = (n + 31) >> 5;
  const long long stride = (long long)gridDim.x * NT;
  for (long long g = (long long)blockIdx.x * NT + threadIdx.x; g < groups; g += stride) {
    uint32_t d[B + 1];
    const uint32_t* src = dense + g * B;
#pragma unroll
    for (int i = 0; i < B; ++i) d[i] = src[i];
    d[B] = 0;
    const long long left = n - (g << 5);
    auto rec = [&](int k) __attribute__((always_inline)) -> unsigned {
      const int bit = k * B, i = bit >> 5, sh = bit & 31;
      if (sh + B <= 32) return __builtin_amdgcn_ubfe(d[i], (unsigned)sh, (unsigned)B);
      return __builtin_amdgcn_alignbit(d[i + 1], d[i], (unsigned)sh) & M;
    };
    if (left >= 32) {  // every group but the last: no per-record predicate
#pragma unroll
      for (int k = 0; k < 32; ++k) {
        const unsigned r = rec(k);
        atomicAdd(&s_joint[(r ^ (r >> S)) * R + rep], 1u);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 32; ++k)
        if (k < left) {
        const unsigned r = rec(k);
        atomicAdd(&s_joint[(r ^ (r >> S)) * R + rep], 1u);
      }
    }
  }
  __syncthreads();
  for (int p = threadIdx.x; p < J; p += NT) {
    unsigned cnt = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) cnt += s_joint[p * R + r];
    if (!cnt) continue;
    unsigned ju = (unsigned)p;
#pragma unroll
    for (int t = S; t < B; t += S) ju ^= (unsigned)p >> t;
    const int j = (int)ju;
    int c = 0;
    if (n_classes > 1) {
      const unsigned lb = __builtin_amdgcn_ubfe((unsigned)j, (unsigned)spec.lsh, (unsigned)n_classes);
      if (lb == 1u) c = 0;
      else if (lb == 2u) c = 1;
      else continue;
    }
    unsigned int* row = s_small + c * total_bins;
    for (int kf = 0; kf < nfeat; ++kf) {
      const int code = (int)__builtin_amdgcn_ubfe((unsigned)j, (unsigned)spec.sh[kf], (unsigned)spec.w[kf]);
      if (code < bins[kf]) atomicAdd(&row[offs[kf] + code], cnt);
    }
    if (count_labels) atomicAdd(&row[total_bins - 1], cnt);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n_classes * total_bins; i += NT) {
    const unsigned cnt = s_small[i];
    if (cnt) atomicAdd(&out[i], (unsigned long long)cnt);
  }
}

// dense[g * B + i]: record k of group g at bits [k B, k B + B) of the group's B dwords
__global__ __launch_bounds__(HB) void pack_dense_kernel(const uint16_t* __restrict__ words, long long n, int B,
                                                        uint32_t* __restrict__ dense) {
  const long long groups = (n + 31) >> 5;
  const long long stride = (long long)gridDim.x * HB;
  for (long long g = (long long)blockIdx.x * HB + threadIdx.x; g < groups; g += stride) {
    uint32_t d[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) d[i] = 0;
    for (int k = 0; k < 32; ++k) {
      const long long r = (g << 5) + k;
      const uint32_t v = r < n ? ((uint32_t)words[r] & ((1u << B) - 1u)) : 0u;
      const int bit = k * B, i = bit >> 5, sh = bit & 31;
#pragma unroll
      for (int q = 0; q < 16; ++q) {  // register-indexed writes unrolled (no scratch)
        if (q == i) d[q] |= v << sh;
        if (q == i + 1 && sh + B > 32) d[q] |= v >> (32 - sh);
      }
    }
    for (int i = 0; i < B; ++i) dense[g * B + i] = d[i];
  }
}

int hist_joint_lds(int nbits, int n_classes, int total_bins) {
  return (int)(sizeof(unsigned) * ((size_t(1) << nbits) + (size_t)n_classes * total_bins));
}

struct RowPackLaunch {
  const uint16_t* words;
  long long n;
  RowPackSpec spec;
  const int* bins;
  const int* offs;
  int total_bins, count_labels;
  unsigned long long* out;
  hipStream_t stream;
};

template <int NF, int C, int NM>
void launch_rowpack(const RowPackLaunch& a) {
  static const int res = av::resident_blocks((const void*)hist_rowpack_kernel<NF, C, NM>, HB, 0);
  const int grid = std::min(av::stream_grid(std::max(1LL, a.n >> 3), HB, 4, 4096), res);
  hist_rowpack_kernel<NF, C, NM><<<grid, HB, 0, a.stream>>>(a.words, a.n, a.spec, a.bins, a.offs, a.total_bins,
                                                            a.count_labels, a.out);
  AV_HIP_CHECK(hipGetLastError());
}

template <int NF, int NM>
void launch_rowpack_c2(int nm, const RowPackLaunch& a) {
  if constexpr (NM > NF) {
    throw std::runtime_error("row-packed histogram: bad merged-feature count");
  } else {
    if (nm == NM) launch_rowpack<NF, 2, NM>(a);
    else launch_rowpack_c2<NF, NM + 1>(nm, a);
  }
}

template <int NF>
void launch_rowpack_nf(int n_classes, int nm, const RowPackLaunch& a) {
  if (n_classes == 1) launch_rowpack<NF, 1, 0>(a);
  else launch_rowpack_c2<NF, 0>(nm, a);
}

// General path: LDS-privatised table with R replicas (one per wave when it fits) so that lanes of
// different waves never contend; replicas are summed once per block.
__global__ __launch_bounds__(HB) void hist_lds_kernel(
    const uint8_t* __restrict__ codes, long long ld, long long n, const uint8_t* __restrict__ labels,
    const int* __restrict__ bins, const int* __restrict__ offs, int nfeat, int total_bins,
    int n_classes, int count_labels, int replicas, unsigned long long* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned int s_tab[];
  const int tab = n_classes * total_bins;
  for (int i = threadIdx.x; i < tab * replicas; i += HB) s_tab[i] = 0;
  __syncthreads();
  unsigned int* my = s_tab + (av::wave_id() % replicas) * tab;
  const long long stride = (long long)gridDim.x * HB;
  for (long long r = (long long)blockIdx.x * HB + threadIdx.x; r < n; r += stride) {
    const unsigned c = labels ? labels[r] : 0u;
    if (c >= (unsigned)n_classes) continue;
    for (int f = 0; f < nfeat; ++f) {
      const unsigned v = codes[(long long)f * ld + r];
      if (v < (unsigned)bins[f]) atomicAdd(&my[c * total_bins + offs[f] + v], 1u);
    }
    if (count_labels) atomicAdd(&my[c * total_bins + total_bins - 1], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < tab; i += HB) {
    unsigned long long s = 0;
    for (int q = 0; q < replicas; ++q) s += s_tab[q * tab + i];
    if (s) atomicAdd(&out[i], s);
  }
}

// Fallback for tables larger than LDS: global 64-bit atomics.
__global__ __launch_bounds__(HB) void hist_global_kernel(
    const uint8_t* __restrict__ codes, long long ld, long long n, const uint8_t* __restrict__ labels,
    const int* __restrict__ bins, const int* __restrict__ offs, int nfeat, int total_bins,
    int n_classes, int count_labels, unsigned long long* __restrict__ out) {
  const long long stride = (long long)gridDim.x * HB;
  for (long long r = (long long)blockIdx.x * HB + threadIdx.x; r < n; r += stride) {
    const unsigned c = labels ? labels[r] : 0u;
    if (c >= (unsigned)n_classes) continue;
    for (int f = 0; f < nfeat; ++f) {
      const unsigned v = codes[(long long)f * ld + r];
      if (v < (unsigned)bins[f])
        atomicAdd(&out[(long long)c * total_bins + offs[f] + v], 1ull);
    }
    if (count_labels) atomicAdd(&out[(long long)c * total_bins + total_bins - 1], 1ull);
  }
}

// ---------------------------------------------------------------------------------------------
// K3: pair histograms.  pairs[p] = (fa, fb); out[p][c][ba][bb] at offset poff[p].
// grid = (row_blocks, n_pairs); LDS table per block (replicated per wave when it fits).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(HB) void pair_hist_kernel(
    const uint8_t* __restrict__ codes, long long ld, long long n, const uint8_t* __restrict__ labels,
    const int* __restrict__ bins, const int* __restrict__ pairs, const long long* __restrict__ poff,
    int n_classes, int replicas, unsigned long long* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned int s_tab[];
  const int p = blockIdx.y;
  const int fa = pairs[2 * p], fb = pairs[2 * p + 1];
  const int Ba = bins[fa], Bb = bins[fb];
  const int tab = n_classes * Ba * Bb;
  for (int i = threadIdx.x; i < tab * replicas; i += HB) s_tab[i] = 0;
  __syncthreads();
  unsigned int* my = s_tab + (av::wave_id() % replicas) * tab;
  const uint8_t* ca = codes + (long long)fa * ld;
  const uint8_t* cb = codes + (long long)fb * ld;
  const long long stride = (long long)gridDim.x * HB;
  for (long long r = (long long)blockIdx.x * HB + threadIdx.x; r < n; r += stride) {
    const unsigned c = labels ? labels[r] : 0u;
    const unsigned a = ca[r], b = cb[r];
    if (c < (unsigned)n_classes && a < (unsigned)Ba && b < (unsigned)Bb)
      atomicAdd(&my[(c * Ba + a) * Bb + b], 1u);
  }
  __syncthreads();
  unsigned long long* o = out + poff[p];
  for (int i = threadIdx.x; i < tab; i += HB) {
    unsigned long long s = 0;
    for (int q = 0; q < replicas; ++q) s += s_tab[q * tab + i];
    if (s) atomicAdd(&o[i], s);
  }
}

// ---------------------------------------------------------------------------------------------
// K4: Markov bigram counts.  states int16 [N][L] row-major (padding value < 0 ends a sequence),
// labels (optional) uint8 [N] select one of C models.  out[c][s][s'].
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(HB) void bigram_kernel(const int16_t* __restrict__ st, long long n,
                                                    int L, const uint8_t* __restrict__ labels,
                                                    int n_classes, int S, int replicas,
                                                    unsigned long long* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned int s_tab[];
  const int tab = n_classes * S * S;
  const bool use_lds = replicas > 0;
  if (use_lds) {
    for (int i = threadIdx.x; i < tab * replicas; i += HB) s_tab[i] = 0;
    __syncthreads();
  }
  unsigned int* my = use_lds ? s_tab + (av::wave_id() % replicas) * tab : nullptr;
  const long long total = n * (long long)(L - 1);
  const long long stride = (long long)gridDim.x * HB;
  for (long long e = (long long)blockIdx.x * HB + threadIdx.x; e < total; e += stride) {
    const long long r = e / (L - 1);
    const int j = (int)(e - r * (L - 1));
    const int a = st[r * L + j], b = st[r * L + j + 1];
    if (a < 0 || b < 0 || a >= S || b >= S) continue;
    const unsigned c = labels ? labels[r] : 0u;
    if (c >= (unsigned)n_classes) continue;
    const int idx = (c * S + a) * S + b;
    if (use_lds) atomicAdd(&my[idx], 1u);
    else atomicAdd(&out[idx], 1ull);
  }
  if (use_lds) {
    __syncthreads();
    for (int i = threadIdx.x; i < tab; i += HB) {
      unsigned long long s = 0;
      for (int q = 0; q < replicas; ++q) s += s_tab[q * tab + i];
      if (s) atomicAdd(&out[i], s);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Class-conditional moments (count, sum, sum of squares) of continuous features — deterministic:
// per-block partials in a fixed order, then an ordered cross-block reduction (no float atomics).
// x f32 [F][ld]; part f64 [blocks][C][F][3]; out f64 [C][F][3].
// ---------------------------------------------------------------------------------------------
constexpr int MC = 8;  // classes per pass held in registers

__global__ __launch_bounds__(HB) void moments_partial_kernel(
    const float* __restrict__ x, long long ld, long long n, int nfeat,
    const uint8_t* __restrict__ labels, int c0, int nc, int n_classes, double* __restrict__ part) {
  __shared__ double s_red[HB / AV_WAVE][MC][3];
  const long long per_block = (n + gridDim.x - 1) / gridDim.x;
  const long long r0 = (long long)blockIdx.x * per_block;
  const long long r1 = min(n, r0 + per_block);
  for (int f = 0; f < nfeat; ++f) {
    double cnt[MC], sm[MC], sq[MC];
#pragma unroll
    for (int k = 0; k < MC; ++k) { cnt[k] = 0; sm[k] = 0; sq[k] = 0; }
    const float* xf = x + (long long)f * ld;
    for (long long r = r0 + threadIdx.x; r < r1; r += HB) {
      const int c = (labels ? (int)labels[r] : 0) - c0;
      const double v = (double)xf[r];
#pragma unroll
      for (int k = 0; k < MC; ++k) {
        const bool m = (k == c) && (k < nc);
        cnt[k] += m ? 1.0 : 0.0;
        sm[k] += m ? v : 0.0;
        sq[k] += m ? v * v : 0.0;
      }
    }
#pragma unroll
    for (int k = 0; k < MC; ++k) {
      cnt[k] = av::wave_sum(cnt[k]);
      sm[k] = av::wave_sum(sm[k]);
      sq[k] = av::wave_sum(sq[k]);
    }
    if (av::lane_id() == 0) {
#pragma unroll
      for (int k = 0; k < MC; ++k) {
        s_red[av::wave_id()][k][0] = cnt[k];
        s_red[av::wave_id()][k][1] = sm[k];
        s_red[av::wave_id()][k][2] = sq[k];
      }
    }
    __syncthreads();
    if (threadIdx.x < nc * 3) {
      const int k = threadIdx.x / 3, q = threadIdx.x % 3;
      double s = 0;
      for (int w = 0; w < HB / AV_WAVE; ++w) s += s_red[w][k][q];
      part[(((long long)blockIdx.x * n_classes + (c0 + k)) * nfeat + f) * 3 + q] = s;
    }
    __syncthreads();
  }
}

__global__ void moments_reduce_kernel(const double* __restrict__ part, int nblocks, int len,
                                      double* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= len) return;
  double s = 0;
  for (int b = 0; b < nblocks; ++b) s += part[(long long)b * len + i];
  out[i] += s;
}

}  // namespace

// ============================================================================================
// host launchers
// ============================================================================================
namespace avk {

void class_histogram(const uint8_t* codes, long long ld, long long n, const uint8_t* labels,
                     const int* d_bins, const int* d_offs, const int* h_bins, int nfeat,
                     int total_bins, int n_classes, int count_labels, unsigned long long* out,
                     int mode, hipStream_t stream) {
  if (n <= 0 || (nfeat <= 0 && !count_labels)) return;
  int max_cb = 0;
  for (int f = 0; f < nfeat; ++f) max_cb = std::max(max_cb, n_classes * h_bins[f]);
  const bool aligned = (ld % 16 == 0) && ((uintptr_t)codes % 16 == 0) &&
                       (labels == nullptr || (uintptr_t)labels % 16 == 0);
  int max_b = 0;
  for (int f = 0; f < nfeat; ++f) max_b = std::max(max_b, h_bins[f]);
  if (mode == 0 && aligned && nfeat > 0 && max_b <= 7 && n_classes <= 4) {
    const uint8_t* lab = n_classes > 1 ? labels : nullptr;
    if (n_classes > 1 && labels == nullptr) n_classes = 1;
    switch (n_classes) {
      case 1: launch_split<1>(codes, ld, n, lab, d_bins, d_offs, nfeat, total_bins, count_labels, out, stream); break;
      case 2: launch_split<2>(codes, ld, n, lab, d_bins, d_offs, nfeat, total_bins, count_labels, out, stream); break;
      case 3: launch_split<3>(codes, ld, n, lab, d_bins, d_offs, nfeat, total_bins, count_labels, out, stream); break;
      default: launch_split<4>(codes, ld, n, lab, d_bins, d_offs, nfeat, total_bins, count_labels, out, stream); break;
    }
    return;
  }
  if ((mode == 0 || mode == 3) && max_cb <= 16 && n_classes <= 16 && aligned && nfeat > 0) {
    const long long nvec = n >> 4;
    const int grid = av::stream_grid(std::max(1LL, nvec), HB, 4, 2048);
    for (int f0 = 0; f0 < nfeat; f0 += 8) {
      const int nf = std::min(8, nfeat - f0);
      if (nf <= 1)
        hist_packed_kernel<1><<<grid, HB, 0, stream>>>(codes, ld, n, labels, d_bins, d_offs, f0, nf,
                                                      total_bins, n_classes, count_labels, out);
      else if (nf <= 2)
        hist_packed_kernel<2><<<grid, HB, 0, stream>>>(codes, ld, n, labels, d_bins, d_offs, f0, nf,
                                                      total_bins, n_classes, count_labels, out);
      else if (nf <= 4)
        hist_packed_kernel<4><<<grid, HB, 0, stream>>>(codes, ld, n, labels, d_bins, d_offs, f0, nf,
                                                      total_bins, n_classes, count_labels, out);
      else
        hist_packed_kernel<8><<<grid, HB, 0, stream>>>(codes, ld, n, labels, d_bins, d_offs, f0, nf,
                                                      total_bins, n_classes, count_labels, out);
      AV_HIP_CHECK(hipGetLastError());
    }
    return;
  }
  const long long tab_bytes = 4LL * n_classes * total_bins;
  const int grid = av::stream_grid(n, HB, 8, 2048);
  if (mode != 2 && tab_bytes <= 64 * 1024) {
    int replicas = (int)std::min<long long>(HB / AV_WAVE, (64 * 1024) / tab_bytes);
    replicas = std::max(1, replicas);
    hist_lds_kernel<<<grid, HB, tab_bytes * replicas, stream>>>(codes, ld, n, labels, d_bins, d_offs,
                                                               nfeat, total_bins, n_classes,
                                                               count_labels, replicas, out);
  } else {
    hist_global_kernel<<<grid, HB, 0, stream>>>(codes, ld, n, labels, d_bins, d_offs, nfeat,
                                                total_bins, n_classes, count_labels, out);
  }
  AV_HIP_CHECK(hipGetLastError());
}

void pair_histogram(const uint8_t* codes, long long ld, long long n, const uint8_t* labels,
                    const int* d_bins, const int* d_pairs, const long long* d_poff, int n_pairs,
                    int max_tab, int n_classes, unsigned long long* out, hipStream_t stream) {
  if (n <= 0 || n_pairs <= 0) return;
  const long long tab_bytes = 4LL * max_tab;
  if (tab_bytes > 160 * 1024) throw std::runtime_error("pair_histogram: table exceeds LDS");
  int replicas = (int)std::max<long long>(1, std::min<long long>(HB / AV_WAVE, (64 * 1024) / tab_bytes));
  const int rows_blocks = std::max(1, std::min(1024, (int)((n + HB * 16 - 1) / (HB * 16))));
  const int gx = std::max(1, std::min(rows_blocks, std::max(1, 2048 / n_pairs)));
  dim3 grid(gx, n_pairs);
  pair_hist_kernel<<<grid, HB, tab_bytes * replicas, stream>>>(codes, ld, n, labels, d_bins, d_pairs,
                                                              d_poff, n_classes, replicas, out);
  AV_HIP_CHECK(hipGetLastError());
}

void bigram_histogram(const int16_t* states, long long n, int L, const uint8_t* labels,
                      int n_classes, int S, unsigned long long* out, hipStream_t stream) {
  if (n <= 0 || L < 2) return;
  const long long tab_bytes = 4LL * n_classes * S * S;
  int replicas = 0;
  if (tab_bytes <= 64 * 1024)
    replicas = (int)std::max<long long>(1, std::min<long long>(HB / AV_WAVE, (64 * 1024) / tab_bytes));
  const int grid = av::stream_grid(n * (L - 1), HB, 8, 2048);
  bigram_kernel<<<grid, HB, replicas ? tab_bytes * replicas : 0, stream>>>(states, n, L, labels,
                                                                           n_classes, S, replicas, out);
  AV_HIP_CHECK(hipGetLastError());
}

void class_moments(const float* x, long long ld, long long n, int nfeat, const uint8_t* labels,
                   int n_classes, double* part, int nblocks, double* out, hipStream_t stream) {
  if (n <= 0 || nfeat <= 0) return;
  for (int c0 = 0; c0 < n_classes; c0 += MC) {
    const int nc = std::min(MC, n_classes - c0);
    moments_partial_kernel<<<nblocks, HB, 0, stream>>>(x, ld, n, nfeat, labels, c0, nc, n_classes,
                                                        part);
    AV_HIP_CHECK(hipGetLastError());
  }
  const int len = n_classes * nfeat * 3;
  moments_reduce_kernel<<<(len + 255) / 256, 256, 0, stream>>>(part, nblocks, len, out);
  AV_HIP_CHECK(hipGetLastError());
}

int moments_blocks(long long n) { return av::stream_grid(n, HB, 16, 1024); }

void class_histogram_rowpacked(const uint16_t* words, long long n, const int* h_shift, const int* h_width, int nfeat,
                               int label_shift, int label_width, const int* d_bins, const int* d_offs, int total_bins,
                               int n_classes, int count_labels, unsigned long long* out, hipStream_t stream) {
  if (n <= 0 || nfeat <= 0) return;
  if (nfeat > 8 || n_classes < 1 || n_classes > 2) throw std::runtime_error("row-packed histogram: F <= 8, C <= 2");
  RowPackSpec spec{};
  for (int k = 0; k < nfeat; ++k) {
    if (h_width[k] < 1 || h_width[k] > 3) throw std::runtime_error("row-packed histogram: field widths 1..3 bits");
    spec.sh[k] = h_shift[k];
    spec.w[k] = h_width[k];
  }
  if (n_classes > 1 && (label_width != n_classes || label_shift != 0))
    throw std::runtime_error("row-packed histogram: the class is C one-hot bits at bit 0");
  for (int k = 0; k < nfeat; ++k)
    if (n_classes > 1 && h_shift[k] < 2) throw std::runtime_error("row-packed histogram: fields start at bit 2");
  spec.lsh = n_classes > 1 ? label_shift : 0;
  int nm = 0;  // leading features whose (class, code) share one slot (kernel order puts them first)
  if (n_classes == 2)
    while (nm < nfeat && h_width[nm] <= 2) ++nm;
  // records of <= 15 bits: one LDS atomic per record into the joint table (AVMI_ROWPACK_KERNEL=nibble
  // keeps the VALU nibble-counter kernel)
  int nbits = n_classes > 1 ? label_shift + label_width : 1;
  for (int k = 0; k < nfeat; ++k) nbits = std::max(nbits, h_shift[k] + h_width[k]);
  const char* kenv = std::getenv("AVMI_ROWPACK_KERNEL");
  const bool force_nibble = kenv && std::string(kenv) == "nibble";
  const int jlds = hist_joint_lds(nbits, n_classes, total_bins);
  if (!force_nibble && nbits <= 15 && jlds <= 136 * 1024) {
    if (jlds > 64 * 1024)
      AV_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(hist_joint_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, jlds));
    const int res = av::resident_blocks((const void*)hist_joint_kernel, HB, (size_t)jlds);
    const int grid = std::max(1, std::min(av::stream_grid(std::max(1LL, n >> 3), HB, 4, 4096), res));
    hist_joint_kernel<<<grid, HB, (size_t)jlds, stream>>>(words, n, nbits, spec, nfeat, n_classes, d_bins, d_offs,
                                                          total_bins, count_labels, out);
    AV_HIP_CHECK(hipGetLastError());
    return;
  }
  const RowPackLaunch a{words, n, spec, d_bins, d_offs, total_bins, count_labels, out, stream};
  switch (nfeat) {
    case 1: launch_rowpack_nf<1>(n_classes, nm, a); break;
    case 2: launch_rowpack_nf<2>(n_classes, nm, a); break;
    case 3: launch_rowpack_nf<3>(n_classes, nm, a); break;
    case 4: launch_rowpack_nf<4>(n_classes, nm, a); break;
    case 5: launch_rowpack_nf<5>(n_classes, nm, a); break;
    case 6: launch_rowpack_nf<6>(n_classes, nm, a); break;
    case 7: launch_rowpack_nf<7>(n_classes, nm, a); break;
    default: launch_rowpack_nf<8>(n_classes, nm, a); break;
  }
}


long long dense_words(long long n, int B) { return ((n + 31) >> 5) * (long long)B; }

void pack_dense(const uint16_t* words, long long n, int B, uint32_t* dense, hipStream_t stream) {
  if (n <= 0) return;
  if (B < 1 || B > 15) throw std::runtime_error("pack_dense: 1..15 bits per record");
  pack_dense_kernel<<<av::stream_grid((n + 31) >> 5, HB, 1, 4096), HB, 0, stream>>>(words, n, B, dense);
  AV_HIP_CHECK(hipGetLastError());
}

template <int B, int R, int NT>
static void launch_joint_dense_r(const uint32_t* dense, long long n, const RowPackSpec& spec, int nfeat, int n_classes,
                                 const int* bins, const int* offs, int total_bins, int count_labels,
                                 unsigned long long* out, hipStream_t stream) {
  const int lds = (int)(sizeof(unsigned) * ((size_t)R * (size_t(1) << B) + (size_t)n_classes * total_bins));
  if (lds > 160 * 1024) throw std::runtime_error("dense histogram: replicated table exceeds LDS");
  auto kern = hist_joint_dense_kernel<B, R, NT>;
  if (lds > 64 * 1024)
    AV_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                     lds));
  const int res = av::resident_blocks((const void*)kern, NT, (size_t)lds);
  const int grid = std::max(1, std::min(av::stream_grid(std::max(1LL, (n + 31) >> 5), NT, 1, 8192), res));
  kern<<<grid, NT, (size_t)lds, stream>>>(dense, n, spec, nfeat, n_classes, bins, offs, total_bins, count_labels, out);
  AV_HIP_CHECK(hipGetLastError());
}

// replicas: AVMI_JOINT_REPLICAS (1, 2 or 4), else the most that fit 128 KiB of LDS
template <int B>
static void launch_joint_dense(const uint32_t* dense, long long n, const RowPackSpec& spec, int nfeat, int n_classes,
                               const int* bins, const int* offs, int total_bins, int count_labels,
                               unsigned long long* out, hipStream_t stream) {
  int R = (B <= 13) ? 4 : (B == 14 ? 2 : 1);
  if (const char* e = std::getenv("AVMI_JOINT_REPLICAS")) R = std::atoi(e);
  if (R >= 4 && B <= 13)
    launch_joint_dense_r<B, 4, 1024>(dense, n, spec, nfeat, n_classes, bins, offs, total_bins, count_labels, out, stream);
  else if (R >= 2 && B <= 14)
    launch_joint_dense_r<B, 2, 512>(dense, n, spec, nfeat, n_classes, bins, offs, total_bins, count_labels, out, stream);
  else
    launch_joint_dense_r<B, 1, HB>(dense, n, spec, nfeat, n_classes, bins, offs, total_bins, count_labels, out, stream);
}

void class_histogram_dense(const uint32_t* dense, long long n, int B, const int* h_shift, const int* h_width,
                           int nfeat, int label_shift, int label_width, const int* d_bins, const int* d_offs,
                           int total_bins, int n_classes, int count_labels, unsigned long long* out,
                           hipStream_t stream) {
  if (n <= 0 || nfeat <= 0) return;
  if (nfeat > 8 || n_classes < 1 || n_classes > 2) throw std::runtime_error("dense histogram: F <= 8, C <= 2");
  if (n_classes > 1 && (label_width != n_classes || label_shift != 0))
    throw std::runtime_error("dense histogram: the class is C one-hot bits at bit 0");
  RowPackSpec spec{};
  int need = n_classes > 1 ? label_width : 1;
  for (int k = 0; k < nfeat; ++k) {
    spec.sh[k] = h_shift[k];
    spec.w[k] = h_width[k];
    need = std::max(need, h_shift[k] + h_width[k]);
  }
  spec.lsh = n_classes > 1 ? label_shift : 0;
  if (need > B) throw std::runtime_error("dense histogram: fields exceed the record width");
  switch (B) {
#define AV_DENSE(BB) \
  case BB: launch_joint_dense<BB>(dense, n, spec, nfeat, n_classes, d_bins, d_offs, total_bins, count_labels, out, stream); break;
    AV_DENSE(4) AV_DENSE(5) AV_DENSE(6) AV_DENSE(7) AV_DENSE(8) AV_DENSE(9) AV_DENSE(10) AV_DENSE(11)
    AV_DENSE(12) AV_DENSE(13) AV_DENSE(14) AV_DENSE(15)
#undef AV_DENSE
    default: throw std::runtime_error("dense histogram: 4..15 bits per record");
  }
}

}  // namespace avk
