// Sequence-mining kernels for CDNA4 (gfx950): K5 n-gram counting, K16 uniformisation power
// chain, K19 dot-matrix window matching.
//
// K5  n-gram hash counting — every contiguous window of length min_len..max_len of every state
//     sequence, counted in ONE pass.  Reference: ProbabilisticSuffixTreeGenerator emits each
//     sub-sequence as a key and sums in a combiner/reducer
//     (J/markov/ProbabilisticSuffixTreeGenerator.java:140-194, 252-305); TimeDelayEmbeddingModel
//     histograms fixed-size symbol windows (S/sequence/TimeDelayEmbeddingModel.scala:69-97).
//     Here a lane owns one (row, start) position and builds the keys of all lengths incrementally
//     (key_k = key_{k-1} * base + s).  Keys are inserted into a workgroup-private open-addressing
//     table in LDS (64-bit ds_cmpst + 32-bit ds_add: the few hot short n-grams are combined on
//     chip), which is flushed once into a global open-addressing table in HBM; a key that finds no
//     LDS slot within the probe budget goes straight to the global table.  Key layout:
//     [len:6][group * base^max_len + packed] with packed = sum s_j base^(k-1-j), base = S + 1 —
//     the same packing as the host oracle so decoded n-grams are identical.
// K16 uniformisation (CTMC) — for a stochastic P (S <= 64) and per-problem Poisson weights,
//     A = sum_k w1[k] P^k and B = sum_k w2[k] P^k, with P^k built by repeated multiplication
//     (S/markov/ContTimeStateTransitionStats.scala:96-112 powers, :161-236 weighted sums).  One
//     workgroup per problem: P and the running power live in LDS (fp64), lane j owns column j and
//     16 rows; the accumulators stay in registers, no power is ever written to HBM.
// K19 dot-matrix matching — number of equal length-w windows between every pair of sequences
//     (S/sequence/DotMatrixMatching.scala:176-252, all pairs via bucket-pair replication :76-99).
//     Windows are pre-mapped to dense int32 ids; a workgroup owns a 16 x 16 tile of sequence pairs,
//     stages the id rows of its 16 + 16 sequences in LDS in chunks, and each lane counts the
//     matches of one pair.
#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

constexpr unsigned long long EMPTY = ~0ull;
constexpr int NG_BLOCK = 256;
constexpr int NG_LDS_SLOTS = 2048;  // 2048 x (8 + 4) B = 24 KiB
constexpr int NG_LDS_PROBES = 16;

__device__ __forceinline__ unsigned long long mix64(unsigned long long k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

__device__ __forceinline__ void global_insert(unsigned long long* keys, unsigned* counts, unsigned long long cap,
                                              unsigned long long key, unsigned c, int* overflow) {
  unsigned long long h = mix64(key) & (cap - 1);
  for (unsigned long long probe = 0; probe < cap; ++probe) {
    const unsigned long long prev = atomicCAS(&keys[h], EMPTY, key);
    if (prev == EMPTY || prev == key) {
      atomicAdd(&counts[h], c);
      return;
    }
    h = (h + 1) & (cap - 1);
  }
  atomicOr(overflow, 1);  // table full: host retries with a larger one
}

__global__ __launch_bounds__(NG_BLOCK) void ngram_count_kernel(const short* __restrict__ st, long long n, int L,
                                                               int S, int min_len, int max_len,
                                                               const int* __restrict__ group,
                                                               unsigned long long group_mul,
                                                               unsigned long long* __restrict__ keys,
                                                               unsigned* __restrict__ counts,
                                                               unsigned long long cap, int* overflow) {
  __shared__ unsigned long long s_key[NG_LDS_SLOTS];
  __shared__ unsigned s_cnt[NG_LDS_SLOTS];
  for (int i = threadIdx.x; i < NG_LDS_SLOTS; i += NG_BLOCK) {
    s_key[i] = EMPTY;
    s_cnt[i] = 0;
  }
  __syncthreads();
  const unsigned long long base = (unsigned long long)S + 1;
  const long long total = n * (long long)L;
  const long long stride = (long long)gridDim.x * NG_BLOCK;
  for (long long item = (long long)blockIdx.x * NG_BLOCK + threadIdx.x; item < total; item += stride) {
    const long long row = item / L;
    const int p = (int)(item - row * L);
    const short* r = st + row * L;
    const unsigned long long goff = group ? (unsigned long long)group[row] * group_mul : 0ull;
    unsigned long long packed = 0;
    for (int k = 1; k <= max_len; ++k) {
      if (p + k > L) break;
      const int s = r[p + k - 1];
      if (s < 0 || s >= S) break;  // a window may not span an invalid / padding state
      packed = packed * base + (unsigned long long)s;
      if (k < min_len) continue;
      const unsigned long long key = ((unsigned long long)k << 58) | (goff + packed);
      unsigned h = (unsigned)mix64(key) & (NG_LDS_SLOTS - 1);
      bool done = false;
      for (int q = 0; q < NG_LDS_PROBES; ++q) {
        const unsigned long long prev = atomicCAS(&s_key[h], EMPTY, key);
        if (prev == EMPTY || prev == key) {
          atomicAdd(&s_cnt[h], 1u);
          done = true;
          break;
        }
        h = (h + 1) & (NG_LDS_SLOTS - 1);
      }
      if (!done) global_insert(keys, counts, cap, key, 1u, overflow);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NG_LDS_SLOTS; i += NG_BLOCK) {
    const unsigned long long k = s_key[i];
    if (k != EMPTY) global_insert(keys, counts, cap, k, s_cnt[i], overflow);
  }
}

__global__ __launch_bounds__(256) void hash_compact_kernel(const unsigned long long* __restrict__ keys,
                                                           const unsigned* __restrict__ counts,
                                                           unsigned long long cap,
                                                           long long* __restrict__ out_keys,
                                                           long long* __restrict__ out_counts,
                                                           unsigned long long* __restrict__ n_out) {
  const unsigned long long stride = (unsigned long long)gridDim.x * 256;
  for (unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x; i < cap; i += stride) {
    const unsigned long long k = keys[i];
    const bool live = k != EMPTY;
    // one atomic per wave: ballot + popcount prefix
    const unsigned long long m = __ballot(live);
    if (m == 0) continue;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((long long)m) - 1;
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(n_out, (unsigned long long)__popcll(m));
    base = __shfl(base, leader, 64);
    if (live) {
      const unsigned long long below = m & ((1ull << lane) - 1);
      const unsigned long long pos = base + __popcll(below);
      out_keys[pos] = (long long)k;
      out_counts[pos] = (long long)counts[i];
    }
  }
}

// ------------------------------------------------------------------------------------------
// K16
// ------------------------------------------------------------------------------------------
constexpr int UN_MAXS = 64;
constexpr int UN_ROWS = UN_MAXS / 4;  // rows per lane (4 waves)

__global__ __launch_bounds__(256) void uniformization_kernel(const double* __restrict__ P, int S,
                                                             const double* __restrict__ w1,
                                                             const double* __restrict__ w2,
                                                             const int* __restrict__ steps, int ldw,
                                                             double* __restrict__ out) {
  __shared__ double sP[UN_MAXS * UN_MAXS];
  __shared__ double sC[UN_MAXS * UN_MAXS];
  const int prob = blockIdx.x;
  const int j = threadIdx.x & 63, i0 = threadIdx.x >> 6;
  for (int t = threadIdx.x; t < S * S; t += 256) {
    sP[t] = P[t];
    const int r = t / S, c = t - r * S;
    sC[t] = r == c ? 1.0 : 0.0;  // P^0
  }
  __syncthreads();
  const double* a1 = w1 + (long long)prob * ldw;
  const double* a2 = w2 + (long long)prob * ldw;
  const int Lp = steps[prob];
  double acc1[UN_ROWS], acc2[UN_ROWS], nxt[UN_ROWS];
#pragma unroll
  for (int q = 0; q < UN_ROWS; ++q) {
    const int i = i0 + 4 * q;
    const double c0 = (i < S && j < S) ? sC[i * S + j] : 0.0;
    acc1[q] = a1[0] * c0;
    acc2[q] = a2[0] * c0;
  }
  for (int k = 1; k <= Lp; ++k) {
#pragma unroll
    for (int q = 0; q < UN_ROWS; ++q) nxt[q] = 0.0;
    if (j < S) {
      for (int m = 0; m < S; ++m) {
        const double p = sP[m * S + j];  // lanes read consecutive columns: conflict-free
#pragma unroll
        for (int q = 0; q < UN_ROWS; ++q) {
          const int i = i0 + 4 * q;
          if (i < S) nxt[q] = fma(sC[i * S + m], p, nxt[q]);  // wave-uniform address: broadcast
        }
      }
    }
    __syncthreads();
    const double b1 = a1[k], b2 = a2[k];
#pragma unroll
    for (int q = 0; q < UN_ROWS; ++q) {
      const int i = i0 + 4 * q;
      if (i < S && j < S) {
        sC[i * S + j] = nxt[q];
        acc1[q] = fma(b1, nxt[q], acc1[q]);
        acc2[q] = fma(b2, nxt[q], acc2[q]);
      }
    }
    __syncthreads();
  }
  double* o = out + (long long)prob * 2 * S * S;
#pragma unroll
  for (int q = 0; q < UN_ROWS; ++q) {
    const int i = i0 + 4 * q;
    if (i < S && j < S) {
      o[i * S + j] = acc1[q];
      o[S * S + i * S + j] = acc2[q];
    }
  }
}

// ------------------------------------------------------------------------------------------
// K19
// ------------------------------------------------------------------------------------------
constexpr int DM_T = 16;     // 16 x 16 sequence pairs per workgroup
constexpr int DM_CH = 256;   // window ids staged per chunk

__global__ __launch_bounds__(256) void dot_matrix_kernel(const int* __restrict__ A, int n, int Wa,
                                                         const int* __restrict__ B, int m, int Wb,
                                                         int* __restrict__ hits) {
  __shared__ int sa[DM_T][DM_CH + 1];
  __shared__ int sb[DM_T][DM_CH + 1];  // +1: the 16 rows read together fall in different banks
  const int ti = threadIdx.x >> 4, tj = threadIdx.x & 15;
  const int i0 = blockIdx.y * DM_T, j0 = blockIdx.x * DM_T;
  int cnt = 0;
  for (int pa = 0; pa < Wa; pa += DM_CH) {
    const int ca = min(DM_CH, Wa - pa);
    __syncthreads();
    for (int t = threadIdx.x; t < DM_T * DM_CH; t += 256) {
      const int r = t / DM_CH, c = t - r * DM_CH;
      sa[r][c] = (i0 + r < n && c < ca) ? A[(long long)(i0 + r) * Wa + pa + c] : -1;
    }
    for (int pb = 0; pb < Wb; pb += DM_CH) {
      const int cb = min(DM_CH, Wb - pb);
      __syncthreads();
      for (int t = threadIdx.x; t < DM_T * DM_CH; t += 256) {
        const int r = t / DM_CH, c = t - r * DM_CH;
        sb[r][c] = (j0 + r < m && c < cb) ? B[(long long)(j0 + r) * Wb + pb + c] : -2;
      }
      __syncthreads();
      for (int p = 0; p < ca; ++p) {
        const int a = sa[ti][p];
        if (a < 0) continue;
        for (int q = 0; q < cb; ++q) cnt += (sb[tj][q] == a);
      }
    }
  }
  const int i = i0 + ti, jj = j0 + tj;
  if (i < n && jj < m) hits[(long long)i * m + jj] = cnt;
}

}  // namespace

namespace avk {

void ngram_count(const short* st, long long n, int L, int S, int min_len, int max_len, const int* group,
                 unsigned long long group_mul, unsigned long long* keys, unsigned* counts, unsigned long long cap,
                 int* overflow, hipStream_t stream) {
  if (cap == 0 || (cap & (cap - 1))) throw std::runtime_error("ngram_count: capacity must be a power of two");
  if (min_len < 1 || max_len < min_len || max_len > 63) throw std::runtime_error("ngram_count: bad lengths");
  const long long items = n * (long long)L;
  const int grid = av::stream_grid(items, NG_BLOCK, 8, 1024);
  ngram_count_kernel<<<grid, NG_BLOCK, 0, stream>>>(st, n, L, S, min_len, max_len, group, group_mul, keys, counts,
                                                    cap, overflow);
  AV_HIP_CHECK(hipGetLastError());
}

void hash_compact(const unsigned long long* keys, const unsigned* counts, unsigned long long cap, long long* out_keys,
                  long long* out_counts, unsigned long long* n_out, hipStream_t stream) {
  const int grid = av::stream_grid((long long)cap, 256, 4, 2048);
  hash_compact_kernel<<<grid, 256, 0, stream>>>(keys, counts, cap, out_keys, out_counts, n_out);
  AV_HIP_CHECK(hipGetLastError());
}

void uniformization(const double* P, int S, const double* w1, const double* w2, const int* steps, int ldw, int B,
                    double* out, hipStream_t stream) {
  if (S < 1 || S > UN_MAXS) throw std::runtime_error("uniformization: 1 <= S <= 64");
  uniformization_kernel<<<B, 256, 0, stream>>>(P, S, w1, w2, steps, ldw, out);
  AV_HIP_CHECK(hipGetLastError());
}

void dot_matrix(const int* A, int n, int Wa, const int* B, int m, int Wb, int* hits, hipStream_t stream) {
  dim3 grid((m + DM_T - 1) / DM_T, (n + DM_T - 1) / DM_T);
  if (grid.y > 65535) throw std::runtime_error("dot_matrix: too many query sequences for one launch");
  dot_matrix_kernel<<<grid, 256, 0, stream>>>(A, n, Wa, B, m, Wb, hits);
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
