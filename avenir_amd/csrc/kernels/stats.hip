// K26 rank statistics for CDNA4 (gfx950): tie-averaged ranks and Kendall pair counts.
//
// Reference: P/mlextra/daexp.py getSpearmanRankCorr / getKendalRankCorr / testTwoSampleMw /
// testTwoSampleKw (:1093-1175, :1458-1836) call scipy.stats on host arrays.  Here the data stays on
// the device; only scalar statistics come back (p-values are closed-form functions of them,
// analytics/explorer.py).
//   * rank_avg_kernel   : from a sorted copy of the sample (values + the sort permutation), every
//     element's average rank over its tie run, (lo + 1 + hi) / 2 with lo / hi the run bounds found
//     by two binary searches (each element independent: no scan, any n), scattered back to the
//     original order; the run's first element adds the tie terms sum (t^3 - t), sum t (t - 1),
//     sum t (t - 1)(t - 2) and sum t (t - 1)(2t + 5) (fp64, exact for t < 2^17) used by the
//     Spearman / Mann-Whitney / Kruskal-Wallis / Kendall variance corrections, and the element's
//     group (sample id) accumulates its rank into per-group rank sums.
//   * kendall_pairs_kernel : all pairs i < j of (x, y), tiled 256 x 256: a workgroup stages a
//     column tile in LDS and every thread compares its row against it, counting concordant,
//     discordant, x-tied, y-tied and both-tied pairs in registers (u32 per thread, at most 256
//     pairs per tile), reduced per workgroup and added to u64 totals — exact integer counts,
//     O(n^2) work spread over (n / 256)^2 / 2 workgroups.
//   * inv_merge_local_kernel / inv_merge_level_kernel : strict inversions of a sequence (Knight's
//     Kendall count: y ordered by (x, y)) by a bottom-up merge sort whose merges are merge-path
//     rank computations: a left-run element lands at its index + #(right < v), a right-run element
//     at its index + #(left <= v) and contributes #(left > v) inversions.  Runs up to 1,024 values
//     are merged inside one workgroup in LDS (10 levels, one launch), longer runs one launch per
//     level; counts are wave-reduced into one u64.  O(n log^2 n) work in 1 + log2(n / 1024) launches
//     (the tensor path was a batched sort + searchsorted per level).
// Index safety: binary searches stay in [0, n); merge levels work on m = a power of two >= 1024
// values (padded with +inf by the caller), so every run and its partner lie inside [0, m); perm[i] < n is the caller's permutation of 0..n-1;
// group ids >= n_groups are ignored; pair tiles only touch rows / columns < n.
#include <algorithm>
#include <stdexcept>

#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

constexpr int RK_T = 256;
constexpr int RK_MAXG = 256;  // group rank sums privatised in LDS up to this many groups

__device__ __forceinline__ long long lower_bound_d(const double* v, long long n, double key) {
  long long lo = 0, hi = n;
  while (lo < hi) {
    const long long mid = (lo + hi) >> 1;
    if (v[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ long long upper_bound_d(const double* v, long long n, double key) {
  long long lo = 0, hi = n;
  while (lo < hi) {
    const long long mid = (lo + hi) >> 1;
    if (v[mid] <= key) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// sorted [n] ascending, perm [n] (sorted position -> original index), group [n] (original order)
// or null; out ranks [n] (original order); tie[4] += tie terms; gsum[n_groups] += rank sums.
__global__ __launch_bounds__(RK_T) void rank_avg_kernel(const double* __restrict__ sorted,
                                                        const long long* __restrict__ perm, long long n,
                                                        const int* __restrict__ group, int n_groups,
                                                        double* __restrict__ ranks, double* __restrict__ tie,
                                                        double* __restrict__ gsum) {
  __shared__ double s_g[RK_MAXG];
  __shared__ double s_t[4][RK_T / 64];
  const bool lds_groups = group && n_groups <= RK_MAXG;
  if (lds_groups)
    for (int k = threadIdx.x; k < n_groups; k += RK_T) s_g[k] = 0.0;
  __syncthreads();
  double t3 = 0.0, t2 = 0.0, t21 = 0.0, t25 = 0.0;
  const long long stride = (long long)gridDim.x * RK_T;
  for (long long i = (long long)blockIdx.x * RK_T + threadIdx.x; i < n; i += stride) {
    const double v = sorted[i];
    const long long lo = lower_bound_d(sorted, n, v), hi = upper_bound_d(sorted, n, v);
    const double r = 0.5 * (double)(lo + 1 + hi);
    const long long o = perm[i];
    ranks[o] = r;
    if (group) {
      const int gg = group[o];
      if (gg >= 0 && gg < n_groups) {
        if (lds_groups) atomicAdd(&s_g[gg], r);   // block-private group sums (ds_add_f64)
        else atomicAdd(&gsum[gg], r);
      }
    }
    if (i == lo) {
      const double t = (double)(hi - lo);
      t3 += t * t * t - t;
      t2 += t * (t - 1.0);
      t21 += t * (t - 1.0) * (t - 2.0);
      t25 += t * (t - 1.0) * (2.0 * t + 5.0);
    }
  }
  // block sums, one atomic per block and term / group
  for (int o = 32; o > 0; o >>= 1) {
    t3 += __shfl_xor(t3, o, 64);
    t2 += __shfl_xor(t2, o, 64);
    t21 += __shfl_xor(t21, o, 64);
    t25 += __shfl_xor(t25, o, 64);
  }
  const int w = threadIdx.x >> 6;
  if (av::lane_id() == 0) {
    s_t[0][w] = t3;
    s_t[1][w] = t2;
    s_t[2][w] = t21;
    s_t[3][w] = t25;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    double s = 0.0;
    for (int q = 0; q < RK_T / 64; ++q) s += s_t[threadIdx.x][q];
    if (s != 0.0) atomicAdd(&tie[threadIdx.x], s);
  }
  if (lds_groups)
    for (int k = threadIdx.x; k < n_groups; k += RK_T)
      if (s_g[k] != 0.0) atomicAdd(&gsum[k], s_g[k]);
}

constexpr int KT = 256;  // tile edge: rows per workgroup = columns per LDS stage

__device__ __forceinline__ int cmp3(double a, double b) { return (a > b) - (a < b); }

// blockIdx.x enumerates upper-triangular tile pairs (bi <= bj) of the (n / KT)^2 grid.
// out[0] concordant, [1] discordant, [2] tied in x only, [3] tied in y only, [4] tied in both.
__global__ __launch_bounds__(KT) void kendall_pairs_kernel(const double* __restrict__ x, const double* __restrict__ y,
                                                           long long n, int nt,
                                                           unsigned long long* __restrict__ out) {
  __shared__ double sx[KT], sy[KT];
  __shared__ unsigned red[5][KT / 64];
  long long p = blockIdx.x;
  int bi = 0;
  while (p >= nt - bi) { p -= nt - bi; ++bi; }
  const int bj = bi + (int)p;
  const long long i = (long long)bi * KT + threadIdx.x;
  const long long j0 = (long long)bj * KT;
  if (j0 + threadIdx.x < n) {
    sx[threadIdx.x] = x[j0 + threadIdx.x];
    sy[threadIdx.x] = y[j0 + threadIdx.x];
  }
  __syncthreads();
  unsigned c[5] = {0u, 0u, 0u, 0u, 0u};
  if (i < n) {
    const double xi = x[i], yi = y[i];
    const int jn = (int)min((long long)KT, n - j0);
    for (int k = 0; k < jn; ++k) {
      if (j0 + k <= i) continue;  // each unordered pair once (diagonal tiles)
      const int a = cmp3(xi, sx[k]), b = cmp3(yi, sy[k]);
      const int s = a * b;
      c[0] += s > 0;
      c[1] += s < 0;
      c[2] += (a == 0) & (b != 0);
      c[3] += (a != 0) & (b == 0);
      c[4] += (a == 0) & (b == 0);
    }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    unsigned v = c[q];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[q][w] = v;
  }
  __syncthreads();
  if (threadIdx.x < 5) {
    unsigned long long s = 0;
    for (int q = 0; q < KT / 64; ++q) s += red[threadIdx.x][q];
    if (s) atomicAdd(&out[threadIdx.x], s);
  }
}

constexpr int IM_T = 1024;

__device__ __forceinline__ int lb_run(const double* v, int n, double key) {   // #(v < key)
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (v[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ int ub_run(const double* v, int n, double key) {   // #(v <= key)
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (v[mid] <= key) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ void inv_add(unsigned long long c, unsigned long long* inv) {
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(inv, c);
}

// every 1,024-value block of in, sorted through runs of 1, 2, ..., 512 in LDS -> out
__global__ __launch_bounds__(IM_T) void inv_merge_local_kernel(const double* __restrict__ in, double* __restrict__ out,
                                                               unsigned long long* __restrict__ inv) {
  __shared__ double buf[2][IM_T];
  const long long base = (long long)blockIdx.x * IM_T;
  const int t = threadIdx.x;
  buf[0][t] = in[base + t];
  __syncthreads();
  unsigned long long c = 0;
  int cur = 0;
  for (int s = 1; s < IM_T; s <<= 1) {
    const double* src = buf[cur];
    const int p = t & ~(2 * s - 1), w = t - p;
    const double v = src[t];
    int pos;
    if (w < s) {
      pos = w + lb_run(src + p + s, s, v);
    } else {
      const int u = ub_run(src + p, s, v);
      pos = (w - s) + u;
      c += (unsigned long long)(s - u);
    }
    buf[cur ^ 1][p + pos] = v;
    cur ^= 1;
    __syncthreads();
  }
  out[base + t] = buf[cur][t];
  inv_add(c, inv);
}

// one merge level of runs of s (>= 1,024) values: in -> out, m values in all
__global__ __launch_bounds__(256) void inv_merge_level_kernel(const double* __restrict__ in, double* __restrict__ out,
                                                              long long m, long long s,
                                                              unsigned long long* __restrict__ inv) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  unsigned long long c = 0;
  if (i < m) {
    const long long p = i & ~(2 * s - 1), w = i - p;
    const double v = in[i];
    long long pos;
    if (w < s) {
      pos = w + lower_bound_d(in + p + s, s, v);
    } else {
      const long long u = upper_bound_d(in + p, s, v);
      pos = (w - s) + u;
      c = (unsigned long long)(s - u);
    }
    out[p + pos] = v;
  }
  inv_add(c, inv);
}

}  // namespace

namespace avk {

void rank_avg(const double* sorted, const long long* perm, long long n, const int* group, int n_groups, double* ranks,
              double* tie, double* gsum, hipStream_t stream) {
  if (n <= 0) return;
  rank_avg_kernel<<<av::stream_grid(n, RK_T, 4, 4096), RK_T, 0, stream>>>(sorted, perm, n, group, n_groups, ranks, tie,
                                                                          gsum);
  AV_HIP_CHECK(hipGetLastError());
}

void kendall_pairs(const double* x, const double* y, long long n, unsigned long long* out, hipStream_t stream) {
  if (n <= 1) return;
  const long long nt = (n + KT - 1) / KT;
  const long long tiles = nt * (nt + 1) / 2;
  if (tiles > 0x7fffffffLL) throw std::runtime_error("kendall_pairs: n too large");
  kendall_pairs_kernel<<<(unsigned)tiles, KT, 0, stream>>>(x, y, n, (int)nt, out);
  AV_HIP_CHECK(hipGetLastError());
}

int inv_merge_block() { return IM_T; }

// strict inversions of a[0, m) (m a power of two >= IM_T); a and tmp are clobbered.  Returns the
// buffer holding the sorted sequence (a or tmp).
double* inversions(double* a, double* tmp, long long m, unsigned long long* inv, hipStream_t stream) {
  if (m < IM_T || (m & (m - 1))) throw std::runtime_error("inversions: m must be a power of two >= 1024");
  inv_merge_local_kernel<<<(unsigned)(m / IM_T), IM_T, 0, stream>>>(a, tmp, inv);
  AV_HIP_CHECK(hipGetLastError());
  double* src = tmp;
  double* dst = a;
  for (long long s = IM_T; s < m; s <<= 1) {
    inv_merge_level_kernel<<<(unsigned)((m + 255) / 256), 256, 0, stream>>>(src, dst, m, s, inv);
    AV_HIP_CHECK(hipGetLastError());
    std::swap(src, dst);
  }
  return src;
}

}  // namespace avk
