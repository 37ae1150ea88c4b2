// K28 text kernels for CDNA4 (gfx950): TF-IDF rows, TextRank power iteration, skip-gram negative
// sampling.
//
// Reference: python/text/preprocess.py:380-524 (TfIdf / term-frequency vectors, host Counters),
// python/text/summ.py TextRank (networkx pagerank over a sentence-similarity graph) and
// python/text/wv.py:36-153 (gensim word2vec / doc2vec).
//   * tfidf_df_kernel   : document frequencies of a CSR count matrix (every column id once per row):
//     a workgroup counts a chunk of <= 65,535 entries into an LDS table of 16-bit counters (two per
//     word, 65,536 ids per 128 KB window, up to 4 windows re-reading the L2-resident chunk) and
//     flushes one global atomic per non-zero bin, so a hot word costs one atomic per chunk instead
//     of one per document (a global-atomic bincount serialises every occurrence on one address);
//     ids past the windows use global atomics.
//   * tfidf_rows_kernel : one wavefront per document row: w = tf * idf(df[col]) with the idf formula
//     inline (smooth: ln((1+D)/(1+df)) + 1, else ln(D/df) + 1; tf = count, or 1 + ln count when
//     sublinear — scikit-learn's sublinear_tf), then the row's L2 (or L1) norm as a wave reduction and
//     the normalised weights written in place.  Both kernels check their indices on the device and
//     raise a status bit instead of touching memory out of range; the binding reads it once.
//   * pagerank_kernel   : the whole power iteration in ONE persistent workgroup: r lives in LDS,
//     every iteration is a column sweep of the row-stochastic matrix (thread j owns columns
//     j, j + 1024, ... — consecutive threads read consecutive addresses of a row), and the L1
//     change is reduced on the device, so there is no host synchronisation per iteration.
//   * sgns_grad_kernel / sgns_apply_kernel : one wavefront per (centre, context) pair of a
//     mini-batch: the context and `neg` negatives drawn on the device (Philox keyed by (seed, step,
//     pair) + an alias table of the unigram^0.75 noise distribution), dot products as wave
//     reductions, the logistic gradients accumulated per row with float atomics; the apply pass
//     moves each touched row by the mean of its updates (the tensor path's averaged SGD);
//     d <= 256 (each lane owns d / 64 coordinates).  PV-DBOW (doc2vec) is the same pair kernel
//     with the document matrix as the centre table (summed, not averaged: few rows per doc).
// Index safety: CSR column ids < V (checked by the binding), alias indices < V, pair ids < V / D.
#include <algorithm>

#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

constexpr int DF_T = 512;
constexpr int DF_WIN = 65536;            // column ids per LDS window: two 16-bit counters per word (128 KB)
constexpr int DF_CHUNK = 65535;          // nnz per chunk: a 16-bit counter cannot carry into its neighbour
constexpr int DF_MAX_WIN = 4;            // ids >= 4 * 65536 are counted with global atomics

__global__ __launch_bounds__(DF_T) void tfidf_df_kernel(const long long* __restrict__ col, long long nnz, long long V,
                                                        int* __restrict__ df, int* __restrict__ status) {
  __shared__ unsigned h[DF_WIN / 2];
  const int nwin = (int)min<long long>((V + DF_WIN - 1) / DF_WIN, DF_MAX_WIN);
  const long long lds_end = (long long)nwin * DF_WIN;
  int bad = 0;
  for (long long c0 = (long long)blockIdx.x * DF_CHUNK; c0 < nnz; c0 += (long long)gridDim.x * DF_CHUNK) {
    const long long c1 = min(nnz, c0 + DF_CHUNK);
    for (int w = 0; w < nwin; ++w) {
      for (int i = threadIdx.x; i < DF_WIN / 2; i += DF_T) h[i] = 0u;
      __syncthreads();
      const long long lo = (long long)w * DF_WIN, hi = lo + DF_WIN;
      for (long long k = c0 + threadIdx.x; k < c1; k += DF_T) {
        const long long c = col[k];
        if (c < 0 || c >= V) {
          bad = 1;                        // never counted
        } else if (c >= lo && c < hi) {
          const int b = (int)(c - lo);
          atomicAdd(&h[b >> 1], 1u << ((b & 1) * 16));
        } else if (w == 0 && c >= lds_end) {  // ids past the LDS windows, once
          atomicAdd(df + c, 1);
        }
      }
      __syncthreads();
      for (int i = threadIdx.x; i < DF_WIN / 2; i += DF_T) {
        const unsigned v = h[i];
        if (v & 0xFFFFu) atomicAdd(df + lo + 2 * i, (int)(v & 0xFFFFu));
        if (v >> 16) atomicAdd(df + lo + 2 * i + 1, (int)(v >> 16));
      }
      __syncthreads();
    }
  }
  if (bad) atomicOr(status, 1);
}

__global__ __launch_bounds__(256) void tfidf_rows_kernel(const long long* __restrict__ crow,
                                                         const long long* __restrict__ col, float* __restrict__ val,
                                                         const int* __restrict__ df, long long n_rows, long long nnz,
                                                         long long V, float n_docs, int smooth, int sublinear, int norm,
                                                         int* __restrict__ status) {
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n_rows) return;
  const int lane = threadIdx.x & 63;
  const long long b = crow[row], e = crow[row + 1];
  if (b < 0 || e > nnz || b > e) {
    if (lane == 0) atomicOr(status, 2);
    return;
  }
  float acc = 0.f;
  for (long long k = b + lane; k < e; k += 64) {
    const long long c = col[k];
    const float tf = sublinear ? (val[k] > 0.f ? 1.f + logf(val[k]) : 0.f) : val[k];
    float idf = 0.f;
    if (c >= 0 && c < V) {
      const float d = (float)df[c];
      idf = smooth ? logf((1.f + n_docs) / (1.f + d)) + 1.f : logf(n_docs / fmaxf(d, 1.f)) + 1.f;
    }
    const float w = tf * idf;
    val[k] = w;
    acc += norm == 2 ? w * w : fabsf(w);
  }
  if (norm == 0) return;
  acc = av::wave_sum(acc);
  const float s = norm == 2 ? sqrtf(acc) : acc;
  const float inv = 1.f / fmaxf(s, 1e-12f);
  for (long long k = b + lane; k < e; k += 64) val[k] *= inv;
}

constexpr int PR_T = 1024;
constexpr int PR_MAXN = 8192;  // r (fp64) in LDS

__global__ __launch_bounds__(PR_T) void pagerank_kernel(const double* __restrict__ P, int n, double d, int iters,
                                                        double tol, double* __restrict__ r_out,
                                                        int* __restrict__ it_out) {
  __shared__ double r[PR_MAXN];
  __shared__ double red[PR_T / 64];
  const int tid = threadIdx.x;
  for (int j = tid; j < n; j += PR_T) r[j] = 1.0 / n;
  __syncthreads();
  constexpr int PER = PR_MAXN / PR_T;
  double nr[PER];
  int it = 0;
  for (; it < iters; ++it) {
    double diff = 0.0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int j = tid + q * PR_T;
      nr[q] = 0.0;
      if (j < n) {
        double s = 0.0;
        for (int i = 0; i < n; ++i) s += P[(long long)i * n + j] * r[i];
        nr[q] = (1.0 - d) / n + d * s;
        diff += fabs(nr[q] - r[j]);
      }
    }
    for (int o = 32; o > 0; o >>= 1) diff += __shfl_xor(diff, o, 64);
    if ((tid & 63) == 0) red[tid >> 6] = diff;
    __syncthreads();  // every r[i] read of this iteration is done
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int j = tid + q * PR_T;
      if (j < n) r[j] = nr[q];
    }
    double tot = 0.0;
    for (int w = 0; w < PR_T / 64; ++w) tot += red[w];
    __syncthreads();  // r updated; red reusable
    if (tot < tol) { ++it; break; }
  }
  for (int j = tid; j < n; j += PR_T) r_out[j] = r[j];
  if (tid == 0) *it_out = it;
}

// Multi-workgroup power iteration for graphs above the single-workgroup size: per iteration
//   pr_partial_kernel  : column sums of P[rows of chunk y, j] * r[i] (r chunk staged in LDS), one
//                        partial per (row chunk, column) — every CU streams a slab of P;
//   pr_finalize_kernel : nr[j] = (1 - d) / n + d * sum_y partial[y][j] (fixed order), per-block
//                        L1 change partials;
//   pr_status_kernel   : one block sums the change partials (fixed order) and raises the done flag
//                        at the first iteration under tol.
// Every kernel returns at once once the flag is up, so the host enqueues all iterations without a
// synchronisation per iteration and reads the iteration count once at the end.
constexpr int PRM_T = 256;
constexpr int PRM_ROWS = 256;

__global__ __launch_bounds__(PRM_T) void pr_partial_kernel(const double* __restrict__ P, const double* __restrict__ r,
                                                           double* __restrict__ partial, int n,
                                                           const int* __restrict__ done) {
  if (*done) return;
  __shared__ double rs[PRM_ROWS];
  const int j = blockIdx.x * PRM_T + threadIdx.x;
  const int i0 = blockIdx.y * PRM_ROWS, i1 = min(n, i0 + PRM_ROWS);
  for (int i = i0 + threadIdx.x; i < i1; i += PRM_T) rs[i - i0] = r[i];
  __syncthreads();
  if (j >= n) return;
  double s = 0.0;
  for (int i = i0; i < i1; ++i) s += P[(long long)i * n + j] * rs[i - i0];
  partial[(long long)blockIdx.y * n + j] = s;
}

__global__ __launch_bounds__(PRM_T) void pr_finalize_kernel(const double* __restrict__ partial, int R,
                                                            const double* __restrict__ r, double* __restrict__ nr,
                                                            int n, double d, double* __restrict__ dpart,
                                                            const int* __restrict__ done) {
  if (*done) return;
  __shared__ double red[PRM_T / 64];
  const int j = blockIdx.x * PRM_T + threadIdx.x;
  double diff = 0.0;
  if (j < n) {
    double s = 0.0;
    for (int y = 0; y < R; ++y) s += partial[(long long)y * n + j];
    const double v = (1.0 - d) / n + d * s;
    nr[j] = v;
    diff = fabs(v - r[j]);
  }
  for (int o = 32; o > 0; o >>= 1) diff += __shfl_xor(diff, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = diff;
  __syncthreads();
  if (threadIdx.x == 0) dpart[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(64) void pr_status_kernel(const double* __restrict__ dpart, int nb, double tol, int k,
                                                       int* __restrict__ done, int* __restrict__ it_out) {
  if (*done) return;
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int b = 0; b < nb; ++b) t += dpart[b];
    *it_out = k + 1;
    if (t < tol) *done = 1;
  }
}

// Hot rows: the negatives follow unigram^0.75 and the contexts / centres the unigram itself, so a
// few frequent words collect most of a batch's gradient atomics, all on the same addresses (the
// grad kernel was 82 % of an epoch, serialised on them).  Rows with hot[row] = s >= 0 (the H most
// probable words) accumulate instead into SG_R replicas [SG_R][H][dp] chosen by the pair index,
// counts likewise after the table's rows; the apply pass folds the replicas back (and zeroes them).
constexpr int SG_R = 16;

// alias table: prob[V] (float), alias[V] (int); draw: k = u1 * V, take k if u2 < prob[k] else alias[k].
// One mini-batch: every pair's gradients are ADDED into gIn / gOut with per-row counts (float
// atomics); sgns_apply_kernel then moves each touched row by the MEAN of its updates.  A device
// batch touches a frequent word many times, and summing those steps (Hogwild over thousands of
// concurrent waves) diverges on small vocabularies; the mean keeps the step size independent of the
// batch size — the same update as the tensor path of text/models.py.
template <int DV>
__global__ __launch_bounds__(256) void sgns_grad_kernel(const float* __restrict__ Win, const float* __restrict__ Wout,
                                                        float* __restrict__ gIn, float* __restrict__ gOut,
                                                        float* __restrict__ cIn, float* __restrict__ cOut,
                                                        const int* __restrict__ centre, const int* __restrict__ context,
                                                        long long n_pairs, const float* __restrict__ aprob,
                                                        const int* __restrict__ alias, int V, int neg, float lr,
                                                        unsigned long long seed, unsigned long long step,
                                                        const int* __restrict__ hot, int H, float* __restrict__ gOutHot,
                                                        float* __restrict__ gInHot, long long rows_in) {
  const long long pr = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (pr >= n_pairs) return;
  const int lane = threadIdx.x & 63;
  const int rep = (int)(pr & (SG_R - 1));
  const int c = centre[pr];
  const float* wc = Win + (long long)c * (DV * 64);
  float v[DV], grad[DV];
#pragma unroll
  for (int k = 0; k < DV; ++k) {
    v[k] = wc[lane + 64 * k];
    grad[k] = 0.f;
  }
  for (int t = 0; t <= neg; ++t) {
    int o;
    float label;
    if (t == 0) {
      o = context[pr];
      label = 1.f;
    } else {
      // the same draw on every lane (wave-uniform counter): no broadcast needed
      const av::u4 rr = av::philox_draw(seed, step, (unsigned long long)(pr * 64 + t));
      int k = (int)(av::u32_to_unit(rr.x) * (float)V);
      k = k >= V ? V - 1 : k;
      o = av::u32_to_unit(rr.y) < aprob[k] ? k : alias[k];
      label = 0.f;
    }
    const float* wo = Wout + (long long)o * (DV * 64);
    float u[DV], dot = 0.f;
#pragma unroll
    for (int k = 0; k < DV; ++k) {
      u[k] = wo[lane + 64 * k];
      dot += u[k] * v[k];
    }
    dot = av::wave_sum(dot);
    const float g = (label - 1.f / (1.f + __expf(-dot))) * lr;
    int hs = hot ? hot[o] : -1;
    hs = hs < H ? hs : -1;
    float* go = hs >= 0 ? gOutHot + (long long)(rep * H + hs) * (DV * 64) : gOut + (long long)o * (DV * 64);
#pragma unroll
    for (int k = 0; k < DV; ++k) {
      grad[k] += g * u[k];
      atomicAdd(&go[lane + 64 * k], g * v[k]);
    }
    if (lane == 0) atomicAdd(&cOut[hs >= 0 ? (long long)V + rep * H + hs : (long long)o], 1.f);
  }
  int hc = (hot && gInHot) ? hot[c] : -1;
  hc = hc < H ? hc : -1;
  float* gc = hc >= 0 ? gInHot + (long long)(rep * H + hc) * (DV * 64) : gIn + (long long)c * (DV * 64);
#pragma unroll
  for (int k = 0; k < DV; ++k) atomicAdd(&gc[lane + 64 * k], grad[k]);
  if (lane == 0) atomicAdd(&cIn[hc >= 0 ? rows_in + rep * H + hc : (long long)c], 1.f);
}

// W[r] += g[r] / max(count[r], 1) (mean_in: the centre table of doc2vec sums instead), g -> 0;
// hot rows (hot[r] = s >= 0, gHot != null) first fold their SG_R replicas (zeroing them) and
// counts (stored after the table's rows; zeroed by the caller with the counts)
__global__ __launch_bounds__(256) void sgns_apply_kernel(float* __restrict__ W, float* __restrict__ g,
                                                         const float* __restrict__ cnt, long long rows, int dp,
                                                         int mean, const int* __restrict__ hot, int H,
                                                         float* __restrict__ gHot, float* __restrict__ zero_next,
                                                         long long n_zero) {
  const long long total = rows * dp;
  const long long stride = (long long)gridDim.x * 256;
  // the other count buffer (ping-pong: the previous batch's, no longer read) is cleared for the next
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; zero_next && i < n_zero; i += stride)
    zero_next[i] = 0.f;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += stride) {
    const long long r = i / dp;
    float gv = g[i];
    float cv = cnt[r];
    const int hs = (hot && gHot) ? hot[r] : -1;
    if (hs >= 0 && hs < H) {
      const int col = (int)(i - r * dp);
#pragma unroll 4
      for (int q = 0; q < SG_R; ++q) {
        float* p = gHot + (long long)(q * H + hs) * dp + col;
        gv += *p;
        *p = 0.f;
        cv += cnt[rows + q * H + hs];
      }
    }
    if (gv != 0.f) {
      W[i] += mean ? gv / fmaxf(cv, 1.f) : gv;
      g[i] = 0.f;
    }
  }
}

}  // namespace

namespace avk {

void tfidf_csr(const long long* crow, const long long* col, float* val, long long n_rows, long long nnz, long long V,
               int smooth, int sublinear, int norm, int* df, int* status, hipStream_t stream) {
  if (nnz > 0) {
    const long long blocks = std::min<long long>(1024, (nnz + DF_CHUNK - 1) / DF_CHUNK);
    tfidf_df_kernel<<<(unsigned)blocks, DF_T, 0, stream>>>(col, nnz, V, df, status);
    AV_HIP_CHECK(hipGetLastError());
  }
  if (n_rows <= 0) return;
  tfidf_rows_kernel<<<(unsigned)((n_rows + 3) / 4), 256, 0, stream>>>(crow, col, val, df, n_rows, nnz, V,
                                                                      (float)n_rows, smooth, sublinear, norm, status);
  AV_HIP_CHECK(hipGetLastError());
}

int pagerank_max_n() { return PR_MAXN; }

void pagerank(const double* P, int n, double d, int iters, double tol, double* r, int* it, hipStream_t stream) {
  if (n <= 0) return;
  if (n > PR_MAXN) throw std::runtime_error("pagerank: n exceeds the LDS-resident vector");
  pagerank_kernel<<<1, PR_T, 0, stream>>>(P, n, d, iters, tol, r, it);
  AV_HIP_CHECK(hipGetLastError());
}

int sgns_hot_replicas() { return SG_R; }

void sgns_step(float* Win, float* Wout, float* gIn, float* gOut, float* cIn, float* cOut, int dim, long long rows_in,
               const int* centre, const int* context, long long n_pairs, const float* aprob, const int* alias, int V,
               int neg, float lr, int mean_in, unsigned long long seed, unsigned long long step, const int* hot, int H,
               float* gOutHot, float* gInHot, float* cIn_next, long long n_cin, float* cOut_next, long long n_cout,
               hipStream_t stream) {
  if (n_pairs <= 0) return;
  const unsigned grid = (unsigned)((n_pairs + 3) / 4);
#define AV_SG(DV) sgns_grad_kernel<DV><<<grid, 256, 0, stream>>>(Win, Wout, gIn, gOut, cIn, cOut, centre, context, \
      n_pairs, aprob, alias, V, neg, lr, seed, step, hot, H, gOutHot, gInHot, rows_in)
  switch (dim) {
    case 64: AV_SG(1); break;
    case 128: AV_SG(2); break;
    case 192: AV_SG(3); break;
    case 256: AV_SG(4); break;
    default: throw std::runtime_error("sgns_step: padded dim must be 64, 128, 192 or 256");
  }
#undef AV_SG
  AV_HIP_CHECK(hipGetLastError());
  sgns_apply_kernel<<<av::stream_grid(rows_in * dim, 256, 4, 4096), 256, 0, stream>>>(Win, gIn, cIn, rows_in, dim,
                                                                                       mean_in, hot, H, gInHot,
                                                                                       cIn_next, n_cin);
  AV_HIP_CHECK(hipGetLastError());
  sgns_apply_kernel<<<av::stream_grid((long long)V * dim, 256, 4, 4096), 256, 0, stream>>>(Wout, gOut, cOut, V, dim, 1,
                                                                                           hot, H, gOutHot, cOut_next,
                                                                                           n_cout);
  AV_HIP_CHECK(hipGetLastError());
}

int pagerank_multi_rows() { return PRM_ROWS; }

// Iterations [k0, k1).  buf: 2 x n (buf[0] = the start vector, filled by the caller), partial:
// ceil(n / 256) x n, dpart: ceil(n / 256), state: 2 ints zeroed before the first batch (done,
// iterations).  The result is in buf[iterations & 1].
void pagerank_multi(const double* P, int n, double d, int k0, int k1, double tol, double* buf, double* partial,
                    double* dpart, int* state, hipStream_t stream) {
  if (n <= 0) return;
  const int nb = (n + PRM_T - 1) / PRM_T, R = (n + PRM_ROWS - 1) / PRM_ROWS;
  for (int k = k0; k < k1; ++k) {
    const double* r = buf + (long long)(k & 1) * n;
    double* nr = buf + (long long)((k + 1) & 1) * n;
    pr_partial_kernel<<<dim3((unsigned)nb, (unsigned)R), PRM_T, 0, stream>>>(P, r, partial, n, state);
    pr_finalize_kernel<<<(unsigned)nb, PRM_T, 0, stream>>>(partial, R, r, nr, n, d, dpart, state);
    pr_status_kernel<<<1, 64, 0, stream>>>(dpart, nb, tol, k, state, state + 1);
  }
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
