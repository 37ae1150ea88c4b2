// Device-resident gradient boosting round for CDNA4 (gfx950): K9g.
//
// Reference: P/supv/gbt.py wraps scikit-learn's GradientBoostingClassifier (deviance loss, one
// regression tree per class and stage, Newton leaf values); one stage is a host loop there.  Here a
// boosting round is a FIXED sequence of launches with static shapes, so the whole round is captured
// in one HIP graph and replayed per stage (models/tree.py GradientBoostedTrees._fit_device):
//   1. gbt_grad_kernel   : g = p - y, h = max(p(1 - p), 1e-6) of the current raw scores (sigmoid, or
//      softmax over K classes for class k), the row subsample as a counter hash of (seed, round,
//      GLOBAL row) (world-size invariant, no RNG state), and the training loss of the scores left by
//      the previous round accumulated on the device (no host sync per round);
//   2. per level: node_grad_hist (tree.hip; at levels >= 1 only the LEFT children are histogrammed,
//      right = parent - left, exact in fixed point), the split scan as batched tensor math, and
//   3. gbt_assign_kernel : rows move to their child slot (heap layout: children of slot s are 2s and
//      2s + 1), and rows that reach a leaf (stopped node, missing code, or the last level) add
//      lr * leaf value to their score in the same pass — no separate tree-inference pass.
// Index safety: slots at level l are < 2^l and heap indices < 2^(D+1) - 1 by construction (the
// binding checks D); a missing / out-of-range code never indexes the segment arrays.
#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

constexpr int GT = 256;

__device__ __forceinline__ unsigned mix32(unsigned long long z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  z ^= z >> 31;
  return (unsigned)(z >> 32);
}

__global__ __launch_bounds__(GT) void gbt_grad_kernel(const float* __restrict__ F, int K, int k,
                                                      const uint8_t* __restrict__ y, long long n, long long row_off,
                                                      unsigned long long seed, unsigned rate32, float* __restrict__ g,
                                                      float* __restrict__ h, double* __restrict__ loss) {
  double acc = 0.0;
  const long long stride = (long long)gridDim.x * GT;
  for (long long r = (long long)blockIdx.x * GT + threadIdx.x; r < n; r += stride) {
    const int yr = y[r];
    float p, lr_loss;
    if (K == 1) {
      const float f = F[r];
      p = 1.0f / (1.0f + __expf(-f));
      // BCE with logits, stable: max(f, 0) - f*y + log(1 + exp(-|f|))
      lr_loss = fmaxf(f, 0.0f) - f * (float)yr + log1pf(__expf(-fabsf(f)));
    } else {
      const float* fr = F + r * K;
      float m = fr[0];
      for (int j = 1; j < K; ++j) m = fmaxf(m, fr[j]);
      float s = 0.0f;
      for (int j = 0; j < K; ++j) s += __expf(fr[j] - m);
      p = __expf(fr[k] - m) / s;
      lr_loss = (m + __logf(s)) - fr[yr < K ? yr : 0];
    }
    const float target = K == 1 ? (float)yr : (yr == k ? 1.0f : 0.0f);
    float gr = p - target;
    float hr = fmaxf(p * (1.0f - p), 1e-6f);
    if (rate32 != 0xFFFFFFFFu) {
      const unsigned u = mix32(seed + (unsigned long long)(row_off + r) * 0x9E3779B97F4A7C15ULL);
      if (u >= rate32) { gr = 0.0f; hr = 0.0f; }
    }
    g[r] = gr;
    h[r] = hr;
    acc += (double)lr_loss;
  }
  if (loss) {
    // block sum, ONE atomic per block (the loss is a report, not part of the model; one atomic per
    // wave serialised ~260 k same-address atomics at 16.7 M rows)
    __shared__ double red[GT / 64];
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (av::lane_id() == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      double s = 0.0;
      for (int w = 0; w < GT / 64; ++w) s += red[w];
      atomicAdd(loss, s);
    }
  }
}

// rows of slot s at level `level` (heap index hb + s, hb = 2^level - 1)
__global__ __launch_bounds__(GT) void gbt_assign_kernel(const uint8_t* __restrict__ codes, long long ld, long long n,
                                                        int* __restrict__ node, const int* __restrict__ feat,
                                                        const int* __restrict__ thr, const double* __restrict__ value,
                                                        const int* __restrict__ bins, int level, int last, float lr,
                                                        float* __restrict__ F, int K, int k) {
  const int hb = (1 << level) - 1;
  const int hc = (2 << level) - 1;  // first heap index of the next level
  const long long stride = (long long)gridDim.x * GT;
  for (long long r = (long long)blockIdx.x * GT + threadIdx.x; r < n; r += stride) {
    const int s = node[r];
    if (s < 0) continue;
    const int i = hb + s;
    const int f = feat[i];
    int nxt = -1;
    double v = value[i];
    if (f >= 0) {
      const unsigned c = codes[(long long)f * ld + r];
      if (c < (unsigned)bins[f]) {
        const int child = 2 * s + (c > (unsigned)thr[i] ? 1 : 0);
        if (last) v = value[hc + child];
        else nxt = child;
      }
    }
    if (nxt < 0) F[r * K + k] += lr * (float)v;
    node[r] = nxt;
  }
}

// Split scoring of one level, one workgroup per node (replaces ~25 small tensor ops per level):
//   * the node's [TB][2] fixed-point (g, h) histogram: given (level 0 / no subtraction), or built
//     from the parent level's histogram and the left-children histogram (odd slot = parent - left,
//     exact in int64) and written out as the next level's parent;
//   * per feature, the exact int64 prefix over its bins (one thread per feature);
//   * gain = gl^2 / max(hl + l2, 1e-12) + gr^2 / max(hr + l2, 1e-12) - parent over every threshold
//     position (fp64, no FMA contraction, the expression order of the host twin in models/tree.py),
//     argmax with ties to the lowest position;
//   * the node's feature / threshold and its two children's Newton values into the heap.
// Positions p < nb are the features' bins in histogram order (pstart / pend: the feature's first
// and last bin, pvalid: p < pend); slot `tot` holds the rows whose feature-0 code is missing, so
// feature 0's bins + `tot` are the node total (node_grad_hist_kernel tot_slot).
constexpr int GS_T = 256;

__global__ __launch_bounds__(GS_T) void gbt_split_kernel(const long long* __restrict__ hist,
                                                         const long long* __restrict__ parent,
                                                         const long long* __restrict__ left,
                                                         long long* __restrict__ out_hist, int TB, int tot,
                                                         const int* __restrict__ pfeat, const int* __restrict__ pthr,
                                                         const int* __restrict__ pstart, const int* __restrict__ pend,
                                                         const unsigned char* __restrict__ pvalid, int nb, double l2,
                                                         double invS, int hb, int hc, int level0,
                                                         int* __restrict__ feat, int* __restrict__ thr,
                                                         double* __restrict__ val) {
#pragma clang fp contract(off)
  extern __shared__ long long gs_smem[];
  long long* sh = gs_smem;            // [TB][2]
  long long* cs = gs_smem + 2 * TB;   // [nb][2] per-feature prefix sums
  __shared__ double bg[GS_T / 64];
  __shared__ int bp[GS_T / 64];
  const int a = blockIdx.x, tid = threadIdx.x;
  const long long w2 = 2LL * TB;
  for (int i = tid; i < 2 * TB; i += GS_T) {
    long long v;
    if (hist) {
      v = hist[a * w2 + i];
    } else {
      const long long l = left[(long long)(a >> 1) * w2 + i];
      v = (a & 1) ? parent[(long long)(a >> 1) * w2 + i] - l : l;
    }
    sh[i] = v;
    if (out_hist) out_hist[a * w2 + i] = v;
  }
  __syncthreads();
  for (int p = tid; p < nb; p += GS_T) {
    if (pstart[p] != p) continue;  // one thread per feature
    const int e = min(max(pend[p], p), nb - 1);
    long long g = 0, h = 0;
    for (int q = p; q <= e; ++q) {
      g += sh[2 * q];
      h += sh[2 * q + 1];
      cs[2 * q] = g;
      cs[2 * q + 1] = h;
    }
  }
  __syncthreads();
  // node total = feature 0's bins (positions 0..pend[0]) + the slot of rows missing feature 0
  const int e0 = min(max(pend[0], 0), nb - 1);
  const double G = (double)(cs[2 * e0] + sh[2 * tot]) * invS, H = (double)(cs[2 * e0 + 1] + sh[2 * tot + 1]) * invS;
  const double par = G * G / fmax(H + l2, 1e-12);
  double best = -INFINITY;
  int bpos = 0x7fffffff;
  for (int p = tid; p < nb; p += GS_T) {
    const int e = min(max(pend[p], p), nb - 1);
    const double gl = (double)cs[2 * p] * invS, hl = (double)cs[2 * p + 1] * invS;
    const double gr = (double)(cs[2 * e] - cs[2 * p]) * invS, hr = (double)(cs[2 * e + 1] - cs[2 * p + 1]) * invS;
    double gain = -INFINITY;
    if (hl > 1e-12 && hr > 1e-12 && pvalid[p]) gain = gl * gl / fmax(hl + l2, 1e-12) + gr * gr / fmax(hr + l2, 1e-12) - par;
    if (gain > best) { best = gain; bpos = p; }  // p ascends per thread: the first maximum stays
  }
  // block argmax, ties -> lowest position
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double ob = __shfl_xor(best, o, 64);
    const int op = __shfl_xor(bpos, o, 64);
    if (ob > best || (ob == best && op < bpos)) { best = ob; bpos = op; }
  }
  if ((tid & 63) == 0) { bg[tid >> 6] = best; bp[tid >> 6] = bpos; }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < GS_T / 64; ++w)
      if (bg[w] > best || (bg[w] == best && bp[w] < bpos)) { best = bg[w]; bpos = bp[w]; }
    const bool split = isfinite(best) && best > 1e-12;
    const int p = bpos < nb ? bpos : 0;
    feat[hb + a] = split ? pfeat[p] : -1;
    thr[hb + a] = pthr[p];
    const int e = min(max(pend[p], p), nb - 1);
    const double gl = (double)cs[2 * p] * invS, hl = (double)cs[2 * p + 1] * invS;
    const double gr = (double)(cs[2 * e] - cs[2 * p]) * invS, hr = (double)(cs[2 * e + 1] - cs[2 * p + 1]) * invS;
    val[hc + 2 * a] = split ? -gl / fmax(hl + l2, 1e-12) : 0.0;
    val[hc + 2 * a + 1] = split ? -gr / fmax(hr + l2, 1e-12) : 0.0;
    if (level0) val[0] = -G / fmax(H + l2, 1e-12);
  }
}

}  // namespace

namespace avk {

void gbt_split(const long long* hist, const long long* parent, const long long* left, long long* out_hist, int A,
               int TB, int tot, const int* pfeat, const int* pthr, const int* pstart, const int* pend,
               const unsigned char* pvalid, int nb, double l2, double invS, int hb, int hc, int level0, int* feat,
               int* thr, double* val, hipStream_t stream) {
  if (A <= 0) return;
  const size_t lds = sizeof(long long) * 2 * ((size_t)TB + nb);
  if (lds > 160 * 1024) throw std::runtime_error("gbt_split: histogram exceeds LDS");
  gbt_split_kernel<<<A, GS_T, lds, stream>>>(hist, parent, left, out_hist, TB, tot, pfeat, pthr, pstart, pend, pvalid,
                                             nb, l2, invS, hb, hc, level0, feat, thr, val);
  AV_HIP_CHECK(hipGetLastError());
}

void gbt_grad(const float* F, int K, int k, const uint8_t* y, long long n, long long row_off, unsigned long long seed,
              unsigned rate32, float* g, float* h, double* loss, hipStream_t stream) {
  if (n <= 0) return;
  gbt_grad_kernel<<<av::stream_grid(n, GT, 4, 4096), GT, 0, stream>>>(F, K, k, y, n, row_off, seed, rate32, g, h,
                                                                      loss);
  AV_HIP_CHECK(hipGetLastError());
}

void gbt_assign(const uint8_t* codes, long long ld, long long n, int* node, const int* feat, const int* thr,
                const double* value, const int* bins, int level, int last, float lr, float* F, int K, int k,
                hipStream_t stream) {
  if (n <= 0) return;
  gbt_assign_kernel<<<av::stream_grid(n, GT, 4, 4096), GT, 0, stream>>>(codes, ld, n, node, feat, thr, value, bins,
                                                                        level, last, lr, F, K, k);
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
