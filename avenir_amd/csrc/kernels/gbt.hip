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
    // per-wave sum, one atomic per wave (the loss is a report, not part of the model)
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (av::lane_id() == 0) atomicAdd(loss, acc);
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

}  // namespace

namespace avk {

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
