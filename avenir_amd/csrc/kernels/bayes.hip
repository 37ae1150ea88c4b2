// Naive Bayes batched inference (K-gather-product in log space + arbitration + confusion matrix).
//
// Reference behaviour: BayesianPredictor.predictClassValue scores every class as
// P(f|c) * P(c) / P(f) (J/bayesian/BayesianPredictor.java:396-421) and arbitrates by max
// (defaultArbitrate :342-370) or by misclassification cost (costArbitrate :375-391).  Here one
// thread scores one record for all classes with the [C][TB] log-probability table staged in LDS;
// continuous features use the class-conditional Gaussian (BayesianModel/FeatureCount).
#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

constexpr int PB = 256;

__global__ __launch_bounds__(PB) void nb_predict_kernel(
    const uint8_t* __restrict__ codes, long long ld, long long n, int nfeat,
    const int* __restrict__ offs, const float* __restrict__ logp /*[C][TB]*/,
    const float* __restrict__ logfp /*[TB] feature prior*/, int total_bins,
    const float* __restrict__ x /*[Fc][ldx]*/, long long ldx, int ncont,
    const float* __restrict__ gmean /*[C][Fc]*/, const float* __restrict__ ginvstd,
    const float* __restrict__ glognorm /*[C][Fc] = -log(std*sqrt(2pi))*/,
    const float* __restrict__ pmean /*[Fc] prior*/, const float* __restrict__ pinvstd,
    const float* __restrict__ plognorm, const float* __restrict__ logprior /*[C]*/, int C,
    int ref_scale, float* __restrict__ post /*[N][C] or null*/, int* __restrict__ pred,
    const uint8_t* __restrict__ labels, unsigned long long* __restrict__ confusion /*[C][C]*/) {
  extern __shared__ __attribute__((aligned(16))) float s_lp[];
  float* s_fp = s_lp + C * total_bins;
  int* s_off = reinterpret_cast<int*>(s_fp + total_bins);
  unsigned int* s_conf = reinterpret_cast<unsigned int*>(s_off + nfeat);
  for (int i = threadIdx.x; i < C * total_bins; i += PB) s_lp[i] = logp[i];
  for (int i = threadIdx.x; i < total_bins; i += PB) s_fp[i] = logfp ? logfp[i] : 0.f;
  for (int i = threadIdx.x; i < nfeat; i += PB) s_off[i] = offs[i];
  if (confusion)
    for (int i = threadIdx.x; i < C * C; i += PB) s_conf[i] = 0;
  __syncthreads();

  const long long stride = (long long)gridDim.x * PB;
  for (long long r = (long long)blockIdx.x * PB + threadIdx.x; r < n; r += stride) {
    // feature prior log P(f) (only for the reference-compatible ratio output)
    float lfp = 0.f;
    if (ref_scale) {
      for (int f = 0; f < nfeat; ++f) {
        const unsigned v = codes[(long long)f * ld + r];
        if (v != 255u) lfp += s_fp[s_off[f] + v];
      }
      for (int j = 0; j < ncont; ++j) {
        const float z = (x[(long long)j * ldx + r] - pmean[j]) * pinvstd[j];
        lfp += plognorm[j] - 0.5f * z * z;
      }
    }
    float best = -INFINITY, mx = -INFINITY, se = 0.f;
    int arg = 0;
    for (int c = 0; c < C; ++c) {
      float s = logprior[c];
      const float* lp = s_lp + c * total_bins;
      for (int f = 0; f < nfeat; ++f) {
        const unsigned v = codes[(long long)f * ld + r];
        if (v != 255u) s += lp[s_off[f] + v];
      }
      for (int j = 0; j < ncont; ++j) {
        const float z = (x[(long long)j * ldx + r] - gmean[c * ncont + j]) * ginvstd[c * ncont + j];
        s += glognorm[c * ncont + j] - 0.5f * z * z;
      }
      if (s > best) { best = s; arg = c; }
      // online log-sum-exp
      if (s > mx) { se = se * __expf(mx - s) + 1.f; mx = s; }
      else se += __expf(s - mx);
      if (post && ref_scale) post[r * C + c] = __expf(s - lfp);
    }
    pred[r] = arg;
    if (post && !ref_scale) {
      const float lse = mx + __logf(se);
      for (int c = 0; c < C; ++c) {
        float s = logprior[c];
        const float* lp = s_lp + c * total_bins;
        for (int f = 0; f < nfeat; ++f) {
          const unsigned v = codes[(long long)f * ld + r];
          if (v != 255u) s += lp[s_off[f] + v];
        }
        for (int j = 0; j < ncont; ++j) {
          const float z = (x[(long long)j * ldx + r] - gmean[c * ncont + j]) * ginvstd[c * ncont + j];
          s += glognorm[c * ncont + j] - 0.5f * z * z;
        }
        post[r * C + c] = __expf(s - lse);
      }
    }
    if (confusion) {
      const unsigned a = labels[r];
      if (a < (unsigned)C) atomicAdd(&s_conf[a * C + arg], 1u);
    }
  }
  if (confusion) {
    __syncthreads();
    for (int i = threadIdx.x; i < C * C; i += PB)
      if (s_conf[i]) atomicAdd(&confusion[i], (unsigned long long)s_conf[i]);
  }
}

}  // namespace

namespace avk {

void nb_predict(const uint8_t* codes, long long ld, long long n, int nfeat, const int* offs,
                const float* logp, const float* logfp, int total_bins, const float* x, long long ldx,
                int ncont, const float* gmean, const float* ginvstd, const float* glognorm,
                const float* pmean, const float* pinvstd, const float* plognorm,
                const float* logprior, int C, int ref_scale, float* post, int* pred,
                const uint8_t* labels, unsigned long long* confusion, hipStream_t stream) {
  if (n <= 0) return;
  const size_t lds = sizeof(float) * ((size_t)C * total_bins + total_bins) + sizeof(int) * nfeat +
                     sizeof(unsigned) * (confusion ? C * C : 0);
  if (lds > 160 * 1024) throw std::runtime_error("nb_predict: model table exceeds LDS");
  const int grid = av::stream_grid(n, PB, 4, 4096);
  nb_predict_kernel<<<grid, PB, lds, stream>>>(codes, ld, n, nfeat, offs, logp, logfp, total_bins, x,
                                               ldx, ncont, gmean, ginvstd, glognorm, pmean, pinvstd,
                                               plognorm, logprior, C, ref_scale, post, pred, labels,
                                               confusion);
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
