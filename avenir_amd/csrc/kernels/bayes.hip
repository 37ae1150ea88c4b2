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

// Wide tables (uint16 / int32 codes: categoricals beyond 255 values).  The [C][TB] table no longer
// fits LDS (10^5-value fields), so the model is read through L2 in the transposed layout
// logpT [TB][C]: one record-feature gather fetches the C class terms of its value from one
// contiguous run (one cache line for C <= 32), and the per-class scores live in registers
// (compile-time unrolled over NBW_MAXC with a C guard, so no scratch).  Codes >= bins[f] (missing
// or unknown) contribute nothing, as in the CPU oracle.
constexpr int NBW_MAXC = 32;

template <typename CT>
__global__ __launch_bounds__(PB) void nb_predict_wide_kernel(
    const CT* __restrict__ codes, long long ld, long long n, int nfeat, const int* __restrict__ offs,
    const int* __restrict__ bins, const float* __restrict__ logpT /*[TB][C]*/, const float* __restrict__ logfp,
    const float* __restrict__ x, long long ldx, int ncont, const float* __restrict__ gmean,
    const float* __restrict__ ginvstd, const float* __restrict__ glognorm, const float* __restrict__ pmean,
    const float* __restrict__ pinvstd, const float* __restrict__ plognorm, const float* __restrict__ logprior, int C,
    int ref_scale, float* __restrict__ post, int* __restrict__ pred, const uint8_t* __restrict__ labels,
    unsigned long long* __restrict__ confusion) {
  __shared__ unsigned s_conf[NBW_MAXC * NBW_MAXC];
  if (confusion)
    for (int i = threadIdx.x; i < C * C; i += PB) s_conf[i] = 0;
  __syncthreads();
  const long long stride = (long long)gridDim.x * PB;
  for (long long r = (long long)blockIdx.x * PB + threadIdx.x; r < n; r += stride) {
    float s[NBW_MAXC];
#pragma unroll
    for (int c = 0; c < NBW_MAXC; ++c) s[c] = c < C ? logprior[c] : -INFINITY;
    float lfp = 0.f;
    for (int f = 0; f < nfeat; ++f) {
      const unsigned v = (unsigned)codes[(long long)f * ld + r];
      if (v >= (unsigned)bins[f]) continue;
      const long long idx = (long long)offs[f] + v;
      const float* row = logpT + idx * C;
#pragma unroll
      for (int c = 0; c < NBW_MAXC; ++c)
        if (c < C) s[c] += row[c];
      if (ref_scale) lfp += logfp[idx];
    }
    for (int j = 0; j < ncont; ++j) {
      const float xv = x[(long long)j * ldx + r];
#pragma unroll
      for (int c = 0; c < NBW_MAXC; ++c)
        if (c < C) {
          const float z = (xv - gmean[c * ncont + j]) * ginvstd[c * ncont + j];
          s[c] += glognorm[c * ncont + j] - 0.5f * z * z;
        }
      if (ref_scale) {
        const float z = (xv - pmean[j]) * pinvstd[j];
        lfp += plognorm[j] - 0.5f * z * z;
      }
    }
    float best = -INFINITY;
    int arg = 0;
#pragma unroll
    for (int c = 0; c < NBW_MAXC; ++c)
      if (c < C && s[c] > best) { best = s[c]; arg = c; }
    pred[r] = arg;
    if (post) {
      float sub = lfp;
      if (!ref_scale) {
        float se = 0.f;
#pragma unroll
        for (int c = 0; c < NBW_MAXC; ++c)
          if (c < C) se += __expf(s[c] - best);
        sub = best + __logf(se);
      }
#pragma unroll
      for (int c = 0; c < NBW_MAXC; ++c)
        if (c < C) post[r * C + c] = __expf(s[c] - sub);
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

// Model finalisation: [C, TB+1] int64 counts (last column = class counts) -> float log tables.
// One workgroup per feature (+1 for the class prior); fp64 sums, floor at log_floor.  Replaces
// ~40 tiny torch launches in the training step (BayesianDistribution reducer + the predictor's
// table load, J/bayesian/BayesianDistribution.java:243-320).
__global__ __launch_bounds__(256) void nb_finalize_kernel(const long long* __restrict__ counts, int C, int TB,
                                                          const int* __restrict__ offs,
                                                          const int* __restrict__ bins, int F, float laplace,
                                                          float log_floor, float* __restrict__ logp,
                                                          float* __restrict__ logfp, float* __restrict__ logprior) {
  __shared__ double red[4];
  const int ld = TB + 1;
  const int f = blockIdx.x;
  auto block_sum = [&](double v) -> double {
    v = av::wave_sum(v);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    const double t = red[0] + red[1] + red[2] + red[3];
    __syncthreads();
    return t;
  };
  if (f == F) {  // class prior
    double v = 0.0;
    for (int c = threadIdx.x; c < C; c += 256) v += (double)counts[(long long)c * ld + TB];
    const double tot = block_sum(v);
    for (int c = threadIdx.x; c < C; c += 256) {
      const double p = tot > 0.0 ? (double)counts[(long long)c * ld + TB] / tot : 0.0;
      logprior[c] = fmaxf((float)log(fmax(p, 1e-300)), log_floor);
    }
    return;
  }
  const int o = offs[f], b = bins[f];
  // P(value | class) per class row
  for (int c = 0; c < C; ++c) {
    double v = 0.0;
    for (int j = threadIdx.x; j < b; j += 256) v += (double)counts[(long long)c * ld + o + j] + laplace;
    const double tot = block_sum(v);
    for (int j = threadIdx.x; j < b; j += 256) {
      const double x = (double)counts[(long long)c * ld + o + j] + laplace;
      const float lv = tot > 0.0 ? (float)log(fmax(x / tot, 1e-300)) : log_floor;
      logp[(long long)c * TB + o + j] = fmaxf(lv, log_floor);
    }
  }
  // P(value) over all classes
  double v = 0.0;
  for (int j = threadIdx.x; j < b; j += 256) {
    double s = laplace;
    for (int c = 0; c < C; ++c) s += (double)counts[(long long)c * ld + o + j];
    v += s;
  }
  const double tot = block_sum(v);
  for (int j = threadIdx.x; j < b; j += 256) {
    double s = laplace;
    for (int c = 0; c < C; ++c) s += (double)counts[(long long)c * ld + o + j];
    const float lv = tot > 0.0 ? (float)log(fmax(s / tot, 1e-300)) : log_floor;
    logfp[o + j] = fmaxf(lv, log_floor);
  }
}

}  // namespace

namespace avk {

void nb_finalize(const long long* counts, int C, int TB, const int* offs, const int* bins, int F, float laplace,
                 float log_floor, float* logp, float* logfp, float* logprior, hipStream_t stream) {
  nb_finalize_kernel<<<F + 1, 256, 0, stream>>>(counts, C, TB, offs, bins, F, laplace, log_floor, logp, logfp,
                                                 logprior);
  AV_HIP_CHECK(hipGetLastError());
}


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

template <typename CT>
static void nb_predict_wide_t(const CT* codes, long long ld, long long n, int nfeat, const int* offs, const int* bins,
                              const float* logpT, const float* logfp, const float* x, long long ldx, int ncont,
                              const float* gmean, const float* ginvstd, const float* glognorm, const float* pmean,
                              const float* pinvstd, const float* plognorm, const float* logprior, int C,
                              int ref_scale, float* post, int* pred, const uint8_t* labels,
                              unsigned long long* confusion, hipStream_t stream) {
  const int grid = av::stream_grid(n, PB, 4, 4096);
  nb_predict_wide_kernel<CT><<<grid, PB, 0, stream>>>(codes, ld, n, nfeat, offs, bins, logpT, logfp, x, ldx, ncont,
                                                      gmean, ginvstd, glognorm, pmean, pinvstd, plognorm, logprior, C,
                                                      ref_scale, post, pred, labels, confusion);
}

int nb_predict_wide_max_classes() { return NBW_MAXC; }

void nb_predict_wide(const void* codes, int code_bytes, long long ld, long long n, int nfeat, const int* offs,
                     const int* bins, const float* logpT, const float* logfp, const float* x, long long ldx, int ncont,
                     const float* gmean, const float* ginvstd, const float* glognorm, const float* pmean,
                     const float* pinvstd, const float* plognorm, const float* logprior, int C, int ref_scale,
                     float* post, int* pred, const uint8_t* labels, unsigned long long* confusion,
                     hipStream_t stream) {
  if (n <= 0) return;
  if (C < 1 || C > NBW_MAXC) throw std::runtime_error("nb_predict_wide: 1..32 classes");
  if (code_bytes == 4)
    nb_predict_wide_t<int>(static_cast<const int*>(codes), ld, n, nfeat, offs, bins, logpT, logfp, x, ldx, ncont, gmean,
                           ginvstd, glognorm, pmean, pinvstd, plognorm, logprior, C, ref_scale, post, pred, labels,
                           confusion, stream);
  else if (code_bytes == 2)
    nb_predict_wide_t<uint16_t>(static_cast<const uint16_t*>(codes), ld, n, nfeat, offs, bins, logpT, logfp, x, ldx,
                                ncont, gmean, ginvstd, glognorm, pmean, pinvstd, plognorm, logprior, C, ref_scale,
                                post, pred, labels, confusion, stream);
  else
    nb_predict_wide_t<uint8_t>(static_cast<const uint8_t*>(codes), ld, n, nfeat, offs, bins, logpT, logfp, x, ldx,
                               ncont, gmean, ginvstd, glognorm, pmean, pinvstd, plognorm, logprior, C, ref_scale, post,
                               pred, labels, confusion, stream);
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
