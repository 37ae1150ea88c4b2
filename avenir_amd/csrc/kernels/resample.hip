// K25: class-based re-sampling on the device for CDNA4 (gfx950).
//
// Reference: ClassBasedOverSampler (SMOTE) interpolates a minority record with one of its
// same-class neighbours and copies categorical values from either side, one synthetic record per
// draw of a java.util.Random (J/explore/ClassBasedOverSampler.java:125-200); UnderSamplingBalancer
// keeps a majority record with probability minCount / count (J/explore/UnderSamplingBalancer.java:
// 95-133); BaggingSampler draws bootstrap positions within batches (J/explore/BaggingSampler.java:
// 117-122).  Here every random draw is counter-based Philox4x32-10 keyed by (seed, stream, GLOBAL
// record index), so a rank produces exactly the records a single process would produce for the
// rows it owns — results do not depend on the world size — and the host twin
// (ops/random.philox4x32) reproduces them bit for bit.
//   * resample_uniform_kernel : u(seed, stream, base + i) in (0, 1] for i < n (undersampling and
//     bagging masks / positions);
//   * smote_kernel            : one thread per (source row, copy): neighbour pick (uniform, or the
//     reference's exponential rank pick), gap, categorical coin from ONE Philox draw, then the
//     interpolated numeric row and the categorical row written in one pass.
// Index safety: source rows < m, picks < n_nbr[row] <= k (a row with no neighbour copies itself),
// every output index < m * mult.
#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

constexpr int RS_T = 256;

__global__ __launch_bounds__(RS_T) void resample_uniform_kernel(unsigned long long seed, unsigned long long stream,
                                                                long long base, long long n, float* __restrict__ out) {
  const long long s = (long long)gridDim.x * RS_T;
  for (long long i = (long long)blockIdx.x * RS_T + threadIdx.x; i < n; i += s)
    out[i] = av::u32_to_unit(av::philox_draw(seed, stream, (unsigned long long)(base + i)).x);
}

// X [m, D] source rows, Xn [m, k, D] their neighbours' rows, nn [m] neighbours per row; Cs [m, Dc] /
// Cn [m, k, Dc] categorical codes (Dc may be 0).  Output row o = r * mult + j, counter
// (gbase + r) * mult + j: x.x -> neighbour pick, x.y -> gap, x.z -> categorical coin.
__global__ __launch_bounds__(RS_T) void smote_kernel(const float* __restrict__ X, const float* __restrict__ Xn,
                                                     const int* __restrict__ nn, const int* __restrict__ Cs,
                                                     const int* __restrict__ Cn, long long m, int k, int D, int Dc,
                                                     int mult, long long gbase, unsigned long long seed,
                                                     int exponential, float exp_mean, float* __restrict__ outX,
                                                     int* __restrict__ outC, int* __restrict__ outPick) {
  const long long total = m * mult;
  const long long s = (long long)gridDim.x * RS_T;
  for (long long o = (long long)blockIdx.x * RS_T + threadIdx.x; o < total; o += s) {
    const long long r = o / mult;
    const int j = (int)(o - r * mult);
    const av::u4 d = av::philox_draw(seed, 0x5EED0025ull, (unsigned long long)((gbase + r) * mult + j));
    const int cnt = nn[r];
    int pick = 0;
    if (cnt > 0) {
      if (exponential) {  // ClassBasedOverSampler exponential pick: round(-mean * ln u) - 1, clipped
        const double e = -(double)exp_mean * log((double)av::u32_to_unit(d.x));
        pick = (int)rint(e) - 1;
        pick = pick < 0 ? 0 : (pick >= cnt ? cnt - 1 : pick);
      } else {
        pick = (int)(av::u32_to_unit(d.x) * (float)cnt);
        pick = pick >= cnt ? cnt - 1 : pick;
      }
    }
    const float gap = av::u32_to_unit(d.y) - (1.0f / 16777216.0f);  // [0, 1)
    const float* src = X + r * D;
    const float* nb = cnt > 0 ? Xn + (r * k + pick) * D : src;
    float* dst = outX + o * D;
    {
      // no contraction into an FMA: the host twin rounds the product and the sum separately
#pragma clang fp contract(off)
      for (int c = 0; c < D; ++c) dst[c] = src[c] + gap * (nb[c] - src[c]);
    }
    if (Dc > 0) {
      const bool take_src = (d.z >> 31) != 0;
      const int* cs = Cs + r * Dc;
      const int* cn = cnt > 0 ? Cn + (r * k + pick) * Dc : cs;
      int* cd = outC + o * Dc;
      for (int c = 0; c < Dc; ++c) cd[c] = take_src ? cs[c] : cn[c];
    }
    if (outPick) outPick[o] = cnt > 0 ? pick : -1;
  }
}

}  // namespace

namespace avk {

void resample_uniform(unsigned long long seed, unsigned long long stream, long long base, long long n, float* out,
                      hipStream_t st) {
  if (n <= 0) return;
  resample_uniform_kernel<<<av::stream_grid(n, RS_T, 4, 4096), RS_T, 0, st>>>(seed, stream, base, n, out);
  AV_HIP_CHECK(hipGetLastError());
}

void smote(const float* X, const float* Xn, const int* nn, const int* Cs, const int* Cn, long long m, int k, int D,
           int Dc, int mult, long long gbase, unsigned long long seed, int exponential, float exp_mean, float* outX,
           int* outC, int* outPick, hipStream_t st) {
  if (m <= 0 || mult <= 0) return;
  smote_kernel<<<av::stream_grid(m * mult, RS_T, 1, 8192), RS_T, 0, st>>>(X, Xn, nn, Cs, Cn, m, k, D, Dc, mult, gbase,
                                                                          seed, exponential, exp_mean, outX, outC,
                                                                          outPick);
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
