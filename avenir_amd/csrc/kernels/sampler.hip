// K21: device random samplers on counter-based Philox4x32-10 (CDNA4, gfx950).
//
// Replaces the reference's per-call Python samplers (python/lib/sampler.py:180-920) and the
// per-record JVM samplers used by SMOTE / bagging / MC (J/explore, P/mlextra/mcsim.py:184-212):
// every element i of a draw is a pure function of (seed, offset, i), so a Monte-Carlo run sharded
// over any number of GPUs / workgroups reproduces the single-device stream exactly.
#include <algorithm>

#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

enum Dist : int {
  UNIFORM = 0,      // p0 = lo, p1 = hi
  NORMAL = 1,       // p0 = mean, p1 = sd
  EXPONENTIAL = 2,  // p0 = rate
  LOGNORMAL = 3,    // p0 = mu, p1 = sigma (of the underlying normal)
  GAMMA = 4,        // p0 = shape k, p1 = scale theta   (Marsaglia-Tsang)
  POISSON = 5,      // p0 = lambda                      (inversion for small, transformed rejection otherwise)
  PARETO = 6,       // p0 = shape a, p1 = scale xm
  TRIANGULAR = 7,   // p0 = lo, p1 = mode, p2 = hi
  BERNOULLI = 8,    // p0 = p
  TABLE = 9,        // inverse CDF over a bin table: cdf[nbins], p0 = lo, p1 = bin width
  UNIFORM_INT = 10  // p0 = lo, p1 = hi inclusive
};

__device__ __forceinline__ float normal_bm(av::u4 r) {
  const float u1 = av::u32_to_unit(r.x), u2 = av::u32_to_unit(r.y);
  return sqrtf(-2.f * __logf(u1)) * __cosf(6.283185307f * u2);
}

__device__ float gamma_mt(float k, unsigned long long seed, unsigned long long offset, unsigned long long idx) {
  // Marsaglia & Tsang (2000); k < 1 boosted by U^(1/k).  Each retry draws a fresh Philox block.
  float boost = 1.f;
  if (k < 1.f) {
    const av::u4 b = av::philox_draw(seed, offset ^ 0x5bd1e995ull, idx);
    boost = __powf(av::u32_to_unit(b.x), 1.f / k);
    k += 1.f;
  }
  const float d = k - 1.f / 3.f, c = 1.f / sqrtf(9.f * d);
  for (unsigned t = 0; t < 64; ++t) {
    const av::u4 r = av::philox_draw(seed, offset + ((unsigned long long)(t + 1) << 40), idx);
    const float x = normal_bm(r);
    const float v0 = 1.f + c * x;
    if (v0 <= 0.f) continue;
    const float v = v0 * v0 * v0;
    const float u = av::u32_to_unit(r.z);
    if (__logf(u) < 0.5f * x * x + d - d * v + d * __logf(v)) return d * v * boost;
  }
  return d * boost;  // practically unreachable
}

__device__ float poisson_draw(float lam, unsigned long long seed, unsigned long long offset, unsigned long long idx) {
  if (lam < 30.f) {  // inversion by sequential search
    const av::u4 r = av::philox_draw(seed, offset, idx);
    const float u = av::u32_to_unit(r.x);
    float p = __expf(-lam), s = p;
    int k = 0;
    while (u > s && k < 1000) {
      ++k;
      p *= lam / (float)k;
      s += p;
    }
    return (float)k;
  }
  // PTRS (Hormann 1993): transformed rejection with squeeze
  const float slam = sqrtf(lam), loglam = __logf(lam);
  const float b = 0.931f + 2.53f * slam, a = -0.059f + 0.02483f * b, invalpha = 1.1239f + 1.1328f / (b - 3.4f),
              vr = 0.9277f - 3.6224f / (b - 2.f);
  for (unsigned t = 0; t < 64; ++t) {
    const av::u4 r = av::philox_draw(seed, offset + ((unsigned long long)(t + 1) << 40), idx);
    const float u = av::u32_to_unit(r.x) - 0.5f, v = av::u32_to_unit(r.y);
    const float us = 0.5f - fabsf(u);
    const float k = floorf((2.f * a / us + b) * u + lam + 0.43f);
    if (us >= 0.07f && v <= vr) return k;
    if (k < 0.f || (us < 0.013f && v > us)) continue;
    if (__logf(v) + __logf(invalpha) - __logf(a / (us * us) + b) <= -lam + k * loglam - lgammaf(k + 1.f)) return k;
  }
  return lam;
}

// fp64 Gaussian pairs of Philox(seed, offset, index_base + i): the device twin of
// csrc/host/random.cpp (same counters, 53-bit uniforms, Box-Muller in double precision)
__device__ __forceinline__ double unit53(uint32_t a, uint32_t b) {
  const unsigned long long m = ((unsigned long long)a << 21) ^ (unsigned long long)(b >> 11);
  return ((double)(m & ((1ull << 53) - 1)) + 1.0) * (1.0 / 9007199254740992.0);
}

__global__ __launch_bounds__(256) void philox_normal_kernel(unsigned long long seed, unsigned long long offset,
                                                            unsigned long long index_base, long long n,
                                                            double* __restrict__ out, int pairs) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const av::u4 r = av::philox_draw(seed, offset, index_base + (unsigned long long)i);
    const double u1 = unit53(r.x, r.y), u2 = unit53(r.z, r.w);
    const double rad = sqrt(-2.0 * log(u1)), a = 6.283185307179586476925 * u2;
    if (pairs) {
      out[2 * i] = rad * cos(a);
      out[2 * i + 1] = rad * sin(a);
    } else {
      out[i] = rad * cos(a);
    }
  }
}

__global__ __launch_bounds__(256) void sample_kernel(int dist, long long n, const float* __restrict__ p,
                                                     const float* __restrict__ table, int nbins,
                                                     unsigned long long seed, unsigned long long offset,
                                                     float* __restrict__ out) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const av::u4 r = av::philox_draw(seed, offset, (unsigned long long)i);
    float v = 0.f;
    switch (dist) {
      case UNIFORM: v = p[0] + (p[1] - p[0]) * (av::u32_to_unit(r.x) - 0.5f / 16777216.f); break;
      case NORMAL: v = p[0] + p[1] * normal_bm(r); break;
      case EXPONENTIAL: v = -__logf(av::u32_to_unit(r.x)) / p[0]; break;
      case LOGNORMAL: v = __expf(p[0] + p[1] * normal_bm(r)); break;
      case GAMMA: v = gamma_mt(p[0], seed, offset, (unsigned long long)i) * p[1]; break;
      case POISSON: v = poisson_draw(p[0], seed, offset, (unsigned long long)i); break;
      case PARETO: v = p[1] / __powf(av::u32_to_unit(r.x), 1.f / p[0]); break;
      case TRIANGULAR: {
        const float lo = p[0], md = p[1], hi = p[2], u = av::u32_to_unit(r.x);
        const float fc = (md - lo) / (hi - lo);
        v = u < fc ? lo + sqrtf(u * (hi - lo) * (md - lo)) : hi - sqrtf((1.f - u) * (hi - lo) * (hi - md));
        break;
      }
      case BERNOULLI: v = av::u32_to_unit(r.x) <= p[0] ? 1.f : 0.f; break;
      case TABLE: {
        // binary search in the normalised CDF, uniform within the bin
        const float u = av::u32_to_unit(r.x);
        int lo = 0, hi = nbins - 1;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (table[mid] >= u) hi = mid;
          else lo = mid + 1;
        }
        v = p[0] + ((float)lo + av::u32_to_unit(r.y) - 0.5f / 16777216.f) * p[1];
        break;
      }
      case UNIFORM_INT: {
        const float span = p[1] - p[0] + 1.f;
        v = p[0] + fminf(floorf(av::u32_to_unit(r.x) * span - 0.5f / 16777216.f * span), span - 1.f);
        break;
      }
      default: break;
    }
    out[i] = v;
  }
}

}  // namespace

namespace avk {

void philox_normal(unsigned long long seed, unsigned long long offset, unsigned long long index_base, long long n,
                   double* out, int pairs, hipStream_t stream) {
  if (n <= 0) return;
  const long long blocks = std::min<long long>((n + 255) / 256, 4096);
  philox_normal_kernel<<<(unsigned)blocks, 256, 0, stream>>>(seed, offset, index_base, n, out, pairs);
  AV_HIP_CHECK(hipGetLastError());
}

void sample(int dist, long long n, const float* params, const float* table, int nbins, unsigned long long seed,
            unsigned long long offset, float* out, hipStream_t stream) {
  if (n <= 0) return;
  sample_kernel<<<av::stream_grid(n, 256, 4, 8192), 256, 0, stream>>>(dist, n, params, table, nbins, seed, offset,
                                                                      out);
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
