// K16: fused k-means Lloyd step — assignment + SSE + centroid partial sums in ONE pass (CDNA4).
//
// Reference: KmeansCluster (J/cluster/KmeansCluster.java, one MR job per iteration: mapper
// assigns each record to its nearest centroid, reducer averages) and the Spark job that runs many
// (k, init-group) instances (S/cluster/KmeansCluster.scala:103-156).
//
// Design: centroids (k x D, padded D) and their squared norms live in LDS; each lane owns one row
// at a time, keeps the row in registers (vector loads of its D floats), computes ||x||^2 - 2 x.c +
// ||c||^2 against every centroid from LDS broadcast reads, takes the argmin, and adds the row into a
// per-workgroup LDS accumulator [k][D+1] (f32 ds_add over at most n / 256 rows per workgroup,
// summed across workgroups in fp64) — the data is read exactly once per iteration.  Workgroup partials are summed in fp64 on
// the device.  Sizes: D in {2,4,8,16,32,64} (host pads), k * (D + 1) <= 12288.
#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

constexpr int KB = 256;

template <int D>
__global__ __launch_bounds__(KB) void kmeans_step_kernel(const float* __restrict__ X, long long n,
                                                         const float* __restrict__ C, int k,
                                                         int* __restrict__ assign, float* __restrict__ partial,
                                                         double* __restrict__ sse_partial) {
  extern __shared__ float lds[];
  float* cen = lds;                 // [k][D]
  float* cnorm = cen + k * D;       // [k]
  float* acc = cnorm + k;           // [k][D + 1]  (last column = count)
  __shared__ double red[KB / 64];
  for (int i = threadIdx.x; i < k * D; i += KB) cen[i] = C[i];
  for (int i = threadIdx.x; i < k * (D + 1); i += KB) acc[i] = 0.f;
  __syncthreads();
  for (int j = threadIdx.x; j < k; j += KB) {
    float s = 0.f;
    for (int d = 0; d < D; ++d) s = fmaf(cen[j * D + d], cen[j * D + d], s);
    cnorm[j] = s;
  }
  __syncthreads();
  double sse = 0.0;
  const long long stride = (long long)gridDim.x * KB;
  for (long long r = (long long)blockIdx.x * KB + threadIdx.x; r < n; r += stride) {
    float x[D];
    if constexpr (D % 4 == 0) {
#pragma unroll
      for (int d = 0; d < D; d += 4) {
        const float4 v = *reinterpret_cast<const float4*>(X + r * D + d);
        x[d] = v.x; x[d + 1] = v.y; x[d + 2] = v.z; x[d + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int d = 0; d < D; ++d) x[d] = X[r * D + d];
    }
    float xn = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) xn = fmaf(x[d], x[d], xn);
    float best = INFINITY;
    int bj = 0;
    for (int j = 0; j < k; ++j) {
      float dot = 0.f;
#pragma unroll
      for (int d = 0; d < D; ++d) dot = fmaf(x[d], cen[j * D + d], dot);
      const float dist = cnorm[j] - 2.f * dot;
      if (dist < best) { best = dist; bj = j; }
    }
    if (assign) assign[r] = bj;
    sse += (double)fmaxf(best + xn, 0.f);
    float* a = acc + bj * (D + 1);
#pragma unroll
    for (int d = 0; d < D; ++d) atomicAdd(&a[d], x[d]);
    atomicAdd(&a[D], 1.f);
  }
  sse = av::wave_sum(sse);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sse;
  __syncthreads();
  float* out = partial + (long long)blockIdx.x * k * (D + 1);
  for (int i = threadIdx.x; i < k * (D + 1); i += KB) out[i] = acc[i];
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int q = 0; q < KB / 64; ++q) s += red[q];
    sse_partial[blockIdx.x] = s;
  }
}

}  // namespace

namespace avk {

int kmeans_grid(long long n) {
  // ~16K rows per workgroup (never fewer than 256 workgroups, at most 4096)
  long long g = (n + 16383) / 16384;
  return (int)std::max(256LL, std::min(g, 4096LL));
}

void kmeans_step(const float* X, long long n, int D, const float* C, int k, int* assign, float* partial,
                 double* sse_partial, int grid, hipStream_t stream) {
  const size_t lds = sizeof(float) * ((size_t)k * D + k + (size_t)k * (D + 1));
  if (lds > 64 * 1024) throw std::runtime_error("kmeans_step: k * D too large for LDS");
  switch (D) {
#define AVK_KM(DD) \
  case DD: kmeans_step_kernel<DD><<<grid, KB, lds, stream>>>(X, n, C, k, assign, partial, sse_partial); break;
    AVK_KM(2) AVK_KM(4) AVK_KM(8) AVK_KM(16) AVK_KM(32) AVK_KM(64)
#undef AVK_KM
    default: throw std::runtime_error("kmeans_step: D must be 2, 4, 8, 16, 32 or 64");
  }
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
