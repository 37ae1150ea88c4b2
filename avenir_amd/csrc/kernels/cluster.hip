// K16: fused k-means Lloyd step for MANY k-means runs at once — assignment + SSE + centroid
// partial sums in ONE pass over the data (CDNA4, gfx950).
//
// Reference: KmeansCluster (J/cluster/KmeansCluster.java, one MR job per iteration: mapper
// assigns each record to its nearest centroid, reducer averages) and the Spark job that runs many
// (numClusters, initGroup) instances keyed by group (S/cluster/KmeansCluster.scala:103-156).
//
// Design: the centroids of all R runs (concatenated [K_total][D], run r owns rows
// [roff[r], roff[r+1])) and their squared norms live in LDS; each lane owns one data row at a time,
// keeps it in registers (float4 loads), computes ||c||^2 - 2 x.c against every centroid from LDS
// broadcast reads, takes the per-run argmin, and adds the row into the per-workgroup LDS
// accumulator of the winning centroid of every run ([K_total][D+1], f32 ds_add; the last column
// counts).  The data is read ONCE per iteration for all runs; workgroup partials are summed in
// fp64 on the device.  D in {2,4,8,16,32,64} (host pads with zeros), R <= 16,
// K_total * (2D + 2) floats <= 64 KiB.
#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

constexpr int KB = 256;
constexpr int MAX_RUNS = 16;  // per-run SSE lives in (statically indexed) registers

template <int D>
__global__ __launch_bounds__(KB) void kmeans_step_kernel(const float* __restrict__ X, long long n,
                                                         const float* __restrict__ C, const int* __restrict__ roff,
                                                         int R, int* __restrict__ assign,
                                                         float* __restrict__ partial,
                                                         double* __restrict__ sse_partial) {
  extern __shared__ float lds[];
  __shared__ int s_off[MAX_RUNS + 1];
  __shared__ double red[KB / 64][MAX_RUNS];
  for (int i = threadIdx.x; i <= R; i += KB) s_off[i] = roff[i];
  __syncthreads();
  const int K = s_off[R];
  float* cen = lds;                 // [K][D]
  float* cnorm = cen + K * D;       // [K]
  float* acc = cnorm + K;           // [K][D + 1]
  for (int i = threadIdx.x; i < K * D; i += KB) cen[i] = C[i];
  for (int i = threadIdx.x; i < K * (D + 1); i += KB) acc[i] = 0.f;
  __syncthreads();
  for (int j = threadIdx.x; j < K; j += KB) {
    float s = 0.f;
    for (int d = 0; d < D; ++d) s = fmaf(cen[j * D + d], cen[j * D + d], s);
    cnorm[j] = s;
  }
  __syncthreads();
  double sse[MAX_RUNS];
#pragma unroll
  for (int r = 0; r < MAX_RUNS; ++r) sse[r] = 0.0;
  const long long stride = (long long)gridDim.x * KB;
  for (long long row = (long long)blockIdx.x * KB + threadIdx.x; row < n; row += stride) {
    float x[D];
    if constexpr (D % 4 == 0) {
#pragma unroll
      for (int d = 0; d < D; d += 4) {
        const float4 v = *reinterpret_cast<const float4*>(X + row * D + d);
        x[d] = v.x; x[d + 1] = v.y; x[d + 2] = v.z; x[d + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int d = 0; d < D; ++d) x[d] = X[row * D + d];
    }
    float xn = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) xn = fmaf(x[d], x[d], xn);
#pragma unroll
    for (int r = 0; r < MAX_RUNS; ++r) {
      if (r >= R) break;
      float best = INFINITY;
      int bj = s_off[r];
      for (int j = s_off[r]; j < s_off[r + 1]; ++j) {
        float dot = 0.f;
#pragma unroll
        for (int d = 0; d < D; ++d) dot = fmaf(x[d], cen[j * D + d], dot);
        const float dist = cnorm[j] - 2.f * dot;
        if (dist < best) { best = dist; bj = j; }
      }
      if (assign) assign[(long long)r * n + row] = bj - s_off[r];
      sse[r] += (double)fmaxf(best + xn, 0.f);
      float* a = acc + bj * (D + 1);
#pragma unroll
      for (int d = 0; d < D; ++d) atomicAdd(&a[d], x[d]);
      atomicAdd(&a[D], 1.f);
    }
  }
#pragma unroll
  for (int r = 0; r < MAX_RUNS; ++r) {
    if (r >= R) break;
    const double v = av::wave_sum(sse[r]);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][r] = v;
  }
  __syncthreads();
  float* out = partial + (long long)blockIdx.x * K * (D + 1);
  for (int i = threadIdx.x; i < K * (D + 1); i += KB) out[i] = acc[i];
  for (int r = threadIdx.x; r < R; r += KB) {
    double s = 0.0;
    for (int q = 0; q < KB / 64; ++q) s += red[q][r];
    sse_partial[(long long)blockIdx.x * R + r] = s;
  }
}

}  // namespace

namespace avk {

int kmeans_grid(long long n) {
  // ~16K rows per workgroup, between 256 and 4096 workgroups
  long long g = (n + 16383) / 16384;
  return (int)std::max(256LL, std::min(g, 4096LL));
}

void kmeans_step(const float* X, long long n, int D, const float* C, const int* roff, int R, int K, int* assign,
                 float* partial, double* sse_partial, int grid, hipStream_t stream) {
  if (R < 1 || R > MAX_RUNS) throw std::runtime_error("kmeans_step: 1 <= runs <= 16");
  const size_t lds = sizeof(float) * ((size_t)K * D + K + (size_t)K * (D + 1));
  if (lds > 64 * 1024) throw std::runtime_error("kmeans_step: total centroids * D too large for LDS");
  switch (D) {
#define AVK_KM(DD)                                                                                          \
  case DD:                                                                                                  \
    kmeans_step_kernel<DD><<<grid, KB, lds, stream>>>(X, n, C, roff, R, assign, partial, sse_partial); \
    break;
    AVK_KM(2) AVK_KM(4) AVK_KM(8) AVK_KM(16) AVK_KM(32) AVK_KM(64)
#undef AVK_KM
    default: throw std::runtime_error("kmeans_step: D must be 2, 4, 8, 16, 32 or 64");
  }
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
