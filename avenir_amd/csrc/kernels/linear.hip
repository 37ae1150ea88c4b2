// K13: fused generalised-linear-model gradient (CDNA4, gfx950).
//
// Reference: LogisticRegressor.aggregate (J/regress/LogisticRegressor.java:61-73) computes, per
// record, sigma(w.x) and accumulates x * (y - sigma) — one mapper pass per Hadoop job
// (J/regress/LogisticRegressionJob.java:143-195).  Here ONE pass over the column-major feature
// matrix X [D, ld] (the framework's SoA layout: a wave's loads of one feature are contiguous) yields
//   g = sum_i sw_i * x_i * e_i        (e = y - sigma(z) | y - z | hinge subgradient y*[y z < 1])
//   loss = sum_i sw_i * l_i           (logistic NLL | squared/2 | hinge)
//   h_i = sw_i * sigma'(z_i)          (optional per-row curvature, for the Newton/IRLS Hessian GEMM)
// Each lane owns VEC consecutive rows (vector loads), keeps w and its gradient partials in
// registers, and the block reduces through wave DPP sums + LDS into one double partial row;
// partial rows are summed on device (deterministic: no float atomics).
#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

__device__ __forceinline__ float softplus(float z) {
  return z > 0.f ? z + log1pf(__expf(-z)) : log1pf(__expf(z));
}

template <int D, int VEC>
__global__ __launch_bounds__(256) void glm_grad_kernel(const float* __restrict__ X, long long ld, long long n,
                                                       const float* __restrict__ y, const float* __restrict__ sw,
                                                       const float* __restrict__ w, int mode,
                                                       double* __restrict__ partial, float* __restrict__ hw) {
  typedef float vf __attribute__((ext_vector_type(VEC)));
  __shared__ float red[4][D + 1];
  float wr[D];
#pragma unroll
  for (int k = 0; k < D; ++k) wr[k] = w[k];
  float g[D];
#pragma unroll
  for (int k = 0; k < D; ++k) g[k] = 0.f;
  float loss = 0.f;
  const long long nq = (n + VEC - 1) / VEC;
  const long long stride = (long long)gridDim.x * 256;
  for (long long q = (long long)blockIdx.x * 256 + threadIdx.x; q < nq; q += stride) {
    const long long r0 = q * VEC;
    vf xv[D];
#pragma unroll
    for (int k = 0; k < D; ++k) xv[k] = *reinterpret_cast<const vf*>(X + (long long)k * ld + r0);
    const vf yv = *reinterpret_cast<const vf*>(y + r0);
    vf sv;
    if (sw) sv = *reinterpret_cast<const vf*>(sw + r0);
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      if (r0 + v >= n) break;
      float z = 0.f;
#pragma unroll
      for (int k = 0; k < D; ++k) z = fmaf(wr[k], xv[k][v], z);
      const float yy = yv[v];
      const float s = sw ? sv[v] : 1.f;
      float e, l, h;
      if (mode == 0) {
        const float p = 1.f / (1.f + __expf(-z));
        e = yy - p;
        l = softplus(z) - yy * z;
        h = p * (1.f - p);
      } else if (mode == 1) {
        e = yy - z;
        l = 0.5f * e * e;
        h = 1.f;
      } else {
        const float m = yy * z;
        e = m < 1.f ? yy : 0.f;
        l = fmaxf(0.f, 1.f - m);
        h = 0.f;
      }
      e *= s;
#pragma unroll
      for (int k = 0; k < D; ++k) g[k] = fmaf(xv[k][v], e, g[k]);
      loss = fmaf(l, s, loss);
      if (hw) hw[r0 + v] = h * s;
    }
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    const float t = av::wave_sum(g[k]);
    if (lane == 0) red[wid][k] = t;
  }
  {
    const float t = av::wave_sum(loss);
    if (lane == 0) red[wid][D] = t;
  }
  __syncthreads();
  if (threadIdx.x <= D) {
    double acc = 0.0;
    for (int q = 0; q < 4; ++q) acc += (double)red[q][threadIdx.x];
    partial[(long long)blockIdx.x * (D + 1) + threadIdx.x] = acc;
  }
}

// Weighted Gram matrix G = sum_i h_i x_i x_i^T for D <= 32 (Newton / IRLS Hessian, ridge
// normal equations) on the matrix cores: each wave stages a 32-feature x 64-row tile of the
// column-major X in LDS (coalesced 256-B feature rows), then issues 32
// v_mfma_f32_32x32x2_f32 with A[i][k] = h_k x_k[i], B[k][j] = x_k[j] (k = row).  Each wave keeps
// its own 32x32 accumulator across all its tiles and writes it once; partials are summed in fp64
// on the device.  Replaces a skinny [D, n] x [n, D] library GEMM (K = n) that hipBLASLt rejects.
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(256) void gram_mfma_kernel(const float* __restrict__ X, long long ld, long long n, int D,
                                                        const float* __restrict__ h, float* __restrict__ partial) {
  __shared__ float tile[4][32][65];  // per wave: [feature][row] (+1 pad against bank conflicts)
  __shared__ float hs[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long long ntiles = (n + 63) / 64;
  const long long gw = (long long)blockIdx.x * 4 + w, nw = (long long)gridDim.x * 4;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  for (long long t = gw; t < ntiles; t += nw) {
    const long long row = t * 64 + lane;
    const bool ok = row < n;
    hs[w][lane] = ok ? (h ? h[row] : 1.f) : 0.f;
    for (int i = 0; i < 32; ++i) tile[w][i][lane] = (ok && i < D) ? X[(long long)i * ld + row] : 0.f;
    __builtin_amdgcn_s_waitcnt(0);  // LDS writes of this wave visible to its own lanes (wave-private tile)
    __builtin_amdgcn_wave_barrier();
#pragma unroll 8
    for (int kk = 0; kk < 32; ++kk) {
      const int r = 2 * kk + (lane >> 5);
      const float xv = tile[w][lane & 31][r];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xv * hs[w][r], xv, acc, 0, 0, 0);
    }
    __builtin_amdgcn_wave_barrier();
  }
  float* out = partial + gw * 1024;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    out[row * 32 + (lane & 31)] = acc[r];
  }
}

// D > 32: the Gram matrix in 32 x 32 blocks.  blockIdx.y enumerates the upper-triangular block
// pairs (bi <= bj); each wave stages the 32-feature x 64-row tiles of feature blocks bi and bj
// and accumulates G[bi, bj] = sum_k h_k x_k[bi] x_k[bj]^T with the same MFMA as above.  Partials
// per (wave, pair) are summed in fp64 on the device and mirrored into the lower triangle.
__global__ __launch_bounds__(256) void gram_mfma_pair_kernel(const float* __restrict__ X, long long ld, long long n,
                                                             int D, int nb, const float* __restrict__ h,
                                                             float* __restrict__ partial) {
  __shared__ float tile[4][2][32][65];
  __shared__ float hs[4][64];
  int p = blockIdx.y, bi = 0;
  while (p >= nb - bi) { p -= nb - bi; ++bi; }
  const int bj = bi + p;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long long ntiles = (n + 63) / 64;
  const long long gw = (long long)blockIdx.x * 4 + w, nw = (long long)gridDim.x * 4;
  const int sb = bi == bj ? 0 : 1;  // diagonal pairs read one tile twice
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  for (long long t = gw; t < ntiles; t += nw) {
    const long long row = t * 64 + lane;
    const bool ok = row < n;
    hs[w][lane] = ok ? (h ? h[row] : 1.f) : 0.f;
    for (int i = 0; i < 32; ++i) {
      const int fa = bi * 32 + i, fb = bj * 32 + i;
      tile[w][0][i][lane] = (ok && fa < D) ? X[(long long)fa * ld + row] : 0.f;
      if (sb) tile[w][1][i][lane] = (ok && fb < D) ? X[(long long)fb * ld + row] : 0.f;
    }
    __builtin_amdgcn_s_waitcnt(0);  // wave-private tiles: own LDS writes visible to own lanes
    __builtin_amdgcn_wave_barrier();
#pragma unroll 8
    for (int kk = 0; kk < 32; ++kk) {
      const int r = 2 * kk + (lane >> 5);
      const float xa = tile[w][0][lane & 31][r];
      const float xb = tile[w][sb][lane & 31][r];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xa * hs[w][r], xb, acc, 0, 0, 0);
    }
    __builtin_amdgcn_wave_barrier();
  }
  float* out = partial + (gw * gridDim.y + blockIdx.y) * 1024;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    out[row * 32 + (lane & 31)] = acc[r];
  }
}

// D in (32, 256]: the same one-pass gradient with the feature loop tiled through LDS.  A block
// walks row tiles of TR = 128 rows (grid-stride): the [D, TR] tile of the column-major X is staged
// in LDS with coalesced 512-B feature-row segments, two threads per row compute z = w.x over the
// tile (half the features each, one shuffle to combine), the loss and e = sw * f(z) (e to LDS),
// then thread k < D accumulates g_k += sum_r X[k, r] e_r from LDS in a register across all the
// block's tiles.  X is read from HBM exactly once; per-block partials are summed on the device.
constexpr int TR = 128;
constexpr int TDMAX = 256;

__global__ __launch_bounds__(256) void glm_grad_tiled_kernel(const float* __restrict__ X, long long ld, long long n,
                                                             int D, const float* __restrict__ y,
                                                             const float* __restrict__ sw, const float* __restrict__ w,
                                                             int mode, double* __restrict__ partial,
                                                             float* __restrict__ hw) {
  // dynamic LDS sized by D (D * 129 floats: 52 KB at D = 100, so several blocks share a CU)
  extern __shared__ float smem[];
  float* tile = smem;                      // [D][TR + 1]
  float* ws_ = tile + D * (TR + 1);        // [D]
  float* es = ws_ + D;                     // [TR]
  float* red = es + TR;                    // [4]
  const int t = threadIdx.x;
  for (int k = t; k < D; k += 256) ws_[k] = w[k];
  float gk = 0.f, loss = 0.f;
  const long long ntile = (n + TR - 1) / TR;
  const int half = (D + 1) / 2;
  for (long long tt = blockIdx.x; tt < ntile; tt += gridDim.x) {
    const long long r0 = tt * TR;
    __syncthreads();  // the previous tile's tile[] / es[] reads are done
    // stage: thread t loads rows (t & 127) of features k = 2j + (t >> 7)
    for (int k = t >> 7; k < D; k += 2) {
      const long long r = r0 + (t & (TR - 1));
      tile[k * (TR + 1) + (t & (TR - 1))] = r < n ? X[(long long)k * ld + r] : 0.f;
    }
    __syncthreads();
    // z: rows r = t >> 1, the feature half (t & 1)
    const int rr = t >> 1, hsel = t & 1;
    float z = 0.f;
    const int k0 = hsel ? half : 0, k1 = hsel ? D : half;
    for (int k = k0; k < k1; ++k) z = fmaf(ws_[k], tile[k * (TR + 1) + rr], z);
    z += __shfl_xor(z, 1, 64);
    if (hsel == 0) {
      const long long r = r0 + rr;
      float e = 0.f;
      if (r < n) {
        const float yy = y[r];
        const float s = sw ? sw[r] : 1.f;
        float l, h;
        if (mode == 0) {
          const float p = 1.f / (1.f + __expf(-z));
          e = yy - p;
          l = softplus(z) - yy * z;
          h = p * (1.f - p);
        } else if (mode == 1) {
          e = yy - z;
          l = 0.5f * e * e;
          h = 1.f;
        } else {
          const float m = yy * z;
          e = m < 1.f ? yy : 0.f;
          l = fmaxf(0.f, 1.f - m);
          h = 0.f;
        }
        e *= s;
        loss = fmaf(l, s, loss);
        if (hw) hw[r] = h * s;
      }
      es[rr] = e;
    }
    __syncthreads();
    if (t < D) {
#pragma unroll 8
      for (int r = 0; r < TR; ++r) gk = fmaf(tile[t * (TR + 1) + r], es[r], gk);
    }
  }
  const float lw = av::wave_sum(loss);
  if ((t & 63) == 0) red[t >> 6] = lw;
  __syncthreads();
  if (t < D) partial[(long long)blockIdx.x * (D + 1) + t] = (double)gk;
  if (t == 0) partial[(long long)blockIdx.x * (D + 1) + D] = (double)red[0] + red[1] + red[2] + red[3];
}

template <int D, int VEC>
void launch_glm(const float* X, long long ld, long long n, const float* y, const float* sw, const float* w, int mode,
                double* partial, int grid, float* hw, hipStream_t stream) {
  glm_grad_kernel<D, VEC><<<grid, 256, 0, stream>>>(X, ld, n, y, sw, w, mode, partial, hw);
}

}  // namespace

namespace avk {

int glm_grid(long long n) {
  const long long nq = (n + 3) / 4;
  return av::stream_grid(nq, 256, 4, 2048);
}

void glm_grad(const float* X, long long ld, long long n, int D, const float* y, const float* sw, const float* w,
              int mode, double* partial, int grid, float* hw, hipStream_t stream) {
  switch (D) {
    case 4: launch_glm<4, 4>(X, ld, n, y, sw, w, mode, partial, grid, hw, stream); break;
    case 8: launch_glm<8, 4>(X, ld, n, y, sw, w, mode, partial, grid, hw, stream); break;
    case 16: launch_glm<16, 4>(X, ld, n, y, sw, w, mode, partial, grid, hw, stream); break;
    case 32: launch_glm<32, 2>(X, ld, n, y, sw, w, mode, partial, grid, hw, stream); break;
    default:
      if (D > 32 && D <= TDMAX) {
        const size_t lds = sizeof(float) * ((size_t)D * (TR + 1) + D + TR + 4);
        glm_grad_tiled_kernel<<<grid, 256, lds, stream>>>(X, ld, n, D, y, sw, w, mode, partial, hw);
        break;
      }
      throw std::runtime_error("glm_grad: D must be 4, 8, 16, 32 or in (32, 256]");
  }
  AV_HIP_CHECK(hipGetLastError());
}

int gram_grid(long long n) { return av::stream_grid((n + 63) / 64, 4, 1, 1024); }

void weighted_gram(const float* X, long long ld, long long n, int D, const float* h, float* partial, int grid,
                   hipStream_t stream) {
  if (D <= 32) {
    gram_mfma_kernel<<<grid, 256, 0, stream>>>(X, ld, n, D, h, partial);
  } else {
    const int nb = (D + 31) / 32;
    gram_mfma_pair_kernel<<<dim3(grid, nb * (nb + 1) / 2), 256, 0, stream>>>(X, ld, n, D, nb, h, partial);
  }
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
