// K27: fused Linear + bias + activation for the feed-forward network (FeedForwardNetwork,
// P/supv/tnn.py:100-145 builds Linear -> activation pairs; torch runs them as an addmm followed by
// a separate activation kernel, i.e. the [M, N] pre-activation makes a full HBM round trip).
//
// Forward  Y = act(X W^T + b):  X [M, K] row-major, W [N, K] row-major (torch Linear layout).
//   Block = 256 threads = 4 waves over a 64 x 64 output tile; each wave owns a 32 x 32 quarter and
//   accumulates it with the exact-f32 MFMA v_mfma_f32_32x32x2_f32 (same rounding as an fmaf chain)
//   over K chunks of 32 staged in LDS (rows padded to 33 floats: the column-of-rows reads of the
//   A / B operands hit 32 distinct banks).  Bias and activation are applied to the accumulator in
//   registers and Y is stored once.
// Backward dZ = dY * act'(Y), db = colsum(dZ): one pass over dY / Y (the derivative is taken from
//   the stored output, so no pre-activation tensor is kept), per-block column partials reduced on
//   the host side of the op; dX = dZ W and dW = dZ^T X are plain GEMMs (hipBLASLt).
#include <algorithm>
#include <cstdlib>
#include <string>

#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

constexpr int MT = 256;  // threads
constexpr int TM = 64;   // output rows per block
constexpr int TN = 64;   // output cols per block
constexpr int KC = 32;   // K chunk in LDS

typedef float f32x16 __attribute__((ext_vector_type(16)));

// act codes: 0 identity, 1 relu, 2 sigmoid, 3 tanh, 4 leaky relu (0.01), 5 elu (alpha 1),
// 6 gelu (erf form, torch.nn.functional.gelu / BERT's "gelu"; forward only)
__device__ __forceinline__ float act_fwd(float z, int act) {
  switch (act) {
    case 6: return 0.5f * z * (1.f + erff(z * 0.70710678118654752f));
    case 1: return fmaxf(z, 0.f);
    case 2: return 1.f / (1.f + expf(-z));
    case 3: return tanhf(z);
    case 4: return z > 0.f ? z : 0.01f * z;
    case 5: return z > 0.f ? z : expm1f(z);
    default: return z;
  }
}

// derivative expressed through the output y = act(z)
__device__ __forceinline__ float act_grad_from_y(float y, int act) {
  switch (act) {
    case 1: return y > 0.f ? 1.f : 0.f;
    case 2: return y * (1.f - y);
    case 3: return 1.f - y * y;
    case 4: return y > 0.f ? 1.f : 0.01f;
    case 5: return y > 0.f ? 1.f : y + 1.f;
    default: return 1.f;
  }
}

// One K chunk of the X and W tiles held in registers (8 floats of each per thread): loaded for
// chunk c+1 while the MFMAs of chunk c run, then dropped into LDS.  VEC: 16-byte loads (K % 4 == 0).
template <bool VEC>
struct ChunkRegs {
  float x[8], w[8];
  // rows of length K (the stride); columns k >= kend read as zero (the end of a split-K slice)
  __device__ __forceinline__ void load(const float* __restrict__ X, const float* __restrict__ W, long long m0, int n0,
                                       int k0, int M, int N, int K, int kend) {
    const int tid = threadIdx.x;
    if constexpr (VEC) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int e4 = tid + MT * i, row = e4 >> 3, c = (e4 & 7) * 4;
        const long long m = m0 + row;
        const int n = n0 + row, k = k0 + c;
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
        if (m < M && k < kend) a = *reinterpret_cast<const float4*>(X + m * K + k);
        if (n < N && k < kend) b = *reinterpret_cast<const float4*>(W + (long long)n * K + k);
        x[4 * i] = a.x; x[4 * i + 1] = a.y; x[4 * i + 2] = a.z; x[4 * i + 3] = a.w;
        w[4 * i] = b.x; w[4 * i + 1] = b.y; w[4 * i + 2] = b.z; w[4 * i + 3] = b.w;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int e = tid + MT * i, row = e / KC, c = e % KC;
        const long long m = m0 + row;
        const int n = n0 + row, k = k0 + c;
        x[i] = (m < M && k < kend) ? X[m * K + k] : 0.f;
        w[i] = (n < N && k < kend) ? W[(long long)n * K + k] : 0.f;
      }
    }
  }
  __device__ __forceinline__ void store(float (*sX)[KC + 1], float (*sW)[KC + 1]) const {
    const int tid = threadIdx.x;
    if constexpr (VEC) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int e4 = tid + MT * i, row = e4 >> 3, c = (e4 & 7) * 4;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          sX[row][c + j] = x[4 * i + j];
          sW[row][c + j] = w[4 * i + j];
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int e = tid + MT * i, row = e / KC, c = e % KC;
        sX[row][c] = x[i];
        sW[row][c] = w[i];
      }
    }
  }
};

// (a second register set holding chunk c + 2 in flight measured slower at the 128-row split-K
// shapes: 12.1 vs 10.4 us per projection, profiles/r5_bert_kernel_stats_v3.csv)
// SPLIT: blockIdx.z is a slice [z kper, (z + 1) kper) of K and the raw tile goes to
// P[z][M][N] (bias and activation applied by linear_splitk_epilogue_kernel after the slice sum)
template <bool VEC, bool SPLIT>
__global__ __launch_bounds__(MT) void linear_act_fwd_kernel(const float* __restrict__ X, const float* __restrict__ W,
                                                             const float* __restrict__ b, float* __restrict__ Y,
                                                             int M, int N, int K, int act, int kper, int xcd) {
  __shared__ float sX[TM][KC + 1];
  __shared__ float sW[TN][KC + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  int tm = blockIdx.y, tn = blockIdx.x;
  if (xcd) {  // XCD-contiguous ranges of 8-row tile groups: an XCD's L2 holds its X band and reuses
              // each W tile across the group's rows
    const int ntn = gridDim.x, ntm = gridDim.y;
    av::grouped_tile(av::xcd_remap(blockIdx.y * ntn + blockIdx.x, ntm * ntn), ntm, ntn, 8, tm, tn);
  }
  const long long m0 = (long long)tm * TM;
  const int n0 = tn * TN;
  const int kb = SPLIT ? (int)blockIdx.z * kper : 0;
  const int ke = SPLIT ? min(K, kb + kper) : K;
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  ChunkRegs<VEC> pre;
  pre.load(X, W, m0, n0, kb, M, N, K, ke);
  for (int k0 = kb; k0 < ke; k0 += KC) {
    __syncthreads();  // previous chunk's MFMA reads are done
    pre.store(sX, sW);
    __syncthreads();
    if (k0 + KC < ke) pre.load(X, W, m0, n0, k0 + KC, M, N, K, ke);  // in flight during the MFMAs
    const int li = lane & 31, lk = lane >> 5;
#pragma unroll
    for (int k = 0; k < KC; k += 2) {
      const float a = sX[wm * 32 + li][k + lk];  // A[i = lane&31][k = lane>>5]
      const float w = sW[wn * 32 + li][k + lk];  // B[k = lane>>5][j = lane&31]
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, w, acc, 0, 0, 0);
    }
  }
  // epilogue: C/D map col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5)
  const int col = n0 + wn * 32 + (lane & 31);
  if (col >= N) return;
  if constexpr (SPLIT) {
    float* P = Y + (long long)blockIdx.z * M * N;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const long long row = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row < M) P[row * N + col] = acc[r];
    }
  } else {
    const float bias = b ? b[col] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const long long row = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row < M) Y[row * N + col] = act_fwd(acc[r] + bias, act);
    }
  }
}

// Large outputs (>= 1,024 rows and columns): a 128 x 128 tile per workgroup, each wave a 64 x 64
// quarter as 2 x 2 v_mfma_f32_32x32x2_f32 blocks, so every A / B value read from LDS feeds two
// MFMAs and each K chunk brings 16 MACs per staged byte (the 64 x 64 tile: 8).  Chunks of 32 K
// columns register-prefetched during the MFMAs, as the 64 x 64 kernel.  VEC (K % 4 == 0,
// 16-byte-aligned operands) only.
constexpr int TB = 128, KCB = 32, LSB = KCB + 1;
__global__ __launch_bounds__(MT) void linear_act_fwd_big_kernel(const float* __restrict__ X,
                                                                const float* __restrict__ W,
                                                                const float* __restrict__ b, float* __restrict__ Y,
                                                                int M, int N, int K, int act, int xcd) {
  __shared__ float sX[TB][LSB];
  __shared__ float sW[TB][LSB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  int tm = blockIdx.y, tn = blockIdx.x;
  if (xcd) av::grouped_tile(av::xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y), gridDim.y,
                            gridDim.x, 8, tm, tn);
  const long long m0 = (long long)tm * TB;
  const int n0 = tn * TB;
  // thread's staging slots: 4 float4 of X and 4 of W per chunk (rows e >> 3, columns (e & 7) * 4)
  float4 px[4], pw[4];
  auto load = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + MT * i, r = e >> 3, c = (e & 7) * 4, k = k0 + c;
      const long long m = m0 + r;
      const int n = n0 + r;
      px[i] = (m < M && k < K) ? *reinterpret_cast<const float4*>(X + m * K + k) : make_float4(0.f, 0.f, 0.f, 0.f);
      pw[i] = (n < N && k < K) ? *reinterpret_cast<const float4*>(W + (long long)n * K + k)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  load(0);
  const int li = lane & 31, lk = lane >> 5;
  for (int k0 = 0; k0 < K; k0 += KCB) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + MT * i, r = e >> 3, c = (e & 7) * 4;
      sX[r][c] = px[i].x; sX[r][c + 1] = px[i].y; sX[r][c + 2] = px[i].z; sX[r][c + 3] = px[i].w;
      sW[r][c] = pw[i].x; sW[r][c + 1] = pw[i].y; sW[r][c + 2] = pw[i].z; sW[r][c + 3] = pw[i].w;
    }
    __syncthreads();
    if (k0 + KCB < K) load(k0 + KCB);
#pragma unroll
    for (int k = 0; k < KCB; k += 2) {
      float a[2], w[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = sX[wm * 64 + 32 * i + li][k + lk];
#pragma unroll
      for (int j = 0; j < 2; ++j) w[j] = sW[wn * 64 + 32 * j + li][k + lk];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], w[j], acc[i][j], 0, 0, 0);
    }
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = n0 + wn * 64 + 32 * j + (lane & 31);
    if (col >= N) continue;
    const float bias = b ? b[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long long row = m0 + wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row < M) Y[row * N + col] = act_fwd(acc[i][j][r] + bias, act);
      }
  }
}

// ---- split-bf16 tiles: fp32 GEMM on the bf16 matrix cores ----------------------------------------
// CDNA4's fp32 MFMA (v_mfma_f32_32x32x2_f32) runs at the packed-fp32 VALU rate, 1/16 of the bf16
// MFMA.  Every fp32 operand is split ONCE while it is staged into LDS into NS bf16 terms,
// x = x_0 + x_1 (+ x_2), each the round-to-nearest bf16 of the remaining residual (the residual
// x - x_0 is exact in fp32), and the tile is accumulated in fp32 on v_mfma_f32_32x32x16_bf16 over
// the cross products that matter:
//   NS = 2 ("bf16x3"): x_1 w_0 + x_0 w_1 + x_0 w_0 — inputs carried to ~16 significand bits, the
//                      dropped x_1 w_1 ~ 2^-18 |x w|: per-product error ~2^-17 relative;
//   NS = 3 ("bf16x6"): + x_2 w_0 + x_1 w_1 + x_0 w_2 — ~24 bits, fp32-level error.
// bf16 has fp32's exponent range, so no scaling is needed (an input of +-inf yields NaN here).  The
// small terms are accumulated first (products of one term order per pass over the wave's blocks,
// so consecutive MFMAs never hit the same accumulator).
// LDS image per term: [rows][32 k + 8 pad] bf16, 80-byte rows: a lane's fragment (8 consecutive k
// of one row) is one ds_read_b128 and the 16 rows of a 16-lane group land on 16 disjoint 4-bank
// groups (row r at bank 20 r mod 64).  Tile = 64 WB x 64 WB outputs, 4 waves, each a (32 WB)^2
// quarter as WB x WB 32 x 32 blocks; the next chunk's fp32 loads are register-prefetched during
// the MFMAs of the current one (as the fp32 tiles above).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef float f32x2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned pack_bf16(float a, float b) {  // v_cvt_pk_bf16_f32 (RNE)
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2v){a, b}, bf16x2v));
}
__device__ __forceinline__ float bf16_lo(unsigned p) { return __builtin_bit_cast(float, p << 16); }
__device__ __forceinline__ float bf16_hi(unsigned p) { return __builtin_bit_cast(float, p & 0xffff0000u); }

// split 4 consecutive fp32 values into NS bf16 terms and store each term's 8 bytes at `dst[t]`
template <int NS>
__device__ __forceinline__ void split_store4(float4 v, unsigned short* const* dst, int off) {
  float r[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int t = 0; t < NS; ++t) {
    const unsigned p0 = pack_bf16(r[0], r[1]), p1 = pack_bf16(r[2], r[3]);
    *reinterpret_cast<uint2*>(dst[t] + off) = make_uint2(p0, p1);
    if (t + 1 < NS) {
      r[0] -= bf16_lo(p0); r[1] -= bf16_hi(p0);
      r[2] -= bf16_lo(p1); r[3] -= bf16_hi(p1);
    }
  }
}

// SWZ: the term images unpadded, [rows][SKC] bf16, the 16-byte k-segment s of row r stored at
// s ^ ((r / (128 / SKC)) & (SKC / 8 - 1)) — the 16 rows a 16-lane group reads still land on 16
// disjoint 4-bank groups, and the x6 128 x 128 tile drops from 61,440 to 49,152 bytes of LDS, so three
// workgroups fit a CU (with OCC = 3 waves / SIMD asked of the register allocator): 768 output tiles
// (4,096 x 3,072 or 16,384 x 768 outputs) are then one round over 256 CUs instead of 1.5.
template <int WB, int NS, bool SPLIT, int SKC, bool SWZ = false, int OCC = 1>
__global__ __launch_bounds__(MT, OCC) void linear_act_fwd_sbf16_kernel(const float* __restrict__ X,
                                                                  const float* __restrict__ W,
                                                                  const float* __restrict__ b, float* __restrict__ Y,
                                                                  int M, int N, int K, int act, int kper, int xcd) {
  constexpr int TR = 64 * WB;        // tile rows = tile cols
  constexpr int SROW = SWZ ? SKC : SKC + 8;  // LDS row (bf16): swizzled, or 80 / 144 padded bytes
  constexpr int RSH = SKC == 32 ? 2 : 1;     // rows per 256 bytes = 1 << RSH (swizzle period)
  constexpr int F4R = SKC / 4;       // float4 per row and chunk
  constexpr int PF = TR * F4R / MT;  // float4 of each operand per thread and chunk
  __shared__ __attribute__((aligned(16))) unsigned short sX[NS][TR][SROW];
  __shared__ __attribute__((aligned(16))) unsigned short sW[NS][TR][SROW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  int tm = blockIdx.y, tn = blockIdx.x;
  if (xcd) av::grouped_tile(av::xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y), gridDim.y,
                            gridDim.x, 8, tm, tn);
  const long long m0 = (long long)tm * TR;
  const int n0 = tn * TR;
  const int kb = SPLIT ? (int)blockIdx.z * kper : 0;
  const int ke = SPLIT ? min(K, kb + kper) : K;
  float4 px[PF], pw[PF];
  auto load = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int e = tid + MT * i, r = e / F4R, k = k0 + (e % F4R) * 4;
      const long long m = m0 + r;
      const int n = n0 + r;
      px[i] = (m < M && k < ke) ? *reinterpret_cast<const float4*>(X + m * K + k) : make_float4(0.f, 0.f, 0.f, 0.f);
      pw[i] = (n < N && k < ke) ? *reinterpret_cast<const float4*>(W + (long long)n * K + k)
                                : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  f32x16 acc[WB][WB];
#pragma unroll
  for (int i = 0; i < WB; ++i)
#pragma unroll
    for (int j = 0; j < WB; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  unsigned short* dX[NS];
  unsigned short* dW[NS];
#pragma unroll
  for (int t = 0; t < NS; ++t) {
    dX[t] = &sX[t][0][0];
    dW[t] = &sW[t][0][0];
  }
  load(kb);
  const int li = lane & 31, lh = (lane >> 5) * 8;
  for (int k0 = kb; k0 < ke; k0 += SKC) {
    __syncthreads();  // the previous chunk's fragment reads are done
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int e = tid + MT * i, r = e / F4R, k4 = (e % F4R) * 4;
      const int off = SWZ ? r * SROW + ((((k4 >> 3) ^ (r >> RSH)) & (SKC / 8 - 1)) << 3) + (k4 & 7)
                          : r * SROW + k4;
      split_store4<NS>(px[i], dX, off);
      split_store4<NS>(pw[i], dW, off);
    }
    __syncthreads();
    if (k0 + SKC < ke) load(k0 + SKC);  // in flight during the MFMAs
#pragma unroll
    for (int ks = 0; ks < SKC; ks += 16) {
      bf16x8 a[NS][WB], w[NS][WB];
      auto col = [&](int r) __attribute__((always_inline)) {
        return SWZ ? ((((ks + lh) >> 3) ^ (r >> RSH)) & (SKC / 8 - 1)) << 3 : ks + lh;
      };
#pragma unroll
      for (int t = 0; t < NS; ++t) {
#pragma unroll
        for (int i = 0; i < WB; ++i) {
          const int r = wm * 32 * WB + 32 * i + li;
          a[t][i] = *reinterpret_cast<const bf16x8*>(&sX[t][r][col(r)]);
        }
#pragma unroll
        for (int j = 0; j < WB; ++j) {
          const int r = wn * 32 * WB + 32 * j + li;
          w[t][j] = *reinterpret_cast<const bf16x8*>(&sW[t][r][col(r)]);
        }
      }
      // term orders, smallest first: (order 2: x2w0, x1w1, x0w2), (order 1: x1w0, x0w1), (order 0)
#pragma unroll
      for (int ord = NS - 1; ord >= 0; --ord)
#pragma unroll
        for (int ta = ord; ta >= 0; --ta) {
          const int tw = ord - ta;
#pragma unroll
          for (int i = 0; i < WB; ++i)
#pragma unroll
            for (int j = 0; j < WB; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ta][i], w[tw][j], acc[i][j], 0, 0, 0);
        }
    }
  }
  // epilogue: C/D map of 32x32x16 (as 32x32x2) col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5)
#pragma unroll
  for (int j = 0; j < WB; ++j) {
    const int col = n0 + wn * 32 * WB + 32 * j + (lane & 31);
    if (col >= N) continue;
    if constexpr (SPLIT) {
      float* P = Y + (long long)blockIdx.z * M * N;
#pragma unroll
      for (int i = 0; i < WB; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const long long row = m0 + wm * 32 * WB + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (row < M) P[row * N + col] = acc[i][j][r];
        }
    } else {
      const float bias = b ? b[col] : 0.f;
#pragma unroll
      for (int i = 0; i < WB; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const long long row = m0 + wm * 32 * WB + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (row < M) Y[row * N + col] = act_fwd(acc[i][j][r] + bias, act);
        }
    }
  }
}

// Y[e] = act(sum_s P[s][e] + b[e % N]): the S slices summed in slice order (deterministic), the
// loads of 8 slices issued together
__global__ __launch_bounds__(256) void linear_splitk_epilogue_kernel(const float* __restrict__ P,
                                                                     const float* __restrict__ b,
                                                                     float* __restrict__ Y, long long MN, int N,
                                                                     int S, int act) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= MN) return;
  float s = 0.f;
  int k = 0;
  for (; k + 8 <= S; k += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = P[(long long)(k + u) * MN + e];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; k < S; ++k) s += P[(long long)k * MN + e];
  Y[e] = act_fwd(s + (b ? b[e % N] : 0.f), act);
}

// dZ = dY * act'(Y); partial[blockIdx.y][n] = sum over this block's `rows` rows of dZ[., n].
// `rows` (linear_act_bwd_rows: 16..256) gives small M enough workgroups, and a thread's rows are
// walked 4 at a time with their loads issued together: a DQN layer (256 x 128) took 20.5 us in 2
// workgroups of 64 dependent row iterations (profiles/r6_dqn_kernel_stats.csv)
constexpr int BR_ROWS = 256;
__global__ __launch_bounds__(MT) void linear_act_bwd_kernel(const float* __restrict__ dY, const float* __restrict__ Y,
                                                             float* __restrict__ dZ, float* __restrict__ partial,
                                                             int M, int N, int act, int rows) {
  __shared__ float s[MT / 64][64];
  const int c = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + c;
  const long long r0 = (long long)blockIdx.y * rows;
  const long long r1 = r0 + rows < M ? r0 + rows : M;
  float acc = 0.f;
  if (n < N) {
    for (long long m0 = r0 + rg; m0 < r1; m0 += 4 * (MT / 64)) {
      float dy[4], yv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long long m = m0 + u * (MT / 64);
        dy[u] = m < r1 ? dY[m * N + n] : 0.f;
        yv[u] = m < r1 ? Y[m * N + n] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long long m = m0 + u * (MT / 64);
        if (m < r1) {
          const float g = dy[u] * act_grad_from_y(yv[u], act);
          dZ[m * N + n] = g;
          acc += g;
        }
      }
    }
  }
  s[rg][c] = acc;
  __syncthreads();
  if (rg == 0 && n < N) {
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < MT / 64; ++j) t += s[j][c];
    partial[(long long)blockIdx.y * N + n] = t;
  }
}

// Weight gradient with the activation derivative fused in: dW = dZ^T X, db = colsum(dZ), dZ =
// dY * act'(Y) computed while the tile is staged (and written once, by the k-tile-0 blocks, for the
// dX GEMM).  Block = 4 waves over a 64 (n) x 64 (k) tile of dW and one slice of rows of M; chunks of
// 32 rows of dZ and X go through LDS and feed v_mfma_f32_32x32x2_f32 with m as the contraction
// index; every slice writes a partial tile, summed in a fixed order by linear_act_wgrad_reduce_kernel
// (deterministic).  The library GEMM this replaces (dZ^T X with M = 65,536 rows reduced inside a
// couple of output tiles) ran at ~2.5 TFLOP/s.
constexpr int MC = 32;
constexpr int WPT = (MC * 64) / MT;  // elements of each staged array per thread and chunk

struct WgradRegs {  // one chunk of dY, Y (n-tile columns) and X (k-tile columns) in flight
  float dy[WPT], y[WPT], x[WPT];
  __device__ __forceinline__ void load(const float* __restrict__ dY, const float* __restrict__ Y,
                                       const float* __restrict__ X, long long m0, long long r1, int n0, int k0, int N,
                                       int K) {
#pragma unroll
    for (int i = 0; i < WPT; ++i) {
      const int e = threadIdx.x + MT * i, row = e >> 6, c = e & 63;
      const long long m = m0 + row;
      const int n = n0 + c, k = k0 + c;
      const bool okz = m < r1 && n < N;
      dy[i] = okz ? dY[m * N + n] : 0.f;
      y[i] = okz ? Y[m * N + n] : 0.f;
      x[i] = (m < r1 && k < K) ? X[m * K + k] : 0.f;
    }
  }
};

__global__ __launch_bounds__(MT) void linear_act_wgrad_kernel(const float* __restrict__ dY, const float* __restrict__ Y,
                                                               const float* __restrict__ X, float* __restrict__ dZ,
                                                               float* __restrict__ pW, int M, int N, int K,
                                                               int rows_per_slice, int act) {
  __shared__ float sZ[MC][TN + 1];
  __shared__ float sX[MC][TN + 1];
  __shared__ float sB[MT / 64][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave >> 1, wk = wave & 1;
  const int n0 = blockIdx.x * 64, k0 = blockIdx.y * 64;
  const long long sl = blockIdx.z;
  const long long r0 = sl * rows_per_slice, r1 = min((long long)M, r0 + rows_per_slice);
  const bool lead = blockIdx.y == 0;
  const long long row_stride = (long long)N * K + N;  // dW partial then db partial
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  float bacc = 0.f;  // column tid & 63 of this thread's rows
  const int li = lane & 31, lm = lane >> 5;
  WgradRegs pre;
  if (r0 < r1) pre.load(dY, Y, X, r0, r1, n0, k0, N, K);
  for (long long m0 = r0; m0 < r1; m0 += MC) {
    __syncthreads();  // the previous chunk's MFMA reads are done
#pragma unroll
    for (int i = 0; i < WPT; ++i) {
      const int e = tid + MT * i, row = e >> 6, c = e & 63;
      const float z = pre.dy[i] * act_grad_from_y(pre.y[i], act);  // 0 outside the tile (dy = 0)
      if (lead && dZ && m0 + row < r1 && n0 + c < N) dZ[(m0 + row) * N + n0 + c] = z;
      sZ[row][c] = z;
      bacc += z;
      sX[row][c] = pre.x[i];
    }
    __syncthreads();
    if (m0 + MC < r1) pre.load(dY, Y, X, m0 + MC, r1, n0, k0, N, K);  // in flight during the MFMAs
#pragma unroll
    for (int mm = 0; mm < MC; mm += 2) {
      const float a = sZ[mm + lm][wn * 32 + li];  // A[i = n][k = m]
      const float b = sX[mm + lm][wk * 32 + li];  // B[k = m][j = k]
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
  }
  const int col = k0 + wk * 32 + (lane & 31);
  if (col < K) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int n = n0 + wn * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (n < N) pW[sl * row_stride + (long long)n * K + col] = acc[r];
    }
  }
  if (lead) {  // bias partial in the tail of the slice row
    sB[wave][lane] = bacc;
    __syncthreads();
    if (wave == 0 && n0 + lane < N)
      pW[sl * row_stride + (long long)N * K + n0 + lane] = sB[0][lane] + sB[1][lane] + sB[2][lane] + sB[3][lane];
  }
}

// out[y][e] = sum of in[s][e] over slices s in [y * span, (y + 1) * span), e < E: a block = 64
// elements x 16 slice groups, the group sums combined in a fixed order (deterministic).  Two passes
// (span 64, then the rest) keep every thread's serial chain short at any slice count.
constexpr int RG = 16;
__global__ __launch_bounds__(64 * RG) void slice_sum_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                            int S, int span, long long E) {
  __shared__ float sw[RG][64];
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
  const long long e = (long long)blockIdx.x * 64 + c;
  const int s0 = blockIdx.y * span, s1 = min(S, s0 + span);
  float t = 0.f;
  if (e < E)
    for (int s = s0 + g; s < s1; s += RG) t += in[(long long)s * E + e];
  sw[g][c] = t;
  __syncthreads();
  if (g == 0 && e < E) {
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < RG; ++k) a += sw[k][c];
    out[(long long)blockIdx.y * E + e] = a;
  }
}

// ---- pre-split ("planes") path of the split-bf16 tiles at large shapes ------------------------
// The in-loop split of linear_act_fwd_sbf16_kernel spends ~1.1k VALU cycles per wave and K chunk
// and a register-staged, single-buffered chunk that exposes the L2 / MALL latency: at 4,096 x 3,072
// x 768 (x6) its MFMA pipes are busy 34 % of the kernel (profiles/r6_k27_pmc_4096x3072x768.jsonl).
// Here one streaming pass writes each operand as NS bf16 term planes, and the GEMM tile reads them
// through a 3-stage LDS ring filled by global_load_lds_dwordx4 (no VGPR staging, no VALU in the K
// loop): stage t + 2 is in flight while stage t feeds the MFMAs, one counted vmcnt and one barrier
// per 32-deep K step.  Plane layout [t][Rp / 16][Kp / 32][16][32] (rows zero-padded to Rp, a
// multiple of 128, K to Kp, a multiple of 32): each 16-row x 32-k block is one contiguous KiB, so a
// DMA wave-instruction reads 8 whole 128-byte lines (row-major planes cost 16 half-used lines per
// instruction, the other halves re-fetched a stage later: 204 vs 147 us for the in-loop split tile
// at 4,096 x 3,072 x 768).

// in [R][K] fp32 -> out planes (layout above, blocks of RPB = 512 / BK rows x BK k); one thread per
// 8 k of one row, a wave per 1-KiB block
template <int NS, int BK>
__global__ __launch_bounds__(256) void sbf16_split_rows_kernel(const float* __restrict__ in,
                                                               unsigned short* __restrict__ out, long long R, int K,
                                                               long long Rp, int Kp, bool vec) {
  // grid (Rp / RPB, ceil(kb / 4)): wave w of a workgroup writes block (blockIdx.x, 4 blockIdx.y + w)
  constexpr int SEGS = BK / 8, RPB = 512 / BK;
  const int kb = Kp / BK, lane = threadIdx.x & 63;
  const int kc = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (kc >= kb) return;
  const int seg = lane % SEGS, rr = lane / SEGS;
  const long long blk = (long long)blockIdx.x * kb + kc;
  const long long r = (long long)blockIdx.x * RPB + rr;
  const int k = kc * BK + seg * 8;
  float v[8];
  if (r >= R) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.f;
  } else {
    const float* src = in + r * K + k;
    if (vec && k + 8 <= K) {
      const float4 a = *reinterpret_cast<const float4*>(src), c = *reinterpret_cast<const float4*>(src + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = c.x; v[5] = c.y; v[6] = c.z; v[7] = c.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = k + j < K ? src[j] : 0.f;
    }
  }
  const long long plane = Rp * (long long)Kp;
  unsigned short* dst = out + blk * 512 + rr * BK + seg * 8;
#pragma unroll
  for (int t = 0; t < NS; ++t) {
    uint4 u;
    u.x = pack_bf16(v[0], v[1]); u.y = pack_bf16(v[2], v[3]);
    u.z = pack_bf16(v[4], v[5]); u.w = pack_bf16(v[6], v[7]);
    *reinterpret_cast<uint4*>(dst + t * plane) = u;
    if (t + 1 < NS) {
      v[0] -= bf16_lo(u.x); v[1] -= bf16_hi(u.x); v[2] -= bf16_lo(u.y); v[3] -= bf16_hi(u.y);
      v[4] -= bf16_lo(u.z); v[5] -= bf16_hi(u.z); v[6] -= bf16_lo(u.w); v[7] -= bf16_hi(u.w);
    }
  }
}

// 16-byte k-segment swizzle of a tile row in LDS (conflict-free ds_read_b128 of 16 rows per lane
// group): 4 segments per row (BK 32) -> seg ^ ((row >> 2) & 3); 2 (BK 16) -> seg ^ ((row >> 3) & 1)
template <int BK>
__device__ __forceinline__ int seg_swz(int row, int seg) {
  if constexpr (BK == 32) return seg ^ ((row >> 2) & 3);
  else return seg ^ ((row >> 3) & 1);
}

// 128 x 128 output tile, 4 waves as 2 x 2, each 64 x 64 (2 x 2 v_mfma_f32_32x32x16_bf16 blocks).
// LDS stage = 2 NS plane tiles (X terms, then W terms) of [128 rows][BK bf16], the k-segments of a
// row swizzled (seg_swz).  LDS-DMA writes lane-linearly (1 KiB = one plane block per
// wave-instruction), so the swizzle goes on the SOURCE address: lane i of an instruction fetches
// row i / SEGS, segment seg_swz(row, i % SEGS) of its block.  NST-stage ring: BK 32 (48 KiB stages
// at x6) fits one workgroup per CU, BK 16 two (x6) or three (x3).  All LDS is one __shared__ array
// and the K loop has no VGPR-destination global load, so the compiler's waits stay the counted
// ones written here.  ABL (A/B of the pipeline's parts): 1 drops the MFMAs, 2 the K loop's DMA.
// (s_setprio 1 around each MFMA group measured slower: 118 -> 128 us x6, 77 -> 81 us x3.)
template <int NS, int BK, int NST, int ABL = 0>
__global__ __launch_bounds__(MT) void linear_act_fwd_planes_kernel(const unsigned short* __restrict__ Xp,
                                                                   const unsigned short* __restrict__ Wp,
                                                                   const float* __restrict__ b, float* __restrict__ Y,
                                                                   int M, int N, int Kp, int act, int xcd) {
  constexpr int TR = 128, SEGS = BK / 8, RPB = 512 / BK, PLANE = TR * BK * 2, STAGE = 2 * NS * PLANE;
  constexpr int PER_WAVE = 2 * NS * (TR / RPB) / 4;  // LDS-DMA instructions per wave and stage
  __shared__ __attribute__((aligned(1024))) unsigned char lds[NST * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  int tm = blockIdx.y, tn = blockIdx.x;
  if (xcd) av::grouped_tile(av::xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y), gridDim.y,
                            gridDim.x, 8, tm, tn);
  const long long m0 = (long long)tm * TR;
  const int n0 = tn * TR;
  const long long kb = Kp / BK;
  const long long xplane = (long long)gridDim.y * TR * Kp, wplane = (long long)gridDim.x * TR * Kp;
  // this lane's source in its block for each of the wave's DMA instructions (+ 512 per stage)
  const int lrow = lane / SEGS, lseg = seg_swz<BK>(lrow, lane % SEGS);
  const unsigned short* src[PER_WAVE];
  int dst[PER_WAVE];
#pragma unroll
  for (int q = 0; q < PER_WAVE; ++q) {
    const int j = wave + 4 * q, pt = j / (TR / RPB), rb = j % (TR / RPB);
    if (pt < NS) src[q] = Xp + pt * xplane + ((m0 / RPB + rb) * kb) * 512 + lrow * BK + lseg * 8;
    else src[q] = Wp + (pt - NS) * wplane + ((n0 / RPB + rb) * kb) * 512 + lrow * BK + lseg * 8;
    dst[q] = pt * PLANE + rb * 1024;
  }
  auto issue = [&](int t) __attribute__((always_inline)) {
    unsigned char* base = lds + (t % NST) * STAGE;
#pragma unroll
    for (int q = 0; q < PER_WAVE; ++q)
      __builtin_amdgcn_global_load_lds((const void*)(src[q] + (long long)t * 512),
                                       (__attribute__((address_space(3))) void*)(base + dst[q]), 16, 0, 0);
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int T = Kp / BK;
  issue(0);
  if (NST == 3 && T > 1) {
    issue(1);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_WAVE) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  const int li = lane & 31, lh = lane >> 5;
  for (int t = 0; t < T; ++t) {
    if (ABL != 2 && t + NST - 1 < T) issue(t + NST - 1);
    const unsigned char* sb = lds + (t % NST) * STAGE;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 a[NS][2], w[NS][2];
#pragma unroll
      for (int p = 0; p < NS; ++p) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int r = wm * 64 + 32 * i + li;
          a[p][i] = *reinterpret_cast<const bf16x8*>(sb + p * PLANE + (r * SEGS + seg_swz<BK>(r, ks * 2 + lh)) * 16);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int r = wn * 64 + 32 * j + li;
          w[p][j] = *reinterpret_cast<const bf16x8*>(sb + (NS + p) * PLANE + (r * SEGS + seg_swz<BK>(r, ks * 2 + lh)) * 16);
        }
      }
      // term orders, smallest first (as linear_act_fwd_sbf16_kernel)
#pragma unroll
      for (int ord = NS - 1; ord >= 0; --ord)
#pragma unroll
        for (int ta = ord; ta >= 0; --ta)
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              if constexpr (ABL == 1) asm volatile("" ::"v"(a[ta][i]), "v"(w[ord - ta][j]));
              else acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ta][i], w[ord - ta][j], acc[i][j], 0, 0, 0);
            }
    }
    // retire this wave's DMA of stage t + 1 (stage t + 2's stays in flight), then one barrier: after
    // it every wave's stage t + 1 has landed and every wave is done reading stage t (re-filled at t + 1)
    if (NST == 3 && t + 2 < T) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_WAVE) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = n0 + wn * 64 + 32 * j + (lane & 31);
    if (col >= N) continue;
    const float bias = b ? b[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long long row = m0 + wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row < M) Y[row * N + col] = act_fwd(acc[i][j][r] + bias, act);
      }
  }
}

}  // namespace

namespace avk {

// AVMI_XCD_TILES=0 restores the dispatch order (A/B switch)
static bool xcd_tiles_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("AVMI_XCD_TILES");
    return !(e && e[0] == '0');
  }();
  return on;
}

// AVMI_BIG_TILES=0: the 64 x 64 tile for every shape (A/B switch)
static bool big_tiles_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("AVMI_BIG_TILES");
    return !(e && e[0] == '0');
  }();
  return on;
}

// workgroups the split-K slices aim at (AVMI_SPLITK_TARGET, default 512): fewer slices mean longer
// slices but less partial traffic for the slice sum / fused LayerNorm that follows (BERT B 1 x S 128,
// 3 interleaved runs each: 512 -> 1.018 ms, 384 -> 1.014 ms per pass, within noise:
// profiles/r5_splitk_target_ab.jsonl)
static long long split_target() {
  static const long long t = [] {
    const char* e = std::getenv("AVMI_SPLITK_TARGET");
    const long long v = e ? std::atoll(e) : 512;
    return v >= 64 ? v : 512;
  }();
  return t;
}

// fp32 GEMM arithmetic of the K27 tiles (AVMI_F32_GEMM, read once): "f32" = exact-f32 MFMA,
// "bf16x3" = split-bf16 with 3 products, "bf16x6" = split-bf16 with 6 products (default: the error
// of the exact-f32 tiles or lower, faster at every measured shape: profiles/r6_gemm_*.jsonl)
int f32_gemm_mode() {
  static const int mode = [] {
    const char* e = std::getenv("AVMI_F32_GEMM");
    if (e == nullptr) return 6;
    const std::string v(e);
    if (v == "f32") return 0;
    if (v == "bf16x3") return 3;
    return 6;
  }();
  return mode;
}

// K chunk of the split-bf16 tiles (AVMI_SBF16_KC = 32 | 64 overrides): x3 64 (a few % faster at
// the large shapes), x6 32 (at 64 its 128 x 128 tile drops to one wave per SIMD: up to 20 % slower;
// profiles/r6_gemm_bf16x*_kc*.jsonl)
// the swizzled three-per-CU x6 tile (AVMI_SBF16_SWZ = 0 turns it off)
static bool sbf16_swz() {
  static const bool on = [] {
    const char* e = std::getenv("AVMI_SBF16_SWZ");
    return e == nullptr || std::atoi(e) != 0;
  }();
  return on;
}

// AVMI_SBF16_SMALLK_KC64=0: the x6 64 x 64 tile keeps 32-deep chunks at K <= 128 (A/B switch)
static bool small_k_kc64() {
  static const bool on = [] {
    const char* e = std::getenv("AVMI_SBF16_SMALLK_KC64");
    return !(e && e[0] == '0');
  }();
  return on;
}

static int sbf16_kc(int mode) {
  static const int kc = [] {
    const char* e = std::getenv("AVMI_SBF16_KC");
    return e ? std::atoi(e) : 0;
  }();
  if (kc == 32 || kc == 64) return kc;
  return mode == 3 ? 64 : 32;
}

int linear_act_fwd_slices(int M, int N, int K) {
  const long long tiles = (long long)((M + TM - 1) / TM) * ((N + TN - 1) / TN);
  // (K < 512: at most 16 chunks per tile, where the extra epilogue launch costs more than the
  // parallelism gains — the LSTM's dx = dZ W_ih at 5,000 x 5 x 400)
  if (tiles >= 256 || K < 16 * KC) return 1;
  // a few output tiles over a long K (a query's rows through a BERT projection: 2 x 12 tiles
  // over K = 3,072): split K so ~512 workgroups cover the 256 CUs, each slice >= 4 chunks.
  // (Tried and measured slower: one-shot slices that issue all 128 K-columns' loads at once, 16.6
  // -> 20.8 us at 128 x 768 x 3,072 — so not per-chunk latency; likely the re-reads of X by every N tile and of W by
  // both M tiles, an estimated ~38 MB of L2 / MALL traffic: profiles/r5_splitk_oneshot_ab.jsonl)
  long long s = (split_target() + tiles - 1) / tiles;
  s = std::min<long long>(s, K / (4 * KC));
  return (int)std::max(1LL, std::min(s, 64LL));
}

int linear_splitk_partial(const float* X, const float* W, float* partial, int M, int N, int K, int S,
                          hipStream_t stream, int prec) {
  const int kper = ((K + S - 1) / S + KC - 1) / KC * KC;
  S = (K + kper - 1) / kper;  // no empty slice
  if (M <= 0 || N <= 0) return S;
  const bool vec = (K % 4 == 0) && (reinterpret_cast<uintptr_t>(X) % 16 == 0) &&
                   (reinterpret_cast<uintptr_t>(W) % 16 == 0);
  dim3 grid((unsigned)((N + TN - 1) / TN), (unsigned)((M + TM - 1) / TM), (unsigned)S);
  const int mode = prec >= 0 ? prec : f32_gemm_mode();
  if (vec && mode == 3)
    (sbf16_kc(mode) == 32 ? linear_act_fwd_sbf16_kernel<1, 2, true, 32><<<grid, MT, 0, stream>>>(X, W, nullptr, partial, M, N, K, 0, kper, 0) : linear_act_fwd_sbf16_kernel<1, 2, true, 64><<<grid, MT, 0, stream>>>(X, W, nullptr, partial, M, N, K, 0, kper, 0));
  else if (vec && mode == 6)
    (sbf16_kc(mode) == 32 ? linear_act_fwd_sbf16_kernel<1, 3, true, 32><<<grid, MT, 0, stream>>>(X, W, nullptr, partial, M, N, K, 0, kper, 0) : linear_act_fwd_sbf16_kernel<1, 3, true, 64><<<grid, MT, 0, stream>>>(X, W, nullptr, partial, M, N, K, 0, kper, 0));
  else if (vec) linear_act_fwd_kernel<true, true><<<grid, MT, 0, stream>>>(X, W, nullptr, partial, M, N, K, 0, kper, 0);
  else linear_act_fwd_kernel<false, true><<<grid, MT, 0, stream>>>(X, W, nullptr, partial, M, N, K, 0, kper, 0);
  AV_HIP_CHECK(hipGetLastError());
  return S;
}

// the pre-split planes path (AVMI_SBF16_PLANES=0 turns it off): split-bf16 modes, outputs of at
// least 1,024 x 1,024 (where the 128 x 128 tiles are taken)
static bool planes_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("AVMI_SBF16_PLANES");
    return !(e && e[0] == '0');
  }();
  return on;
}

// fewest 128 x 128 output tiles that take the planes path (AVMI_PLANES_MIN_TILES overrides): the
// planes tile runs three workgroups per CU (768 in one round), the in-loop x3 tile two (512), the
// in-loop x6 tile three.  Measured (profiles/r6_k27_thresh_bf16x*_p*.jsonl, planes vs in-loop):
// x3 576 tiles 74 vs 104 us, 768 96 vs 116, 1,152 123 vs 160, 512 82 vs 71, 384 67 vs 61;
// x6 768 139 vs 146, 576 111 vs 112, 512 118 vs 107, 384 88 vs 85.  So x3 from 513, x6 from 640.
static long long planes_min_tiles(int mode) {
  static const long long n = [] {
    const char* e = std::getenv("AVMI_PLANES_MIN_TILES");
    return e ? std::atoll(e) : -1LL;
  }();
  return n >= 0 ? n : (mode == 3 ? 513LL : 640LL);
}

long long linear_act_fwd_planes_bytes(int M, int N, int K, int prec) {
  const int mode = prec >= 0 ? prec : f32_gemm_mode();
  if (mode == 0 || !planes_enabled() || M <= 0 || N <= 0 || K <= 0 || K > (1 << 20)) return 0;
  M = std::min(M, 1 << 22);  // linear_act_fwd runs larger M in row chunks of 2^22 over one scratch
  const long long tiles = ((long long)M + 127) / 128 * (((long long)N + 127) / 128);
  if (tiles < planes_min_tiles(mode)) return 0;
  const long long Kp = ((long long)K + 31) / 32 * 32;
  const long long Mp = ((long long)M + 127) / 128 * 128, Np = ((long long)N + 127) / 128 * 128;
  const long long bytes = (mode == 6 ? 3LL : 2LL) * (Mp + Np) * Kp * 2;
  // scratch bound (the in-loop tile needs none): 1.5x the operands' fp32 bytes, at most 2 GiB
  return bytes <= (2LL << 30) ? bytes : 0;
}

// K step of the planes tile (AVMI_PLANES_BK = 16 | 32, default 16)
static int planes_bk() {
  static const int bk = [] {
    const char* e = std::getenv("AVMI_PLANES_BK");
    return e && std::atoi(e) == 32 ? 32 : 16;
  }();
  return bk;
}

// LDS stages of the BK 16 ring (AVMI_PLANES_NST = 2 | 3, default 2)
static int planes_nst() {
  static const int n = [] {
    const char* e = std::getenv("AVMI_PLANES_NST");
    return e && std::atoi(e) == 3 ? 3 : 2;
  }();
  return n;
}

// the NS term planes of rows [R][K] (layout of the BK tile) into `out`
template <int NS, int BK>
static void split_rows(const float* A, int R, int K, void* out, hipStream_t stream) {
  const int Kp = (K + 31) / 32 * 32;
  const long long Rp = ((long long)R + 127) / 128 * 128;
  const bool vec = K % 4 == 0 && reinterpret_cast<uintptr_t>(A) % 16 == 0;
  const unsigned gk = (unsigned)((Kp / BK + 3) / 4);
  sbf16_split_rows_kernel<NS, BK><<<dim3((unsigned)(Rp / (512 / BK)), gk), 256, 0, stream>>>(
      A, static_cast<unsigned short*>(out), R, K, Rp, Kp, vec);
  AV_HIP_CHECK(hipGetLastError());
}

template <int NS, int BK, int NST>
static void linear_act_fwd_planes(const float* X, const float* W, const float* b, float* Y, int M, int N, int K,
                                  int act, hipStream_t stream, void* planes, const void* w_planes) {
  const int Kp = (K + 31) / 32 * 32;
  const long long Mp = ((long long)M + 127) / 128 * 128;
  unsigned short* Xp = static_cast<unsigned short*>(planes);
  const unsigned short* Wp = static_cast<const unsigned short*>(w_planes);
  split_rows<NS, BK>(X, M, K, Xp, stream);
  if (Wp == nullptr) {
    unsigned short* w = Xp + NS * Mp * Kp;
    split_rows<NS, BK>(W, N, K, w, stream);
    Wp = w;
  }
  dim3 grid((unsigned)((N + 127) / 128), (unsigned)((M + 127) / 128));
  const int xcd = xcd_tiles_enabled() && grid.x * grid.y >= 64 ? 1 : 0;
  static const int abl = [] { const char* e = std::getenv("AVMI_PLANES_ABL"); return e ? std::atoi(e) : 0; }();
  if (abl == 1) linear_act_fwd_planes_kernel<NS, BK, NST, 1><<<grid, MT, 0, stream>>>(Xp, Wp, b, Y, M, N, Kp, act, xcd);
  else if (abl == 2) linear_act_fwd_planes_kernel<NS, BK, NST, 2><<<grid, MT, 0, stream>>>(Xp, Wp, b, Y, M, N, Kp, act, xcd);
  else linear_act_fwd_planes_kernel<NS, BK, NST><<<grid, MT, 0, stream>>>(Xp, Wp, b, Y, M, N, Kp, act, xcd);
  AV_HIP_CHECK(hipGetLastError());
}

long long sbf16_weight_planes_bytes(int N, int K, int prec) {
  const int mode = prec >= 0 ? prec : f32_gemm_mode();
  if (mode == 0 || !planes_enabled() || N <= 0 || K <= 0 || K > (1 << 20)) return 0;
  const long long Kp = ((long long)K + 31) / 32 * 32, Np = ((long long)N + 127) / 128 * 128;
  return (mode == 6 ? 3LL : 2LL) * Np * Kp * 2;
}

void sbf16_weight_planes(const float* W, int N, int K, int prec, void* out, hipStream_t stream) {
  if (sbf16_weight_planes_bytes(N, K, prec) == 0) return;
  const bool x6 = (prec >= 0 ? prec : f32_gemm_mode()) == 6;
  if (planes_bk() == 32) (x6 ? split_rows<3, 32> : split_rows<2, 32>)(W, N, K, out, stream);
  else (x6 ? split_rows<3, 16> : split_rows<2, 16>)(W, N, K, out, stream);
}

void linear_act_fwd(const float* X, const float* W, const float* b, float* Y, int M, int N, int K, int act,
                    hipStream_t stream, float* partial, int S, int prec, void* planes, const void* w_planes) {
  if (M <= 0 || N <= 0) return;
  // row chunks of 2^22: the tile grids put the row tiles on grid.y (<= 65,535 tiles of 64 rows)
  constexpr int MAXR = 1 << 22;
  if (M > MAXR) {
    for (int m0 = 0; m0 < M; m0 += MAXR)
      linear_act_fwd(X + (long long)m0 * K, W, b, Y + (long long)m0 * N, std::min(MAXR, M - m0), N, K, act, stream,
                     nullptr, 1, prec, planes, w_planes);
    return;
  }
  const bool vec = (K % 4 == 0) && (reinterpret_cast<uintptr_t>(X) % 16 == 0) &&
                   (reinterpret_cast<uintptr_t>(W) % 16 == 0);
  if (planes != nullptr && S <= 1 && linear_act_fwd_planes_bytes(M, N, K, prec) > 0) {
    const bool x6 = (prec >= 0 ? prec : f32_gemm_mode()) == 6;
    if (planes_bk() == 32) (x6 ? linear_act_fwd_planes<3, 32, 3> : linear_act_fwd_planes<2, 32, 3>)(X, W, b, Y, M, N, K, act, stream, planes, w_planes);
    else if (planes_nst() == 3) (x6 ? linear_act_fwd_planes<3, 16, 3> : linear_act_fwd_planes<2, 16, 3>)(X, W, b, Y, M, N, K, act, stream, planes, w_planes);
    else (x6 ? linear_act_fwd_planes<3, 16, 2> : linear_act_fwd_planes<2, 16, 2>)(X, W, b, Y, M, N, K, act, stream, planes, w_planes);
    return;
  }
  if (S > 1 && partial != nullptr) {
    S = linear_splitk_partial(X, W, partial, M, N, K, S, stream, prec);
    const long long MN = (long long)M * N;
    linear_splitk_epilogue_kernel<<<(unsigned)((MN + 255) / 256), 256, 0, stream>>>(partial, b, Y, MN, N, S, act);
    AV_HIP_CHECK(hipGetLastError());
    return;
  }
  const int mode = prec >= 0 ? prec : f32_gemm_mode();
  if (vec && M >= 1024 && N >= 1024 && big_tiles_enabled()) {
    dim3 gb((unsigned)((N + TB - 1) / TB), (unsigned)((M + TB - 1) / TB));
    const int xcd = xcd_tiles_enabled() && gb.x * gb.y >= 64 ? 1 : 0;
    if (mode == 3) (sbf16_kc(mode) == 32 ? linear_act_fwd_sbf16_kernel<2, 2, false, 32><<<gb, MT, 0, stream>>>(X, W, b, Y, M, N, K, act, K, xcd) : linear_act_fwd_sbf16_kernel<2, 2, false, 64><<<gb, MT, 0, stream>>>(X, W, b, Y, M, N, K, act, K, xcd));
    else if (mode == 6 && sbf16_kc(mode) == 32 && sbf16_swz())
      linear_act_fwd_sbf16_kernel<2, 3, false, 32, true, 3><<<gb, MT, 0, stream>>>(X, W, b, Y, M, N, K, act, K, xcd);
    else if (mode == 6) (sbf16_kc(mode) == 32 ? linear_act_fwd_sbf16_kernel<2, 3, false, 32><<<gb, MT, 0, stream>>>(X, W, b, Y, M, N, K, act, K, xcd) : linear_act_fwd_sbf16_kernel<2, 3, false, 64><<<gb, MT, 0, stream>>>(X, W, b, Y, M, N, K, act, K, xcd));
    else linear_act_fwd_big_kernel<<<gb, MT, 0, stream>>>(X, W, b, Y, M, N, K, act, xcd);
    AV_HIP_CHECK(hipGetLastError());
    return;
  }
  dim3 grid((unsigned)((N + TN - 1) / TN), (unsigned)((M + TM - 1) / TM));
  const int xcd = xcd_tiles_enabled() && grid.x * grid.y >= 64 ? 1 : 0;
  if (vec && mode == 3) (sbf16_kc(mode) == 32 ? linear_act_fwd_sbf16_kernel<1, 2, false, 32><<<grid, MT, 0, stream>>>(X, W, b, Y, M, N, K, act, K, xcd) : linear_act_fwd_sbf16_kernel<1, 2, false, 64><<<grid, MT, 0, stream>>>(X, W, b, Y, M, N, K, act, K, xcd));
  // (x6, 64 x 64 tile: K <= 128 in 64-deep chunks — the latency-bound small GEMMs of the DQN /
  // autoencoder layers take half the chunk round trips; graphed DQN update 266 -> 262 us, ~1 %:
  // profiles/r6_rl_kc64_ab.jsonl)
  else if (vec && mode == 6) ((sbf16_kc(mode) == 32 && !(K <= 128 && small_k_kc64())) ? linear_act_fwd_sbf16_kernel<1, 3, false, 32><<<grid, MT, 0, stream>>>(X, W, b, Y, M, N, K, act, K, xcd) : linear_act_fwd_sbf16_kernel<1, 3, false, 64><<<grid, MT, 0, stream>>>(X, W, b, Y, M, N, K, act, K, xcd));
  else if (vec) linear_act_fwd_kernel<true, false><<<grid, MT, 0, stream>>>(X, W, b, Y, M, N, K, act, K, xcd);
  else linear_act_fwd_kernel<false, false><<<grid, MT, 0, stream>>>(X, W, b, Y, M, N, K, act, K, xcd);
  AV_HIP_CHECK(hipGetLastError());
}

// rows per workgroup: ~512 workgroups over the (64-column, row-block) grid, 16..256 rows each
int linear_act_bwd_rows(int M, int N) {
  const long long nb = (N + 63) / 64;
  long long r = 16;
  while (r < BR_ROWS && ((long long)M + r - 1) / r * nb > 512) r *= 2;
  return (int)r;
}
int linear_act_bwd_blocks(int M, int N) {
  const int r = linear_act_bwd_rows(M, N);
  return (M + r - 1) / r;
}

void linear_act_bwd(const float* dY, const float* Y, float* dZ, float* partial, int M, int N, int act,
                    hipStream_t stream) {
  if (M <= 0 || N <= 0) return;
  dim3 grid((unsigned)((N + 63) / 64), (unsigned)linear_act_bwd_blocks(M, N));
  linear_act_bwd_kernel<<<grid, MT, 0, stream>>>(dY, Y, dZ, partial, M, N, act, linear_act_bwd_rows(M, N));
  AV_HIP_CHECK(hipGetLastError());
}

// slices of M for the weight gradient: about 512 blocks over the (n, k) tiles, >= 256 rows each
int linear_act_wgrad_slices(int M, int N, int K) {  // ~1024 blocks, >= 64 rows per slice
  const long long tiles = (long long)((N + 63) / 64) * ((K + 63) / 64);
  long long S = std::max(1LL, 1024 / std::max(1LL, tiles));
  S = std::min(S, std::max(1LL, ((long long)M + 63) / 64));
  return (int)S;
}

void linear_act_wgrad(const float* dY, const float* Y, const float* X, float* dZ, float* pW, float* tmp, float* out,
                      int M, int N, int K, int act, hipStream_t stream) {
  if (N <= 0 || K <= 0) return;
  const int S = linear_act_wgrad_slices(M, N, K);
  int rows = (int)((((long long)M + S - 1) / S + MC - 1) / MC * MC);
  if (rows < MC) rows = MC;
  dim3 grid((unsigned)((N + 63) / 64), (unsigned)((K + 63) / 64), (unsigned)S);
  linear_act_wgrad_kernel<<<grid, MT, 0, stream>>>(dY, Y, X, dZ, pW, M, N, K, rows, act);
  AV_HIP_CHECK(hipGetLastError());
  const long long E = (long long)N * K + N;
  const unsigned ex = (unsigned)((E + 63) / 64);
  const int S2 = (S + 63) / 64;
  if (S2 == 1) {  // <= 64 slices: one fixed-order pass straight into out (the second was a copy)
    slice_sum_kernel<<<dim3(ex, 1), 64 * RG, 0, stream>>>(pW, out, S, 64, E);
    AV_HIP_CHECK(hipGetLastError());
    return;
  }
  slice_sum_kernel<<<dim3(ex, (unsigned)S2), 64 * RG, 0, stream>>>(pW, tmp, S, 64, E);
  AV_HIP_CHECK(hipGetLastError());
  slice_sum_kernel<<<dim3(ex, 1), 64 * RG, 0, stream>>>(tmp, out, S2, S2, E);
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
