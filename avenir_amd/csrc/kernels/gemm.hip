// Split-K fp32 "Aᵀ·B" GEMM for weight gradients: C[M, N] = Σ_k A[k, m] · B[k, n] with A [K, M] and
// B [K, N] both row-major over the long reduction dimension K (e.g. the LSTM's dW = dzᵀ·[h_{t-1} | x | 1]
// over all B·T rows: K = 5,000, M = 4H = 400, N = H + I + 1 ≈ 106).  Such a product has few output
// tiles (7 x 2 here) and a long K: hipBLASLt's pick ran at ~30 TFLOP/s (26 us, the LSTM trace).  Here
// the K range is split over S slices so the grid has hundreds of workgroups; each workgroup stages
// 32-row chunks of its A and B columns with coalesced row loads (the next chunk register-prefetched
// during the MFMAs), multiplies a 64 x 64 output tile on v_mfma_f32_32x32x2_f32 (exact-f32 products,
// one 32 x 32 quarter per wave) and writes its partial tile; a second kernel sums the S partials of
// every output in slice order (deterministic, no float atomics).
//
// Split-bf16 variant (avenir_sbf16.h): the same grid and slices, but each thread loads 8 CONSECUTIVE
// K rows of one column (still 256-byte coalesced row segments per wave and row), splits them into
// bf16 terms and stores each term's 8 k values as one 16-byte row segment of a transposed
// [column][32 k + 8 pad] image (80-byte rows: conflict-free ds_read_b128 fragments), multiplied on
// v_mfma_f32_32x32x16_bf16: 3 (bf16x3) or 6 (bf16x6) MFMAs per 16 k instead of 8 fp32 MFMAs at
// 1/16 the rate.
#include "avenir_common.h"
#include "avenir_kernels.h"
#include "avenir_sbf16.h"

namespace {

constexpr int GT = 256;   // threads
constexpr int TM = 64;    // output rows (A columns) per workgroup
constexpr int TN = 64;    // output cols (B columns) per workgroup
constexpr int KC = 32;    // K rows per LDS chunk

typedef float f32x16 __attribute__((ext_vector_type(16)));

// one K chunk of the A and B tiles in registers: KC rows x 64 columns each = 2048 floats per
// operand, 8 per thread (rows tid / 64 + 4 i, column tid % 64: coalesced 256-byte row segments)
struct TnChunk {
  float a[8], b[8];
  __device__ __forceinline__ void load(const float* __restrict__ A, const float* __restrict__ B, int k0, int k1, int m0,
                                       int n0, int M, int N) {
    const int c = threadIdx.x & 63, r0 = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int k = k0 + r0 + 4 * i;
      const bool kin = k < k1;
      a[i] = (kin && m0 + c < M) ? A[(long long)k * M + m0 + c] : 0.f;
      b[i] = (kin && n0 + c < N) ? B[(long long)k * N + n0 + c] : 0.f;
    }
  }
  __device__ __forceinline__ void store(float (*sA)[TM + 1], float (*sB)[TN + 1]) const {
    const int c = threadIdx.x & 63, r0 = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sA[r0 + 4 * i][c] = a[i];
      sB[r0 + 4 * i][c] = b[i];
    }
  }
};

// grid (N tiles, M tiles, S slices); partial [S, M, N]
__global__ __launch_bounds__(GT) void gemm_tn_partial_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                             float* __restrict__ partial, int K, int M, int N,
                                                             int kper) {
  __shared__ float sA[KC][TM + 1];
  __shared__ float sB[KC][TN + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * TM, n0 = blockIdx.x * TN;
  const int k0 = blockIdx.z * kper, k1 = min(K, k0 + kper);
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  TnChunk pre;
  if (k0 < k1) pre.load(A, B, k0, k1, m0, n0, M, N);
  for (int kc = k0; kc < k1; kc += KC) {
    __syncthreads();  // the previous chunk's operand reads are done
    pre.store(sA, sB);
    __syncthreads();
    if (kc + KC < k1) pre.load(A, B, kc + KC, k1, m0, n0, M, N);  // in flight during the MFMAs
    const int li = lane & 31, lk = lane >> 5;
#pragma unroll
    for (int k = 0; k < KC; k += 2) {
      // A operand: A'[i = m][k] = A[k][m]; B operand: B[k][j = n]
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(sA[k + lk][wm * 32 + li], sB[k + lk][wn * 32 + li], acc, 0, 0, 0);
    }
  }
  // C/D map of 32x32x2: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
  const int n = n0 + wn * 32 + (lane & 31);
  if (n >= N) return;
  float* P = partial + (long long)blockIdx.z * M * N;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (m < M) P[(long long)m * N + n] = acc[r];
  }
}

template <int NS>
__global__ __launch_bounds__(GT) void gemm_tn_sbf16_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                           float* __restrict__ partial, int K, int M, int N, int kper) {
  constexpr int SROW = KC + 8;  // bf16 per LDS row: 80 bytes
  __shared__ __attribute__((aligned(16))) unsigned short sA[NS][TM][SROW];
  __shared__ __attribute__((aligned(16))) unsigned short sB[NS][TN][SROW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * TM, n0 = blockIdx.x * TN;
  const int k0 = blockIdx.z * kper, k1 = min(K, k0 + kper);
  const int c = tid & 63, r0 = (tid >> 6) * 8;  // column c, K rows r0 .. r0 + 7 of the chunk
  float a[8], b[8];
  auto load = [&](int kc) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = kc + r0 + j;
      const bool kin = k < k1;
      a[j] = (kin && m0 + c < M) ? A[(long long)k * M + m0 + c] : 0.f;
      b[j] = (kin && n0 + c < N) ? B[(long long)k * N + n0 + c] : 0.f;
    }
  };
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  if (k0 < k1) load(k0);
  const int li = lane & 31, lh = (lane >> 5) * 8;
  for (int kc = k0; kc < k1; kc += KC) {
    __syncthreads();  // the previous chunk's fragment reads are done
    {
      sbf::u32x4 ta[NS], tb[NS];
      sbf::split8<NS>(a, ta);
      sbf::split8<NS>(b, tb);
#pragma unroll
      for (int t = 0; t < NS; ++t) {
        *reinterpret_cast<sbf::u32x4*>(&sA[t][c][r0]) = ta[t];
        *reinterpret_cast<sbf::u32x4*>(&sB[t][c][r0]) = tb[t];
      }
    }
    __syncthreads();
    if (kc + KC < k1) load(kc + KC);  // in flight during the MFMAs
#pragma unroll
    for (int ks = 0; ks < KC; ks += 16) {
      sbf::bf16x8 fa[NS], fb[NS];
#pragma unroll
      for (int t = 0; t < NS; ++t) {
        fa[t] = *reinterpret_cast<const sbf::bf16x8*>(&sA[t][wm * 32 + li][ks + lh]);
        fb[t] = *reinterpret_cast<const sbf::bf16x8*>(&sB[t][wn * 32 + li][ks + lh]);
      }
      sbf::mfma32_terms<NS>(fa, fb, acc);
    }
  }
  const int n = n0 + wn * 32 + (lane & 31);
  if (n >= N) return;
  float* P = partial + (long long)blockIdx.z * M * N;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (m < M) P[(long long)m * N + n] = acc[r];
  }
}

// C[e] = Σ_s partial[s][e] in slice order; the loads of 8 slices are issued together (a plain
// loop left one dependent load chain per output: 14.6 us for 42 k outputs x 74 slices)
__global__ __launch_bounds__(256) void gemm_tn_reduce_kernel(const float* __restrict__ partial, float* __restrict__ C,
                                                            long long MN, int S) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= MN) return;
  float s = 0.f;
  int k = 0;
  for (; k + 8 <= S; k += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = partial[(long long)(k + u) * MN + e];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; k < S; ++k) s += partial[(long long)k * MN + e];
  C[e] = s;
}

}  // namespace

namespace avk {

int gemm_tn_slices(int K, int M, int N) {
  const long long tiles = (long long)((M + TM - 1) / TM) * ((N + TN - 1) / TN);
  // one workgroup per CU (256), each slice at least 4 chunks of K: more slices only moved the time
  // into the partial traffic and the slice sum (74 slices of 2 chunks: 17.6 + 14.6 us at K = 5,000)
  long long s = (256 + tiles - 1) / tiles;
  // a long K (65,536 sequences x T 5 = 327,680 rows): one workgroup per CU is ONE wave per SIMD and
  // the staging latency is exposed (0.89 ms, MFMA busy 28 %, profiles/r5_round5_kernels_pmc.jsonl);
  // four per CU once every slice still holds >= 16 chunks (the partials stay < 1/16 of the input)
  const long long s4 = (1024 + tiles - 1) / tiles;
  if ((long long)K >= s4 * 16 * KC) s = s4;
  s = std::min<long long>(s, std::max(1, K / (4 * KC)));
  return (int)std::max(1LL, std::min(s, 128LL));
}

int gemm_tn_mode() {
  static const int mode = sbf::env_mode("AVMI_GEMM_TN", f32_gemm_mode());
  return mode;
}

void gemm_tn(const float* A, const float* B, float* C, float* partial, int K, int M, int N, int S, hipStream_t stream,
             int prec) {
  if (M <= 0 || N <= 0) return;
  if (S < 1) throw std::runtime_error("gemm_tn: S >= 1");
  const int kper = ((K + S - 1) / S + KC - 1) / KC * KC;
  const dim3 grid((unsigned)((N + TN - 1) / TN), (unsigned)((M + TM - 1) / TM), (unsigned)S);
  const int mode = prec >= 0 ? prec : gemm_tn_mode();
  if (mode == 3) gemm_tn_sbf16_kernel<2><<<grid, GT, 0, stream>>>(A, B, partial, K, M, N, kper);
  else if (mode == 6) gemm_tn_sbf16_kernel<3><<<grid, GT, 0, stream>>>(A, B, partial, K, M, N, kper);
  else gemm_tn_partial_kernel<<<grid, GT, 0, stream>>>(A, B, partial, K, M, N, kper);
  AV_HIP_CHECK(hipGetLastError());
  const long long MN = (long long)M * N;
  gemm_tn_reduce_kernel<<<(unsigned)((MN + 255) / 256), 256, 0, stream>>>(partial, C, MN, S);
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
