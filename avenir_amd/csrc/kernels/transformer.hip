// Transformer-encoder epilogues for the BERT encoder of semantic search (the
// reference's P/app/ssearch.py:184-300 embeds documents with spaCy-transformers' BERT).  The GEMMs
// run on the f32-MFMA tile kernel of mlp.hip (bias + GELU in its epilogue); what is left between
// them is memory-bound row work that torch would run as 3-4 separate passes:
//   * add_layernorm_kernel: out = LN(x + residual) * gamma + beta — one wave per row, the row held
//     in registers (4 floats per lane per 256 columns), mean then centred variance (two-pass, fp32,
//     like torch's LayerNorm), one read of each input and one write;
//   * embed_layernorm_kernel: out = LN(word[id] + position[s] + token_type[tt]) — the three table
//     gathers, the sum and the normalisation of BertEmbeddings in one pass.
// H <= 1024 and H % 4 == 0 (checked by the binding).
#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

constexpr int LN_MAXV = 4;  // float4 chunks per lane: H <= 64 * 4 * 4 = 1024

// lane l holds columns 4 (l + 64 i) .. +3 for i < ceil(H / 256); chunks starting at or past H are
// zeros and take no part in the statistics or the write
__device__ __forceinline__ void ln_row(const float4 (&v)[LN_MAXV], int H, const float* __restrict__ gamma,
                                       const float* __restrict__ beta, float eps, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);  // zeros past H
  const float mean = av::wave_sum(s) / (float)H;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i)
    if (4 * (lane + 64 * i) < H) {
      const float a = v[i].x - mean, b = v[i].y - mean, c = v[i].z - mean, d = v[i].w - mean;
      q += (a * a + b * b) + (c * c + d * d);
    }
  const float rstd = rsqrtf(av::wave_sum(q) / (float)H + eps);
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c0 = 4 * (lane + 64 * i);
    if (c0 < H) {
      const float4 g = *reinterpret_cast<const float4*>(gamma + c0), bb = *reinterpret_cast<const float4*>(beta + c0);
      float4 o;
      o.x = (v[i].x - mean) * rstd * g.x + bb.x;
      o.y = (v[i].y - mean) * rstd * g.y + bb.y;
      o.z = (v[i].z - mean) * rstd * g.z + bb.z;
      o.w = (v[i].w - mean) * rstd * g.w + bb.w;
      *reinterpret_cast<float4*>(out + c0) = o;
    }
  }
}

// one wave per row: out = LN(x + res) where x is either a plain [rows, H] tensor (S = 1, no bias)
// or the S split-K partial products of a projection summed in slice order plus its bias — the
// same additions in the same order as mlp.hip's split epilogue followed by this kernel, so the
// fused and the two-kernel paths agree bit for bit
// RPB rows (waves) per block: 1 when rows are few (a query's 128 rows: one wave per CU instead of
// four rows packed on 32 CUs)
template <int RPB>
__global__ __launch_bounds__(64 * RPB) void add_layernorm_kernel(const float* __restrict__ x, int S, long long sstride,
                                                                 const float* __restrict__ bias,
                                                                 const float* __restrict__ res,
                                                                 const float* __restrict__ gamma,
                                                                 const float* __restrict__ beta,
                                                                 float* __restrict__ out, long long rows, int H,
                                                                 float eps) {
  const long long row = (long long)blockIdx.x * RPB + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  // every chunk's slice loads of a batch are issued together (a 128 x 768 projection summed over 21
  // slices was ~18 dependent load round trips per row, 8.2 us: profiles/r6_bert1_kernel_stats.csv);
  // each element still adds its slices in slice order
  float4 v[LN_MAXV];
  const float* __restrict__ px = x + row * H + 4 * lane;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i)
    v[i] = 4 * (lane + 64 * i) < H ? *reinterpret_cast<const float4*>(px + 256 * i) : make_float4(0.f, 0.f, 0.f, 0.f);
  int k = 1;
  for (; k + 4 <= S; k += 4) {
    float4 p[LN_MAXV][4];
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i)
#pragma unroll
      for (int u = 0; u < 4; ++u)
        p[i][u] = 4 * (lane + 64 * i) < H ? *reinterpret_cast<const float4*>(px + 256 * i + (k + u) * sstride)
                                          : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        v[i].x += p[i][u].x; v[i].y += p[i][u].y; v[i].z += p[i][u].z; v[i].w += p[i][u].w;
      }
  }
  for (; k < S; ++k) {
    float4 p[LN_MAXV];
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i)
      p[i] = 4 * (lane + 64 * i) < H ? *reinterpret_cast<const float4*>(px + 256 * i + k * sstride)
                                     : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
      v[i].x += p[i].x; v[i].y += p[i].y; v[i].z += p[i].z; v[i].w += p[i].w;
    }
  }
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c0 = 4 * (lane + 64 * i);
    if (c0 < H) {
      if (bias) {
        const float4 bb = *reinterpret_cast<const float4*>(bias + c0);
        v[i].x += bb.x; v[i].y += bb.y; v[i].z += bb.z; v[i].w += bb.w;
      }
      if (res) {
        const float4 b = *reinterpret_cast<const float4*>(res + row * H + c0);
        v[i] = make_float4(v[i].x + b.x, v[i].y + b.y, v[i].z + b.z, v[i].w + b.w);
      }
    }
  }
  ln_row(v, H, gamma, beta, eps, out + row * H);
}

void launch_add_layernorm(const float* x, int S, long long sstride, const float* bias, const float* res,
                          const float* gamma, const float* beta, float* out, long long rows, int H, float eps,
                          hipStream_t stream) {
  if (rows <= 4096)
    add_layernorm_kernel<1><<<(unsigned)rows, 64, 0, stream>>>(x, S, sstride, bias, res, gamma, beta, out, rows, H, eps);
  else
    add_layernorm_kernel<4><<<(unsigned)((rows + 3) / 4), 256, 0, stream>>>(x, S, sstride, bias, res, gamma, beta, out,
                                                                          rows, H, eps);
}

__global__ __launch_bounds__(256) void embed_layernorm_kernel(const long long* __restrict__ ids,
                                                              const long long* __restrict__ tt,
                                                              const float* __restrict__ word,
                                                              const float* __restrict__ pos,
                                                              const float* __restrict__ type,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ beta, float* __restrict__ out,
                                                              long long rows, int S, int H, float eps,
                                                              long long nword, int ntype) {
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  // ids are range-checked by the binding unless the caller validated them already (host tensors
  // before their upload); the clamp keeps every gather inside the tables either way
  const long long id = min(max(ids[row], 0LL), nword - 1);
  const long long t = tt ? min(max(tt[row], 0LL), (long long)ntype - 1) : 0;
  const int s = (int)(row % S);
  float4 v[LN_MAXV];
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c0 = 4 * (lane + 64 * i);
    v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c0 < H) {
      const float4 a = *reinterpret_cast<const float4*>(word + id * H + c0);
      const float4 b = *reinterpret_cast<const float4*>(pos + (long long)s * H + c0);
      const float4 c = *reinterpret_cast<const float4*>(type + t * H + c0);
      v[i] = make_float4((a.x + c.x) + b.x, (a.y + c.y) + b.y, (a.z + c.z) + b.z, (a.w + c.w) + b.w);
    }
  }
  ln_row(v, H, gamma, beta, eps, out + row * H);
}

// Multi-head attention, head dim 64, fp32: ctx = softmax(q k^T * scale + key_bias) v with an online
// (running max / sum) softmax over key blocks of 64, straight from the fused Q/K/V projection
// [B*S, 3H] into [B*S, H] (no head transposes).  A workgroup is 4 waves over 16 QG queries of one
// (batch, head): wave w owns query group w % QG and, when KSPLIT = 2, every other key block
// (w / QG): the two halves' (max, sum, O) are merged through LDS at the end, so a short sequence
// (a query's 128 tokens: 2 key blocks) has each wave's dependent chain cut to one block.  Per key
// block and wave:
//   * S^T = K Q^T on v_mfma_f32_16x16x4_f32 (A = K rows from LDS, B = the wave's scaled Q fragment
//     held in 16 VGPRs; the 4 key sub-tiles are 4 independent accumulator chains): lane (quad, col)
//     ends with the scores of query col against keys 16 n + 4 quad + r — a query's scores sit in
//     ONE column of lanes, so its max and sum are two cross-quad shuffles;
//   * those exp'ed scores ARE the A operand of O += P V (query col, keys 4 quad + r of step (n, r)),
//     so P never leaves registers; the running-max rescale of O rows moves through 4 shuffles.
constexpr int AD = 64, AKB = 64, AKS = AD + 4;
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int QG, int KSPLIT>
__global__ __launch_bounds__(256) void attn_f32_kernel(const float* __restrict__ qkv, const float* __restrict__ kbias,
                                                       float* __restrict__ out, int S, int nh, float scale) {
  static_assert(QG * KSPLIT == 4, "4 waves");
  __shared__ float sK[KSPLIT * AKB][AKS];
  __shared__ float sV[KSPLIT * AKB][AKS];
  __shared__ float sB[KSPLIT * AKB];
  __shared__ float sML[2][QG][16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int col = lane & 15, quad = lane >> 4;
  const int qg = w % QG, kh = w / QG;
  const int h = blockIdx.y, b = blockIdx.z;
  const int H = nh * AD;
  const long long ld = 3LL * H;
  const float* __restrict__ base = qkv + (long long)b * S * ld;
  const int q0 = blockIdx.x * (16 * QG) + 16 * qg;
  float qf[16];
  {
    const int q = q0 + col;
#pragma unroll
    for (int s = 0; s < 16; ++s) qf[s] = q < S ? base[(long long)q * ld + h * AD + 4 * s + quad] * scale : 0.f;
  }
  float m = -INFINITY, l = 0.f;
  f32x4 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int kb0 = 0; kb0 < S; kb0 += KSPLIT * AKB) {
    __syncthreads();  // the previous blocks' K / V reads are done
#pragma unroll
    for (int i = 0; i < 4 * KSPLIT; ++i) {
      const int e = tid + 256 * i, r = e >> 4, c4 = (e & 15) * 4, key = kb0 + r;
      float4 kv = make_float4(0.f, 0.f, 0.f, 0.f), vv = kv;
      if (key < S) {
        kv = *reinterpret_cast<const float4*>(base + (long long)key * ld + H + h * AD + c4);
        vv = *reinterpret_cast<const float4*>(base + (long long)key * ld + 2 * H + h * AD + c4);
      }
      *reinterpret_cast<float4*>(&sK[r][c4]) = kv;
      *reinterpret_cast<float4*>(&sV[r][c4]) = vv;
    }
    if (tid < KSPLIT * AKB)
      sB[tid] = kb0 + tid < S ? (kbias ? kbias[(long long)b * S + kb0 + tid] : 0.f) : -INFINITY;
    __syncthreads();
    const int kb = kb0 + kh * AKB;  // this wave's key block
    if (kb >= S) continue;          // wave-uniform: past the sequence
    const int kr = kh * AKB;        // its rows in sK / sV
    f32x4 st[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) st[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 16; ++s)
#pragma unroll
      for (int n = 0; n < 4; ++n)
        st[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(sK[kr + 16 * n + col][4 * s + quad], qf[s], st[n], 0, 0, 0);
    float mb = -INFINITY;
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        st[n][r] += sB[kr + 16 * n + 4 * quad + r];
        mb = fmaxf(mb, st[n][r]);
      }
    mb = fmaxf(mb, __shfl_xor(mb, 16, 64));
    mb = fmaxf(mb, __shfl_xor(mb, 32, 64));
    const float mnew = fmaxf(m, mb);  // finite: key kb < S has a finite bias
    const float alpha = expf(m - mnew);
    float ls = 0.f;
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = expf(st[n][r] - mnew);
        st[n][r] = p;
        ls += p;
      }
    ls += __shfl_xor(ls, 16, 64);
    ls += __shfl_xor(ls, 32, 64);
    l = l * alpha + ls;
    m = mnew;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float ar = __shfl(alpha, 4 * quad + r, 64);  // alpha of O row 4 quad + r
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[dt][r] *= ar;
    }
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
          o[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(st[n][r], sV[kr + 16 * n + 4 * quad + r][16 * dt + col], o[dt],
                                                       0, 0, 0);
  }
  if constexpr (KSPLIT == 2) {
    // merge the two key halves: wave (qg, 1) hands (m, l, O) to wave (qg, 0) through LDS
    __syncthreads();
    float(*sO)[16][AKS] = reinterpret_cast<float(*)[16][AKS]>(&sK[0][0]);  // [QG][16][AKS] over sK
    if (kh == 1) {
      if (quad == 0) {
        sML[0][qg][col] = m;
        sML[1][qg][col] = l;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) sO[qg][4 * quad + r][16 * dt + col] = o[dt][r];
    }
    __syncthreads();
    if (kh == 1) return;
    const float m1 = sML[0][qg][col], l1 = sML[1][qg][col];
    const float mm = fmaxf(m, m1);
    const float a0 = expf(m - mm), a1 = expf(m1 - mm);  // a half that saw no keys: m = -inf -> 0
    l = l * a0 + l1 * a1;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float b0 = __shfl(a0, 4 * quad + r, 64), b1 = __shfl(a1, 4 * quad + r, 64);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[dt][r] = o[dt][r] * b0 + sO[qg][4 * quad + r][16 * dt + col] * b1;
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float inv = 1.f / __shfl(l, 4 * quad + r, 64);
    const int q = q0 + 4 * quad + r;
    if (q < S) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) out[((long long)b * S + q) * H + h * AD + 16 * dt + col] = o[dt][r] * inv;
    }
  }
}

}  // namespace

namespace avk {

void add_layernorm(const float* x, const float* res, const float* gamma, const float* beta, float* out, long long rows,
                   int H, float eps, hipStream_t stream) {
  if (rows <= 0) return;
  if (H < 4 || H > 1024 || H % 4) throw std::runtime_error("add_layernorm: 4 <= H <= 1024, H % 4 == 0");
  launch_add_layernorm(x, 1, 0, nullptr, res, gamma, beta, out, rows, H, eps, stream);
  AV_HIP_CHECK(hipGetLastError());
}

void embed_layernorm(const long long* ids, const long long* tt, const float* word, const float* pos, const float* type,
                     const float* gamma, const float* beta, float* out, long long rows, int S, int H, float eps,
                     long long nword, int ntype, hipStream_t stream) {
  if (rows <= 0) return;
  if (nword < 1 || ntype < 1) throw std::runtime_error("embed_layernorm: empty embedding table");
  if (H < 4 || H > 1024 || H % 4) throw std::runtime_error("embed_layernorm: 4 <= H <= 1024, H % 4 == 0");
  embed_layernorm_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, stream>>>(ids, tt, word, pos, type, gamma, beta, out,
                                                                         rows, S, H, eps, nword, ntype);
  AV_HIP_CHECK(hipGetLastError());
}

void add_layernorm_slices(const float* partial, int S, long long sstride, const float* bias, const float* res,
                          const float* gamma, const float* beta, float* out, long long rows, int H, float eps,
                          hipStream_t stream) {
  if (rows <= 0) return;
  if (H < 4 || H > 1024 || H % 4) throw std::runtime_error("add_layernorm: 4 <= H <= 1024, H % 4 == 0");
  launch_add_layernorm(partial, S, sstride, bias, res, gamma, beta, out, rows, H, eps, stream);
  AV_HIP_CHECK(hipGetLastError());
}

void attention_f32(const float* qkv, const float* kbias, float* out, int B, int S, int nh, float scale,
                   hipStream_t stream) {
  if (B <= 0 || S <= 0 || nh <= 0) return;
  // few (batch, head, 64-query) blocks -> split each query group's keys over two waves
  const long long blocks64 = (long long)((S + 63) / 64) * nh * B;
  if (blocks64 < 512 && S > AKB) {
    const dim3 grid((unsigned)((S + 31) / 32), (unsigned)nh, (unsigned)B);
    attn_f32_kernel<2, 2><<<grid, 256, 0, stream>>>(qkv, kbias, out, S, nh, scale);
  } else {
    const dim3 grid((unsigned)((S + 63) / 64), (unsigned)nh, (unsigned)B);
    attn_f32_kernel<4, 1><<<grid, 256, 0, stream>>>(qkv, kbias, out, S, nh, scale);
  }
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
