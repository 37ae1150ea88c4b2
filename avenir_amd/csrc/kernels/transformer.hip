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

// one wave per row
__global__ __launch_bounds__(256) void add_layernorm_kernel(const float* __restrict__ x, const float* __restrict__ res,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, float* __restrict__ out,
                                                            long long rows, int H, float eps) {
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  float4 v[LN_MAXV];
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c0 = 4 * (lane + 64 * i);
    v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c0 < H) {
      const float4 a = *reinterpret_cast<const float4*>(x + row * H + c0);
      const float4 b = res ? *reinterpret_cast<const float4*>(res + row * H + c0) : make_float4(0.f, 0.f, 0.f, 0.f);
      v[i] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
    }
  }
  ln_row(v, H, gamma, beta, eps, out + row * H);
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

}  // namespace

namespace avk {

void add_layernorm(const float* x, const float* res, const float* gamma, const float* beta, float* out, long long rows,
                   int H, float eps, hipStream_t stream) {
  if (rows <= 0) return;
  if (H < 4 || H > 1024 || H % 4) throw std::runtime_error("add_layernorm: 4 <= H <= 1024, H % 4 == 0");
  add_layernorm_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, stream>>>(x, res, gamma, beta, out, rows, H, eps);
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

}  // namespace avk
