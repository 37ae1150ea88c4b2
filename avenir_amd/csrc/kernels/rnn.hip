// K27 — persistent fused LSTM recurrence on the bf16 matrix cores (forward + backward).
//
// Replaces the per-timestep cell loop of the reference's LstmNetwork (P/supv/lstm.py:228-300,
// torch.nn.LSTM on the CPU) and, on the GPU, the MIOpen RNN path that launches several kernels per
// timestep.  The input projection x·W_ihᵀ + b for ALL timesteps is one library GEMM outside this
// kernel (K = input size, fully parallel); only the sequential part lives here:
//
//   forward : z_t = xw_t + h_{t-1}·W_hhᵀ ; i,f,o = σ(z), g = tanh(z) ; c_t = f c_{t-1} + i g ;
//             h_t = o tanh(c_t)
//   backward: dz_t from (dh_t, dc_t, saved gates) ; dh_{t-1} = dz_t·W_hh ; dc_{t-1} = dc_t f
//   (weight gradients dW_hh = Σ_t dz_tᵀ h_{t-1}, dW_ih, db, dx are library GEMMs over B·T rows).
//
// Mapping (CDNA4): one workgroup owns RT tiles of 16 sequences for the WHOLE sequence, so there is
// no inter-workgroup synchronisation.  Wave w owns hidden units [16w, 16w+16) for all four gates:
// its W_hh slice stays in VGPRs as v_mfma_f32_16x16x32_bf16 A-fragments for every timestep (HP/2
// VGPRs), the cell state c stays in VGPRs in the MFMA accumulator layout, and the accumulators are
// initialised with xw_t so the input projection and both biases are added for free.  Only h_t
// (bf16) goes through LDS — double-buffered, one barrier per timestep.  Padded hidden units
// (H < HP) carry zero weights and zero inputs, so their h and c stay 0.
#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned short f2bf(float f) {  // round to nearest even
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}
__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }
__device__ __forceinline__ float tanhf_(float x) {
  const float e = __expf(-2.f * fabsf(x));
  return copysignf((1.f - e) / (1.f + e), x);
}

__device__ __forceinline__ uint2 pack4_bf16(float a, float b, float c, float d) {
  return make_uint2((uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16), (uint32_t)f2bf(c) | ((uint32_t)f2bf(d) << 16));
}
__device__ __forceinline__ uint2 pack4_bf16(f32x4 v) { return pack4_bf16(v[0], v[1], v[2], v[3]); }
__device__ __forceinline__ f32x4 unpack4_bf16(uint2 u) {
  return f32x4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
               __uint_as_float(u.y & 0xffff0000u)};
}

// Layouts.  "Kernel order" of the 4·HP gate columns is kc = 64·w + 16·g + i for hidden unit
// u = 16·w + i and gate g (i, f, g, o), so the four gates of a wave's 16 units are one contiguous
// 256-B run per sequence (saved gates, dz, bias).
//   x      [B, T, I] fp32 layer input (I <= IP = 32·IS)
//   wfrag  [NW][4][KS+IS][64] bf16x8: A-fragments of [W_hh | W_ih] for (wave, gate, k-step):
//          k-steps 0..KS-1 cover the HP recurrent inputs, KS..KS+IS-1 the IP layer inputs
//   bias   [4HP] fp32 kernel order (b_ih + b_hh, zero for padded units)
//   h0, c0 [B, H] or null (zeros)
//   hseq   [B, T, H] fp32 out;  cseq [B, T, HP] fp32 out
//   gates  [B, T, 4HP] bf16 kernel order (post-activation, for the backward) out or null
//   hx     [B, T, HP+IP] bf16 out or null: row (b, t) = [h_{t-1} | x_t | 1 | 0…] — the MFMA
//          B-operand of step t, written once so the backward gets dW_hh, dW_ih and db from ONE GEMM
//          dzᵀ·hx (the 1 sits in the first padding column of x when I < IP)
// Per step: z = bias + [W_hh | W_ih]·[h_{t-1}; x_t]ᵀ — the input projection is fused (no
// B·T·4H intermediate), x_{t+1} is loaded into registers during step t and staged into the other
// LDS buffer next to h_t.  The product is computed transposed (A = weights, B = [h; x]ᵀ from LDS)
// so each lane's four accumulator registers are four CONSECUTIVE hidden units of one sequence
// (row = unit 4·(lane>>4) + r, column = sequence lane & 15): global accesses are 8/16-B vectors
// and h_t goes to LDS as one 8-B write.  Offsets are 32-bit relative to the workgroup's first
// sequence (host checks 16·RT·T·4HP < 2^31).  Sequences past B are clamped for loads, masked for
// stores.
template <int KS, int IS, int RT>
__global__ __launch_bounds__(128 * KS) void lstm_fwd_kernel(const float* __restrict__ x, int I,
                                                            const bf16x8* __restrict__ wfrag,
                                                            const float* __restrict__ bias,
                                                            const float* __restrict__ h0,
                                                            const float* __restrict__ c0, int B, int T,
                                                            int H, float* __restrict__ hseq,
                                                            float* __restrict__ cseq,
                                                            unsigned short* __restrict__ gates,
                                                            unsigned short* __restrict__ hx) {
  constexpr int HP = 32 * KS, IP = 32 * IS, KP = HP + IP, KT = KS + IS, G4P = 4 * HP;
  constexpr int LDS_ROW = KP + 8;                        // +16 B per row against bank conflicts
  constexpr int NT = 128 * KS;                           // threads
  constexpr int XCH = RT * 16 * (IP / 4);                // float4 chunks of x per step
  constexpr int XPT = (XCH + NT - 1) / NT;               // chunks per thread
  __shared__ __attribute__((aligned(16))) unsigned short sbuf[2][RT * 16][LDS_ROW];
  __shared__ __attribute__((aligned(16))) float bias_s[G4P];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int col = lane & 15, quad = lane >> 4;
  const int u0 = 16 * w + 4 * quad;  // this lane's four units
  const int kc0 = 64 * w + 4 * quad;  // kernel-order column of gate 0, unit u0
  const long long row0 = (long long)blockIdx.x * (RT * 16);
  const int TG = T * G4P, THP = T * HP, TH = T * H, TI = T * I, TKP = T * KP;
  const bool vec_h = (H & 3) == 0;
  const float* xb = x + row0 * TI;
  float* hsb = hseq + row0 * TH;
  float* csb = cseq + row0 * THP;
  unsigned short* gtb = gates ? gates + row0 * TG : nullptr;
  unsigned short* hxb = hx ? hx + row0 * TKP : nullptr;

  bf16x8 wf[4][KT];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int ks = 0; ks < KT; ++ks) wf[g][ks] = wfrag[((w * 4 + g) * KT + ks) * 64 + lane];
  for (int i = tid; i < G4P; i += NT) bias_s[i] = bias[i];

  int lrow[RT];
  bool rok[RT];
  f32x4 c[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const int lr = rt * 16 + col;
    rok[rt] = row0 + lr < B;
    lrow[rt] = rok[rt] ? lr : (int)(B - 1 - row0);
    const long long grow = row0 + lrow[rt];
    float hv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool ok = u0 + r < H;
      c[rt][r] = (ok && c0) ? c0[grow * H + u0 + r] : 0.f;
      hv[r] = (ok && h0) ? h0[grow * H + u0 + r] : 0.f;
    }
    *reinterpret_cast<uint2*>(&sbuf[0][lr][u0]) = pack4_bf16(hv[0], hv[1], hv[2], hv[3]);
  }

  // x staging: chunk e -> (tile row e / (IP/4), features 4·(e % (IP/4)) ..); padding -> 0, the
  // first padding feature -> 1 (bias column of hx)
  f32x4 xr[XPT];
  auto load_x = [&](int t) {
#pragma unroll
    for (int j = 0; j < XPT; ++j) {
      const int e = tid + j * NT;
      const int r = e / (IP / 4), f0 = 4 * (e % (IP / 4));
      if (e < XCH) {
        const int rr = row0 + r < B ? r : (int)(B - 1 - row0);
        const float* src = xb + rr * TI + t * I;
#pragma unroll
        for (int q = 0; q < 4; ++q) xr[j][q] = f0 + q < I ? src[f0 + q] : (f0 + q == I ? 1.f : 0.f);
      }
    }
  };
  auto stage_x = [&](int buf) {
#pragma unroll
    for (int j = 0; j < XPT; ++j) {
      const int e = tid + j * NT;
      if (e < XCH) {
        const int r = e / (IP / 4), f0 = 4 * (e % (IP / 4));
        *reinterpret_cast<uint2*>(&sbuf[buf][r][HP + f0]) = pack4_bf16(xr[j]);
      }
    }
  };
  load_x(0);
  stage_x(0);
  if (T > 1) load_x(1);
  __syncthreads();

  for (int t = 0; t < T; ++t) {
    const int cur = t & 1;
    if (hxb) {  // the B-operand rows of this step, for the weight-gradient GEMM
      constexpr int CH = RT * 16 * (KP / 8);
      for (int e = tid; e < CH; e += NT) {
        const int r = e / (KP / 8), k0 = 8 * (e % (KP / 8));
        if (row0 + r < B)
          *reinterpret_cast<uint4*>(hxb + r * TKP + t * KP + k0) = *reinterpret_cast<const uint4*>(&sbuf[cur][r][k0]);
      }
    }
    f32x4 acc[RT][4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 bv = *reinterpret_cast<const f32x4*>(&bias_s[kc0 + 16 * g]);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) acc[rt][g] = bv;
    }
    // x_{t+1} -> the other buffer (read by no one until after this step's barrier).  Kept BEFORE
    // the MFMAs: the accumulators must be consumed in the same basic block as the MFMAs that write
    // them, where the compiler's hazard recognizer pads the MFMA -> VALU read latency (a branch in
    // between let the last step read unfinished accumulators).
    if (t + 1 < T) {
      stage_x(cur ^ 1);
      if (t + 2 < T) load_x(t + 2);
    }
#pragma unroll
    for (int ks = 0; ks < KT; ++ks)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const bf16x8 hb = *reinterpret_cast<const bf16x8*>(&sbuf[cur][rt * 16 + col][32 * ks + 8 * quad]);
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[rt][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[g][ks], hb, acc[rt][g], 0, 0, 0);
      }
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      f32x4 ig, fg, gg, og, hn;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        ig[r] = sigmoidf_(acc[rt][0][r]);
        fg[r] = sigmoidf_(acc[rt][1][r]);
        gg[r] = tanhf_(acc[rt][2][r]);
        og[r] = sigmoidf_(acc[rt][3][r]);
        c[rt][r] = fg[r] * c[rt][r] + ig[r] * gg[r];
        hn[r] = og[r] * tanhf_(c[rt][r]);
      }
      *reinterpret_cast<uint2*>(&sbuf[cur ^ 1][rt * 16 + col][u0]) = pack4_bf16(hn);
      if (rok[rt]) {
        *reinterpret_cast<f32x4*>(csb + lrow[rt] * THP + t * HP + u0) = c[rt];
        float* hp = hsb + lrow[rt] * TH + t * H + u0;
        if (vec_h) {
          if (u0 < H) *reinterpret_cast<f32x4*>(hp) = hn;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (u0 + r < H) hp[r] = hn[r];
        }
        if (gtb) {
          unsigned short* gp = gtb + lrow[rt] * TG + t * G4P + kc0;
          *reinterpret_cast<uint2*>(gp) = pack4_bf16(ig);
          *reinterpret_cast<uint2*>(gp + 16) = pack4_bf16(fg);
          *reinterpret_cast<uint2*>(gp + 32) = pack4_bf16(gg);
          *reinterpret_cast<uint2*>(gp + 48) = pack4_bf16(og);
        }
      }
    }
    __syncthreads();
  }
}

// dhseq  [B, T, H]   gradient of the loss w.r.t. every h_t returned by the forward
// gates  [B, T, 4HP] bf16 post-activation gates (kernel order);  cseq [B, T, HP];  c0 [B, H] or null
// dhn/dcn [B, H]     gradient w.r.t. the final (h_T, c_T) or null
// wfragT [NW][4KS][64] bf16x8: A-fragment of W_hhᵀ for dhᵀ = W_hhᵀ·dzᵀ (k runs over the 4·HP gate
//                    rows, gate-major: k = g·HP + u)
// dz     [B, T, 4HP] bf16 out, kernel order (pre-activation gate gradients, the operand of the
//        weight-gradient GEMMs);  dh0/dc0 [B, H] fp32 out
// Step t's inputs (gates, c_t, c_{t-1}, dh_t) are prefetched during step t+1.
template <int KS, int RT>
__global__ __launch_bounds__(128 * KS) void lstm_bwd_kernel(
    const float* __restrict__ dhseq, const unsigned short* __restrict__ gates, const float* __restrict__ cseq,
    const float* __restrict__ c0, const float* __restrict__ dhn, const float* __restrict__ dcn,
    const bf16x8* __restrict__ wfragT, int B, int T, int H, unsigned short* __restrict__ dz,
    float* __restrict__ dh0, float* __restrict__ dc0) {
  constexpr int HP = 32 * KS, G4P = 4 * HP, LDZ = G4P + 8;
  __shared__ __attribute__((aligned(16))) unsigned short zbuf[RT * 16][LDZ];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = lane & 15, quad = lane >> 4;
  const int u0 = 16 * w + 4 * quad, kc0 = 64 * w + 4 * quad;
  const long long row0 = (long long)blockIdx.x * (RT * 16);
  const int TG = T * G4P, THP = T * HP, TH = T * H;
  const bool vec_h = (H & 3) == 0;
  const unsigned short* gtb = gates + row0 * TG;
  const float* csb = cseq + row0 * THP;
  const float* dhb = dhseq + row0 * TH;
  unsigned short* dzb = dz + row0 * TG;

  bf16x8 wb[4 * KS];
#pragma unroll
  for (int ks = 0; ks < 4 * KS; ++ks) wb[ks] = wfragT[(w * 4 * KS + ks) * 64 + lane];

  int lrow[RT];
  bool rok[RT];
  f32x4 dhr[RT], dcc[RT], cinit[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const int lr = rt * 16 + col;
    rok[rt] = row0 + lr < B;
    lrow[rt] = rok[rt] ? lr : (int)(B - 1 - row0);
    const long long grow = row0 + lrow[rt];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool ok = u0 + r < H;
      dhr[rt][r] = (ok && dhn) ? dhn[grow * H + u0 + r] : 0.f;
      dcc[rt][r] = (ok && dcn) ? dcn[grow * H + u0 + r] : 0.f;
      cinit[rt][r] = (ok && c0) ? c0[grow * H + u0 + r] : 0.f;
    }
  }

  f32x4 pg[RT][4], pc[RT], pp[RT], pd[RT];
  auto fetch = [&](int t) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const unsigned short* gp = gtb + lrow[rt] * TG + t * G4P + kc0;
#pragma unroll
      for (int g = 0; g < 4; ++g) pg[rt][g] = unpack4_bf16(*reinterpret_cast<const uint2*>(gp + 16 * g));
      const float* cp = csb + lrow[rt] * THP + t * HP + u0;
      pc[rt] = *reinterpret_cast<const f32x4*>(cp);
      pp[rt] = t > 0 ? *reinterpret_cast<const f32x4*>(cp - HP) : cinit[rt];
      const float* dp = dhb + lrow[rt] * TH + t * H + u0;
      if (vec_h) {
        pd[rt] = u0 < H ? *reinterpret_cast<const f32x4*>(dp) : f32x4{0.f, 0.f, 0.f, 0.f};
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) pd[rt][r] = u0 + r < H ? dp[r] : 0.f;
      }
    }
  };
  fetch(T - 1);
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) dhr[rt] += pd[rt];

  for (int t = T - 1; t >= 0; --t) {
    f32x4 zi[RT], zf[RT], zg[RT], zo[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float ig = pg[rt][0][r], fg = pg[rt][1][r], gg = pg[rt][2][r], og = pg[rt][3][r];
        const float dh = dhr[rt][r];  // = dh_t from above + recurrent dh (folded after the MFMA)
        const float tc = tanhf_(pc[rt][r]);
        const float dc = dcc[rt][r] + dh * og * (1.f - tc * tc);
        zo[rt][r] = dh * tc * og * (1.f - og);
        zi[rt][r] = dc * gg * ig * (1.f - ig);
        zg[rt][r] = dc * ig * (1.f - gg * gg);
        zf[rt][r] = dc * pp[rt][r] * fg * (1.f - fg);
        dcc[rt][r] = dc * fg;
      }
    if (t > 0) {
      fetch(t - 1);
    } else {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) pd[rt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const uint2 bi = pack4_bf16(zi[rt]), bf = pack4_bf16(zf[rt]), bg = pack4_bf16(zg[rt]), bo = pack4_bf16(zo[rt]);
      unsigned short* zr = &zbuf[rt * 16 + col][u0];
      *reinterpret_cast<uint2*>(zr) = bi;
      *reinterpret_cast<uint2*>(zr + HP) = bf;
      *reinterpret_cast<uint2*>(zr + 2 * HP) = bg;
      *reinterpret_cast<uint2*>(zr + 3 * HP) = bo;
      if (rok[rt]) {
        unsigned short* zp = dzb + lrow[rt] * TG + t * G4P + kc0;
        *reinterpret_cast<uint2*>(zp) = bi;
        *reinterpret_cast<uint2*>(zp + 16) = bf;
        *reinterpret_cast<uint2*>(zp + 32) = bg;
        *reinterpret_cast<uint2*>(zp + 48) = bo;
      }
    }
    __syncthreads();
    f32x4 acc[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc[rt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4 * KS; ++ks)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const bf16x8 zb = *reinterpret_cast<const bf16x8*>(&zbuf[rt * 16 + col][32 * ks + 8 * quad]);
        acc[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[ks], zb, acc[rt], 0, 0, 0);
      }
    // consume the accumulators in this basic block (hazard padding, see the forward kernel); pd
    // holds dh_{t-1} from above (zero after the last step)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) dhr[rt] = acc[rt] + pd[rt];
    __syncthreads();  // zbuf is rewritten by the next timestep
  }
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
    if (rok[rt]) {
      const long long grow = row0 + lrow[rt];
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (u0 + r < H) {
          dh0[grow * H + u0 + r] = dhr[rt][r];
          dc0[grow * H + u0 + r] = dcc[rt][r];
        }
    }
}

template <int KS, int IS, int RT>
void launch_fwd(const float* x, int I, const void* wfrag, const float* bias, const float* h0, const float* c0, int B,
                int T, int H, float* hseq, float* cseq, unsigned short* gates, unsigned short* hx, hipStream_t s) {
  const int grid = (B + 16 * RT - 1) / (16 * RT);
  lstm_fwd_kernel<KS, IS, RT><<<grid, 128 * KS, 0, s>>>(x, I, reinterpret_cast<const bf16x8*>(wfrag), bias, h0, c0,
                                                       B, T, H, hseq, cseq, gates, hx);
}

template <int KS, int RT>
void launch_bwd(const float* dhseq, const unsigned short* gates, const float* cseq, const float* c0, const float* dhn,
                const float* dcn, const void* wfragT, int B, int T, int H, unsigned short* dz, float* dh0, float* dc0,
                hipStream_t s) {
  const int grid = (B + 16 * RT - 1) / (16 * RT);
  lstm_bwd_kernel<KS, RT><<<grid, 128 * KS, 0, s>>>(dhseq, gates, cseq, c0, dhn, dcn,
                                                   reinterpret_cast<const bf16x8*>(wfragT), B, T, H, dz, dh0, dc0);
}

#define AV_LSTM_FWD_IS(KS_, RT_, ...)                                            \
  switch (IS) {                                                                   \
    case 1: launch_fwd<KS_, 1, RT_>(__VA_ARGS__); break;                          \
    case 2: launch_fwd<KS_, 2, RT_>(__VA_ARGS__); break;                          \
    case 4: launch_fwd<KS_, 4, RT_>(__VA_ARGS__); break;                          \
    default: throw std::runtime_error("lstm: input size must be <= 128");         \
  }

#define AV_LSTM_DISPATCH(FN, ...)                                  \
  switch (KS * 8 + RT) {                                           \
    case 1 * 8 + 1: FN<1, 1>(__VA_ARGS__); break;                  \
    case 1 * 8 + 2: FN<1, 2>(__VA_ARGS__); break;                  \
    case 2 * 8 + 1: FN<2, 1>(__VA_ARGS__); break;                  \
    case 2 * 8 + 2: FN<2, 2>(__VA_ARGS__); break;                  \
    case 4 * 8 + 1: FN<4, 1>(__VA_ARGS__); break;                  \
    default: throw std::runtime_error("lstm: unsupported (KS, RT)"); \
  }

}  // namespace

namespace avk {

// Rows per workgroup: two 16-row tiles share each wave's weight registers when H <= 64 and the
// batch still fills the chip; at HP = 128 the weight fragments (64 VGPRs) leave room for one tile.
int lstm_row_tiles(long long B, int KS) { return (KS <= 2 && B >= 16384) ? 2 : 1; }

static void check_offsets(int T, int KS, int RT) {
  if ((long long)16 * RT * T * 128 * KS >= (1LL << 31))
    throw std::runtime_error("lstm: T * H too large for 32-bit per-workgroup offsets");
}

void lstm_fwd(const float* x, int I, int IS, const void* wfrag, const float* bias, const float* h0, const float* c0,
              int B, int T, int H, int KS, int RT, float* hseq, float* cseq, unsigned short* gates, unsigned short* hx,
              hipStream_t s) {
  check_offsets(T, KS + IS, RT);
  switch (KS * 8 + RT) {
    case 1 * 8 + 1: AV_LSTM_FWD_IS(1, 1, x, I, wfrag, bias, h0, c0, B, T, H, hseq, cseq, gates, hx, s) break;
    case 1 * 8 + 2: AV_LSTM_FWD_IS(1, 2, x, I, wfrag, bias, h0, c0, B, T, H, hseq, cseq, gates, hx, s) break;
    case 2 * 8 + 1: AV_LSTM_FWD_IS(2, 1, x, I, wfrag, bias, h0, c0, B, T, H, hseq, cseq, gates, hx, s) break;
    case 2 * 8 + 2: AV_LSTM_FWD_IS(2, 2, x, I, wfrag, bias, h0, c0, B, T, H, hseq, cseq, gates, hx, s) break;
    case 4 * 8 + 1: AV_LSTM_FWD_IS(4, 1, x, I, wfrag, bias, h0, c0, B, T, H, hseq, cseq, gates, hx, s) break;
    default: throw std::runtime_error("lstm: unsupported (KS, RT)");
  }
  AV_HIP_CHECK(hipGetLastError());
}

void lstm_bwd(const float* dhseq, const unsigned short* gates, const float* cseq, const float* c0, const float* dhn,
              const float* dcn, const void* wfragT, int B, int T, int H, int KS, int RT, unsigned short* dz,
              float* dh0, float* dc0, hipStream_t s) {
  check_offsets(T, KS, RT);
  AV_LSTM_DISPATCH(launch_bwd, dhseq, gates, cseq, c0, dhn, dcn, wfragT, B, T, H, dz, dh0, dc0, s)
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
