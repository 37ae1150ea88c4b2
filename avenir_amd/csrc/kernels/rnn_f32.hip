// K27 (fp32) — persistent fused LSTM recurrence on the f32 matrix cores, forward + backward.
//
// The fp32 twin of rnn.hip for the reference's numerics (P/supv/lstm.py:275-339 trains an fp32
// torch.nn.LSTM): every product is v_mfma_f32_16x16x4_f32 — a k-ordered chain of f32 fmas, one
// rounding per product, no reduced-precision operand — and every stored intermediate is fp32.
//
//   forward : z_t = xw_t + h_{t-1}·W_hhᵀ ; i,f,o = σ(z), g = tanh(z) ; c_t = f c_{t-1} + i g ;
//             h_t = o tanh(c_t)
//   backward: dz_t from (dh_t, dc_t, saved gates) ; dh_{t-1} = dz_t·W_hh ; dc_{t-1} = dc_t f
//
// Split (MI355X): the input projection xw = x·W_ihᵀ + b of ALL timesteps is one fp32 library GEMM
// outside the kernel (fully parallel; with f32 operands the recurrent weights alone take HP VGPRs,
// so [W_hh | W_ih] no longer both fit in registers as in the bf16 kernel).  Only the sequential
// part lives here.  One workgroup owns RT tiles of 16 sequences for the whole sequence; wave w owns
// hidden units [16w, 16w+16) of all four gates with its W_hh slice in VGPRs as f32 A-fragments
// (lane l of k-step s: W[row 16w + (l&15)][k 4s + (l>>4)]), the cell state in VGPRs in the
// accumulator layout (row = unit 4(l>>4) + r, column = sequence l&15 — the same C/D map as the bf16
// kernel, so the gate math is shared), and the accumulators start from xw_t.  h_t goes through LDS
// as fp32 (double-buffered, one barrier per step); the B operand of k-step s is one float per lane,
// h[seq l&15][unit 4s + (l>>4)] (rows padded to HP + 2 floats: conflict-free per half-wave).
// Weight-gradient GEMMs (dzᵀ·h_{t-1}, dzᵀ·x, Σdz) and dx = dz·W_ih run as fp32 library GEMMs on dz in
// torch gate order; lstm_pack_f32_kernel re-lays the parameters for a step in one launch.
#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// gate nonlinearities with the hardware reciprocal (v_rcp_f32, 1 ulp) instead of the IEEE
// division sequence (~10 instructions each, 5 per hidden unit per step on the recurrence's path)
__device__ __forceinline__ float sigm(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float tanh_(float x) {
  const float e = __expf(-2.f * fabsf(x));
  return copysignf((1.f - e) * __builtin_amdgcn_rcpf(1.f + e), x);
}

// Layouts (kernel order of the 4·HP gate columns: kc = 64·w + 16·g + i for unit u = 16·w + i, gate g):
//   xw     [B, T, 4HP] fp32, kernel order: x_t·W_ihᵀ + b_ih + b_hh (zero for padded units)  (PX = 0)
//   x      [B, T, I] fp32 (PX = 1: the input itself, I <= 8; also copied into hx when training)
//   wxfrag [NW][4][2][64] fp32 (PX = 1): A-fragments of W_ih, lane l of k-step s: W_ih[g·H + 16w + (l&15)][4s + (l>>4)]
//   biask  [4HP] fp32 kernel order (PX = 1): b_ih + b_hh, the accumulators' start
//   wfrag  [NW][4][KS4][64] fp32: A-fragment of W_hh for (wave, gate, k-step of 4), KS4 = HP / 4
//   h0, c0 [B, H] or null;  hseq [B, T, H], cseq [B, T, HP] fp32 out
//   gates  [B, T, 4HP] fp32 post-activation (kernel order) out or null
//   hx     [B, T, H + I + 1] fp32 out or null: [h_{t-1} | x_t | 1] (h0 / zeros at t = 0) — the B
//          operand rows of the backward's ONE weight-gradient GEMM (dW_hh, dW_ih and db together)
struct F32Fwd {
  const float* xw;
  const float* x;
  const float* wxfrag;
  const float* biask;
  const float* wfrag;
  const float* h0;
  const float* c0;
  int B, T, H, I;
  float* hseq;
  float* cseq;
  float* gates;
  float* hx;
};

// PX = 1: the input projection of a narrow input (I <= 8) runs INSIDE the recurrence as two extra
// MFMA k-steps per gate (x_t as the B operand, W_ih fragments in 8 VGPRs), so the layer needs no
// projection GEMM and no B·T·4HP xw tensor.
template <int KS, int RT, int PX>
__global__ __launch_bounds__(128 * KS) void lstm_fwd_f32_kernel(const F32Fwd a) {
  // h rows padded to HP + 2 floats: the B-operand read of k-step s (lane (quad, col) reads row col,
  // column 4 s + quad) hits bank 2 col + quad: distinct within each half-wave (HP + 1 put (col, quad)
  // and (col + 1, quad - 1) on one bank: 3.9 conflict cycles per LDS instruction measured)
  constexpr int HP = 32 * KS, KS4 = HP / 4, G4P = 4 * HP, NT = 128 * KS, LROW = HP + 2;
  __shared__ float sbuf[2][RT * 16][LROW];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int col = lane & 15, quad = lane >> 4;
  const int u0 = 16 * w + 4 * quad, kc0 = 64 * w + 4 * quad;
  const int B = a.B, T = a.T, H = a.H, I = a.I;
  const long long row0 = (long long)blockIdx.x * (RT * 16);
  const long long TG = (long long)T * G4P, THP = (long long)T * HP, TH = (long long)T * H, TI = (long long)T * I;
  const int HXS = H + I + 1;
  const long long THX = (long long)T * HXS;
  const bool vec_h = (H & 3) == 0;
  float* __restrict__ hx = a.hx;

  float wf[4][KS4];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int s = 0; s < KS4; ++s) wf[g][s] = a.wfrag[((w * 4 + g) * KS4 + s) * 64 + lane];
  float wx[4][2];
  f32x4 bk[4];
  if constexpr (PX) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
#pragma unroll
      for (int s = 0; s < 2; ++s) wx[g][s] = a.wxfrag[((w * 4 + g) * 2 + s) * 64 + lane];
      bk[g] = *reinterpret_cast<const f32x4*>(a.biask + kc0 + 16 * g);
    }
  }

  int lrow[RT];
  bool rok[RT];
  f32x4 c[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const int lr = rt * 16 + col;
    rok[rt] = row0 + lr < B;
    lrow[rt] = rok[rt] ? lr : (int)(B - 1 - row0);
    const long long grow = row0 + lrow[rt];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool ok = u0 + r < H;
      c[rt][r] = (ok && a.c0) ? a.c0[grow * H + u0 + r] : 0.f;
      const float hv = (ok && a.h0) ? a.h0[grow * H + u0 + r] : 0.f;
      sbuf[0][lr][u0 + r] = hv;
      if (hx && ok && rok[rt]) hx[grow * THX + u0 + r] = hv;
    }
  }
  if (hx) {  // the [x_t | 1] columns of every step of this workgroup's rows
    const int rows = (int)min((long long)RT * 16, (long long)B - row0), per = I + 1;
    for (int e = tid; e < rows * T * per; e += NT) {
      const int r = e / (T * per), rest = e - r * (T * per), t = rest / per, i = rest - t * per;
      const long long grow = row0 + r;
      hx[grow * THX + (long long)t * HXS + H + i] = i < I ? a.x[grow * TI + (long long)t * I + i] : 1.f;
    }
  }
  // xw_t (PX = 0) or x_t (PX = 1) of this lane, prefetched one step ahead
  f32x4 xn[RT][4];
  float xi[RT][2];
  auto load_in = [&](int t) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      if constexpr (PX) {
        const float* src = a.x + (row0 + lrow[rt]) * TI + (long long)t * I;
#pragma unroll
        for (int s = 0; s < 2; ++s) xi[rt][s] = 4 * s + quad < I ? src[4 * s + quad] : 0.f;
      } else {
        const float* src = a.xw + (row0 + lrow[rt]) * TG + (long long)t * G4P + kc0;
#pragma unroll
        for (int g = 0; g < 4; ++g) xn[rt][g] = *reinterpret_cast<const f32x4*>(src + 16 * g);
      }
    }
  };
  load_in(0);
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    const int cur = t & 1;
    f32x4 acc[RT][4];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        if constexpr (PX) {
          acc[rt][g] = bk[g];
#pragma unroll
          for (int s = 0; s < 2; ++s) acc[rt][g] = __builtin_amdgcn_mfma_f32_16x16x4f32(wx[g][s], xi[rt][s], acc[rt][g], 0, 0, 0);
        } else {
          acc[rt][g] = xn[rt][g];
        }
      }
    if (t + 1 < T) load_in(t + 1);
#pragma unroll
    for (int s = 0; s < KS4; ++s)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const float hb = sbuf[cur][rt * 16 + col][4 * s + quad];
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[rt][g] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[g][s], hb, acc[rt][g], 0, 0, 0);
      }
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      f32x4 ig, fg, gg, og, hn;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        ig[r] = sigm(acc[rt][0][r]);
        fg[r] = sigm(acc[rt][1][r]);
        gg[r] = tanh_(acc[rt][2][r]);
        og[r] = sigm(acc[rt][3][r]);
        c[rt][r] = fg[r] * c[rt][r] + ig[r] * gg[r];
        hn[r] = og[r] * tanh_(c[rt][r]);
        sbuf[cur ^ 1][rt * 16 + col][u0 + r] = hn[r];
      }
      if (rok[rt]) {
        *reinterpret_cast<f32x4*>(a.cseq + lrow[rt] * THP + (long long)t * HP + u0 + row0 * THP) = c[rt];
        float* hp = a.hseq + (row0 + lrow[rt]) * TH + (long long)t * H + u0;
        if (vec_h) {
          if (u0 < H) *reinterpret_cast<f32x4*>(hp) = hn;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (u0 + r < H) hp[r] = hn[r];
        }
        if (hx && t + 1 < T) {
          float* pp = hx + (row0 + lrow[rt]) * THX + (long long)(t + 1) * HXS + u0;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (u0 + r < H) pp[r] = hn[r];
        }
        if (a.gates) {
          float* gp = a.gates + (row0 + lrow[rt]) * TG + (long long)t * G4P + kc0;
          *reinterpret_cast<f32x4*>(gp) = ig;
          *reinterpret_cast<f32x4*>(gp + 16) = fg;
          *reinterpret_cast<f32x4*>(gp + 32) = gg;
          *reinterpret_cast<f32x4*>(gp + 48) = og;
        }
      }
    }
    __syncthreads();
  }
}

// dhseq [B, T, H]; gates [B, T, 4HP] fp32 kernel order; cseq [B, T, HP]; c0 / dhn / dcn [B, H] or null
// wfragT [NW][4HP/4][64] fp32: A-fragment of W_hhᵀ for dhᵀ = W_hhᵀ·dzᵀ, k over the 4·HP gate rows
//        gate-major (k = g·HP + u): lane l of k-step s holds W_hh[k = 4s + (l>>4)][unit 16w + (l&15)]
// dz [B, T, 4H] fp32 out in torch.nn.LSTM gate order (column g·H + u, padding dropped), so the
//    weight-gradient GEMMs land in the parameters' own row order; dh0 / dc0 [B, H] out
template <int KS, int RT>
__global__ __launch_bounds__(128 * KS) void lstm_bwd_f32_kernel(
    const float* __restrict__ dhseq, const float* __restrict__ gates, const float* __restrict__ cseq,
    const float* __restrict__ c0, const float* __restrict__ dhn, const float* __restrict__ dcn,
    const float* __restrict__ wfragT, int B, int T, int H, float* __restrict__ dz, float* __restrict__ dh0,
    float* __restrict__ dc0) {
  // dz rows padded to 4 HP + 2 floats (bank 2 col + quad for the B-operand reads, as the forward)
  constexpr int HP = 32 * KS, G4P = 4 * HP, KB = G4P / 4, LZ = G4P + 2;
  __shared__ float zbuf[RT * 16][LZ];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = lane & 15, quad = lane >> 4;
  const int u0 = 16 * w + 4 * quad, kc0 = 64 * w + 4 * quad;
  const long long row0 = (long long)blockIdx.x * (RT * 16);
  const long long TG = (long long)T * G4P, THP = (long long)T * HP, TH = (long long)T * H, T4H = 4 * TH;
  const bool vec_h = (H & 3) == 0;

  float wb[KB];
#pragma unroll
  for (int s = 0; s < KB; ++s) wb[s] = wfragT[(w * KB + s) * 64 + lane];

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
      const long long grow = row0 + lrow[rt];
      const float* gp = gates + grow * TG + (long long)t * G4P + kc0;
#pragma unroll
      for (int g = 0; g < 4; ++g) pg[rt][g] = *reinterpret_cast<const f32x4*>(gp + 16 * g);
      const float* cp = cseq + grow * THP + (long long)t * HP + u0;
      pc[rt] = *reinterpret_cast<const f32x4*>(cp);
      pp[rt] = t > 0 ? *reinterpret_cast<const f32x4*>(cp - HP) : cinit[rt];
      const float* dp = dhseq + grow * TH + (long long)t * H + u0;
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
        const float dh = dhr[rt][r];
        const float tc = tanh_(pc[rt][r]);
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
      float* zr = &zbuf[rt * 16 + col][u0];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        zr[r] = zi[rt][r];
        zr[HP + r] = zf[rt][r];
        zr[2 * HP + r] = zg[rt][r];
        zr[3 * HP + r] = zo[rt][r];
      }
      if (rok[rt] && u0 < H) {
        float* zp = dz + (row0 + lrow[rt]) * T4H + (long long)t * 4 * H + u0;
        if (vec_h) {
          *reinterpret_cast<f32x4*>(zp) = zi[rt];
          *reinterpret_cast<f32x4*>(zp + H) = zf[rt];
          *reinterpret_cast<f32x4*>(zp + 2 * H) = zg[rt];
          *reinterpret_cast<f32x4*>(zp + 3 * H) = zo[rt];
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (u0 + r < H) {
              zp[r] = zi[rt][r];
              zp[H + r] = zf[rt][r];
              zp[2 * H + r] = zg[rt][r];
              zp[3 * H + r] = zo[rt][r];
            }
        }
      }
    }
    __syncthreads();
    f32x4 acc[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc[rt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KB; ++s)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
        acc[rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(wb[s], zbuf[rt * 16 + col][4 * s + quad], acc[rt], 0, 0, 0);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) dhr[rt] = acc[rt] + pd[rt];
    __syncthreads();
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

// One launch re-lays the parameters for a step (replacing ~a dozen small copy / scatter launches):
//   wfrag  [NW][4][HP/4][64]  forward A-fragments of W_hh (lane l, k-step s: W_hh[g·H + 16w + (l&15)][4s + (l>>4)])
//   wfragT [NW][HP][64]       backward A-fragments of W_hhᵀ (k = 4s + (l>>4) over the gate-major 4·HP rows)
//   wihk   [4HP, I]           W_ih rows in kernel gate order (the input-projection GEMM's operand)
//   biask  [4HP]              b_ih + b_hh in kernel gate order
//   wxfrag [NW][4][2][64]     (I <= 8, else null) W_ih A-fragments of the in-kernel projection
// Padded units / columns are zero.  Flat grid-stride over the outputs.
__global__ __launch_bounds__(256) void lstm_pack_f32_kernel(const float* __restrict__ w_ih,
                                                            const float* __restrict__ w_hh,
                                                            const float* __restrict__ b_ih,
                                                            const float* __restrict__ b_hh, int H, int I, int HP,
                                                            float* __restrict__ wfrag, float* __restrict__ wfragT,
                                                            float* __restrict__ wihk, float* __restrict__ biask,
                                                            float* __restrict__ wxfrag) {
  const long long n1 = 4LL * HP * HP, n3 = 4LL * HP * I, n5 = wxfrag ? (long long)(HP / 16) * 4 * 2 * 64 : 0;
  const long long n = 2 * n1 + n3 + 4 * HP + n5;
  const int KS4 = HP / 4;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    if (e < n1) {
      const int lane = (int)(e & 63);
      const long long rest = e >> 6;
      const int s = (int)(rest % KS4), g = (int)((rest / KS4) & 3), w = (int)(rest / (4 * KS4));
      const int u = 16 * w + (lane & 15), k = 4 * s + (lane >> 4);
      wfrag[e] = (u < H && k < H) ? w_hh[(long long)(g * H + u) * H + k] : 0.f;
    } else if (e < 2 * n1) {
      const long long f = e - n1;
      const int lane = (int)(f & 63);
      const long long rest = f >> 6;
      const int s = (int)(rest % HP), w = (int)(rest / HP);
      const int k = 4 * s + (lane >> 4), g = k / HP, uu = k % HP, cu = 16 * w + (lane & 15);
      wfragT[f] = (uu < H && cu < H) ? w_hh[(long long)(g * H + uu) * H + cu] : 0.f;
    } else if (e >= 2 * n1 + n3 + 4 * HP) {
      const long long f = e - (2 * n1 + n3 + 4 * HP);
      const int lane = (int)(f & 63);
      const long long rest = f >> 6;
      const int s = (int)(rest & 1), g = (int)((rest >> 1) & 3), w = (int)(rest >> 3);
      const int u = 16 * w + (lane & 15), k = 4 * s + (lane >> 4);
      wxfrag[f] = (u < H && k < I) ? w_ih[(long long)(g * H + u) * I + k] : 0.f;
    } else {
      const long long f = e - 2 * n1;
      const int kc = f < n3 ? (int)(f / I) : (int)(f - n3);
      const int w = kc >> 6, g = (kc >> 4) & 3, u = 16 * w + (kc & 15);
      if (f < n3) {
        const int j = (int)(f % I);
        wihk[f] = u < H ? w_ih[(long long)(g * H + u) * I + j] : 0.f;
      } else {
        float b = 0.f;
        if (u < H) b = (b_ih ? b_ih[g * H + u] : 0.f) + (b_hh ? b_hh[g * H + u] : 0.f);
        biask[kc] = b;
      }
    }
  }
}

}  // namespace

namespace avk {

void lstm_pack_f32(const float* w_ih, const float* w_hh, const float* b_ih, const float* b_hh, int H, int I, int KS,
                   float* wfrag, float* wfragT, float* wihk, float* biask, float* wxfrag, hipStream_t s) {
  const int HP = 32 * KS;
  const long long n = 8LL * HP * HP + 4LL * HP * I + 4LL * HP + (wxfrag ? (HP / 16) * 4 * 2 * 64 : 0);
  const int grid = (int)std::min<long long>((n + 255) / 256, 2048);
  lstm_pack_f32_kernel<<<grid, 256, 0, s>>>(w_ih, w_hh, b_ih, b_hh, H, I, HP, wfrag, wfragT, wihk, biask, wxfrag);
  AV_HIP_CHECK(hipGetLastError());
}

// RT = 1 throughout: the f32 weight fragments take HP (forward) / 4·HP/4 (backward) VGPRs per
// lane, leaving no room for a second tile's accumulators at HP = 128.
void lstm_fwd_f32(const float* xw, const float* x, const float* wxfrag, const float* biask, const float* wfrag,
                  const float* h0, const float* c0, int B, int T, int H, int I, int KS, float* hseq, float* cseq,
                  float* gates, float* hx, hipStream_t s) {
  const int grid = (B + 15) / 16;
  const F32Fwd a{xw, x, wxfrag, biask, wfrag, h0, c0, B, T, H, I, hseq, cseq, gates, hx};
  const bool px = xw == nullptr;
  if (px && (I > 8 || !x || !wxfrag || !biask)) throw std::runtime_error("lstm_fwd_f32: in-kernel projection needs I <= 8");
#define AV_LF(KS_, NT_) \
  (px ? lstm_fwd_f32_kernel<KS_, 1, 1><<<grid, NT_, 0, s>>>(a) : lstm_fwd_f32_kernel<KS_, 1, 0><<<grid, NT_, 0, s>>>(a))
  switch (KS) {
    case 1: AV_LF(1, 128); break;
    case 2: AV_LF(2, 256); break;
    case 4: AV_LF(4, 512); break;
    default: throw std::runtime_error("lstm_fwd_f32: KS in {1, 2, 4}");
  }
#undef AV_LF
  AV_HIP_CHECK(hipGetLastError());
}

void lstm_bwd_f32(const float* dhseq, const float* gates, const float* cseq, const float* c0, const float* dhn,
                  const float* dcn, const float* wfragT, int B, int T, int H, int KS, float* dz, float* dh0,
                  float* dc0, hipStream_t s) {
  const int grid = (B + 15) / 16;
  switch (KS) {
    case 1:
      lstm_bwd_f32_kernel<1, 1><<<grid, 128, 0, s>>>(dhseq, gates, cseq, c0, dhn, dcn, wfragT, B, T, H, dz, dh0, dc0);
      break;
    case 2:
      lstm_bwd_f32_kernel<2, 1><<<grid, 256, 0, s>>>(dhseq, gates, cseq, c0, dhn, dcn, wfragT, B, T, H, dz, dh0, dc0);
      break;
    case 4:
      lstm_bwd_f32_kernel<4, 1><<<grid, 512, 0, s>>>(dhseq, gates, cseq, c0, dhn, dcn, wfragT, B, T, H, dz, dh0, dc0);
      break;
    default: throw std::runtime_error("lstm_bwd_f32: KS in {1, 2, 4}");
  }
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
