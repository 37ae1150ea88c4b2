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
// its W_hh slice stays in VGPRs as v_mfma_f32_16x16x32_bf16 B-fragments for every timestep (HP/2
// VGPRs), the cell state c stays in VGPRs in the MFMA accumulator layout (row = 4·(lane>>4) + r,
// column = lane & 15), and the accumulators are initialised with xw_t so the input projection and
// both biases are added for free.  Only h_t (bf16) goes through LDS — double-buffered, one barrier
// per timestep.  Padded hidden units (H < HP) carry zero weights and zero inputs, so their h stays 0.
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

// xw     [B, T, 4H] fp32   x_t·W_ihᵀ + b_ih + b_hh (gate order i, f, g, o as torch.nn.LSTM)
// wfrag  [NW][4][KS][64] bf16x8 — B-fragment of W_hh for (wave, gate, k-step), lane-ordered
// h0, c0 [B, H] or null (zeros)
// hseq, cseq [B, T, H] fp32 out;  gates [B, T, 4H] (post-activation, for backward) out or null
// All per-element offsets are 32-bit relative to the workgroup's first row (host checks
// 16·RT·T·4H < 2^31), so loads/stores use an SGPR base + one VGPR offset.  Rows past B are
// clamped for loads and masked for stores.  xw of step t+1 is prefetched during step t.
template <int KS, int RT>
__global__ __launch_bounds__(128 * KS) void lstm_fwd_kernel(const float* __restrict__ xw,
                                                            const bf16x8* __restrict__ wfrag,
                                                            const float* __restrict__ h0,
                                                            const float* __restrict__ c0, int B, int T,
                                                            int H, float* __restrict__ hseq,
                                                            float* __restrict__ cseq,
                                                            float* __restrict__ gates) {
  constexpr int HP = 32 * KS, LDH = HP + 8;  // +16 B per row: A-fragment reads spread over banks
  __shared__ __attribute__((aligned(16))) unsigned short hbuf[2][RT * 16][LDH];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = lane & 15, quad = lane >> 4;
  const int unit = 16 * w + col;
  const bool uok = unit < H;
  const int uc = uok ? unit : 0;
  const long long row0 = (long long)blockIdx.x * (RT * 16);
  const int G4 = 4 * H, TG4 = T * G4, TH = T * H;
  const float* xwb = xw + row0 * TG4;
  float* hsb = hseq + row0 * TH;
  float* csb = cseq + row0 * TH;
  float* gtb = gates ? gates + row0 * TG4 : nullptr;

  bf16x8 wf[4][KS];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) wf[g][ks] = wfrag[((w * 4 + g) * KS + ks) * 64 + lane];

  // per-lane row offsets (row index within the tile, clamped to B - 1 for loads) and store masks
  int lrow[RT][4];
  unsigned smask = 0;
  float c[RT][4];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int lr = rt * 16 + quad * 4 + r;
      const bool ok = row0 + lr < B;
      lrow[rt][r] = ok ? lr : (int)(B - 1 - row0);
      if (ok && uok) smask |= 1u << (rt * 4 + r);
      const long long grow = row0 + lrow[rt][r];
      c[rt][r] = (uok && c0) ? c0[grow * H + uc] : 0.f;
      hbuf[0][lr][unit] = f2bf((uok && h0) ? h0[grow * H + uc] : 0.f);
    }

  float xn[RT][4][4];  // prefetched xw of the next step
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int g = 0; g < 4; ++g) xn[rt][r][g] = uok ? xwb[lrow[rt][r] * TG4 + g * H + uc] : 0.f;
  __syncthreads();

  for (int t = 0; t < T; ++t) {
    const int cur = t & 1;
    f32x4 acc[RT][4];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[rt][g][r] = xn[rt][r][g];
    if (t + 1 < T) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int g = 0; g < 4; ++g)
            xn[rt][r][g] = uok ? xwb[lrow[rt][r] * TG4 + (t + 1) * G4 + g * H + uc] : 0.f;
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(&hbuf[cur][rt * 16 + col][32 * ks + 8 * quad]);
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[rt][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wf[g][ks], acc[rt][g], 0, 0, 0);
      }
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float ig = sigmoidf_(acc[rt][0][r]), fg = sigmoidf_(acc[rt][1][r]);
        const float gg = tanhf_(acc[rt][2][r]), og = sigmoidf_(acc[rt][3][r]);
        const float cn = fg * c[rt][r] + ig * gg;
        const float hn = og * tanhf_(cn);
        c[rt][r] = cn;
        hbuf[cur ^ 1][rt * 16 + quad * 4 + r][unit] = f2bf(hn);
        if (smask >> (rt * 4 + r) & 1u) {
          const int o = lrow[rt][r] * TH + t * H + unit;
          hsb[o] = hn;
          csb[o] = cn;
          if (gtb) {
            float* gp = gtb + lrow[rt][r] * TG4 + t * G4 + unit;
            gp[0] = ig;
            gp[H] = fg;
            gp[2 * H] = gg;
            gp[3 * H] = og;
          }
        }
      }
    __syncthreads();
  }
}

// dhseq  [B, T, H]  gradient of the loss w.r.t. every h_t returned by the forward
// gates  [B, T, 4H] post-activation gates, cseq [B, T, H] cell states, c0 [B, H] or null
// dhn/dcn [B, H]    gradient w.r.t. the final (h_T, c_T) or null
// wfragT [NW][4KS][64] bf16x8 — B-fragment of W_hh for dh = dz·W_hh (k runs over 4·HP gate rows)
// dz     [B, T, 4H] out (pre-activation gate gradients);  dh0/dc0 [B, H] out
// Step t's inputs (gates, c_t, c_{t-1}, dh_t) are prefetched during step t+1.
template <int KS, int RT>
__global__ __launch_bounds__(128 * KS) void lstm_bwd_kernel(
    const float* __restrict__ dhseq, const float* __restrict__ gates, const float* __restrict__ cseq,
    const float* __restrict__ c0, const float* __restrict__ dhn, const float* __restrict__ dcn,
    const bf16x8* __restrict__ wfragT, int B, int T, int H, float* __restrict__ dz,
    float* __restrict__ dh0, float* __restrict__ dc0) {
  constexpr int HP = 32 * KS, K4 = 4 * HP, LDZ = K4 + 8;
  __shared__ __attribute__((aligned(16))) unsigned short zbuf[RT * 16][LDZ];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = lane & 15, quad = lane >> 4;
  const int unit = 16 * w + col;
  const bool uok = unit < H;
  const int uc = uok ? unit : 0;
  const long long row0 = (long long)blockIdx.x * (RT * 16);
  const int G4 = 4 * H, TG4 = T * G4, TH = T * H;
  const float* gtb = gates + row0 * TG4;
  const float* csb = cseq + row0 * TH;
  const float* dhb = dhseq + row0 * TH;
  float* dzb = dz + row0 * TG4;

  bf16x8 wb[4 * KS];
#pragma unroll
  for (int ks = 0; ks < 4 * KS; ++ks) wb[ks] = wfragT[(w * 4 * KS + ks) * 64 + lane];

  int lrow[RT][4];
  unsigned smask = 0;
  float dhr[RT][4], dcc[RT][4], cinit[RT][4];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int lr = rt * 16 + quad * 4 + r;
      const bool ok = row0 + lr < B;
      lrow[rt][r] = ok ? lr : (int)(B - 1 - row0);
      if (ok && uok) smask |= 1u << (rt * 4 + r);
      const long long grow = row0 + lrow[rt][r];
      dhr[rt][r] = (uok && dhn) ? dhn[grow * H + uc] : 0.f;
      dcc[rt][r] = (uok && dcn) ? dcn[grow * H + uc] : 0.f;
      cinit[rt][r] = (uok && c0) ? c0[grow * H + uc] : 0.f;
    }

  // prefetched step inputs: 4 gates, c_t, c_{t-1}, dh_t
  float pg[RT][4][4], pc[RT][4], pp[RT][4], pd[RT][4];
  auto fetch = [&](int t) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int og = lrow[rt][r] * TG4 + t * G4 + uc, oh = lrow[rt][r] * TH + t * H + uc;
#pragma unroll
        for (int g = 0; g < 4; ++g) pg[rt][r][g] = gtb[og + g * H];
        pc[rt][r] = csb[oh];
        pp[rt][r] = t > 0 ? csb[oh - H] : cinit[rt][r];
        pd[rt][r] = dhb[oh];
      }
  };
  fetch(T - 1);

  for (int t = T - 1; t >= 0; --t) {
    float zi[RT][4], zf[RT][4], zg[RT][4], zo[RT][4];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float ig = pg[rt][r][0], fg = pg[rt][r][1], gg = pg[rt][r][2], og = pg[rt][r][3];
        const float dh = pd[rt][r] + dhr[rt][r];
        const float tc = tanhf_(pc[rt][r]);
        const float dc = dcc[rt][r] + dh * og * (1.f - tc * tc);
        const bool on = uok;  // padded units carry zero gradient
        zo[rt][r] = on ? dh * tc * og * (1.f - og) : 0.f;
        zi[rt][r] = on ? dc * gg * ig * (1.f - ig) : 0.f;
        zg[rt][r] = on ? dc * ig * (1.f - gg * gg) : 0.f;
        zf[rt][r] = on ? dc * pp[rt][r] * fg * (1.f - fg) : 0.f;
        dcc[rt][r] = dc * fg;
      }
    if (t > 0) fetch(t - 1);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int lr = rt * 16 + quad * 4 + r;
        zbuf[lr][unit] = f2bf(zi[rt][r]);
        zbuf[lr][HP + unit] = f2bf(zf[rt][r]);
        zbuf[lr][2 * HP + unit] = f2bf(zg[rt][r]);
        zbuf[lr][3 * HP + unit] = f2bf(zo[rt][r]);
        if (smask >> (rt * 4 + r) & 1u) {
          float* zp = dzb + lrow[rt][r] * TG4 + t * G4 + unit;
          zp[0] = zi[rt][r];
          zp[H] = zf[rt][r];
          zp[2 * H] = zg[rt][r];
          zp[3 * H] = zo[rt][r];
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
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(&zbuf[rt * 16 + col][32 * ks + 8 * quad]);
        acc[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wb[ks], acc[rt], 0, 0, 0);
      }
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) dhr[rt][r] = acc[rt][r];
    __syncthreads();  // zbuf is rewritten by the next timestep
  }
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (smask >> (rt * 4 + r) & 1u) {
        const long long grow = row0 + lrow[rt][r];
        dh0[grow * H + unit] = dhr[rt][r];
        dc0[grow * H + unit] = dcc[rt][r];
      }
}

template <int KS, int RT>
void launch_fwd(const float* xw, const void* wfrag, const float* h0, const float* c0, int B, int T, int H,
                float* hseq, float* cseq, float* gates, hipStream_t s) {
  const int grid = (B + 16 * RT - 1) / (16 * RT);
  lstm_fwd_kernel<KS, RT><<<grid, 128 * KS, 0, s>>>(xw, reinterpret_cast<const bf16x8*>(wfrag), h0, c0, B, T, H,
                                                   hseq, cseq, gates);
}

template <int KS, int RT>
void launch_bwd(const float* dhseq, const float* gates, const float* cseq, const float* c0, const float* dhn,
                const float* dcn, const void* wfragT, int B, int T, int H, float* dz, float* dh0, float* dc0,
                hipStream_t s) {
  const int grid = (B + 16 * RT - 1) / (16 * RT);
  lstm_bwd_kernel<KS, RT><<<grid, 128 * KS, 0, s>>>(dhseq, gates, cseq, c0, dhn, dcn,
                                                   reinterpret_cast<const bf16x8*>(wfragT), B, T, H, dz, dh0, dc0);
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

static void check_offsets(int T, int H, int RT) {
  if ((long long)16 * RT * T * 4 * H >= (1LL << 31))
    throw std::runtime_error("lstm: T * H too large for 32-bit per-workgroup offsets");
}

void lstm_fwd(const float* xw, const void* wfrag, const float* h0, const float* c0, int B, int T, int H, int KS,
              int RT, float* hseq, float* cseq, float* gates, hipStream_t s) {
  check_offsets(T, H, RT);
  AV_LSTM_DISPATCH(launch_fwd, xw, wfrag, h0, c0, B, T, H, hseq, cseq, gates, s)
  AV_HIP_CHECK(hipGetLastError());
}

void lstm_bwd(const float* dhseq, const float* gates, const float* cseq, const float* c0, const float* dhn,
              const float* dcn, const void* wfragT, int B, int T, int H, int KS, int RT, float* dz, float* dh0,
              float* dc0, hipStream_t s) {
  check_offsets(T, H, RT);
  AV_LSTM_DISPATCH(launch_bwd, dhseq, gates, cseq, c0, dhn, dcn, wfragT, B, T, H, dz, dh0, dc0, s)
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
