// K12: SMO for kernel SVMs — one persistent workgroup per problem (CDNA4, gfx950).
//
// Reference: Platt's SMO in J/discriminant/SequentialMinimalOptimization.java:77-282 (examine /
// step / error cache, linear kernel only, host loop over records) and the cascade SVM of
// J/discriminant/SupportVectorMachine.java:97-196 (SMO per mapper split, final SMO on the union of
// support vectors).
//
// MI355X design: the Gram matrix K [N, N] of a problem is built by ONE GEMM (hipBLASLt) and
// stays resident in HBM (288 GB holds N ~ 250k in fp32); the SMO loop is a single 1024-thread
// workgroup that never returns to the host: per iteration it
//   1. scans alpha / gradient for the maximal violating index i (first-order, I_up set),
//   2. reads row K[i] and picks j by the second-order gain -(b^2 / a) over I_low,
//   3. solves the two-variable sub-problem with box clipping (thread 0),
//   4. updates the gradient with rows K[i], K[j] (coalesced 64-lane row reads, L2 resident).
// Independent problems (cascade shards, one-vs-rest classes, CV folds) are independent
// workgroups of one launch: blockIdx.x = problem, so B problems fill the 256 CUs.
#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

constexpr int SMO_THREADS = 1024;
constexpr int SMO_WAVES = SMO_THREADS / 64;
constexpr float TAU = 1e-12f;

__device__ __forceinline__ void block_argmax(float& v, int& idx, float* sv, int* si) {
  av::wave_argmax(v, idx);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) { sv[w] = v; si[w] = idx; }
  __syncthreads();
  if (w == 0) {
    v = lane < SMO_WAVES ? sv[lane] : -INFINITY;
    idx = lane < SMO_WAVES ? si[lane] : 0x7fffffff;
    av::wave_argmax(v, idx);
    if (lane == 0) { sv[0] = v; si[0] = idx; }
  }
  __syncthreads();
  v = sv[0];
  idx = si[0];
  __syncthreads();
}

__global__ __launch_bounds__(SMO_THREADS) void smo_kernel(const float* __restrict__ Kall, const float* __restrict__ yall,
                                                          const float* __restrict__ dall, float* __restrict__ aall,
                                                          float* __restrict__ gall, int N, float C, float eps,
                                                          int max_iter, int* __restrict__ iters) {
  __shared__ float sv[SMO_WAVES];
  __shared__ int si[SMO_WAVES];
  __shared__ float upd[3];
  const long long b = blockIdx.x;
  const float* K = Kall + b * (long long)N * N;
  const float* y = yall + b * (long long)N;
  const float* QD = dall + b * (long long)N;
  float* alpha = aall + b * (long long)N;
  float* G = gall + b * (long long)N;
  int it = 0;
  for (; it < max_iter; ++it) {
    // ---- i: max over I_up of -y G ------------------------------------------------------------
    float gmax = -INFINITY;
    int gi = 0x7fffffff;
    for (int t = threadIdx.x; t < N; t += SMO_THREADS) {
      const float yt = y[t];
      if (yt == 0.f) continue;  // padding row
      const float at = alpha[t];
      const bool up = yt > 0.f ? at < C : at > 0.f;
      if (up) {
        const float v = -yt * G[t];
        if (v > gmax || (v == gmax && t < gi)) { gmax = v; gi = t; }
      }
    }
    block_argmax(gmax, gi, sv, si);
    if (gi == 0x7fffffff) break;
    const int i = gi;
    const float* Ki = K + (long long)i * N;
    const float Kii = QD[i];
    // ---- j: second-order selection over I_low; also max of y G over I_low for the stop test --
    float best = -INFINITY;  // maximise b^2 / a
    int bj = 0x7fffffff;
    float gmax2 = -INFINITY;
    for (int t = threadIdx.x; t < N; t += SMO_THREADS) {
      const float yt = y[t];
      if (yt == 0.f) continue;
      const float at = alpha[t];
      const bool low = yt > 0.f ? at > 0.f : at < C;
      if (!low) continue;
      const float yg = yt * G[t];
      gmax2 = fmaxf(gmax2, yg);
      const float bdiff = gmax + yg;
      if (bdiff > 0.f) {
        float a = Kii + QD[t] - 2.f * Ki[t];
        a = a > 0.f ? a : TAU;
        const float gain = bdiff * bdiff / a;
        if (gain > best || (gain == best && t < bj)) { best = gain; bj = t; }
      }
    }
    {
      int dummy = 0;
      block_argmax(gmax2, dummy, sv, si);
    }
    block_argmax(best, bj, sv, si);
    if (gmax + gmax2 < eps || bj == 0x7fffffff) break;
    const int j = bj;
    // ---- two-variable sub-problem (thread 0) ------------------------------------------------
    if (threadIdx.x == 0) {
      const float yi = y[i], yj = y[j];
      const float Gi = G[i], Gj = G[j];
      const float oi = alpha[i], oj = alpha[j];
      float ai = oi, aj = oj;
      const float Kij = Ki[j];
      float quad = Kii + QD[j] - 2.f * Kij;
      quad = quad > 0.f ? quad : TAU;
      if (yi != yj) {
        const float delta = (-Gi - Gj) / quad;
        const float diff = ai - aj;
        ai += delta;
        aj += delta;
        if (diff > 0.f) {
          if (aj < 0.f) { aj = 0.f; ai = diff; }
        } else {
          if (ai < 0.f) { ai = 0.f; aj = -diff; }
        }
        if (diff > 0.f) {
          if (ai > C) { ai = C; aj = C - diff; }
        } else {
          if (aj > C) { aj = C; ai = C + diff; }
        }
      } else {
        const float delta = (Gi - Gj) / quad;
        const float sum = ai + aj;
        ai -= delta;
        aj += delta;
        if (sum > C) {
          if (ai > C) { ai = C; aj = sum - C; }
        } else {
          if (aj < 0.f) { aj = 0.f; ai = sum; }
        }
        if (sum > C) {
          if (aj > C) { aj = C; ai = sum - C; }
        } else {
          if (ai < 0.f) { ai = 0.f; aj = sum; }
        }
      }
      alpha[i] = ai;
      alpha[j] = aj;
      upd[0] = (ai - oi) * yi;  // dalpha_i * y_i
      upd[1] = (aj - oj) * yj;
    }
    __syncthreads();
    const float di = upd[0], dj = upd[1];
    const float* Kj = K + (long long)j * N;
    // G_t += y_t (y_i K_it dalpha_i + y_j K_jt dalpha_j)
    for (int t = threadIdx.x; t < N; t += SMO_THREADS) {
      const float yt = y[t];
      if (yt == 0.f) continue;
      G[t] += yt * (Ki[t] * di + Kj[t] * dj);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) iters[b] = it;
}

// ---------------------------------------------------------------------------------------------
// Working-set (decomposition) SMO inner solver: ONE wavefront per problem solves the Q-variable
// sub-problem of a working set chosen on the device (top violators of the whole problem, see
// models/svm.py::smo_decomposition) with the Q x Q kernel block resident in LDS (64 KB for Q=128).
// Every reduction is a 64-lane shuffle (no barriers), so one SMO step costs a few hundred
// cycles instead of the block-wide scans of smo_kernel over all N; the O(N) work moves to the
// outer loop as one top-k and one batched GEMV per Q-variable step.
//   Kws [B][Q][Q], yws [B][Q] (0 = unused slot), aws [B][Q] in/out, gws [B][Q] (gradient of the
//   full problem restricted to the working set), gap [B] (global violation; the local
//   tolerance is max(eps, 0.1 gap)).
constexpr int WS_Q = 128;

// Converged-problem early exit shared by every kernel of an outer step: once the violation gap of
// problem b (written by the previous step's selection) is below the stopping tolerance, that step's
// sub-problem solve took zero iterations (its local violation <= gap < eps) and changed nothing, so
// the selection, gather, solve and update of every later step are no-ops and return at once.  This
// lets the host queue steps ahead of the convergence test (smo_ws_run) at ~no cost.
// (skip = -inf disables it; a NaN gap counts as converged, as in the host test.)
__device__ __forceinline__ bool ws_done(const float* gap, int b, float skip) {
  return gap != nullptr && skip > -INFINITY && !(gap[b] >= skip);
}

__device__ __forceinline__ unsigned order_key(float f) {  // monotone float -> uint
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Wave max of u32 keys: 4 DPP max steps + the 4 row results over v_readlane (uniform result).
// (old = 0, bound_ctrl: 0 is the identity of an unsigned max, so the DPP move folds into
// v_max_u32_dpp — no separate v_mov + wait state per step)
template <int CTRL>
__device__ __forceinline__ unsigned dpp_max_step(unsigned v) {
  return max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ unsigned wave_max_u32(unsigned v) {
  v = dpp_max_step<0xB1>(v);
  v = dpp_max_step<0x4E>(v);
  v = dpp_max_step<0x124>(v);
  v = dpp_max_step<0x128>(v);
  const unsigned a = (unsigned)__builtin_amdgcn_readlane((int)v, 0), b = (unsigned)__builtin_amdgcn_readlane((int)v, 16);
  const unsigned c = (unsigned)__builtin_amdgcn_readlane((int)v, 32), d = (unsigned)__builtin_amdgcn_readlane((int)v, 48);
  return max(max(a, b), max(c, d));
}

// two independent wave maxima with their DPP steps interleaved (each step's VGPR hazard is covered by
// the other chain's instruction instead of an s_nop)
__device__ __forceinline__ void wave_max2_u32(unsigned& u, unsigned& v) {
  u = dpp_max_step<0xB1>(u);
  v = dpp_max_step<0xB1>(v);
  u = dpp_max_step<0x4E>(u);
  v = dpp_max_step<0x4E>(v);
  u = dpp_max_step<0x124>(u);
  v = dpp_max_step<0x124>(v);
  u = dpp_max_step<0x128>(u);
  v = dpp_max_step<0x128>(v);
  auto rl = [](unsigned x, int l) { return (unsigned)__builtin_amdgcn_readlane((int)x, l); };
  u = max(max(rl(u, 0), rl(u, 16)), max(rl(u, 32), rl(u, 48)));
  v = max(max(rl(v, 0), rl(v, 16)), max(rl(v, 32), rl(v, 48)));
}

// The same maxima finished with the gfx950 row swaps (v_permlane16_swap / v_permlane32_swap)
// instead of 4 v_readlane + SALU max + broadcast: the result lands in every lane, 2 swaps + 2 max.
__device__ __forceinline__ unsigned wave_max_u32_v(unsigned v) {
  v = dpp_max_step<0xB1>(v);
  v = dpp_max_step<0x4E>(v);
  v = dpp_max_step<0x124>(v);
  v = dpp_max_step<0x128>(v);
  const auto p16 = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  v = max((unsigned)p16[0], (unsigned)p16[1]);
  const auto p32 = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return max((unsigned)p32[0], (unsigned)p32[1]);
}
__device__ __forceinline__ void wave_max2_u32_v(unsigned& u, unsigned& v) {
  u = dpp_max_step<0xB1>(u);
  v = dpp_max_step<0xB1>(v);
  u = dpp_max_step<0x4E>(u);
  v = dpp_max_step<0x4E>(v);
  u = dpp_max_step<0x124>(u);
  v = dpp_max_step<0x124>(v);
  u = dpp_max_step<0x128>(u);
  v = dpp_max_step<0x128>(v);
  const auto pu = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  const auto pv = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  u = max((unsigned)pu[0], (unsigned)pu[1]);
  v = max((unsigned)pv[0], (unsigned)pv[1]);
  const auto qu = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  const auto qv = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  u = max((unsigned)qu[0], (unsigned)qu[1]);
  v = max((unsigned)qv[0], (unsigned)qv[1]);
}

__device__ __forceinline__ float order_key_inv(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k ^ 0x80000000u) : ~k);
}

// The SMO iterations of one Q-variable sub-problem, run by ONE wavefront: lane l owns variables
// t = l + 64e; the Q x Q kernel block is in LDS.  Returns the iteration count.
//
// Every VALU instruction of a wave64 costs >= 4 cycles and the loop is one dependent chain, so the
// instruction count IS the iteration time.  The two argmax selections are therefore packed u32
// max reductions: the order-preserving key of the value with its low 7 bits replaced by
// (127 - t) — ties (and values within 2^-16 relative) go to the lowest variable — one DPP chain
// each instead of a (value, index) pair chain; the exact values for the stopping test come from
// the owner lane (i's violation) or from a plain max of exact keys (the low-set maximum).
// A wave-uniform value copied into a VGPR the compiler cannot prove uniform: the two-variable
// update below then compiles to v_cndmask selects instead of ~20 scalar branches per iteration
// (uniform compares of SGPR values become s_cbranch chains otherwise).
__device__ __forceinline__ float as_divergent(float x) {
  float r;
  asm("v_mov_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

template <int E>
__device__ int ws_smo_loop(const float (&Ks)[WS_Q][WS_Q], float (&y)[E], float (&a)[E], float (&g)[E],
                           const float (&qd)[E], float C, float epsl, int max_iter, int lane) {
  static_assert(E * 64 <= 128, "7-bit variable codes");
  auto rdl = [](float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); };
  int it = 0;
  for (; it < max_iter; ++it) {
    unsigned ku = 0u;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      // branch-free set membership (bitwise on the compare masks: no exec-mask branches)
      const bool up = ((y[e] > 0.f) & (a[e] < C)) | ((y[e] < 0.f) & (a[e] > 0.f));
      const unsigned kk = (order_key(-y[e] * g[e]) & ~0x7Fu) | (127u - (unsigned)(lane + 64 * e));
      ku = up ? max(ku, kk) : ku;
    }
    ku = (unsigned)__builtin_amdgcn_readfirstlane((int)wave_max_u32_v(ku));
    if (ku == 0u) break;
    const int i = 127 - (int)(ku & 0x7Fu);
    // i's state from its owner lane (the slot index is wave-uniform)
    const int si = i >> 6;
    float yi = rdl(y[0], i & 63), ai = rdl(a[0], i & 63), gi_ = rdl(g[0], i & 63), Kii = rdl(qd[0], i & 63);
#pragma unroll
    for (int e = 1; e < E; ++e) {
      const float y1 = rdl(y[e], i & 63), a1 = rdl(a[e], i & 63), g1 = rdl(g[e], i & 63), q1 = rdl(qd[e], i & 63);
      yi = e == si ? y1 : yi;
      ai = e == si ? a1 : ai;
      gi_ = e == si ? g1 : gi_;
      Kii = e == si ? q1 : Kii;
    }
    yi = as_divergent(yi);
    ai = as_divergent(ai);
    gi_ = as_divergent(gi_);
    Kii = as_divergent(Kii);
    const float gmax = -yi * gi_;
    unsigned kj = 0u, km = 0u;
    float kit[E];  // row i of the block, kept for K[i][j] (a readlane) and the gradient update
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int t = lane + 64 * e;
      kit[e] = Ks[i][t];
      const bool low = ((y[e] > 0.f) & (a[e] > 0.f)) | ((y[e] < 0.f) & (a[e] < C));
      const float yg = y[e] * g[e];
      const float bd = gmax + yg;
      float q = Kii + qd[e] - 2.f * kit[e];
      q = q > 0.f ? q : TAU;
      // selection only: the hardware reciprocal instead of an IEEE divide; gain >= 0, so its raw
      // bits already order like the value
      const float gain = bd * bd * __builtin_amdgcn_rcpf(q);
      const unsigned kg = (__float_as_uint(gain) & ~0x7Fu) | (127u - (unsigned)t);
      kj = (low && bd > 0.f) ? max(kj, kg) : kj;
      km = low ? max(km, order_key(yg)) : km;
    }
    wave_max2_u32_v(kj, km);
    kj = (unsigned)__builtin_amdgcn_readfirstlane((int)kj);
    const float gmax2 = km ? order_key_inv(km) : -INFINITY;
    if (gmax + gmax2 < epsl || kj == 0u) break;
    const int j = 127 - (int)(kj & 0x7Fu);
    const int sj = j >> 6;
    float yj = rdl(y[0], j & 63), aj = rdl(a[0], j & 63), gj = rdl(g[0], j & 63), Kjj = rdl(qd[0], j & 63);
    float kij = rdl(kit[0], j & 63);  // K[i][j] from the owner lane of the cached row (no LDS round trip)
#pragma unroll
    for (int e = 1; e < E; ++e) {
      const float y1 = rdl(y[e], j & 63), a1 = rdl(a[e], j & 63), g1 = rdl(g[e], j & 63), q1 = rdl(qd[e], j & 63);
      const float k1 = rdl(kit[e], j & 63);
      yj = e == sj ? y1 : yj;
      aj = e == sj ? a1 : aj;
      gj = e == sj ? g1 : gj;
      Kjj = e == sj ? q1 : Kjj;
      kij = e == sj ? k1 : kij;
    }
    yj = as_divergent(yj);
    aj = as_divergent(aj);
    gj = as_divergent(gj);
    Kjj = as_divergent(Kjj);
    kij = as_divergent(kij);
    const float oi = ai, oj = aj;
    float quad = Kii + Kjj - 2.f * kij;
    quad = quad > 0.f ? quad : TAU;
    // num / quad: hardware reciprocal + one residual correction (within an ulp of the IEEE
    // quotient, 4 instructions instead of the 13-instruction divide sequence)
    auto qdiv = [quad](float num) {
      const float r = __builtin_amdgcn_rcpf(quad);
      const float d0 = num * r;
      return fmaf(r, fmaf(-quad, d0, num), d0);
    };
    // LIBSVM's two-variable update and box clipping, both label cases evaluated with selects
    // (wave-uniform values: no branches in the dependent chain)
    const bool opp = yi != yj;
    const float delta = qdiv(opp ? -gi_ - gj : gi_ - gj);
    {
      // opposite labels: ai - aj = diff is kept; same labels: ai + aj = sum is kept
      const float diff = ai - aj, sum = ai + aj;
      float pi = opp ? ai + delta : ai - delta, pj = aj + delta;
      // first clip (conditions combined with bitwise ops: no short-circuit branches)
      const bool dpos = diff > 0.f, spos = sum > C;
      const bool c1 = (opp & dpos & (pj < 0.f)) | (opp & !dpos & (pi < 0.f)) | (!opp & spos & (pi > C)) |
                      (!opp & !spos & (pj < 0.f));
      const float ci = opp ? (dpos ? diff : 0.f) : (spos ? C : sum);
      const float cj = opp ? (dpos ? 0.f : -diff) : (spos ? sum - C : 0.f);
      pi = c1 ? ci : pi;
      pj = c1 ? cj : pj;
      // second clip
      const bool c2 = (opp & dpos & (pi > C)) | (opp & !dpos & (pj > C)) | (!opp & spos & (pj > C)) |
                      (!opp & !spos & (pi < 0.f));
      const float di_ = opp ? (dpos ? C : C + diff) : (spos ? sum - C : 0.f);
      const float dj_ = opp ? (dpos ? C - diff : C) : (spos ? C : sum);
      ai = c2 ? di_ : pi;
      aj = c2 ? dj_ : pj;
    }
    const float di = (ai - oi) * yi, dj = (aj - oj) * yj;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int t = lane + 64 * e;
      if (t == i) a[e] = ai;
      if (t == j) a[e] = aj;
      g[e] += y[e] * (kit[e] * di + Ks[j][t] * dj);
    }
  }
  return it;
}

__global__ __launch_bounds__(64) void smo_ws_kernel(const float* __restrict__ Kall, const float* __restrict__ yall,
                                                    float* __restrict__ aall, const float* __restrict__ gall,
                                                    const float* __restrict__ gap, float C, float eps, int max_iter,
                                                    int* __restrict__ iters) {
  constexpr int Q = WS_Q, E = Q / 64;
  __shared__ __attribute__((aligned(16))) float Ks[Q][Q];
  const int b = blockIdx.x, lane = threadIdx.x;
  const float* Kb = Kall + (long long)b * Q * Q;
  for (int e = lane; e < Q * Q / 4; e += 64)
    reinterpret_cast<float4*>(&Ks[0][0])[e] = reinterpret_cast<const float4*>(Kb)[e];
  float y[E], a[E], g[E], qd[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int t = lane + 64 * e;
    y[e] = yall[b * Q + t];
    a[e] = aall[b * Q + t];
    g[e] = gall[b * Q + t];
  }
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int e = 0; e < E; ++e) qd[e] = Ks[lane + 64 * e][lane + 64 * e];
  const float epsl = fmaxf(eps, 0.1f * gap[b]);
  const int it = ws_smo_loop<E>(Ks, y, a, g, qd, C, epsl, max_iter, lane);
#pragma unroll
  for (int e = 0; e < E; ++e) aall[b * Q + lane + 64 * e] = a[e];
  if (lane == 0) iters[b] = it;
}


// smo_ws_solve_fused_kernel: the sub-problem solve with its gathers and scatters folded in: the
// workgroup's 4 waves gather K[ws, ws] into LDS, wave 0 loads (y, alpha, G) of the working set,
// runs ws_smo_loop, scatters the new alphas, writes dA = (alpha_new - alpha_old) y for the
// gradient update and adds its iteration count to inner_total.
constexpr int SOLVE_T = 1024;  // all 16 waves gather the Q x Q block (memory parallelism), wave 0 solves
__global__ __launch_bounds__(SOLVE_T) void smo_ws_solve_fused_kernel(const float* __restrict__ K, int N,
                                                                 const long long* __restrict__ ws,
                                                                 const bool* __restrict__ ok, float* __restrict__ alpha,
                                                                 const float* __restrict__ G, const float* __restrict__ yv,
                                                                 int ldag, const float* __restrict__ gap, float C,
                                                                 float eps, int max_iter, float* __restrict__ dA,
                                                                 long long* __restrict__ inner_total, long long kbs) {
  constexpr int Q = WS_Q, E = Q / 64;
  __shared__ __attribute__((aligned(16))) float Ks[Q][Q];
  __shared__ long long s_ws[Q];
  __shared__ int s_ok[Q];
  const int b = blockIdx.x, tid = threadIdx.x;
  for (int q = tid; q < Q; q += SOLVE_T) {
    const bool o = ok[(long long)b * Q + q];
    s_ok[q] = o ? 1 : 0;
    s_ws[q] = o ? ws[(long long)b * Q + q] : 0;
  }
  __syncthreads();
  const float* Kb = K + b * kbs;
  // scattered 4-byte gathers from the N x N kernel matrix: 16 per thread, all issued before the
  // LDS stores (latency-bound otherwise)
  constexpr int PER = Q * Q / SOLVE_T;
  float kv[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = tid + i * SOLVE_T;
    kv[i] = Kb[s_ws[e / Q] * N + s_ws[e % Q]];
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = tid + i * SOLVE_T;
    Ks[e / Q][e % Q] = kv[i];
  }
  __syncthreads();
  if (tid >= 64) return;  // wave 0 solves; no block barrier follows
  const int lane = tid;
  float y[E], a[E], g[E], qd[E], a0[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int t = lane + 64 * e;
    const long long n = s_ws[t];
    y[e] = s_ok[t] ? yv[(long long)b * N + n] : 0.f;
    a[e] = alpha[(long long)b * ldag + n];
    g[e] = G[(long long)b * ldag + n];
    a0[e] = a[e];
    qd[e] = Ks[t][t];
  }
  float gp = gap[b];
  if (!isfinite(gp)) gp = 0.f;
  const int it = ws_smo_loop<E>(Ks, y, a, g, qd, C, fmaxf(eps, 0.1f * gp), max_iter, lane);
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int t = lane + 64 * e;
    if (s_ok[t]) alpha[(long long)b * ldag + s_ws[t]] = a[e];
    dA[(long long)b * Q + t] = (a[e] - a0[e]) * y[e];
  }
  if (lane == 0) inner_total[b] += it;
}

// smo_ws_gather_kernel: K[ws, ws] of every problem into a contiguous [B, Q, Q] block, one
// workgroup per (row p, problem): the Q x Q scattered 4-byte reads are spread over Q * B
// workgroups (all CUs) instead of being issued by the one CU that then solves.
__global__ __launch_bounds__(WS_Q) void smo_ws_gather_kernel(const float* __restrict__ K, int N,
                                                             const long long* __restrict__ ws,
                                                             const bool* __restrict__ ok, float* __restrict__ Kws,
                                                             const float* __restrict__ gap, float skip, long long kbs) {
  constexpr int Q = WS_Q;
  const int b = blockIdx.y, p = blockIdx.x, q = threadIdx.x;
  if (ws_done(gap, b, skip)) return;
  const long long* wb = ws + (long long)b * Q;
  const bool* ob = ok + (long long)b * Q;
  const long long rp = ob[p] ? wb[p] : 0, cq = ob[q] ? wb[q] : 0;  // < N (select writes n < N)
  Kws[((long long)b * Q + p) * Q + q] = K[b * kbs + rp * N + cq];
}

// smo_ws_solve_kernel: one wavefront per problem: the gathered Q x Q block into LDS (coalesced
// 16-byte loads), then the sub-problem solve, the alpha scatter, dA and the iteration count.
constexpr int WSS_T = 256;  // 4 waves stage the K block, wave 0 solves
__global__ __launch_bounds__(WSS_T) void smo_ws_solve_kernel(const float* __restrict__ Kws,
                                                          const long long* __restrict__ ws,
                                                          const bool* __restrict__ ok, float* __restrict__ alpha,
                                                          const float* __restrict__ G, const float* __restrict__ yv,
                                                          int N, int ldag, const float* __restrict__ gap, float C,
                                                          float eps, float rel_tol, int max_iter,
                                                          float* __restrict__ dA, long long* __restrict__ inner_total,
                                                          float* __restrict__ gap_out = nullptr) {
  constexpr int Q = WS_Q, E = Q / 64;
  __shared__ __attribute__((aligned(16))) float Ks[Q][Q];
  const int b = blockIdx.x, lane = threadIdx.x;
  // fused merge + gather: ``gap`` is this step's gap (written by the merge), published to the
  // step's ``gap_out`` for the update and the next selection (the merge reads the previous one)
  if (gap_out && threadIdx.x == 0) gap_out[b] = gap[b];
  if (ws_done(gap, b, eps)) {  // converged: zero iterations, alpha unchanged, dA = 0
    for (int t = threadIdx.x; t < Q; t += WSS_T) dA[(long long)b * Q + t] = 0.f;
    return;
  }
  // wave 0's working-set state (dependent ws -> y / alpha / G loads) is issued BEFORE the block
  // staging so that its latency overlaps the copy
  float y[E], a[E], g[E], qd[E], a0[E];
  bool okv[E];
  long long wsv[E];
  if (threadIdx.x < 64) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int t = lane + 64 * e;
      okv[e] = ok[(long long)b * Q + t];
      wsv[e] = okv[e] ? ws[(long long)b * Q + t] : 0;
      y[e] = okv[e] ? yv[(long long)b * N + wsv[e]] : 0.f;
      a[e] = alpha[(long long)b * ldag + wsv[e]];
      g[e] = G[(long long)b * ldag + wsv[e]];
      a0[e] = a[e];
    }
  }
  const float4* src = reinterpret_cast<const float4*>(Kws + (long long)b * Q * Q);
  float4* dst = reinterpret_cast<float4*>(&Ks[0][0]);
#pragma unroll 4
  for (int e = threadIdx.x; e < Q * Q / 4; e += WSS_T) dst[e] = src[e];
  __syncthreads();
  if (threadIdx.x >= 64) return;  // wave 0 solves; no barrier follows
#pragma unroll
  for (int e = 0; e < E; ++e) qd[e] = Ks[lane + 64 * e][lane + 64 * e];
  float gp = gap[b];
  if (!isfinite(gp)) gp = 0.f;
  const int it = ws_smo_loop<E>(Ks, y, a, g, qd, C, fmaxf(eps, rel_tol * gp), max_iter, lane);
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int t = lane + 64 * e;
    if (okv[e]) alpha[(long long)b * ldag + wsv[e]] = a[e];
    dA[(long long)b * Q + t] = (a[e] - a0[e]) * y[e];
  }
  if (lane == 0) inner_total[b] += it;
}

// ---------------------------------------------------------------------------------------------
// Working-set selection and gradient update for smo_decomposition, one launch each per outer
// step (they replace ~25 small torch ops: the violation values, two top-k sorts, the
// duplicate mask, the [B, Q, N] row gather and the batched GEMV).
//
// smo_ws_select_kernel: one 1024-thread workgroup per problem.  The "up" / "low" violation
// values are computed from (alpha, G, y) once into registers (N <= 16384; else every pass re-reads
// them from L2); the gap is
// max(up) + max(low); the h largest of each set are found by an exact 4-pass 8-bit radix select
// on order-preserving float keys (LDS histogram), collected with LDS counters, and written in
// ascending index order (deterministic working sets).  A low-set index already in the up set is
// masked out (ok = 0), as in the torch path.
// smo_ws_update_kernel: G[n] += y[n] * sum_q dA[q] K[ws[q], n], one thread per n, the Q
// (index, dA) pairs in LDS, K rows read coalesced.
// ---------------------------------------------------------------------------------------------
constexpr int SEL_T = 1024;

__device__ __forceinline__ float ws_violation(int which, float y, float a, float g, float C) {
  if (which == 0) {
    const bool up = y > 0.f ? a < C : (y < 0.f && a > 0.f);
    return up ? -y * g : -INFINITY;
  }
  const bool low = y > 0.f ? a > 0.f : (y < 0.f && a < C);
  return low ? y * g : -INFINITY;
}



template <typename T, typename Op>
__device__ T block_reduce(T v, T* red, Op op) {  // all SEL_T threads; red has >= 17 slots
  constexpr int NW = SEL_T / 64;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = op(v, __shfl_xor(v, o, 64));
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    T r = red[0];
    for (int i = 1; i < NW; ++i) r = op(r, red[i]);
    red[NW] = r;
  }
  __syncthreads();
  const T r = red[NW];
  __syncthreads();
  return r;
}

// PER > 0: every thread caches the up / low violations of its PER rows in registers once, and the
// 13 passes of the selection (max, counts, 4 radix digits, ties, for both sides) read registers
// instead of re-reading alpha / G / y from global memory each pass (latency-bound at one
// workgroup).  PER = 0: no cache (any N).
template <int PER>
__global__ __launch_bounds__(SEL_T) void smo_ws_select_kernel(const float* __restrict__ alpha,
                                                              const float* __restrict__ G,
                                                              const float* __restrict__ y, int N, int ldag, float C,
                                                              int h, long long* __restrict__ ws,
                                                              bool* __restrict__ ok, float* __restrict__ gap,
                                                              float skip) {
  extern __shared__ unsigned in_up[];  // [(N + 31) / 32] bitmap of the selected up set
  __shared__ unsigned hist[256];
  __shared__ float redf[17];
  __shared__ unsigned redu[17];
  __shared__ unsigned s_prefix, s_mask, s_krem, s_gt;
  __shared__ int pick[2][64];
  __shared__ unsigned wcnt[PER > 0 ? PER : 1][SEL_T / 64];
  const int b = blockIdx.x, tid = threadIdx.x;
  if (ws_done(gap, b, skip)) return;
  const float* ab = alpha + (long long)b * ldag;
  const float* gb = G + (long long)b * ldag;
  const float* yb = y + (long long)b * N;
  const int words = (N + 31) / 32;
  for (int i = tid; i < words; i += SEL_T) in_up[i] = 0;
  float cu[PER > 0 ? PER : 1], cl[PER > 0 ? PER : 1];
  if constexpr (PER > 0) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int n = tid + i * SEL_T;
      cu[i] = n < N ? ws_violation(0, yb[n], ab[n], gb[n], C) : -INFINITY;
      cl[i] = n < N ? ws_violation(1, yb[n], ab[n], gb[n], C) : -INFINITY;
    }
  }
  // violation of row n = tid + i * SEL_T on side `which`
  auto viol = [&](int which, int i, int n) -> float {
    if constexpr (PER > 0) {
      float v = -INFINITY;
#pragma unroll
      for (int j = 0; j < PER; ++j)
        if (j == i) v = which ? cl[j] : cu[j];
      return v;
    } else {
      return ws_violation(which, yb[n], ab[n], gb[n], C);
    }
  };

  float mu = -INFINITY, ml = -INFINITY;
  for (int i = 0, n = tid; n < N; ++i, n += SEL_T) {
    mu = fmaxf(mu, viol(0, i, n));
    ml = fmaxf(ml, viol(1, i, n));
  }
  auto fmax_op = [](float p, float q) { return fmaxf(p, q); };
  auto add_op = [](unsigned p, unsigned q) { return p + q; };
  mu = block_reduce(mu, redf, fmax_op);
  ml = block_reduce(ml, redf, fmax_op);
  if (tid == 0) gap[b] = mu + ml;

  int npick[2] = {0, 0};
  for (int which = 0; which < 2; ++which) {
    unsigned e = 0;
    for (int i = 0, n = tid; n < N; ++i, n += SEL_T) e += viol(which, i, n) > -INFINITY ? 1u : 0u;
    e = block_reduce(e, redu, add_op);
    const unsigned k = e < (unsigned)h ? e : (unsigned)h;
    npick[which] = (int)k;
    if (k == 0) continue;  // block-uniform
    if (tid == 0) { s_prefix = 0; s_mask = 0; s_krem = k; }
    for (int d = 3; d >= 0; --d) {
      if (tid < 256) hist[tid] = 0;
      __syncthreads();
      const unsigned prefix = s_prefix, mask = s_mask;
      for (int i = 0, n0 = 0; n0 < N; ++i, n0 += SEL_T) {
        const int n = n0 + tid;
        bool act = false;
        unsigned dg = 0;
        if (n < N) {
          const float v = viol(which, i, n);
          if (v > -INFINITY) {
            const unsigned key = order_key(v);
            act = (key & mask) == prefix;
            dg = (key >> (8 * d)) & 255u;
          }
        }
        // leader aggregation: the lanes sharing the first active lane's digit add with ONE atomic
        // (ties are the common case — every violator ties on the first outer step — and
        // same-address LDS atomics serialise)
        const unsigned long long am = __ballot(act);
        if (am) {
          const int lead = __ffsll((long long)am) - 1;
          const unsigned d0 = (unsigned)__builtin_amdgcn_readlane((int)dg, lead);
          const unsigned long long same = __ballot(act && dg == d0);
          if ((tid & 63) == lead) atomicAdd(&hist[d0], (unsigned)__popcll(same));
          else if (act && dg != d0) atomicAdd(&hist[dg], 1u);
        }
      }
      __syncthreads();
      if (tid < 64) {  // the digit holding the krem-th largest key: one wave scans the 256 bins
        const int l = tid;
        unsigned c[4], sum = 0;
#pragma unroll
        for (int t = 0; t < 4; ++t) {  // lane l holds digits 255 - 4l .. 252 - 4l (descending)
          c[t] = hist[255 - (4 * l + t)];
          sum += c[t];
        }
        unsigned inc = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const unsigned y = __shfl_up(inc, o, 64);
          if (l >= o) inc += y;
        }
        const unsigned krem = s_krem, excl = inc - sum;
        if (excl < krem && krem <= inc) {  // exactly one lane
          unsigned cum = excl;
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            if (cum + c[t] >= krem) {
              const unsigned dg = 255u - (unsigned)(4 * l + t);
              s_prefix = prefix | (dg << (8 * d));
              s_mask = mask | (255u << (8 * d));
              s_krem = krem - cum;
              break;
            }
            cum += c[t];
          }
        }
        if (l == 0) s_gt = 0;
      }
      __syncthreads();
    }
    const unsigned T = s_prefix, krem = s_krem, ngt = k - krem;  // keys > T: exactly ngt of them
    // keys > T are all taken (their slots are re-sorted by index below); among the keys == T the
    // krem SMALLEST indices are taken: the rows are walked in index order, SEL_T at a time, and a
    // block prefix count of the ties (wave ballots + per-wave totals) ranks each tie — the working
    // set no longer depends on the order of LDS atomics (first outer step: every violator ties).
    unsigned eq_base = 0;  // ties seen in earlier SEL_T blocks (block-uniform)
    const int lane = tid & 63, wv = tid >> 6;
    const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
    if constexpr (PER > 0) {
      // register-cached rows: all PER chunks' tie ballots at once, ONE barrier for the per-(chunk,
      // wave) counts, then every tie ranks itself (index order = chunk-major, then thread)
      unsigned long long bal[PER];
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int n = i * SEL_T + tid;
        bool eq = false;
        if (n < N) {
          const float v = viol(which, i, n);
          if (v > -INFINITY) {
            const unsigned key = order_key(v);
            if (key > T) pick[which][atomicAdd(&s_gt, 1u)] = n;
            eq = key == T;
          }
        }
        bal[i] = __ballot(eq);
        if (lane == 0) wcnt[i][wv] = (unsigned)__popcll(bal[i]);
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        unsigned before = eq_base, tot = 0;
        for (int w = 0; w < SEL_T / 64; ++w) {
          const unsigned c = wcnt[i][w];
          if (w < wv) before += c;
          tot += c;
        }
        if ((bal[i] >> lane) & 1ull) {
          const unsigned r = before + (unsigned)__popcll(bal[i] & below);
          if (r < krem) pick[which][ngt + r] = i * SEL_T + tid;
        }
        eq_base += tot;
      }
    }
    for (int n0 = 0, i = 0; PER == 0 && n0 < N; n0 += SEL_T, ++i) {
      const int n = n0 + tid;
      bool eq = false;
      if (n < N) {
        const float v = viol(which, i, n);
        if (v > -INFINITY) {
          const unsigned key = order_key(v);
          if (key > T) pick[which][atomicAdd(&s_gt, 1u)] = n;
          eq = key == T;
        }
      }
      const unsigned long long bal = __ballot(eq);
      if (lane == 0) redu[wv] = (unsigned)__popcll(bal);
      __syncthreads();
      unsigned before = eq_base, tot = 0;
      for (int w = 0; w < SEL_T / 64; ++w) {
        if (w < wv) before += redu[w];
        tot += redu[w];
      }
      if (eq) {
        const unsigned r = before + (unsigned)__popcll(bal & below);
        if (r < krem) pick[which][ngt + r] = n;
      }
      eq_base += tot;
      __syncthreads();  // redu is rewritten by the next block of rows
    }
    __syncthreads();
    if (which == 0 && tid < (int)k) atomicOr(&in_up[pick[0][tid] >> 5], 1u << (pick[0][tid] & 31));
    __syncthreads();
  }
  // ascending index order within each half; unused slots -> (0, not ok)
  if (tid < 2 * h) {
    const int which = tid / h, slot = tid % h, np = npick[which];
    long long* wsb = ws + (long long)b * 2 * h + which * h;
    bool* okb = ok + (long long)b * 2 * h + which * h;
    if (slot < np) {
      const int n = pick[which][slot];
      int rank = 0;
      for (int j = 0; j < np; ++j) rank += pick[which][j] < n ? 1 : 0;
      wsb[rank] = n;
      okb[rank] = which == 0 || !((in_up[n >> 5] >> (n & 31)) & 1u);
    } else {
      wsb[slot] = 0;
      okb[slot] = false;
    }
  }
}

// Register-cached selection with both sides (up / low) selected TOGETHER: one combined reduction
// for the two maxima and the two candidate counts, then every radix digit pass builds the two
// 256-bin histograms in the same sweep and two waves scan them in parallel, and the tie ranking of
// both sides shares one barrier — 12 barriers per launch instead of ~40 (the selection is
// latency-bound at one workgroup).  Same working set as smo_ws_select_kernel.
//
// Element sources (position pos = i * SEL_T + tid, positions ascend with the row index, so tie
// ranking by position = by index):
//   RangeSrc — rows [n0, n1) of the problem (single level, or one part of a two-level selection);
//   CandSrc  — the parts' local top-h candidates concatenated in part order (second level).
// Two-level selection (N > 4096): each part of 2048 / 4096 / 8192 rows (the smallest whose
// candidates fit one workgroup) keeps its local top h per side (the global top h, ties to the
// lowest index, is contained in the union), then ONE workgroup of 256..1024 threads selects over
// the parts x h candidates — the parts run on different CUs with 2..8 register rows per thread.
struct RangeSrc {
  int n0, n1;
  __device__ int row(int, int pos) const { const int n = n0 + pos; return n < n1 ? n : -1; }
};
struct CandSrc {
  const int* cand;  // [parts][2][h] local picks (ascending row index), this problem
  const int* cnt;   // [parts][2]
  int parts, h;
  __device__ int row(int w, int pos) const {
    for (int q = 0; q < parts; ++q) {
      const int c = cnt[q * 2 + w];
      if (pos < c) return cand[(q * 2 + w) * h + pos];
      pos -= c;
    }
    return -1;
  }
};

template <int PER, bool PARTIAL, int NT, class Src>
__device__ void ws_select2_body(const Src& src, const float* __restrict__ ab, const float* __restrict__ gb,
                                const float* __restrict__ yb, int N, float C, int h, long long* __restrict__ wsb,
                                bool* __restrict__ okb, float* __restrict__ gapb, int* __restrict__ cand_out,
                                int* __restrict__ cnt_out, unsigned* in_up, float* __restrict__ candv_out = nullptr) {
  __shared__ unsigned hist[2][256];
  __shared__ float redf[2][NT / 64];
  __shared__ unsigned redu[2][NT / 64];
  __shared__ unsigned s_prefix[2], s_mask[2], s_krem[2], s_gt[2];
  __shared__ int pick[2][64];
  __shared__ float pickv[2][64];  // the picks' violation values (PARTIAL: handed to the merge)
  __shared__ unsigned wcnt[2][PER][NT / 64];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (!PARTIAL)
    for (int i = tid; i < (N + 31) / 32; i += NT) in_up[i] = 0;
  float cv[2][PER];
  int rid[2][PER];  // row of each register slot (the candidate source is walked once)
#pragma unroll
  for (int w = 0; w < 2; ++w)
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int n = src.row(w, i * NT + tid);
      rid[w][i] = n;
      cv[w][i] = n >= 0 ? ws_violation(w, yb[n], ab[n], gb[n], C) : -INFINITY;
    }
  // ---- maxima and candidate counts of both sides: one barrier ---------------------------------
  float m[2] = {-INFINITY, -INFINITY};
  unsigned e[2] = {0u, 0u};
#pragma unroll
  for (int w = 0; w < 2; ++w)
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      m[w] = fmaxf(m[w], cv[w][i]);
      e[w] += cv[w][i] > -INFINITY ? 1u : 0u;
    }
#pragma unroll
  for (int w = 0; w < 2; ++w) {
    for (int o = 32; o > 0; o >>= 1) {
      m[w] = fmaxf(m[w], __shfl_xor(m[w], o, 64));
      e[w] += __shfl_xor(e[w], o, 64);
    }
    if (lane == 0) { redf[w][wv] = m[w]; redu[w][wv] = e[w]; }
  }
  if (tid < 2) { s_prefix[tid] = 0; s_mask[tid] = 0; }
  __syncthreads();
  unsigned k[2];
#pragma unroll
  for (int w = 0; w < 2; ++w) {
    float mm = -INFINITY;
    unsigned ee = 0;
    for (int q = 0; q < NT / 64; ++q) { mm = fmaxf(mm, redf[w][q]); ee += redu[w][q]; }
    m[w] = mm;
    k[w] = ee < (unsigned)h ? ee : (unsigned)h;
  }
  if (!PARTIAL && tid == 0) *gapb = m[0] + m[1];
  if (tid < 2) s_krem[tid] = k[tid];
  // ---- 4 radix digit passes, both sides per pass ------------------------------------------------
  for (int d = 3; d >= 0; --d) {
    for (int q = tid; q < 512; q += NT) hist[q >> 8][q & 255] = 0;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < 2; ++w) {
      if (k[w] == 0) continue;  // block-uniform
      const unsigned prefix = s_prefix[w], mask = s_mask[w];
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const float v = cv[w][i];
        bool act = false;
        unsigned dg = 0;
        if (v > -INFINITY) {
          const unsigned key = order_key(v);
          act = (key & mask) == prefix;
          dg = (key >> (8 * d)) & 255u;
        }
        const unsigned long long am = __ballot(act);
        if (am) {
          const int lead = __ffsll((long long)am) - 1;
          const unsigned d0 = (unsigned)__builtin_amdgcn_readlane((int)dg, lead);
          const unsigned long long same = __ballot(act && dg == d0);
          if (lane == lead) atomicAdd(&hist[w][d0], (unsigned)__popcll(same));
          else if (act && dg != d0) atomicAdd(&hist[w][dg], 1u);
        }
      }
    }
    __syncthreads();
    if (wv < 2 && k[wv] > 0) {  // wave w scans side w's 256 bins
      const int w = wv, l = lane;
      const unsigned prefix = s_prefix[w], mask = s_mask[w];
      unsigned c[4], sum = 0;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        c[t] = hist[w][255 - (4 * l + t)];
        sum += c[t];
      }
      unsigned inc = sum;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned yv = __shfl_up(inc, o, 64);
        if (l >= o) inc += yv;
      }
      const unsigned krem = s_krem[w], excl = inc - sum;
      if (excl < krem && krem <= inc) {
        unsigned cum = excl;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if (cum + c[t] >= krem) {
            const unsigned dg = 255u - (unsigned)(4 * l + t);
            s_prefix[w] = prefix | (dg << (8 * d));
            s_mask[w] = mask | (255u << (8 * d));
            s_krem[w] = krem - cum;
            break;
          }
          cum += c[t];
        }
      }
      if (l == 0) s_gt[w] = 0;
    }
    __syncthreads();
  }
  // ---- keys above the threshold, and ties by ascending position, both sides: one barrier -------
  const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
  // tie flags are recomputed in the ranking pass (cheap) rather than kept in registers
  auto is_tie = [&](int w, int i) -> bool {
    return k[w] > 0 && cv[w][i] > -INFINITY && order_key(cv[w][i]) == s_prefix[w];
  };
#pragma unroll
  for (int w = 0; w < 2; ++w) {
    const unsigned T = s_prefix[w];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      if (k[w] > 0 && cv[w][i] > -INFINITY && order_key(cv[w][i]) > T) {
        const unsigned slot = atomicAdd(&s_gt[w], 1u);
        pick[w][slot] = rid[w][i];
        pickv[w][slot] = cv[w][i];
      }
      const unsigned long long bal = __ballot(is_tie(w, i));
      if (lane == 0) wcnt[w][i][wv] = (unsigned)__popcll(bal);
    }
  }
  __syncthreads();
#pragma unroll
  for (int w = 0; w < 2; ++w) {
    const unsigned krem = s_krem[w], ngt = k[w] - krem;
    unsigned eq_base = 0;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      unsigned before = eq_base, tot = 0;
      for (int q = 0; q < NT / 64; ++q) {
        const unsigned c = wcnt[w][i][q];
        if (q < wv) before += c;
        tot += c;
      }
      const bool tie = is_tie(w, i);
      const unsigned long long bal = __ballot(tie);
      if (tie) {
        const unsigned r = before + (unsigned)__popcll(bal & below);
        if (r < krem) {
          pick[w][ngt + r] = rid[w][i];
          pickv[w][ngt + r] = cv[w][i];
        }
      }
      eq_base += tot;
    }
  }
  __syncthreads();
  if (PARTIAL) {
    // local picks in ascending row order + counts (the second level concatenates the parts)
    if (tid < 2 * h) {
      const int which = tid / h, slot = tid % h, np = (int)k[which];
      if (slot < np) {
        const int n = pick[which][slot];
        int rank = 0;
        for (int j = 0; j < np; ++j) rank += pick[which][j] < n ? 1 : 0;
        cand_out[which * h + rank] = n;
        if (candv_out) candv_out[which * h + rank] = pickv[which][slot];
      }
    }
    if (tid < 2) cnt_out[tid] = (int)k[tid];
    return;
  }
  if (tid < (int)k[0]) atomicOr(&in_up[pick[0][tid] >> 5], 1u << (pick[0][tid] & 31));
  __syncthreads();
  if (tid < 2 * h) {
    const int which = tid / h, slot = tid % h, np = (int)k[which];
    long long* wsw = wsb + which * h;
    bool* okw = okb + which * h;
    if (slot < np) {
      const int n = pick[which][slot];
      int rank = 0;
      for (int j = 0; j < np; ++j) rank += pick[which][j] < n ? 1 : 0;
      wsw[rank] = n;
      okw[rank] = which == 0 || !((in_up[n >> 5] >> (n & 31)) & 1u);
    } else {
      wsw[slot] = 0;
      okw[slot] = false;
    }
  }
}

// single level: one workgroup per problem over all N rows
template <int PER>
__global__ __launch_bounds__(SEL_T) void smo_ws_select2_kernel(const float* __restrict__ alpha,
                                                               const float* __restrict__ G,
                                                               const float* __restrict__ y, int N, int ldag, float C,
                                                               int h, long long* __restrict__ ws,
                                                               bool* __restrict__ ok, float* __restrict__ gap,
                                                               float skip) {
  extern __shared__ unsigned in_up[];
  const int b = blockIdx.x;
  if (ws_done(gap, b, skip)) return;
  ws_select2_body<PER, false, SEL_T>(RangeSrc{0, N}, alpha + (long long)b * ldag, G + (long long)b * ldag,
                                     y + (long long)b * N, N, C, h, ws + (long long)b * 2 * h,
                                     ok + (long long)b * 2 * h, gap + b, nullptr, nullptr, in_up);
}

// two levels: part p of problem b = rows [p * chunk, (p + 1) * chunk), chunk = PER * SEL_T
template <int PER>
__global__ __launch_bounds__(SEL_T) void smo_ws_select_part_kernel(const float* __restrict__ alpha,
                                                                   const float* __restrict__ G,
                                                                   const float* __restrict__ y, int N, int ldag,
                                                                   float C, int h, int parts, int* __restrict__ cand,
                                                                   int* __restrict__ cnt, float* __restrict__ candv,
                                                                   const float* __restrict__ gap, float skip) {
  const int b = blockIdx.y, p = blockIdx.x;
  if (ws_done(gap, b, skip)) return;
  const int n0 = p * PER * SEL_T, n1 = min(N, n0 + PER * SEL_T);
  ws_select2_body<PER, true, SEL_T>(RangeSrc{n0, n1}, alpha + (long long)b * ldag, G + (long long)b * ldag,
                                    y + (long long)b * N, N, C, h, nullptr, nullptr, nullptr,
                                    cand + ((long long)b * parts + p) * 2 * h, cnt + ((long long)b * parts + p) * 2,
                                    nullptr, candv + ((long long)b * parts + p) * 2 * h);
}

// merge: one workgroup of NT >= parts * h threads over the concatenated candidates
template <int NT>
__global__ __launch_bounds__(NT) void smo_ws_select_merge_kernel(const float* __restrict__ alpha,
                                                                 const float* __restrict__ G,
                                                                 const float* __restrict__ y, int N, int ldag, float C,
                                                                 int h, int parts, const int* __restrict__ cand,
                                                                 const int* __restrict__ cnt,
                                                                 long long* __restrict__ ws, bool* __restrict__ ok,
                                                                 float* __restrict__ gap, float skip) {
  extern __shared__ unsigned in_up[];
  const int b = blockIdx.x;
  if (ws_done(gap, b, skip)) return;  // every thread reads gap[b] before thread 0 rewrites it (after a barrier)
  const CandSrc src{cand + (long long)b * parts * 2 * h, cnt + (long long)b * parts * 2, parts, h};
  ws_select2_body<1, false, NT>(src, alpha + (long long)b * ldag, G + (long long)b * ldag, y + (long long)b * N, N, C,
                                h, ws + (long long)b * 2 * h, ok + (long long)b * 2 * h, gap + b, nullptr, nullptr,
                                in_up);
}

// Wave max of u64 keys: the u32 DPP steps of wave_max_u32 on both halves (the pair compared as
// one 64-bit value), the 4 row results over v_readlane; two independent maxima interleaved.
template <int CTRL>
__device__ __forceinline__ unsigned long long dpp_max64_step(unsigned long long v) {
  const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)v, CTRL, 0xF, 0xF, true);
  const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(v >> 32), CTRL, 0xF, 0xF, true);
  const unsigned long long o = ((unsigned long long)hi << 32) | lo;
  return o > v ? o : v;
}
__device__ __forceinline__ unsigned long long readlane64(unsigned long long v, int l) {
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), l);
  return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ void wave_max2_u64(unsigned long long& u, unsigned long long& v) {
  u = dpp_max64_step<0xB1>(u);
  v = dpp_max64_step<0xB1>(v);
  u = dpp_max64_step<0x4E>(u);
  v = dpp_max64_step<0x4E>(v);
  u = dpp_max64_step<0x124>(u);
  v = dpp_max64_step<0x124>(v);
  u = dpp_max64_step<0x128>(u);
  v = dpp_max64_step<0x128>(v);
  auto m4 = [](unsigned long long x) {
    const unsigned long long a = readlane64(x, 0), b = readlane64(x, 16), c = readlane64(x, 32), d = readlane64(x, 48);
    const unsigned long long ab = a > b ? a : b, cd = c > d ? c : d;
    return ab > cd ? ab : cd;
  };
  u = m4(u);
  v = m4(v);
}

__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
  v = dpp_max64_step<0xB1>(v);
  v = dpp_max64_step<0x4E>(v);
  v = dpp_max64_step<0x124>(v);
  v = dpp_max64_step<0x128>(v);
  const unsigned long long a = readlane64(v, 0), b = readlane64(v, 16), c = readlane64(v, 32), d = readlane64(v, 48);
  const unsigned long long ab = a > b ? a : b, cd = c > d ? c : d;
  return ab > cd ? ab : cd;
}

// Register top-k part selection (two-level selection, first level): part p of problem b owns the
// 64-row blocks p, p + parts, p + 2 parts, .. (block-cyclic: rows of one label or one cluster that
// sit together in the input are spread over the parts), PER blocks per wave.  Every candidate is
// one exact 64-bit key (order_key(violation) << 32 | ~row: larger = more violating, ties to the
// lower row — the order of the radix selection and of the rank merge), so the selection is exact
// and deterministic.  Each wave keeps its HW (<= 4) largest keys per side by HW wave-max steps (the
// owner lane clears the winner), then waves 0 and 1 take the HP largest of the 16 waves' candidates
// of side 0 / 1.  No radix passes and 2 barriers, against 12 for ws_select2_body.  The part's HP
// candidates per side go to the rank merge; the global top h is exact whenever no part holds more
// than HP of them and no 64-row block more than HW (the host sizes HP to 2-4x a part's expected
// share of h; a block's expected share is 64 h / N < 1 here; beyond that the working set is a
// slightly different set of strong violators — any violating set keeps SMO convergent).
template <int PER, int HP, int HW = (HP < 4 ? HP : 4)>
__global__ __launch_bounds__(SEL_T) void smo_ws_topk_part_kernel(const float* __restrict__ alpha,
                                                                 const float* __restrict__ G,
                                                                 const float* __restrict__ y, int N, int ldag, float C,
                                                                 int parts, int* __restrict__ cand,
                                                                 int* __restrict__ cnt, float* __restrict__ candv,
                                                                 const float* __restrict__ gap, float skip) {
  // each wave keeps its HW largest keys per side (a 64-row block holds ~64 h / N of the global
  // top h: far below HW = 4 at N > 4096), the workgroup the HP largest of those 16 x HW
  static_assert(HP >= 4 && HP <= 64 && HW >= 1 && HW <= HP && (16 * HW) % 64 == 0, "HP / HW");
  constexpr int NW = SEL_T / 64, R = NW * HW / 64;
  __shared__ unsigned long long s_k[2][NW * HW];
  const int b = blockIdx.y, p = blockIdx.x;
  if (ws_done(gap, b, skip)) return;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const float* ab = alpha + (long long)b * ldag;
  const float* gb = G + (long long)b * ldag;
  const float* yb = y + (long long)b * N;
  unsigned long long key[2][PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const long long blk = (long long)(j * NW + wv) * parts + p;
    const long long n = blk * 64 + lane;
    key[0][j] = key[1][j] = 0ull;
    if (n < N) {
      const float yn = yb[n], an = ab[n], gn = gb[n];
#pragma unroll
      for (int w = 0; w < 2; ++w) {
        const float v = ws_violation(w, yn, an, gn, C);
        if (v > -INFINITY) key[w][j] = ((unsigned long long)order_key(v) << 32) | (unsigned)~(unsigned)n;
      }
    }
  }
  for (int it = 0; it < HW; ++it) {  // the wave's HW largest per side
    unsigned long long m0 = key[0][0], m1 = key[1][0];
#pragma unroll
    for (int j = 1; j < PER; ++j) {
      m0 = key[0][j] > m0 ? key[0][j] : m0;
      m1 = key[1][j] > m1 ? key[1][j] : m1;
    }
    wave_max2_u64(m0, m1);
#pragma unroll
    for (int j = 0; j < PER; ++j) {  // keys are unique (distinct rows); 0 = empty stays 0
      if (key[0][j] == m0) key[0][j] = 0ull;
      if (key[1][j] == m1) key[1][j] = 0ull;
    }
    if (lane == 0) {
      s_k[0][wv * HW + it] = m0;
      s_k[1][wv * HW + it] = m1;
    }
  }
  __syncthreads();
  if (wv >= 2) return;
  const int w = wv;
  unsigned long long c[R];
#pragma unroll
  for (int r = 0; r < R; ++r) c[r] = s_k[w][lane * R + r];
  int* cb = cand + ((long long)b * parts + p) * 2 * HP + w * HP;
  float* vb = candv + ((long long)b * parts + p) * 2 * HP + w * HP;
  int np = 0;
  for (int it = 0; it < HP; ++it) {
    unsigned long long m = c[0];
#pragma unroll
    for (int r = 1; r < R; ++r) m = c[r] > m ? c[r] : m;
    m = wave_max_u64(m);
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (c[r] == m) c[r] = 0ull;
    if (m == 0ull) break;  // wave-uniform: no further candidates
    if (lane == 0) {
      cb[it] = (int)~(unsigned)m;
      vb[it] = order_key_inv((unsigned)(m >> 32));
    }
    ++np;
  }
  if (lane == 0) cnt[((long long)b * parts + p) * 2 + w] = np;
}

// Streaming top-k part selection for large N (no row cap): the first level of the two-level
// selection when N is too large for register-resident blocks (select_part_per(N) == 0, N > 2^17).
// Part p of problem b owns the 64-row blocks p, p + parts, .. (block-cyclic as above), ``per``
// blocks per wave, walked in chunks of 4 blocks whose alpha / G / y loads are issued together
// (12 loads in flight per lane).  Every lane keeps its own 4 largest keys per side in a sorted
// register list (compare-swap insertion), so the wave's 4 largest per side are exact for ANY per
// (they can all sit in one lane); then waves 0 / 1 take the HP largest of the 16 waves' 4
// candidates, as in smo_ws_topk_part_kernel.  The host picks per so that parts <= 64 and
// parts x HP <= 256 (the 512-thread rank merge).
template <int HP>
__global__ __launch_bounds__(SEL_T) void smo_ws_topk_stream_kernel(const float* __restrict__ alpha,
                                                                   const float* __restrict__ G,
                                                                   const float* __restrict__ y, int N, int ldag,
                                                                   float C, int parts, int per,
                                                                   int* __restrict__ cand, int* __restrict__ cnt,
                                                                   float* __restrict__ candv,
                                                                   const float* __restrict__ gap, float skip) {
  constexpr int NW = SEL_T / 64, HW = 4, CH = 4;
  static_assert(HP >= 4 && HP <= 64, "HP");
  __shared__ unsigned long long s_k[2][NW * HW];
  const int b = blockIdx.y, p = blockIdx.x;
  if (ws_done(gap, b, skip)) return;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const float* ab = alpha + (long long)b * ldag;
  const float* gb = G + (long long)b * ldag;
  const float* yb = y + (long long)b * N;
  unsigned long long top[2][HW];
#pragma unroll
  for (int i = 0; i < HW; ++i) top[0][i] = top[1][i] = 0ull;
  for (int j0 = 0; j0 < per; j0 += CH) {
    float yv[CH], av[CH], gv[CH];
    long long nv[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const long long blk = (long long)((j0 + c) * NW + wv) * parts + p;
      nv[c] = blk * 64 + lane;
      const bool in = j0 + c < per && nv[c] < N;
      yv[c] = in ? yb[nv[c]] : 0.f;
      av[c] = in ? ab[nv[c]] : 0.f;
      gv[c] = in ? gb[nv[c]] : 0.f;
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) {
#pragma unroll
      for (int w = 0; w < 2; ++w) {
        const float v = yv[c] != 0.f ? ws_violation(w, yv[c], av[c], gv[c], C) : -INFINITY;
        unsigned long long k = v > -INFINITY ? ((unsigned long long)order_key(v) << 32) | (unsigned)~(unsigned)nv[c] : 0ull;
#pragma unroll
        for (int i = 0; i < HW; ++i) {  // sorted descending: bubble k into place
          const unsigned long long t = top[w][i];
          const bool gt = k > t;
          top[w][i] = gt ? k : t;
          k = gt ? t : k;
        }
      }
    }
  }
  for (int it = 0; it < HW; ++it) {  // the wave's HW largest per side: pop the lane heads
    unsigned long long m0 = top[0][0], m1 = top[1][0];
    wave_max2_u64(m0, m1);
#pragma unroll
    for (int w = 0; w < 2; ++w) {
      const unsigned long long m = w ? m1 : m0;
      if (m != 0ull && top[w][0] == m) {
#pragma unroll
        for (int i = 0; i + 1 < HW; ++i) top[w][i] = top[w][i + 1];
        top[w][HW - 1] = 0ull;
      }
    }
    if (lane == 0) {
      s_k[0][wv * HW + it] = m0;
      s_k[1][wv * HW + it] = m1;
    }
  }
  __syncthreads();
  if (wv >= 2) return;
  const int w = wv;
  unsigned long long c0 = s_k[w][lane];  // NW * HW = 64 candidates: one per lane
  int* cb = cand + ((long long)b * parts + p) * 2 * HP + w * HP;
  float* vb = candv + ((long long)b * parts + p) * 2 * HP + w * HP;
  int np = 0;
  for (int it = 0; it < HP; ++it) {
    const unsigned long long m = wave_max_u64(c0);
    if (c0 == m) c0 = 0ull;
    if (m == 0ull) break;  // wave-uniform
    if (lane == 0) {
      cb[it] = (int)~(unsigned)m;
      vb[it] = order_key_inv((unsigned)(m >> 32));
    }
    ++np;
  }
  if (lane == 0) cnt[((long long)b * parts + p) * 2 + w] = np;
}

// Rank merge of the parts' candidates (replaces the radix merge for the two-level path): the
// parts hand over (row, violation) pairs, so every candidate's 64-bit key (order_key(v) << 32 |
// ~row: larger = more violating, ties to the lower row — the same order as the radix selection)
// is known without touching alpha / G again.  Thread t ranks candidate t % M of side t / M by
// counting the larger keys of its side (two keys per 16-byte LDS broadcast read, no barriers
// inside); rank < h is selected, the selected rows are put in ascending order by a 64-entry count,
// and the low side's rows already chosen on the up side are marked unused.  3 barriers instead of
// ~14.  NT = 2M threads (M = parts x h candidate slots per side, <= 512).
template <int NT>
__global__ __launch_bounds__(NT) void smo_ws_merge_rank_kernel(int h, int hp, int hs, int parts, const int* __restrict__ cand,
                                                               const int* __restrict__ cnt,
                                                               const float* __restrict__ candv,
                                                               long long* __restrict__ ws, bool* __restrict__ ok,
                                                               float* __restrict__ gap, float skip) {
  constexpr int M = NT / 2;
  __shared__ __attribute__((aligned(16))) unsigned long long key[2][M];
  __shared__ int sel[2][64];
  __shared__ float s_max[2];
  __shared__ int s_cnt[2];
  const int b = blockIdx.x, tid = threadIdx.x;
  if (ws_done(gap, b, skip)) return;
  const int w = tid / M, c = tid % M;
  const int* cb = cand + (long long)b * parts * 2 * hs;
  const float* vb = candv + (long long)b * parts * 2 * hs;
  const int* nb = cnt + (long long)b * parts * 2;
  int row = -1;
  float val = -INFINITY;
  if (c < parts * hp) {  // part q's slot s (hp slots used of the stride hs)
    const int q = c / hp, s = c % hp;
    if (s < nb[q * 2 + w]) {
      row = cb[(q * 2 + w) * hs + s];
      val = vb[(q * 2 + w) * hs + s];
    }
  }
  const unsigned long long mk = row >= 0 ? ((unsigned long long)order_key(val) << 32) | (unsigned)(~row) : 0ull;
  key[w][c] = mk;
  if (tid < 2) {
    int n = 0;
    for (int q = 0; q < parts; ++q) n += nb[q * 2 + tid];
    s_cnt[tid] = n < h ? n : h;
    s_max[tid] = -INFINITY;
  }
  __syncthreads();
  const ulonglong2* kp = reinterpret_cast<const ulonglong2*>(&key[w][0]);
  int rank = 0;
#pragma unroll 8
  for (int e = 0; e < M / 2; ++e) {
    const ulonglong2 kk = kp[e];
    rank += (kk.x > mk ? 1 : 0) + (kk.y > mk ? 1 : 0);
  }
  if (mk != 0ull && rank < h) {
    sel[w][rank] = row;
    if (rank == 0) s_max[w] = val;
  }
  __syncthreads();
  if (tid == 0) gap[b] = s_max[0] + s_max[1];
  if (tid < 2 * h) {
    const int ww = tid / h, slot = tid % h, np = s_cnt[ww];
    long long* wsw = ws + (long long)b * 2 * h + ww * h;
    bool* okw = ok + (long long)b * 2 * h + ww * h;
    if (slot < np) {
      const int n = sel[ww][slot];
      int pos = 0;
      for (int j = 0; j < np; ++j) pos += sel[ww][j] < n ? 1 : 0;
      bool dup = false;
      if (ww == 1)
        for (int j = 0; j < s_cnt[0]; ++j) dup |= sel[0][j] == n;
      wsw[pos] = n;
      okw[pos] = !dup;
    } else {
      wsw[slot] = 0;
      okw[slot] = false;
    }
  }
}

// The rank merge fused into the K[ws, ws] gather: every one of the Q x B gather workgroups repeats
// the (small, deterministic) merge of the parts' candidates in LDS — identical in all of them —
// and gathers its row p of the block; workgroup 0 also writes ws / ok and this step's gap into
// ``gap_next`` (the previous step's gap in ``gap`` stays untouched for the other workgroups'
// converged test; the solve publishes gap_next).  One launch and one dependent global round trip
// less per outer step than merge + gather.
template <int NT>
__global__ __launch_bounds__(NT) void smo_ws_merge_gather_kernel(int h, int hp, int hs, int parts,
                                                                 const int* __restrict__ cand,
                                                                 const int* __restrict__ cnt,
                                                                 const float* __restrict__ candv,
                                                                 long long* __restrict__ ws, bool* __restrict__ ok,
                                                                 const float* __restrict__ gap,
                                                                 float* __restrict__ gap_next, float skip,
                                                                 const float* __restrict__ K, int N, long long kbs,
                                                                 float* __restrict__ Kws) {
  constexpr int M = NT / 2, Q = WS_Q;
  __shared__ __attribute__((aligned(16))) unsigned long long key[2][M];
  __shared__ int sel[2][64];
  __shared__ float s_max[2];
  __shared__ int s_cnt[2];
  __shared__ long long s_ws[Q];
  __shared__ int s_ok[Q];
  const int b = blockIdx.y, p = blockIdx.x, tid = threadIdx.x;
  if (ws_done(gap, b, skip)) return;
  const int w = tid / M, c = tid % M;
  const int* cb = cand + (long long)b * parts * 2 * hs;
  const float* vb = candv + (long long)b * parts * 2 * hs;
  const int* nb = cnt + (long long)b * parts * 2;
  int row = -1;
  float val = -INFINITY;
  if (c < parts * hp) {
    const int q = c / hp, s = c % hp;
    if (s < nb[q * 2 + w]) {
      row = cb[(q * 2 + w) * hs + s];
      val = vb[(q * 2 + w) * hs + s];
    }
  }
  const unsigned long long mk = row >= 0 ? ((unsigned long long)order_key(val) << 32) | (unsigned)(~row) : 0ull;
  key[w][c] = mk;
  if (tid < 2) {
    int n = 0;
    for (int q = 0; q < parts; ++q) n += nb[q * 2 + tid];
    s_cnt[tid] = n < h ? n : h;
    s_max[tid] = -INFINITY;
  }
  __syncthreads();
  const ulonglong2* kp = reinterpret_cast<const ulonglong2*>(&key[w][0]);
  int rank = 0;
#pragma unroll 8
  for (int e = 0; e < M / 2; ++e) {
    const ulonglong2 kk = kp[e];
    rank += (kk.x > mk ? 1 : 0) + (kk.y > mk ? 1 : 0);
  }
  if (mk != 0ull && rank < h) {
    sel[w][rank] = row;
    if (rank == 0) s_max[w] = val;
  }
  __syncthreads();
  const float gnew = s_max[0] + s_max[1];
  if (tid < 2 * h) {
    const int ww = tid / h, slot = tid % h, np = s_cnt[ww];
    if (slot < np) {
      const int n = sel[ww][slot];
      int pos = 0;
      for (int j = 0; j < np; ++j) pos += sel[ww][j] < n ? 1 : 0;
      bool dup = false;
      if (ww == 1)
        for (int j = 0; j < s_cnt[0]; ++j) dup |= sel[0][j] == n;
      s_ws[ww * h + pos] = n;
      s_ok[ww * h + pos] = dup ? 0 : 1;
    } else {
      s_ws[ww * h + slot] = 0;
      s_ok[ww * h + slot] = 0;
    }
  }
  __syncthreads();
  if (p == 0) {
    for (int q = tid; q < 2 * h; q += NT) {
      ws[(long long)b * 2 * h + q] = s_ws[q];
      ok[(long long)b * 2 * h + q] = s_ok[q] != 0;
    }
    if (tid == 0) gap_next[b] = gnew;
  }
  if (!(gnew >= skip) || p >= 2 * h) return;  // converged at this step: the solve and update skip too
  const long long rp = s_ok[p] ? s_ws[p] : 0;
  for (int q = tid; q < 2 * h; q += NT) {
    const long long cq = s_ok[q] ? s_ws[q] : 0;
    Kws[((long long)b * Q + p) * Q + q] = K[b * kbs + rp * N + cq];
  }
}

// G[n] += y[n] * sum_q dA[q] K[ws[q], n].  A workgroup owns 64 consecutive columns n; its 16 waves
// split the non-zero (ws, dA) pairs (compacted in q order by wave 0) into sixteenths, each lane
// streams its column of those <= 8 K rows (coalesced, all loads in flight at once), and the 16
// partials are added in a fixed order (deterministic).  Grid (N / 64, B): >= 128 workgroups at
// N = 8192.  (16 waves rather than 4: the per-wave row chain is the latency, 5.6 -> ~3 us.)
constexpr int UPD_T = 1024;
__global__ __launch_bounds__(UPD_T) void smo_ws_update_kernel(const float* __restrict__ K, const long long* __restrict__ ws,
                                                            const float* __restrict__ dA, const bool* __restrict__ ok,
                                                            const float* __restrict__ y, float* __restrict__ G, int N,
                                                            int ldag, int Q, const float* __restrict__ gap, float skip,
                                                            long long kbs) {
  __shared__ long long s_ws[WS_Q];
  __shared__ float s_d[WS_Q];
  __shared__ float red[UPD_T / 64][64];
  __shared__ int s_cnt;
  const int b = blockIdx.y, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (ws_done(gap, b, skip)) return;
  if (w == 0) {
    int base = 0;
    for (int q0 = 0; q0 < Q; q0 += 64) {
      const int q = q0 + lane;
      float d = 0.f;
      long long r = 0;
      if (q < Q && ok[(long long)b * Q + q]) {
        d = dA[(long long)b * Q + q];
        r = ws[(long long)b * Q + q];
      }
      const bool nz = d != 0.f;
      const unsigned long long bal = __ballot(nz);
      const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
      if (nz) {
        const int k = base + (int)__popcll(bal & below);
        s_ws[k] = r;
        s_d[k] = d;
      }
      base += (int)__popcll(bal);
    }
    if (lane == 0) s_cnt = base;
  }
  __syncthreads();
  constexpr int NW = UPD_T / 64;
  const int cnt = s_cnt, per = (cnt + NW - 1) / NW;
  const int q0 = w * per, q1 = min(cnt, q0 + per);
  const int n = blockIdx.x * 64 + lane;
  float acc = 0.f;
  if (n < N) {
    const float* Kb = K + b * kbs + n;
#pragma unroll 8
    for (int q = q0; q < q1; ++q) acc += s_d[q] * Kb[s_ws[q] * N];
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && n < N) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NW; ++k) s += red[k][lane];
    G[(long long)b * ldag + n] += y[(long long)b * N + n] * s;
  }
}

// RBF kernel matrix K[i][j] = exp(-gamma * |a_i - b_j|^2) in ONE pass for d <= 64: a 64 x 64
// output tile per workgroup, the 64 rows of A and of B staged in LDS (zero-padded to DP), each of the
// 256 threads computes a 4 x 4 block from the squared DIFFERENCES (no |a|^2 + |b|^2 - 2ab
// cancellation) and writes it as 4 row segments (16 threads x 16 B contiguous per row).  The
// GEMM + five elementwise passes of the tensor formula become one write-bound pass (N = 32 768:
// 4 GB written once instead of ~14 passes over 4 GB temporaries).
template <int DP>
__global__ __launch_bounds__(256) void rbf_matrix_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                         int na, int nb, int d, float gamma, float* __restrict__ K) {
  __shared__ float sa[64][DP + 1], sb[64][DP + 1];
  const int i0 = blockIdx.y * 64, j0 = blockIdx.x * 64, tid = threadIdx.x;
  for (int e = tid; e < 64 * DP; e += 256) {
    const int r = e / DP, k = e % DP;
    sa[r][k] = (i0 + r < na && k < d) ? A[(long long)(i0 + r) * d + k] : 0.f;
    sb[r][k] = (j0 + r < nb && k < d) ? B[(long long)(j0 + r) * d + k] : 0.f;
  }
  __syncthreads();
  const int tx = tid & 15, ty = tid >> 4;
  float acc[4][4] = {};
#pragma unroll 4
  for (int k = 0; k < DP; ++k) {
    float av[4], bv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) av[r] = sa[ty * 4 + r][k];
#pragma unroll
    for (int c = 0; c < 4; ++c) bv[c] = sb[tx * 4 + c][k];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float df = av[r] - bv[c];
        acc[r][c] = fmaf(df, df, acc[r][c]);
      }
  }
  const int jc = j0 + tx * 4;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = i0 + ty * 4 + r;
    if (i >= na) continue;
    float o[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) o[c] = expf(-gamma * acc[r][c]);
    float* dst = K + (long long)i * nb + jc;
    if ((nb & 3) == 0 && jc + 3 < nb) {
      *reinterpret_cast<float4*>(dst) = make_float4(o[0], o[1], o[2], o[3]);
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (jc + c < nb) dst[c] = o[c];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Implicit kernel (avk::SvmKerX): the working-set solver recomputes the kernel values it needs
// from the rows of X instead of reading an N x N matrix.  Per outer step it needs K[ws, ws]
// (Q x Q, the sub-problem) and K[ws, :] (Q x N, the gradient update).  Recomputing the Q x N block
// costs Q N D FMAs: at N = 262 144, D = 16, Q = 128 that is 0.5 GFLOP, ~10 us of VALU — less than
// READING those 134 MB from an HBM row cache (27 us at 5 TB/s), so no cache is kept at all and
// memory is O(N D): the N x N matrix (275 GB at N = 262 144) is never formed.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float kfun_dot(int kind, float dot, float ni, float nj, float gamma, float coef0, int deg) {
  switch (kind) {
    case 0:
      return dot;
    case 1: {
      const float base = gamma * dot + coef0;
      float r = 1.f;
      for (int i = 0; i < deg; ++i) r *= base;
      return r;
    }
    case 2:
      return __expf(-gamma * fmaxf(ni + nj - 2.f * dot, 0.f));
    default:
      return tanhf(gamma * dot + coef0);
  }
}

// K[ws_p, ws_q] of every problem: one workgroup per (p, problem), thread q; RBF from the squared
// differences (no cancellation), the others from the dot product
__global__ __launch_bounds__(WS_Q) void smo_ws_gather_x_kernel(const avk::SvmKerX k, const long long* __restrict__ ws,
                                                               const bool* __restrict__ ok, float* __restrict__ Kws,
                                                               int N, const float* __restrict__ gap, float skip) {
  constexpr int Q = WS_Q;
  const int b = blockIdx.y, p = blockIdx.x, q = threadIdx.x;
  if (ws_done(gap, b, skip)) return;
  const long long* wb = ws + (long long)b * Q;
  const bool* ob = ok + (long long)b * Q;
  const long long rp = ob[p] ? wb[p] : 0, rq = ob[q] ? wb[q] : 0;
  const float* X = k.X + (long long)b * k.xbs * k.D;
  const float* xp = X + rp * k.D;
  const float* xq = X + rq * k.D;
  float acc = 0.f;
  if (k.kind == 2) {
    for (int d = 0; d < k.D; ++d) {
      const float df = xp[d] - xq[d];
      acc = fmaf(df, df, acc);
    }
    Kws[((long long)b * Q + p) * Q + q] = __expf(-k.gamma * acc);
    return;
  }
  for (int d = 0; d < k.D; ++d) acc = fmaf(xp[d], xq[d], acc);
  Kws[((long long)b * Q + p) * Q + q] = kfun_dot(k.kind, acc, 0.f, 0.f, k.gamma, k.coef0, k.degree);
}

// compaction of the working set's non-zero (index, dA) pairs into LDS by wave 0 (q order)
__device__ __forceinline__ void ws_compact(const long long* __restrict__ ws, const float* __restrict__ dA,
                                           const bool* __restrict__ ok, int b, int Q, long long* s_ws, float* s_d,
                                           int* s_cnt) {
  const int lane = threadIdx.x & 63;
  int base = 0;
  for (int q0 = 0; q0 < Q; q0 += 64) {
    const int q = q0 + lane;
    float d = 0.f;
    long long r = 0;
    if (q < Q && ok[(long long)b * Q + q]) {
      d = dA[(long long)b * Q + q];
      r = ws[(long long)b * Q + q];
    }
    const bool nz = d != 0.f;
    const unsigned long long bal = __ballot(nz);
    const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
    if (nz) {
      const int kk = base + (int)__popcll(bal & below);
      s_ws[kk] = r;
      s_d[kk] = d;
    }
    base += (int)__popcll(bal);
  }
  if (lane == 0) *s_cnt = base;
}

// G[n] += y[n] sum_q dA_q k(x_ws_q, x_n), D <= DP <= 64: one thread per column n, x_n in registers,
// the (<= Q) working-set rows in LDS (every lane reads the same word: broadcast), RBF from squared
// differences.  Grid (N / 256, B).
constexpr int UPX_T = 256;
template <int DP>
__global__ __launch_bounds__(UPX_T) void smo_ws_update_x_kernel(const avk::SvmKerX k, const long long* __restrict__ ws,
                                                                const float* __restrict__ dA, const bool* __restrict__ ok,
                                                                const float* __restrict__ y, float* __restrict__ G, int N,
                                                                int ldag, int Q, const float* __restrict__ gap,
                                                                float skip) {
  __shared__ long long s_ws[WS_Q];
  __shared__ float s_d[WS_Q];
  __shared__ float s_x[WS_Q][DP];
  __shared__ int s_cnt;
  const int b = blockIdx.y;
  if (ws_done(gap, b, skip)) return;
  if (threadIdx.x < 64) ws_compact(ws, dA, ok, b, Q, s_ws, s_d, &s_cnt);
  __syncthreads();
  const int cnt = s_cnt;
  if (cnt == 0) return;
  const int D = k.D;
  const float* X = k.X + (long long)b * k.xbs * D;
  for (int e = threadIdx.x; e < cnt * DP; e += UPX_T) {
    const int q = e / DP, d = e % DP;
    s_x[q][d] = d < D ? X[s_ws[q] * D + d] : 0.f;
  }
  __syncthreads();
  const int n = blockIdx.x * UPX_T + threadIdx.x;
  if (n >= N) return;
  float xr[DP];
#pragma unroll
  for (int d = 0; d < DP; ++d) xr[d] = d < D ? X[(long long)n * D + d] : 0.f;
  float acc = 0.f;
  if (k.kind == 2) {
    const float ng = -k.gamma;
    for (int q = 0; q < cnt; ++q) {
      float d2 = 0.f;
#pragma unroll
      for (int d = 0; d < DP; ++d) {
        const float df = s_x[q][d] - xr[d];
        d2 = fmaf(df, df, d2);
      }
      acc = fmaf(s_d[q], __expf(ng * d2), acc);
    }
  } else {
    for (int q = 0; q < cnt; ++q) {
      float dot = 0.f;
#pragma unroll
      for (int d = 0; d < DP; ++d) dot = fmaf(s_x[q][d], xr[d], dot);
      acc = fmaf(s_d[q], kfun_dot(k.kind, dot, 0.f, 0.f, k.gamma, k.coef0, k.degree), acc);
    }
  }
  G[(long long)b * ldag + n] += y[(long long)b * N + n] * acc;
}

// ---- kernel-row cache (the reference memoises kernel values, J/discriminant/
// SequentialMinimalOptimization.java:511-524; libsvm keeps an LRU row cache, P/supv/svm.py:83-121).
// svm_cache_lookup_kernel: ONE workgroup.  The slot metadata (tag, stamp) is staged in LDS; each
// active working-set entry (ok, dA != 0: the rows the update reads) looks its row up through
// slot_of (validated against tag) and stamps a hit with this step; a miss takes, among the ways of
// its set (row % nsets) not used this step, the rank-th least recently used, rank = its order among
// this step's misses of the same set (all choices computed from the same pre-update stamps, so no
// two misses take one way), or a transient slot S + q when the set has no free way left.  Metadata
// goes back to global memory at the end; the compact miss list drives the fill kernel.
__global__ __launch_bounds__(1024) void svm_cache_lookup_kernel(avk::SvmCache c, const long long* __restrict__ ws,
                                                                const float* __restrict__ dA,
                                                                const bool* __restrict__ ok, int Q,
                                                                const float* __restrict__ gap, float skip) {
  extern __shared__ int cache_sm[];
  int* s_tag = cache_sm;
  int* s_stamp = cache_sm + c.S;
  __shared__ int s_step, s_set[WS_Q], s_miss[WS_Q], s_choice[WS_Q], s_hits;
  __shared__ long long s_row[WS_Q];
  if (ws_done(gap, 0, skip)) return;
  const int tid = threadIdx.x;
  for (int i = tid; i < c.S; i += 1024) {
    s_tag[i] = c.tag[i];
    s_stamp[i] = c.stamp[i];
  }
  if (tid == 0) {
    s_step = c.step[0] + 1;
    c.step[0] = s_step;
    s_hits = 0;
  }
  __syncthreads();
  const int step = s_step, nsets = c.S / c.ways;
  const bool mine = tid < Q;
  bool active = false, hit = false;
  long long row = 0;
  if (mine) {
    active = ok[tid] && dA[tid] != 0.f;
    row = ws[tid];
    s_row[tid] = row;
    if (active) {
      const int sl = c.slot_of[row];
      hit = sl >= 0 && sl < c.S && s_tag[sl] == (int)row;
      if (hit) {
        s_stamp[sl] = step;
        c.ws_slot[tid] = sl;
        atomicAdd(&s_hits, 1);
      }
    }
    s_miss[tid] = active && !hit;
    s_set[tid] = (int)(row % nsets);
  }
  __syncthreads();
  if (mine && s_miss[tid]) {
    const int set = s_set[tid];
    int rank = 0;
    for (int p = 0; p < tid; ++p) rank += (s_miss[p] && s_set[p] == set) ? 1 : 0;
    int choice = -1;
    for (int w = 0; w < c.ways && choice < 0; ++w) {
      const int sw = set * c.ways + w;
      if (s_stamp[sw] == step) continue;
      int pos = 0;
      for (int v = 0; v < c.ways; ++v) {
        const int sv = set * c.ways + v;
        if (s_stamp[sv] == step) continue;
        pos += (s_stamp[sv] < s_stamp[sw] || (s_stamp[sv] == s_stamp[sw] && v < w)) ? 1 : 0;
      }
      if (pos == rank) choice = sw;
    }
    s_choice[tid] = choice;
  }
  __syncthreads();
  if (mine && s_miss[tid]) {
    const int choice = s_choice[tid];
    int slot = c.S + tid;  // transient row: the set is full this step
    if (choice >= 0) {
      const int old = s_tag[choice];
      if (old >= 0) c.slot_of[old] = -1;
      s_tag[choice] = (int)row;
      s_stamp[choice] = step;
      c.slot_of[row] = choice;
      slot = choice;
    }
    c.ws_slot[tid] = slot;
    int mpos = 0;
    for (int p = 0; p < tid; ++p) mpos += s_miss[p] ? 1 : 0;
    c.miss_q[mpos] = tid;
  }
  __syncthreads();
  for (int i = tid; i < c.S; i += 1024) {
    c.tag[i] = s_tag[i];
    c.stamp[i] = s_stamp[i];
  }
  if (tid == 0) {
    int m = 0;
    for (int p = 0; p < Q; ++p) m += s_miss[p] ? 1 : 0;
    c.miss_cnt[0] = m;
    c.stats[0] += (unsigned long long)s_hits;
    c.stats[1] += (unsigned long long)m;
  }
}

// the missing rows K[ws[q], n] into their slots, D <= DP <= 64: one thread per n, the missing rows
// of X in LDS (broadcast reads), RBF from squared differences.  Grid N / 256.
template <int DP>
__global__ __launch_bounds__(UPX_T) void svm_cache_fill_kernel(const avk::SvmKerX k, avk::SvmCache c,
                                                               const long long* __restrict__ ws, int N,
                                                               const float* __restrict__ gap, float skip) {
  __shared__ float s_x[WS_Q][DP];
  __shared__ long long s_slot[WS_Q];
  if (ws_done(gap, 0, skip)) return;
  const int cnt = c.miss_cnt[0];
  if (cnt == 0) return;
  const int D = k.D;
  for (int e = threadIdx.x; e < cnt * DP; e += UPX_T) {
    const int m = e / DP, d = e % DP;
    const int q = c.miss_q[m];
    s_x[m][d] = d < D ? k.X[ws[q] * D + d] : 0.f;
    if (d == 0) s_slot[m] = c.ws_slot[q];
  }
  __syncthreads();
  const int n = blockIdx.x * UPX_T + threadIdx.x;
  if (n >= N) return;
  float xr[DP];
#pragma unroll
  for (int d = 0; d < DP; ++d) xr[d] = d < D ? k.X[(long long)n * D + d] : 0.f;
  for (int m = 0; m < cnt; ++m) {
    float v;
    if (k.kind == 2) {
      float d2 = 0.f;
#pragma unroll
      for (int d = 0; d < DP; ++d) {
        const float df = s_x[m][d] - xr[d];
        d2 = fmaf(df, df, d2);
      }
      v = __expf(-k.gamma * d2);
    } else {
      float dot = 0.f;
#pragma unroll
      for (int d = 0; d < DP; ++d) dot = fmaf(s_x[m][d], xr[d], dot);
      v = kfun_dot(k.kind, dot, 0.f, 0.f, k.gamma, k.coef0, k.degree);
    }
    c.rows[s_slot[m] * N + n] = v;
  }
}

// The same update for any D through f32 MFMA: the Q x 64 block of dot products of a workgroup (4
// waves x 16 columns, 8 row tiles of 16 per wave) accumulates v_mfma_f32_16x16x4_f32 over D in LDS
// chunks of 64 (working-set rows and the 64 column rows staged per chunk), then the epilogue maps
// each dot product through the kernel, weights it by dA_q and reduces over q: the 4 rows a lane
// holds per tile, then the 4 lane groups (xor-16 / xor-32 shuffles).  C/D map of 16x16x4:
// col = lane & 15, row = 4 (lane >> 4) + reg.
using f32x4 = __attribute__((ext_vector_type(4))) float;
constexpr int UPM_T = 256, UPM_KC = 64;
__global__ __launch_bounds__(UPM_T) void smo_ws_update_x_mfma_kernel(const avk::SvmKerX k,
                                                                     const long long* __restrict__ ws,
                                                                     const float* __restrict__ dA,
                                                                     const bool* __restrict__ ok,
                                                                     const float* __restrict__ y, float* __restrict__ G,
                                                                     int N, int ldag, int Q,
                                                                     const float* __restrict__ gap, float skip) {
  __shared__ long long s_ws[WS_Q];
  __shared__ float s_d[WS_Q];
  __shared__ float s_nq[WS_Q];
  __shared__ float s_a[WS_Q][UPM_KC + 1];
  __shared__ float s_b[64][UPM_KC + 1];
  __shared__ int s_cnt;
  const int b = blockIdx.y, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (ws_done(gap, b, skip)) return;
  if (threadIdx.x < 64) ws_compact(ws, dA, ok, b, Q, s_ws, s_d, &s_cnt);
  __syncthreads();
  const int cnt = s_cnt;
  if (cnt == 0) return;
  const int D = k.D;
  const float* X = k.X + (long long)b * k.xbs * D;
  const float* xn = k.xn + (long long)b * k.xbs;
  for (int q = threadIdx.x; q < WS_Q; q += UPM_T) {
    s_nq[q] = q < cnt ? xn[s_ws[q]] : 0.f;
    if (q >= cnt) s_d[q] = 0.f;
  }
  const int n0 = blockIdx.x * 64;
  const int tiles = (cnt + 15) / 16;
  f32x4 acc[WS_Q / 16];
#pragma unroll
  for (int t = 0; t < WS_Q / 16; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int kc = 0; kc < D; kc += UPM_KC) {
    __syncthreads();  // the previous chunk is consumed
    const int kw = min(UPM_KC, D - kc);
    for (int e = threadIdx.x; e < tiles * 16 * UPM_KC; e += UPM_T) {
      const int q = e / UPM_KC, d = e % UPM_KC;
      s_a[q][d] = (q < cnt && d < kw) ? X[s_ws[q] * D + kc + d] : 0.f;
    }
    for (int e = threadIdx.x; e < 64 * UPM_KC; e += UPM_T) {
      const int c = e / UPM_KC, d = e % UPM_KC;
      s_b[c][d] = (n0 + c < N && d < kw) ? X[(long long)(n0 + c) * D + kc + d] : 0.f;
    }
    __syncthreads();
    const int col = w * 16 + (lane & 15), kq = lane >> 4;
    for (int kk = 0; kk < kw; kk += 4) {
      const float bv = s_b[col][kk + kq];
#pragma unroll
      for (int t = 0; t < WS_Q / 16; ++t)
        if (t < tiles) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(s_a[t * 16 + (lane & 15)][kk + kq], bv, acc[t], 0, 0, 0);
    }
  }
  const int n = n0 + w * 16 + (lane & 15);
  const float nn = n < N ? xn[n] : 0.f;
  float part = 0.f;
#pragma unroll
  for (int t = 0; t < WS_Q / 16; ++t) {
    if (t >= tiles) break;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = t * 16 + 4 * (lane >> 4) + r;
      part = fmaf(s_d[q], kfun_dot(k.kind, acc[t][r], s_nq[q], nn, k.gamma, k.coef0, k.degree), part);
    }
  }
  part += __shfl_xor(part, 16, 64);
  part += __shfl_xor(part, 32, 64);
  if (lane < 16 && n < N) G[(long long)b * ldag + n] += y[(long long)b * N + n] * part;
}

// The cache fill for any D through f32 MFMA (the tiling of smo_ws_update_x_mfma_kernel): the
// workgroup's 64 columns x the step's missing rows (<= 128, 16-row tiles) accumulate
// v_mfma_f32_16x16x4_f32 over D in LDS chunks of 64; the epilogue maps each dot product through
// the kernel (RBF from the norms, as the uncached update) and writes it to the row's slot: per
// missing row, each wave stores 16 consecutive columns.
__global__ __launch_bounds__(UPM_T) void svm_cache_fill_mfma_kernel(const avk::SvmKerX k, avk::SvmCache c,
                                                                    const long long* __restrict__ ws, int N,
                                                                    const float* __restrict__ gap, float skip) {
  __shared__ long long s_row[WS_Q], s_slot[WS_Q];
  __shared__ float s_nq[WS_Q];
  __shared__ float s_a[WS_Q][UPM_KC + 1];
  __shared__ float s_b[64][UPM_KC + 1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (ws_done(gap, 0, skip)) return;
  const int cnt = c.miss_cnt[0];
  if (cnt == 0) return;
  const int D = k.D;
  for (int m = threadIdx.x; m < WS_Q; m += UPM_T) {
    const bool in = m < cnt;
    const long long r = in ? ws[c.miss_q[m]] : 0;
    s_row[m] = r;
    s_slot[m] = in ? c.ws_slot[c.miss_q[m]] : 0;
    s_nq[m] = in ? k.xn[r] : 0.f;
  }
  const int n0 = blockIdx.x * 64;
  const int tiles = (cnt + 15) / 16;
  f32x4 acc[WS_Q / 16];
#pragma unroll
  for (int t = 0; t < WS_Q / 16; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int kc = 0; kc < D; kc += UPM_KC) {
    __syncthreads();  // the previous chunk is consumed (first pass: s_row is written)
    const int kw = min(UPM_KC, D - kc);
    for (int e = threadIdx.x; e < tiles * 16 * UPM_KC; e += UPM_T) {
      const int m = e / UPM_KC, d = e % UPM_KC;
      s_a[m][d] = (m < cnt && d < kw) ? k.X[s_row[m] * D + kc + d] : 0.f;
    }
    for (int e = threadIdx.x; e < 64 * UPM_KC; e += UPM_T) {
      const int cc = e / UPM_KC, d = e % UPM_KC;
      s_b[cc][d] = (n0 + cc < N && d < kw) ? k.X[(long long)(n0 + cc) * D + kc + d] : 0.f;
    }
    __syncthreads();
    const int col = w * 16 + (lane & 15), kq = lane >> 4;
    for (int kk = 0; kk < kw; kk += 4) {
      const float bv = s_b[col][kk + kq];
#pragma unroll
      for (int t = 0; t < WS_Q / 16; ++t)
        if (t < tiles) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(s_a[t * 16 + (lane & 15)][kk + kq], bv, acc[t], 0, 0, 0);
    }
  }
  const int n = n0 + w * 16 + (lane & 15);
  if (n >= N) return;
  const float nn = k.xn[n];
#pragma unroll
  for (int t = 0; t < WS_Q / 16; ++t) {
    if (t >= tiles) break;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = t * 16 + 4 * (lane >> 4) + r;
      if (m < cnt) c.rows[s_slot[m] * N + n] = kfun_dot(k.kind, acc[t][r], s_nq[m], nn, k.gamma, k.coef0, k.degree);
    }
  }
}

// K[i][j] = k(a_i, b_j) for any d by f32 MFMA: a 64 x 64 output tile per workgroup, wave w owns rows
// 16w..16w+15 (4 column tiles of 16), D in LDS chunks of 64; the epilogue applies the kernel
// (RBF from the norms) and writes 16-float row segments.
__global__ __launch_bounds__(256) void kernel_matrix_mfma_kernel(const avk::SvmKerX a, const float* __restrict__ Bx,
                                                                 const float* __restrict__ bn, int na, int nb,
                                                                 float* __restrict__ K) {
  __shared__ float sa[64][UPM_KC + 1], sb[64][UPM_KC + 1];
  const int i0 = blockIdx.y * 64, j0 = blockIdx.x * 64, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int D = a.D;
  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int kc = 0; kc < D; kc += UPM_KC) {
    __syncthreads();
    const int kw = min(UPM_KC, D - kc);
    for (int e = threadIdx.x; e < 64 * UPM_KC; e += 256) {
      const int r = e / UPM_KC, d = e % UPM_KC;
      sa[r][d] = (i0 + r < na && d < kw) ? a.X[(long long)(i0 + r) * D + kc + d] : 0.f;
      sb[r][d] = (j0 + r < nb && d < kw) ? Bx[(long long)(j0 + r) * D + kc + d] : 0.f;
    }
    __syncthreads();
    const int kq = lane >> 4;
    for (int kk = 0; kk < kw; kk += 4) {
      const float av = sa[w * 16 + (lane & 15)][kk + kq];
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, sb[t * 16 + (lane & 15)][kk + kq],
                                                                              acc[t], 0, 0, 0);
    }
  }
  // acc[t][r]: row i = i0 + 16 w + 4 (lane >> 4) + r, column j = j0 + 16 t + (lane & 15)
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int j = j0 + 16 * t + (lane & 15);
    const float nj = j < nb ? bn[j] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 16 * w + 4 * (lane >> 4) + r;
      if (i < na && j < nb)
        K[(long long)i * nb + j] = kfun_dot(a.kind, acc[t][r], a.xn[i], nj, a.gamma, a.coef0, a.degree);
    }
  }
}

}  // namespace

namespace avk {

void rbf_matrix(const float* A, const float* B, int na, int nb, int d, float gamma, float* K, hipStream_t stream) {
  if (na <= 0 || nb <= 0) return;
  const dim3 grid((nb + 63) / 64, (na + 63) / 64);
  if (d <= 8) rbf_matrix_kernel<8><<<grid, 256, 0, stream>>>(A, B, na, nb, d, gamma, K);
  else if (d <= 16) rbf_matrix_kernel<16><<<grid, 256, 0, stream>>>(A, B, na, nb, d, gamma, K);
  else if (d <= 32) rbf_matrix_kernel<32><<<grid, 256, 0, stream>>>(A, B, na, nb, d, gamma, K);
  else if (d <= 64) rbf_matrix_kernel<64><<<grid, 256, 0, stream>>>(A, B, na, nb, d, gamma, K);
  else throw std::runtime_error("rbf_matrix: d <= 64");
  AV_HIP_CHECK(hipGetLastError());
}

void smo_solve(const float* K, const float* y, const float* diag, float* alpha, float* G, int B, int N, float C,
               float eps, int max_iter, int* iters, hipStream_t stream) {
  if (B <= 0 || N <= 0) return;
  smo_kernel<<<B, SMO_THREADS, 0, stream>>>(K, y, diag, alpha, G, N, C, eps, max_iter, iters);
  AV_HIP_CHECK(hipGetLastError());
}

int smo_ws_size() { return WS_Q; }

void smo_ws_gather_x(const SvmKerX& k, const long long* ws, const bool* ok, float* Kws, int B, int N, const float* gap,
                     float skip, hipStream_t stream) {
  if (B <= 0) return;
  smo_ws_gather_x_kernel<<<dim3(WS_Q, B), WS_Q, 0, stream>>>(k, ws, ok, Kws, N, gap, skip);
  AV_HIP_CHECK(hipGetLastError());
}

void smo_ws_update_x(const SvmKerX& k, const long long* ws, const float* dA, const bool* ok, const float* y, float* G,
                     int B, int N, int ldag, int Q, const float* gap, float skip, hipStream_t stream) {
  if (B <= 0 || N <= 0) return;
  if (Q > WS_Q) throw std::runtime_error("smo_ws_update_x: Q <= 128");
  if (k.D > 64 || std::getenv("AVMI_SVM_MFMA_UPDATE")) {
    smo_ws_update_x_mfma_kernel<<<dim3((N + 63) / 64, B), UPM_T, 0, stream>>>(k, ws, dA, ok, y, G, N, ldag, Q, gap, skip);
  } else {
    const dim3 grid((N + UPX_T - 1) / UPX_T, B);
#define AV_UX(DP) smo_ws_update_x_kernel<DP><<<grid, UPX_T, 0, stream>>>(k, ws, dA, ok, y, G, N, ldag, Q, gap, skip)
    if (k.D <= 8) AV_UX(8);
    else if (k.D <= 16) AV_UX(16);
    else if (k.D <= 32) AV_UX(32);
    else AV_UX(64);
#undef AV_UX
  }
  AV_HIP_CHECK(hipGetLastError());
}

void smo_ws_update_cached(const SvmKerX& k, const SvmCache& c, const long long* ws, const float* dA, const bool* ok,
                          const float* y, float* G, int N, int ldag, int Q, const float* gap, float skip,
                          hipStream_t stream) {
  if (N <= 0) return;
  if (Q > WS_Q) throw std::runtime_error("smo_ws_update_cached: Q <= 128");
  if (c.S <= 0 || c.ways <= 0 || c.S % c.ways) throw std::runtime_error("smo_ws_update_cached: S must be a multiple of ways");
  const size_t lds = 2 * sizeof(int) * (size_t)c.S;
  if (lds > 128 * 1024) throw std::runtime_error("smo_ws_update_cached: at most 16384 slots");
  if (lds > 64 * 1024)
    AV_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(svm_cache_lookup_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  svm_cache_lookup_kernel<<<1, 1024, lds, stream>>>(c, ws, dA, ok, Q, gap, skip);
  AV_HIP_CHECK(hipGetLastError());
  const dim3 grid((N + UPX_T - 1) / UPX_T);
  if (k.D <= 64) {
#define AV_CF(DP) svm_cache_fill_kernel<DP><<<grid, UPX_T, 0, stream>>>(k, c, ws, N, gap, skip)
    if (k.D <= 8) AV_CF(8);
    else if (k.D <= 16) AV_CF(16);
    else if (k.D <= 32) AV_CF(32);
    else AV_CF(64);
#undef AV_CF
  } else {
    svm_cache_fill_mfma_kernel<<<dim3((N + 63) / 64), UPM_T, 0, stream>>>(k, c, ws, N, gap, skip);
  }
  AV_HIP_CHECK(hipGetLastError());
  // the dense update reads K[ws_slot[q], n] from the cache rows
  smo_ws_update(c.rows, c.ws_slot, dA, ok, y, G, 1, N, ldag, Q, gap, skip, 0, stream);
}

void svm_kernel_matrix_mfma(const SvmKerX& a, const float* Bx, const float* bn, int na, int nb, float* K,
                            hipStream_t stream) {
  if (na <= 0 || nb <= 0) return;
  kernel_matrix_mfma_kernel<<<dim3((nb + 63) / 64, (na + 63) / 64), 256, 0, stream>>>(a, Bx, bn, na, nb, K);
  AV_HIP_CHECK(hipGetLastError());
}

void smo_ws_solve(const float* Kws, const float* yws, float* aws, const float* gws, const float* gap, int B, float C,
                  float eps, int max_iter, int* iters, hipStream_t stream) {
  if (B <= 0) return;
  smo_ws_kernel<<<B, 64, 0, stream>>>(Kws, yws, aws, gws, gap, C, eps, max_iter, iters);
  AV_HIP_CHECK(hipGetLastError());
}

// "0" / "false" in the environment turns an optional fast path off (A/B measurements)
static bool env_off(const char* name) {
  const char* v = std::getenv(name);
  return v && (v[0] == '0' || v[0] == 'f' || v[0] == 'F' || v[0] == 'n' || v[0] == 'N');
}

// parts of 2048 / 4096 / 8192 rows: the smallest whose candidates (parts x h per side) fit a
// 512-thread merge, else a 1024-thread one
static int select_part_per(int N, int h) {
  for (int cap : {512, SEL_T})
    for (int per = 2; per <= 8; per *= 2) {
      const int parts = (N + per * SEL_T - 1) / (per * SEL_T);
      if (parts * h <= cap) return per;
    }
  return 0;
}

// large N (no register-resident part size): the streaming parts, <= 64 parts x 4 candidates per
// side = 4 x h slots of the [parts][2][h] allocation
static void stream_plan(int N, int* parts, int* per) {
  const long long blocks = ((long long)N + 63) / 64;
  *per = (int)((blocks + 64LL * (SEL_T / 64) - 1) / (64LL * (SEL_T / 64)));  // parts <= 64
  *parts = (int)((blocks + (long long)*per * (SEL_T / 64) - 1) / ((long long)*per * (SEL_T / 64)));
}

int smo_ws_select_parts(int N) {
  const int per = select_part_per(N, 64);
  return per ? (N + per * SEL_T - 1) / (per * SEL_T) : 4;
}

// The rank merge of a two-level selection, when the caller launches it itself (fused with the gather)
struct MergePlan {
  int parts = 0, hp = 0, hs = 0, nt = 0;
  const float* candv = nullptr;
};

static void select_impl(const float* alpha, const float* G, const float* y, int B, int N, int ldag, float C, int h,
                        long long* ws, bool* ok, float* gap, int* cand, int* cnt, float skip, hipStream_t stream,
                        MergePlan* plan);

// cand: [B][parts][2][h] rows followed by [B][parts][2][h] float violation values (candv)
void smo_ws_select(const float* alpha, const float* G, const float* y, int B, int N, int ldag, float C, int h,
                   long long* ws, bool* ok, float* gap, int* cand, int* cnt, float skip, hipStream_t stream) {
  select_impl(alpha, G, y, B, N, ldag, C, h, ws, ok, gap, cand, cnt, skip, stream, nullptr);
}

static void select_impl(const float* alpha, const float* G, const float* y, int B, int N, int ldag, float C, int h,
                        long long* ws, bool* ok, float* gap, int* cand, int* cnt, float skip, hipStream_t stream,
                        MergePlan* plan) {
  if (plan) *plan = MergePlan{};
  if (B <= 0) return;
  const size_t lds = (size_t)((N + 31) / 32) * sizeof(unsigned);
  if (h > 64) throw std::runtime_error("smo_ws_select: h <= 64");
  const int per = select_part_per(N, 64);
  // register top-k parts + rank merge for every two-level size (N > 4096), HW = 4 keys per wave and
  // HP = the power of two <= target / parts per part (target 128 candidates per side: the
  // 256-thread merge).  Against the exact radix parts: N = 8192 18.3-19.3 -> 17.2-18.4 ms, 12000
  // 28.5-29.1 -> 23.4 ms, 16384 37.0 -> 31.2 ms, 32768 76 -> 54 ms (profiles/r4_svm_topk_ab.log,
  // profiles/r4_svm_mid_ab.log, profiles/r4_svm_hw_ab.log).  AVMI_SMO_TOPK=0: the exact radix parts.
  static const int topk_min_n = [] {
    const char* e = std::getenv("AVMI_SMO_TOPK_MIN_N");
    return e && *e ? std::atoi(e) : 4 * 1024 + 1;
  }();
  if (N > 4 * SEL_T && N >= topk_min_n && cand && per && !env_off("AVMI_SMO_TOPK") && h == 64) {
    static const int target = [] {
      const char* e = std::getenv("AVMI_SMO_TOPK_M");
      return e && std::atoi(e) >= 256 ? 256 : 128;
    }();
    static const int force_per = [] {
      const char* e = std::getenv("AVMI_SMO_TOPK_PER");
      const int v = e && *e ? std::atoi(e) : 0;
      return v == 1 || v == 2 || v == 4 ? v : 0;
    }();
    // one 64-row block per wave (N = 32768: 58 ms against 61 ms with 2 and 85 ms with 4 blocks,
    // the HP-step wave loop being the cost), up to 256 candidates per side (512-thread merge)
    const int tper = force_per ? force_per : 1;
    const int tparts = (N + tper * SEL_T - 1) / (tper * SEL_T);
    static const int force_hp = [] {  // A/B: a fixed HP (4..64, power of two)
      const char* e = std::getenv("AVMI_SMO_TOPK_HP");
      const int v = e && *e ? std::atoi(e) : 0;
      return v == 4 || v == 8 || v == 16 || v == 32 || v == 64 ? v : 0;
    }();
    int hp = 64;
    while (hp > 4 && tparts * hp > target) hp >>= 1;
    if (force_hp) hp = force_hp;
    // (33..64 parts keep HP = 4: 256 candidates, the 512-thread merge; more parts: radix parts)
    const int old_parts = (N + per * SEL_T - 1) / (per * SEL_T);
    if (tparts * hp <= 256 && tparts * hp >= h && tparts * hp <= old_parts * h) {
      float* candv = reinterpret_cast<float*>(cand + (long long)B * old_parts * 2 * h);  // the allocation's layout
      const dim3 pg(tparts, B);
#define AV_TK(P, H) smo_ws_topk_part_kernel<P, H><<<pg, SEL_T, 0, stream>>>(alpha, G, y, N, ldag, C, tparts, cand, \
      cnt, candv, gap, skip)
#define AV_TKP(P) do { if (hp == 4) AV_TK(P, 4); else if (hp == 8) AV_TK(P, 8); else if (hp == 16) AV_TK(P, 16); \
      else if (hp == 32) AV_TK(P, 32); else AV_TK(P, 64); } while (0)
      if (tper == 1) AV_TKP(1);
      else if (tper == 2) AV_TKP(2);
      else AV_TKP(4);
#undef AV_TKP
#undef AV_TK
      AV_HIP_CHECK(hipGetLastError());
      if (plan) {
        *plan = MergePlan{tparts, hp, hp, tparts * hp <= 128 ? 256 : 512, candv};
        return;
      }
      if (tparts * hp <= 128)
        smo_ws_merge_rank_kernel<256><<<B, 256, 0, stream>>>(h, hp, hp, tparts, cand, cnt, candv, ws, ok, gap, skip);
      else
        smo_ws_merge_rank_kernel<512><<<B, 512, 0, stream>>>(h, hp, hp, tparts, cand, cnt, candv, ws, ok, gap, skip);
      AV_HIP_CHECK(hipGetLastError());
      return;
    }
  }
  if (!per && cand && h == 64) {
    // large N: streaming parts (<= 64) + the rank merge over <= 256 candidates per side
    int parts = 0, sper = 0;
    stream_plan(N, &parts, &sper);
    const int hp = parts * 4 <= 128 ? (parts * 8 <= 128 ? 8 : 4) : 4;
    float* candv = reinterpret_cast<float*>(cand + (long long)B * smo_ws_select_parts(N) * 2 * h);
    const dim3 pg(parts, B);
    if (hp == 8)
      smo_ws_topk_stream_kernel<8><<<pg, SEL_T, 0, stream>>>(alpha, G, y, N, ldag, C, parts, sper, cand, cnt, candv,
                                                             gap, skip);
    else
      smo_ws_topk_stream_kernel<4><<<pg, SEL_T, 0, stream>>>(alpha, G, y, N, ldag, C, parts, sper, cand, cnt, candv,
                                                             gap, skip);
    AV_HIP_CHECK(hipGetLastError());
    if (plan) {
      *plan = MergePlan{parts, hp, hp, parts * hp <= 128 ? 256 : 512, candv};
      return;
    }
    if (parts * hp <= 128)
      smo_ws_merge_rank_kernel<256><<<B, 256, 0, stream>>>(h, hp, hp, parts, cand, cnt, candv, ws, ok, gap, skip);
    else
      smo_ws_merge_rank_kernel<512><<<B, 512, 0, stream>>>(h, hp, hp, parts, cand, cnt, candv, ws, ok, gap, skip);
    AV_HIP_CHECK(hipGetLastError());
    return;
  }
  if (N > (1 << 18)) throw std::runtime_error("smo_ws_select: N > 2^18 needs the candidate buffers (cand)");
  if (N <= 4 * SEL_T) {
    smo_ws_select2_kernel<4><<<B, SEL_T, lds, stream>>>(alpha, G, y, N, ldag, C, h, ws, ok, gap, skip);
  } else if (cand && per) {
    // two levels: parts on separate CUs, then one merge over <= parts x h candidates per side
    const int parts = (N + per * SEL_T - 1) / (per * SEL_T);
    const dim3 pg(parts, B);
    float* candv = reinterpret_cast<float*>(cand + (long long)B * parts * 2 * h);
#define AV_SP(P) smo_ws_select_part_kernel<P><<<pg, SEL_T, 0, stream>>>(alpha, G, y, N, ldag, C, h, parts, cand, cnt, \
      candv, gap, skip)
    if (per == 2) AV_SP(2);
    else if (per == 4) AV_SP(4);
    else AV_SP(8);
#undef AV_SP
    AV_HIP_CHECK(hipGetLastError());
    const int m = parts * h;
    // rank merge up to 256 candidates per side (N <= 8192: 7.0 us against 10.4 us for the radix
    // merge, profiles/r3_svm_v6_kernel_stats.txt); 512 per side (N = 32768) is an A/B switch
    // (AVMI_SMO_RANK_MERGE_MAX=512) until measured: its O(M^2) LDS reads double again
    static const int rank_max = [] {
      const char* e = std::getenv("AVMI_SMO_RANK_MERGE_MAX");
      return e && std::atoi(e) >= 512 ? 512 : 256;
    }();
    if (m <= rank_max && !env_off("AVMI_SMO_RANK_MERGE")) {
      if (plan) {
        *plan = MergePlan{parts, h, h, m <= 128 ? 256 : (m <= 256 ? 512 : 1024), candv};
        return;
      }
      if (m <= 128) smo_ws_merge_rank_kernel<256><<<B, 256, 0, stream>>>(h, h, h, parts, cand, cnt, candv, ws, ok, gap, skip);
      else if (m <= 256) smo_ws_merge_rank_kernel<512><<<B, 512, 0, stream>>>(h, h, h, parts, cand, cnt, candv, ws, ok, gap, skip);
      else smo_ws_merge_rank_kernel<1024><<<B, 1024, 0, stream>>>(h, h, h, parts, cand, cnt, candv, ws, ok, gap, skip);
      AV_HIP_CHECK(hipGetLastError());
      return;
    }
    if (m <= 256)
      smo_ws_select_merge_kernel<256><<<B, 256, lds, stream>>>(alpha, G, y, N, ldag, C, h, parts, cand, cnt, ws, ok, gap,
                                                                skip);
    else if (m <= 512)
      smo_ws_select_merge_kernel<512><<<B, 512, lds, stream>>>(alpha, G, y, N, ldag, C, h, parts, cand, cnt, ws, ok, gap,
                                                                skip);
    else
      smo_ws_select_merge_kernel<1024><<<B, 1024, lds, stream>>>(alpha, G, y, N, ldag, C, h, parts, cand, cnt, ws, ok,
                                                                 gap, skip);
  } else {
    smo_ws_select_kernel<0><<<B, SEL_T, lds, stream>>>(alpha, G, y, N, ldag, C, h, ws, ok, gap, skip);
  }
  AV_HIP_CHECK(hipGetLastError());
}

void smo_ws_update(const float* K, const long long* ws, const float* dA, const bool* ok, const float* y, float* G,
                   int B, int N, int ldag, int Q, const float* gap, float skip, long long kbs, hipStream_t stream) {
  if (B <= 0 || N <= 0) return;
  smo_ws_update_kernel<<<dim3((N + 63) / 64, B), UPD_T, 0, stream>>>(K, ws, dA, ok, y, G, N, ldag, Q, gap, skip, kbs);
  AV_HIP_CHECK(hipGetLastError());
}

void smo_ws_solve_fused(const float* K, int N, const long long* ws, const bool* ok, float* alpha, const float* G,
                        const float* y, int ldag, const float* gap, int B, float C, float eps, int max_iter, float* dA,
                        long long* inner_total, float* Kws, float rel_tol, long long kbs, hipStream_t stream) {
  if (B <= 0) return;
  if (Kws) {  // spread gather (Q x B workgroups) + one-wave solve
    smo_ws_gather_kernel<<<dim3(WS_Q, B), WS_Q, 0, stream>>>(K, N, ws, ok, Kws, gap, eps, kbs);
    AV_HIP_CHECK(hipGetLastError());
    smo_ws_solve_kernel<<<B, WSS_T, 0, stream>>>(Kws, ws, ok, alpha, G, y, N, ldag, gap, C, eps, rel_tol, max_iter,
                                                 dA, inner_total);
  } else {
    smo_ws_solve_fused_kernel<<<B, SOLVE_T, 0, stream>>>(K, N, ws, ok, alpha, G, y, ldag, gap, C, eps, max_iter, dA,
                                                         inner_total, kbs);
  }
  AV_HIP_CHECK(hipGetLastError());
}

// The whole working-set solve driven from the host without Python or graph capture: blocks of
// `check_every` outer steps (select, gather, solve, update = 5 launches each, ~25 us of host time
// against ~65 us of GPU time per step, so the queue never drains) are enqueued back to back; after
// each block the gaps are copied into pinned host memory behind an event, and the host tests the
// PREVIOUS block's gaps while the current one runs.  Steps queued past convergence are no-ops
// (ws_done), so the one-block look-behind costs a few microseconds of empty launches instead of a
// pipeline drain per test.  Returns the number of outer steps enqueued.
long long smo_ws_run(const float* K, int N, float* alpha, float* G, const float* y, int B, int ldag, float C,
                     float eps, int inner_iter, float rel_tol, long long max_outer, int check_every, long long* ws,
                     bool* ok, float* dA, long long* inner_total, float* gap, int* cand, int* cnt, float* Kws,
                     float* host_gap, long long kbs, hipStream_t caller, const SvmKerX* kx, float* gap_next,
                     const SvmCache* cache) {
  if (B <= 0 || N <= 0 || max_outer <= 0) return 0;
  if (cache && (B != 1 || !kx || kx->xbs != 0)) throw std::runtime_error("smo_ws_run: the row cache needs one problem on X");
  // merge fused into the gather (explicit K, a rank-merge selection, gap_next scratch given)
  const bool fuse = gap_next && !kx && Kws && !env_off("AVMI_SMO_FUSED_GATHER");
  const int Q = WS_Q, h = WS_Q / 2;
  check_every = check_every < 1 ? 1 : check_every;
  hipEvent_t ev[2];
  for (auto& e : ev) AV_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  // a private stream ordered after the caller's work (the caller's may be the null stream, which
  // cannot be captured); the caller's stream is synchronised at the end anyway
  hipStream_t stream = nullptr;
  AV_HIP_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  AV_HIP_CHECK(hipEventRecord(ev[1], caller));
  AV_HIP_CHECK(hipStreamWaitEvent(stream, ev[1], 0));
  if (fuse) AV_HIP_CHECK(hipMemcpyAsync(gap_next, gap, sizeof(float) * B, hipMemcpyDeviceToDevice, stream));
  auto enqueue = [&](long long n) {
    for (long long s = 0; s < n; ++s) {
      if (fuse) {
        MergePlan plan;
        select_impl(alpha, G, y, B, N, ldag, C, h, ws, ok, gap, cand, cnt, eps, stream, &plan);
        if (plan.nt) {
          const dim3 gg(Q, B);
#define AV_MG(NT) smo_ws_merge_gather_kernel<NT><<<gg, NT, 0, stream>>>(h, plan.hp, plan.hs, plan.parts, cand, cnt, \
      plan.candv, ws, ok, gap, gap_next, eps, K, N, kbs, Kws)
          if (plan.nt == 256) AV_MG(256);
          else if (plan.nt == 512) AV_MG(512);
          else AV_MG(1024);
#undef AV_MG
          AV_HIP_CHECK(hipGetLastError());
          smo_ws_solve_kernel<<<B, WSS_T, 0, stream>>>(Kws, ws, ok, alpha, G, y, N, ldag, gap_next, C, eps, rel_tol,
                                                       inner_iter, dA, inner_total, gap);
          AV_HIP_CHECK(hipGetLastError());
        } else {  // a selection without a separate merge (single level): unfused gather + solve
          smo_ws_solve_fused(K, N, ws, ok, alpha, G, y, ldag, gap, B, C, eps, inner_iter, dA, inner_total, Kws,
                             rel_tol, kbs, stream);
        }
        smo_ws_update(K, ws, dA, ok, y, G, B, N, ldag, Q, gap, eps, kbs, stream);
        continue;
      }
      smo_ws_select(alpha, G, y, B, N, ldag, C, h, ws, ok, gap, cand, cnt, eps, stream);
      if (kx) {  // implicit kernel: K[ws, ws] and the gradient update from the rows of X
        smo_ws_gather_x(*kx, ws, ok, Kws, B, N, gap, eps, stream);
        smo_ws_solve_kernel<<<B, WSS_T, 0, stream>>>(Kws, ws, ok, alpha, G, y, N, ldag, gap, C, eps, rel_tol,
                                                     inner_iter, dA, inner_total);
        AV_HIP_CHECK(hipGetLastError());
        if (cache)
          smo_ws_update_cached(*kx, *cache, ws, dA, ok, y, G, N, ldag, Q, gap, eps, stream);
        else
          smo_ws_update_x(*kx, ws, dA, ok, y, G, B, N, ldag, Q, gap, eps, stream);
        continue;
      }
      smo_ws_solve_fused(K, N, ws, ok, alpha, G, y, ldag, gap, B, C, eps, inner_iter, dA, inner_total, Kws, rel_tol,
                         kbs, stream);
      smo_ws_update(K, ws, dA, ok, y, G, B, N, ldag, Q, gap, eps, kbs, stream);
    }
  };
  // One block of steps captured once as a HIP graph (a few microseconds of host time per block
  // instead of five launches per step); the capture records without executing.
  hipGraphExec_t exec = nullptr;
  if (!env_off("AVMI_SMO_RUN_GRAPH") && max_outer >= check_every) {
    hipGraph_t graph = nullptr;
    AV_HIP_CHECK(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
    enqueue(check_every);
    AV_HIP_CHECK(hipStreamEndCapture(stream, &graph));
    AV_HIP_CHECK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    AV_HIP_CHECK(hipGraphDestroy(graph));
  }
  long long outer = 0;
  for (long long blk = 0; outer < max_outer; ++blk) {
    const long long n = std::min<long long>(check_every, max_outer - outer);
    if (exec && n == check_every) AV_HIP_CHECK(hipGraphLaunch(exec, stream));
    else enqueue(n);
    outer += n;
    float* hg = host_gap + (blk & 1) * B;
    AV_HIP_CHECK(hipMemcpyAsync(hg, gap, sizeof(float) * B, hipMemcpyDeviceToHost, stream));
    AV_HIP_CHECK(hipEventRecord(ev[blk & 1], stream));
    if (blk >= 1) {
      AV_HIP_CHECK(hipEventSynchronize(ev[(blk - 1) & 1]));
      const float* pg = host_gap + ((blk - 1) & 1) * B;
      bool done = true;
      for (int b = 0; b < B; ++b) done = done && !(pg[b] >= eps);
      if (done) break;
    }
  }
  AV_HIP_CHECK(hipStreamSynchronize(stream));
  AV_HIP_CHECK(hipStreamDestroy(stream));
  if (exec) AV_HIP_CHECK(hipGraphExecDestroy(exec));
  for (auto& e : ev) AV_HIP_CHECK(hipEventDestroy(e));
  return outer;
}

}  // namespace avk
