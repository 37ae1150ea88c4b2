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
  constexpr int NONE = 0x7fffffff;
  int it = 0;
  for (; it < max_iter; ++it) {
    float gmax = -INFINITY;
    int gi = NONE;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const bool up = y[e] > 0.f ? a[e] < C : (y[e] < 0.f && a[e] > 0.f);
      const float v = -y[e] * g[e];
      if (up && v > gmax) { gmax = v; gi = lane + 64 * e; }
    }
    av::wave_argmax(gmax, gi);
    if (gi == NONE) break;
    const int i = gi;
    const float Kii = Ks[i][i];
    float best = -INFINITY, gmax2 = -INFINITY;
    int bj = NONE;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int t = lane + 64 * e;
      const bool low = y[e] > 0.f ? a[e] > 0.f : (y[e] < 0.f && a[e] < C);
      if (!low) continue;
      const float yg = y[e] * g[e];
      gmax2 = fmaxf(gmax2, yg);
      const float bd = gmax + yg;
      if (bd > 0.f) {
        float q = Kii + qd[e] - 2.f * Ks[i][t];
        q = q > 0.f ? q : TAU;
        const float gain = bd * bd / q;
        if (gain > best) { best = gain; bj = t; }
      }
    }
    gmax2 = av::wave_max(gmax2);
    av::wave_argmax(best, bj);
    if (gmax + gmax2 < epsl || bj == NONE) break;
    const int j = bj;
    // fetch the pair's state from its owner lanes (slot index is wave-uniform)
    const int si = i >> 6, sj = j >> 6;
    float yi = 0.f, ai = 0.f, gi_ = 0.f, yj = 0.f, aj = 0.f, gj = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if (e == si) { yi = __shfl(y[e], i & 63, 64); ai = __shfl(a[e], i & 63, 64); gi_ = __shfl(g[e], i & 63, 64); }
      if (e == sj) { yj = __shfl(y[e], j & 63, 64); aj = __shfl(a[e], j & 63, 64); gj = __shfl(g[e], j & 63, 64); }
    }
    const float oi = ai, oj = aj;
    float quad = Kii + Ks[j][j] - 2.f * Ks[i][j];
    quad = quad > 0.f ? quad : TAU;
    if (yi != yj) {
      const float delta = (-gi_ - gj) / quad, diff = ai - aj;
      ai += delta;
      aj += delta;
      if (diff > 0.f) { if (aj < 0.f) { aj = 0.f; ai = diff; } }
      else if (ai < 0.f) { ai = 0.f; aj = -diff; }
      if (diff > 0.f) { if (ai > C) { ai = C; aj = C - diff; } }
      else if (aj > C) { aj = C; ai = C + diff; }
    } else {
      const float delta = (gi_ - gj) / quad, sum = ai + aj;
      ai -= delta;
      aj += delta;
      if (sum > C) { if (ai > C) { ai = C; aj = sum - C; } }
      else if (aj < 0.f) { aj = 0.f; ai = sum; }
      if (sum > C) { if (aj > C) { aj = C; ai = sum - C; } }
      else if (ai < 0.f) { ai = 0.f; aj = sum; }
    }
    const float di = (ai - oi) * yi, dj = (aj - oj) * yj;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int t = lane + 64 * e;
      if (t == i) a[e] = ai;
      if (t == j) a[e] = aj;
      g[e] += y[e] * (Ks[i][t] * di + Ks[j][t] * dj);
    }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) aall[b * Q + lane + 64 * e] = a[e];
  if (lane == 0) iters[b] = it;
}

}  // namespace

namespace avk {

void smo_solve(const float* K, const float* y, const float* diag, float* alpha, float* G, int B, int N, float C,
               float eps, int max_iter, int* iters, hipStream_t stream) {
  if (B <= 0 || N <= 0) return;
  smo_kernel<<<B, SMO_THREADS, 0, stream>>>(K, y, diag, alpha, G, N, C, eps, max_iter, iters);
  AV_HIP_CHECK(hipGetLastError());
}

int smo_ws_size() { return WS_Q; }

void smo_ws_solve(const float* Kws, const float* yws, float* aws, const float* gws, const float* gap, int B, float C,
                  float eps, int max_iter, int* iters, hipStream_t stream) {
  if (B <= 0) return;
  smo_ws_kernel<<<B, 64, 0, stream>>>(Kws, yws, aws, gws, gap, C, eps, max_iter, iters);
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
