// K20: batched multi-armed bandit action selection for CDNA4 (gfx950).
//
// The reference runs one learner object per group, one action at a time (J/reinforce/*Learner.java,
// driven per event by the Storm bolt, J/storm/ReinforcementLearnerBolt.java:97-129, or per group by
// Spark combineByKey, S/reinforce/MultiArmBandit.scala:86-116).  Here thousands of independent
// learners (groups) decide in one launch: one wavefront per group, lane = arm, all per-arm scores
// computed in parallel, argmax / categorical sampling by wave reductions and a wave prefix scan, and
// counter-based Philox randomness (reproducible for a given seed + round, independent of grid shape).
#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

enum Algo : int {
  EPS_GREEDY = 0, UCB1 = 1, UCB2 = 2, SOFTMAX = 3, THOMPSON = 4, OPT_THOMPSON = 5,
  INTERVAL_EST = 6, SAMPLE_PROB = 100
};

constexpr int BT = 256;

// inclusive prefix sum across the 64 lanes
__device__ __forceinline__ float wave_incl_scan(float v) {
  const int l = av::lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float u = __shfl_up(v, o, 64);
    if (l >= o) v += u;
  }
  return v;
}

// Arm k of a group lives on lane k % 64, slot e = k / 64 (E slots per lane: groups of up to 64 E
// arms).  The categorical pick scans the arms in index order: slot 0 of every lane (arms 0..63),
// then slot 1 (arms 64..127), ...; the first arm whose inclusive prefix exceeds the target.
template <int E>
__device__ __forceinline__ int wave_pick(const float (&w)[E], float u01, int A) {
  float part = 0.f;
#pragma unroll
  for (int e = 0; e < E; ++e) part += w[e];
  const float tot = av::wave_sum(part);
  const float target = u01 * tot;
  float run = 0.f;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const float cum = run + wave_incl_scan(w[e]);
    const unsigned long long m = __ballot(cum > target && w[e] > 0.f);
    if (m) return e * 64 + __ffsll((long long)m) - 1;
    run += av::wave_sum(w[e]);
  }
  return A - 1;
}

// inverse-CDF sample of a reward histogram, uniform within the chosen bin (v = position in bin)
__device__ __forceinline__ float thompson_sample(const unsigned* h, int nb, float bin_width, float u, float v) {
  unsigned tot = 0;
  for (int b = 0; b < nb; ++b) tot += h[b];
  if (tot == 0) return v * bin_width;
  const float target = u * (float)tot;
  float cum = 0.f;
  for (int b = 0; b < nb; ++b) {
    cum += (float)h[b];
    if (cum >= target) return ((float)b + v) * bin_width;
  }
  return ((float)nb - 1.f + v) * bin_width;
}

template <int E>
__global__ __launch_bounds__(BT) void bandit_select_kernel(
    int algo, int G, int A, int batch, const int* __restrict__ trials, const float* __restrict__ rsum,
    const float* __restrict__ probs, const unsigned* __restrict__ hist, int nb, float bin_width,
    const float* __restrict__ fparam /*[8]*/, const int* __restrict__ iparam /*[8]*/,
    float* __restrict__ gstate /*[G][4] float state: temperature, conf limit ...*/,
    int* __restrict__ istate /*[G][4] int state: ucb2 current action, epoch trials, epoch size*/,
    int* __restrict__ epochs /*[G][A] ucb2*/, unsigned long long seed, unsigned long long round,
    int* __restrict__ out /*[G][batch]*/) {
  const int lane = av::lane_id();
  const int g = blockIdx.x * (BT / 64) + av::wave_id();
  if (g >= G) return;
  bool active[E];
  int n[E];
  float mean[E];
  long long base[E];
  unsigned own = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int k = e * 64 + lane;
    active[e] = k < A;
    base[e] = (long long)g * A + k;
    n[e] = active[e] ? trials[base[e]] : 0;
    mean[e] = (active[e] && n[e] > 0) ? rsum[base[e]] / (float)n[e] : 0.f;
    own += (unsigned)n[e];
  }
  const int total = (int)av::wave_sum(own);
  const int min_trial = iparam[0];

  for (int b = 0; b < batch; ++b) {
    const unsigned long long slot0 = ((unsigned long long)g * batch + b) * E * 64;
    const av::u4 r0 = av::philox_draw(seed, round, slot0);  // lane-0 stream
    const float u_a = av::u32_to_unit(r0.x), u_b = av::u32_to_unit(r0.y);
    int action = -1;
    // forced exploration: first arm with fewer than min_trial trials
    if (algo != SAMPLE_PROB && min_trial > 0) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const unsigned long long under = __ballot(active[e] && n[e] < min_trial);
        if (under && action < 0) action = e * 64 + __ffsll((long long)under) - 1;
      }
    }
    if (action < 0) {
      float score[E];
#pragma unroll
      for (int e = 0; e < E; ++e) score[e] = -INFINITY;
      switch (algo) {
        case EPS_GREEDY: {
          // eps(t): none / linear / logLinear reduction with a floor (RandomGreedyLearner)
          const float p0 = fparam[0], c = fparam[1], pmin = fparam[2];
          const int red = iparam[1];
          const float t = (float)max(total, 1);
          float eps = p0;
          if (red == 1) eps = p0 * c / t;
          else if (red == 2) eps = p0 * c * __logf(t) / t;
          eps = fminf(eps, p0);
          if (pmin > 0.f) eps = fmaxf(eps, pmin);
          if (u_a < eps) action = min((int)(u_b * (float)A), A - 1);
#pragma unroll
          for (int e = 0; e < E; ++e) score[e] = active[e] ? mean[e] : -INFINITY;
          break;
        }
        case UCB1: {
          const float t = (float)max(total, 1);
#pragma unroll
          for (int e = 0; e < E; ++e)
            score[e] = active[e] ? (n[e] > 0 ? mean[e] + sqrtf(2.f * __logf(t) / (float)n[e]) : INFINITY) : -INFINITY;
          break;
        }
        case UCB2: {
          int* st = istate + (long long)g * 4;
          const int cur = st[0], et = st[1], es = st[2];
          if (cur >= 0 && et < es) {
            action = cur;
          } else {
            const float alpha = fparam[0];
#pragma unroll
            for (int e = 0; e < E; ++e) {
              const int ep = active[e] ? epochs[base[e]] : 0;
              const float tao = ep == 0 ? 1.f : __powf(1.f + alpha, (float)ep);
              const float a = (1.f + alpha) * __logf(2.718281828f * (float)max(total, 1) / tao) / (2.f * tao);
              score[e] = active[e] ? mean[e] + sqrtf(fmaxf(a, 0.f)) : -INFINITY;
            }
          }
          break;
        }
        case SOFTMAX: {
          const float temp = gstate[(long long)g * 4 + 0];
          float w[E];
#pragma unroll
          for (int e = 0; e < E; ++e) w[e] = active[e] ? __expf(mean[e] / fmaxf(temp, 1e-6f)) : 0.f;
          action = wave_pick<E>(w, u_a, A);
          break;
        }
        case THOMPSON:
        case OPT_THOMPSON: {
          const int min_samples = iparam[2];
          if (total < min_samples) {
            action = min((int)(u_a * (float)A), A - 1);
          } else {
#pragma unroll
            for (int e = 0; e < E; ++e) {
              if (!active[e]) continue;
              const av::u4 r = av::philox_draw(seed, round, slot0 + e * 64 + lane);
              float sv = thompson_sample(hist + base[e] * nb, nb, bin_width, av::u32_to_unit(r.x),
                                         av::u32_to_unit(r.y));
              if (algo == OPT_THOMPSON) sv = fmaxf(sv, mean[e]);
              score[e] = sv;
            }
          }
          break;
        }
        case INTERVAL_EST: {
          // upper bound of the central conf-limit interval of each arm's reward histogram
          const float conf = gstate[(long long)g * 4 + 1];
#pragma unroll
          for (int e = 0; e < E; ++e) {
            if (!active[e]) continue;
            const unsigned* h = hist + base[e] * nb;
            unsigned tot = 0;
            for (int k = 0; k < nb; ++k) tot += h[k];
            if (tot == 0) {
              score[e] = INFINITY;
            } else {
              const float target = (0.5f + 0.5f * conf / 100.f) * (float)tot;
              float cum = 0.f, ub = ((float)nb - 0.5f) * bin_width;
              for (int k = 0; k < nb; ++k) {
                cum += (float)h[k];
                if (cum >= target) { ub = ((float)k + 1.f) * bin_width; break; }
              }
              score[e] = ub;
            }
          }
          break;
        }
        case SAMPLE_PROB: {
          float w[E];
#pragma unroll
          for (int e = 0; e < E; ++e) w[e] = active[e] ? probs[base[e]] : 0.f;
          action = wave_pick<E>(w, u_a, A);
          break;
        }
        default:
          break;
      }
      if (action < 0) {
        // this lane's best arm (lowest index on ties: slots ascend with the arm index), then the
        // wave argmax (lowest index on ties)
        float s = active[0] ? score[0] : -INFINITY;
        int idx = lane;
#pragma unroll
        for (int e = 1; e < E; ++e)
          if (active[e] && score[e] > s) { s = score[e]; idx = e * 64 + lane; }
        av::wave_argmax(s, idx);
        action = idx;
      }
    }
    if (lane == 0) {
      out[(long long)g * batch + b] = action;
      if (algo == UCB2) {
        int* st = istate + (long long)g * 4;
        if (st[0] == action && st[1] < st[2]) {
          st[1] += 1;
        } else {
          const float alpha = fparam[0];
          const int ep = epochs[(long long)g * A + action];
          int es = (int)rintf(__powf(1.f + alpha, (float)(ep + 1)) - __powf(1.f + alpha, (float)ep));
          st[0] = action;
          st[1] = 1;
          st[2] = es < 1 ? 1 : es;
          epochs[(long long)g * A + action] = ep + 1;
        }
      }
    }
  }
}

}  // namespace

namespace avk {

void bandit_select(int algo, int G, int A, int batch, const int* trials, const float* rsum, const float* probs,
                   const unsigned* hist, int nb, float bin_width, const float* fparam, const int* iparam,
                   float* gstate, int* istate, int* epochs, unsigned long long seed, unsigned long long round,
                   int* out, hipStream_t stream) {
  if (G <= 0) return;
  const int E = (A + 63) / 64;
  auto go = [&](auto kern) {
    kern<<<(G + 3) / 4, BT, 0, stream>>>(algo, G, A, batch, trials, rsum, probs, hist, nb, bin_width, fparam, iparam,
                                         gstate, istate, epochs, seed, round, out);
  };
  if (E <= 1) go(bandit_select_kernel<1>);
  else if (E <= 2) go(bandit_select_kernel<2>);
  else if (E <= 4) go(bandit_select_kernel<4>);
  else if (E <= 8) go(bandit_select_kernel<8>);
  else if (E <= 16) go(bandit_select_kernel<16>);
  else throw std::runtime_error("bandit_select: at most 1024 arms per group");
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
