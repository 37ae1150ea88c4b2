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

// index of the first lane whose inclusive prefix >= target (targets in [0, total))
__device__ __forceinline__ int wave_pick(float w, float u01, int A) {
  const float tot = av::wave_sum(w);
  const float cum = wave_incl_scan(w);
  const float target = u01 * tot;
  const unsigned long long m = __ballot(cum > target && w > 0.f);
  return m ? __ffsll((long long)m) - 1 : A - 1;
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
  const bool active = lane < A;
  const long long base = (long long)g * A + lane;
  const int n = active ? trials[base] : 0;
  const float mean = (active && n > 0) ? rsum[base] / (float)n : 0.f;
  const int total = (int)av::wave_sum((unsigned)n);
  const int min_trial = iparam[0];

  for (int b = 0; b < batch; ++b) {
    const av::u4 r = av::philox_draw(seed, round, ((unsigned long long)g * batch + b) * 64 + lane);
    const av::u4 r0 = av::philox_draw(seed, round, ((unsigned long long)g * batch + b) * 64);  // lane-0 stream
    const float u_a = av::u32_to_unit(r0.x), u_b = av::u32_to_unit(r0.y);
    int action = -1;
    // forced exploration: first arm with fewer than min_trial trials
    if (algo != SAMPLE_PROB && min_trial > 0) {
      const unsigned long long under = __ballot(active && n < min_trial);
      if (under) action = __ffsll((long long)under) - 1;
    }
    if (action < 0) {
      float score = -INFINITY;
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
          score = active ? mean : -INFINITY;
          break;
        }
        case UCB1: {
          const float t = (float)max(total, 1);
          score = active ? (n > 0 ? mean + sqrtf(2.f * __logf(t) / (float)n) : INFINITY) : -INFINITY;
          break;
        }
        case UCB2: {
          int* st = istate + (long long)g * 4;
          const int cur = st[0], et = st[1], es = st[2];
          if (cur >= 0 && et < es) {
            action = cur;
          } else {
            const float alpha = fparam[0];
            const int ep = active ? epochs[base] : 0;
            const float tao = ep == 0 ? 1.f : __powf(1.f + alpha, (float)ep);
            const float a = (1.f + alpha) * __logf(2.718281828f * (float)max(total, 1) / tao) / (2.f * tao);
            score = active ? mean + sqrtf(fmaxf(a, 0.f)) : -INFINITY;
          }
          break;
        }
        case SOFTMAX: {
          const float temp = gstate[(long long)g * 4 + 0];
          const float w = active ? __expf(mean / fmaxf(temp, 1e-6f)) : 0.f;
          action = wave_pick(w, u_a, A);
          break;
        }
        case THOMPSON:
        case OPT_THOMPSON: {
          const int min_samples = iparam[2];
          if (total < min_samples) {
            action = min((int)(u_a * (float)A), A - 1);
          } else if (active) {
            float s = thompson_sample(hist + base * nb, nb, bin_width, av::u32_to_unit(r.x), av::u32_to_unit(r.y));
            if (algo == OPT_THOMPSON) s = fmaxf(s, mean);
            score = s;
          }
          break;
        }
        case INTERVAL_EST: {
          // upper bound of the central conf-limit interval of each arm's reward histogram
          const float conf = gstate[(long long)g * 4 + 1];
          if (active) {
            const unsigned* h = hist + base * nb;
            unsigned tot = 0;
            for (int k = 0; k < nb; ++k) tot += h[k];
            if (tot == 0) {
              score = INFINITY;
            } else {
              const float target = (0.5f + 0.5f * conf / 100.f) * (float)tot;
              float cum = 0.f, ub = ((float)nb - 0.5f) * bin_width;
              for (int k = 0; k < nb; ++k) {
                cum += (float)h[k];
                if (cum >= target) { ub = ((float)k + 1.f) * bin_width; break; }
              }
              score = ub;
            }
          }
          break;
        }
        case SAMPLE_PROB: {
          const float w = active ? probs[base] : 0.f;
          action = wave_pick(w, u_a, A);
          break;
        }
        default:
          break;
      }
      if (action < 0) {
        int idx = lane;
        float s = active ? score : -INFINITY;
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
  if (A > 64) throw std::runtime_error("bandit_select: more than 64 arms per group not supported in-kernel");
  bandit_select_kernel<<<(G + 3) / 4, BT, 0, stream>>>(algo, G, A, batch, trials, rsum, probs, hist, nb,
                                                       bin_width, fparam, iparam, gstate, istate, epochs, seed,
                                                       round, out);
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
