// K14 / K15: sequence kernels for CDNA4 (gfx950).
//
// K14  batched log-space Viterbi (and forward log-likelihood): ONE wavefront per sequence, lane j
//      owns state j (j + 64q for S > 64).  Each step is a max-plus (or log-sum-exp) product of the
//      previous [S] vector with the [S, S] log-transition matrix held in LDS: the previous vector is
//      broadcast lane-by-lane with v_readlane (wave-uniform index, no LDS traffic), the column
//      logA[i][j] is a conflict-free LDS read.  Back-pointers go to HBM, lane 0 backtracks.
//      Reference: ViterbiDecoder (probability space, one record at a time),
//      J/markov/ViterbiDecoder.java:53-143, driven by J/markov/ViterbiStatePredictor.java:114-142.
// K15  Markov-chain log-odds classifier: sum over transitions of log(A0[s,s'] / A1[s,s']) with the
//      [S, S] log-ratio table in LDS, one thread per sequence
//      (J/markov/MarkovModelClassifier.java:127-150).
#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

constexpr int VT = 256;  // 4 waves -> 4 sequences per block

template <int QS>
__global__ __launch_bounds__(VT) void viterbi_kernel(const short* __restrict__ obs, long long n, int T, int S,
                                                     int O, const float* __restrict__ logA,
                                                     const float* __restrict__ logB,
                                                     const float* __restrict__ logpi, int mode,
                                                     short* __restrict__ bp, short* __restrict__ path,
                                                     float* __restrict__ score) {
  extern __shared__ __attribute__((aligned(16))) float sA[];  // [S][S]
  for (int i = threadIdx.x; i < S * S; i += VT) sA[i] = logA[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const long long seq = (long long)blockIdx.x * (VT / 64) + (threadIdx.x >> 6);
  if (seq >= n) return;  // wave-uniform exit (after the only block barrier)
  const short* ob = obs + seq * T;
  float delta[QS];
#pragma unroll
  for (int q = 0; q < QS; ++q) {
    const int j = lane + 64 * q;
    const int o0 = ob[0];
    delta[q] = (j < S && o0 >= 0 && o0 < O) ? logpi[j] + logB[(long long)j * O + o0] : -INFINITY;
  }
  int len = (ob[0] >= 0) ? 1 : 0;
  for (int t = 1; t < T; ++t) {
    const int ot = ob[t];
    if (ot < 0 || ot >= O) break;  // wave-uniform (all lanes read the same word)
    float nd[QS];
    short arg[QS];
#pragma unroll
    for (int q = 0; q < QS; ++q) { nd[q] = -INFINITY; arg[q] = 0; }
    if (mode == 0) {
      for (int i = 0; i < S; ++i) {
        // broadcast prev[i] from the lane that owns state i (compile-time register index q)
        float prev = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(delta[0]), i & 63));
#pragma unroll
        for (int q = 1; q < QS; ++q)
          if ((i >> 6) == q) prev = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(delta[q]), i & 63));
#pragma unroll
        for (int q = 0; q < QS; ++q) {
          const int j = lane + 64 * q;
          if (j < S) {
            const float v = prev + sA[i * S + j];
            if (v > nd[q]) { nd[q] = v; arg[q] = (short)i; }
          }
        }
      }
    } else {
      // forward algorithm: log-sum-exp over predecessors (online, numerically stable)
      float se[QS];
#pragma unroll
      for (int q = 0; q < QS; ++q) se[q] = 0.f;
      for (int i = 0; i < S; ++i) {
        float prev = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(delta[0]), i & 63));
#pragma unroll
        for (int q = 1; q < QS; ++q)
          if ((i >> 6) == q) prev = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(delta[q]), i & 63));
#pragma unroll
        for (int q = 0; q < QS; ++q) {
          const int j = lane + 64 * q;
          if (j < S) {
            const float v = prev + sA[i * S + j];
            if (v > nd[q]) { se[q] = se[q] * __expf(nd[q] - v) + 1.f; nd[q] = v; }
            else if (v > -INFINITY) se[q] += __expf(v - nd[q]);
          }
        }
      }
#pragma unroll
      for (int q = 0; q < QS; ++q) nd[q] = (nd[q] > -INFINITY) ? nd[q] + __logf(se[q]) : -INFINITY;
    }
#pragma unroll
    for (int q = 0; q < QS; ++q) {
      const int j = lane + 64 * q;
      if (j < S) {
        delta[q] = nd[q] + logB[(long long)j * O + ot];
        if (mode == 0) bp[(seq * T + t) * S + j] = arg[q];
      }
    }
    ++len;
  }
  // final: best state (Viterbi) or log-sum-exp (forward)
  float best = -INFINITY;
  int barg = 0;
#pragma unroll
  for (int q = 0; q < QS; ++q) {
    const int j = lane + 64 * q;
    if (j < S && delta[q] > best) { best = delta[q]; barg = j; }
  }
  if (mode == 0) {
    av::wave_argmax(best, barg);
    if (lane == 0) {
      score[seq] = best;
      short* pth = path + seq * T;
      for (int t = len; t < T; ++t) pth[t] = -1;
      if (len > 0) {
        int s = barg;
        pth[len - 1] = (short)s;
        for (int t = len - 1; t > 0; --t) {
          s = bp[(seq * T + t) * S + s];
          pth[t - 1] = (short)s;
        }
      }
    }
  } else {
    // wave log-sum-exp of delta
    float m = av::wave_max(best);
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < QS; ++q) {
      const int j = lane + 64 * q;
      if (j < S && delta[q] > -INFINITY) s += __expf(delta[q] - m);
    }
    s = av::wave_sum(s);
    if (lane == 0) score[seq] = (len > 0 && m > -INFINITY) ? m + __logf(s) : -INFINITY;
  }
}

__global__ __launch_bounds__(256) void markov_logodds_kernel(const short* __restrict__ st, long long n, int L,
                                                              const float* __restrict__ lr, int S,
                                                              float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float sL[];
  for (int i = threadIdx.x; i < S * S; i += 256) sL[i] = lr[i];
  __syncthreads();
  const long long stride = (long long)gridDim.x * 256;
  for (long long r = (long long)blockIdx.x * 256 + threadIdx.x; r < n; r += stride) {
    const short* s = st + r * L;
    float acc = 0.f;
    int a = s[0];
    for (int j = 1; j < L; ++j) {
      const int b = s[j];
      if (a < 0 || b < 0 || a >= S || b >= S) break;
      acc += sL[a * S + b];
      a = b;
    }
    out[r] = acc;
  }
}

}  // namespace

namespace avk {

void viterbi(const short* obs, long long n, int T, int S, int O, const float* logA, const float* logB,
             const float* logpi, int mode, short* bp, short* path, float* score, hipStream_t stream) {
  if (n <= 0 || T <= 0) return;
  if ((size_t)S * S * sizeof(float) > 160 * 1024) throw std::runtime_error("viterbi: S too large for LDS");
  const unsigned grid = (unsigned)((n + 3) / 4);
  const size_t lds = (size_t)S * S * sizeof(float);
  if (S <= 64)
    viterbi_kernel<1><<<grid, VT, lds, stream>>>(obs, n, T, S, O, logA, logB, logpi, mode, bp, path, score);
  else if (S <= 128)
    viterbi_kernel<2><<<grid, VT, lds, stream>>>(obs, n, T, S, O, logA, logB, logpi, mode, bp, path, score);
  else if (S <= 192)
    viterbi_kernel<3><<<grid, VT, lds, stream>>>(obs, n, T, S, O, logA, logB, logpi, mode, bp, path, score);
  else
    throw std::runtime_error("viterbi: more than 192 states not supported");
  AV_HIP_CHECK(hipGetLastError());
}

void markov_logodds(const short* states, long long n, int L, const float* lr, int S, float* out,
                    hipStream_t stream) {
  if (n <= 0) return;
  markov_logodds_kernel<<<av::stream_grid(n, 256, 2, 4096), 256, (size_t)S * S * sizeof(float), stream>>>(
      states, n, L, lr, S, out);
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
