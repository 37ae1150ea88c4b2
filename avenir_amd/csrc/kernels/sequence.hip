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
#include <cstdlib>

#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

constexpr int VT = 256;  // 4 waves -> 4 sequences per block

struct ViterbiArgs {
  const short* obs;    // [rows, T] observations, a negative value ends the sequence
  long long n;         // sequences, one wavefront each
  long long obs_div;   // sequence s reads observation row s / obs_div
  long long pi_mod;    // sequence s starts from logpi row s % pi_mod
  int T, S, O, mode;   // mode 0 Viterbi (max-plus), 1 forward (log-sum-exp)
  const float* logA;   // [S, S]
  const float* logB;   // [S, O]
  const float* logpi;  // [pi_mod, S]
  short* bp;           // [n, T, S] back-pointers, or null
  short* path;         // [n, T] decoded path (needs bp), or null
  float* score;        // [n], or null
  float* delta_out;    // [n, S] final delta vector, or null
};

template <int QS>
__global__ __launch_bounds__(VT) void viterbi_kernel(const ViterbiArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sA[];  // [S][S]
  const int S = a.S, T = a.T, O = a.O, mode = a.mode;
  for (int i = threadIdx.x; i < S * S; i += VT) sA[i] = a.logA[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const long long seq = (long long)blockIdx.x * (VT / 64) + (threadIdx.x >> 6);
  if (seq >= a.n) return;  // wave-uniform exit (after the only block barrier)
  const short* ob = a.obs + (seq / a.obs_div) * T;
  const float* logpi = a.logpi + (seq % a.pi_mod) * S;
  const float* logB = a.logB;
  short* bp = a.bp;
  float delta[QS];
#pragma unroll
  for (int q = 0; q < QS; ++q) {
    const int j = lane + 64 * q;
    const int o0 = ob[0];
    delta[q] = (j < S && o0 >= 0 && o0 < O) ? logpi[j] + logB[(long long)j * O + o0] : -INFINITY;
  }
  // an invalid first observation ends the sequence before it starts (len 0, as the host oracle)
  int len = (ob[0] >= 0 && ob[0] < O) ? 1 : 0;
  for (int t = 1; len > 0 && t < T; ++t) {
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
        if (bp) bp[(seq * T + t) * S + j] = arg[q];
      }
    }
    ++len;
  }
  if (a.delta_out) {
#pragma unroll
    for (int q = 0; q < QS; ++q) {
      const int j = lane + 64 * q;
      if (j < S) a.delta_out[seq * S + j] = delta[q];
    }
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
      if (a.score) a.score[seq] = best;
      if (a.path) {
        short* pth = a.path + seq * T;
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
    if (lane == 0 && a.score) a.score[seq] = (len > 0 && m > -INFINITY) ? m + __logf(s) : -INFINITY;
  }
}

// Small state spaces (S <= SP <= 32): 64 / SP sequences share one wavefront, lane group g owns
// sequence g and lane j of the group state j (the one-sequence-per-wave kernel left 56 of 64 lanes
// idle at S = 8).  prev[i] comes from the group's lane i by a shuffle; a group whose sequence ended
// keeps its delta and stops counting; the wave leaves the time loop when no group is active.
template <int SP>
__global__ __launch_bounds__(VT) void viterbi_small_kernel(const ViterbiArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sA[];  // [S][S]
  constexpr int G = 64 / SP;
  const int S = a.S, T = a.T, O = a.O, mode = a.mode;
  for (int i = threadIdx.x; i < S * S; i += VT) sA[i] = a.logA[i];
  __syncthreads();
  const int lane = threadIdx.x & 63, grp = lane / SP, j = lane % SP, base = grp * SP;
  const long long seq = ((long long)blockIdx.x * (VT / 64) + (threadIdx.x >> 6)) * G + grp;
  const bool live = seq < a.n;
  const bool js = live && j < S;
  const short* ob = a.obs + (live ? (seq / a.obs_div) * T : 0);
  const float* logpi = a.logpi + (live ? (seq % a.pi_mod) * S : 0);
  const float* logB = a.logB;
  short* bp = a.bp;
  const int o0 = live ? ob[0] : -1;
  float delta = (js && o0 >= 0 && o0 < O) ? logpi[j] + logB[(long long)j * O + o0] : -INFINITY;
  int len = (live && o0 >= 0 && o0 < O) ? 1 : 0;
  bool act = len > 0;  // an invalid first observation: an empty sequence
  for (int t = 1; t < T; ++t) {
    const int ot = act ? ob[t] : -1;
    if (ot < 0 || ot >= O) act = false;
    if (!__any(act)) break;
    float nd = -INFINITY, se = 0.f;
    short arg = 0;
    for (int i = 0; i < S; ++i) {
      const float prev = __shfl(delta, base + i, 64);
      const float v = prev + (j < S ? sA[i * S + (j < S ? j : 0)] : 0.f);
      if (mode == 0) {
        if (v > nd) { nd = v; arg = (short)i; }
      } else {
        if (v > nd) { se = se * __expf(nd - v) + 1.f; nd = v; }
        else if (v > -INFINITY) se += __expf(v - nd);
      }
    }
    if (mode != 0) nd = (nd > -INFINITY) ? nd + __logf(se) : -INFINITY;
    if (act && j < S) {
      delta = nd + logB[(long long)j * O + ot];
      if (bp) bp[(seq * T + t) * S + j] = arg;
    }
    if (act) ++len;
  }
  if (a.delta_out && js) a.delta_out[seq * S + j] = delta;
  float best = js ? delta : -INFINITY;
  int barg = js ? j : 0;
#pragma unroll
  for (int o = SP / 2; o > 0; o >>= 1) {  // group argmax, ties -> lowest state (as wave_argmax)
    const float v2 = __shfl_xor(best, o, 64);
    const int i2 = __shfl_xor(barg, o, 64);
    if (v2 > best || (v2 == best && i2 < barg)) { best = v2; barg = i2; }
  }
  if (mode == 0) {
    if (live && j == 0) {
      if (a.score) a.score[seq] = best;
      if (a.path) {
        short* pth = a.path + seq * T;
        for (int t = len; t < T; ++t) pth[t] = -1;
        if (len > 0) {
          int st = barg;
          pth[len - 1] = (short)st;
          for (int t = len - 1; t > 0; --t) {
            st = bp[(seq * T + t) * S + st];
            pth[t - 1] = (short)st;
          }
        }
      }
    }
  } else {
    float m = best;  // group max (best is the group's max after the argmax reduction)
    float e = (js && delta > -INFINITY) ? __expf(delta - m) : 0.f;
#pragma unroll
    for (int o = SP / 2; o > 0; o >>= 1) e += __shfl_xor(e, o, 64);
    if (live && j == 0 && a.score) a.score[seq] = (len > 0 && m > -INFINITY) ? m + __logf(e) : -INFINITY;
  }
}

// Chunked-Viterbi back-tracking (sequence_ops.viterbi_long): thread k follows the back-pointers
// of chunk k / per_chunk from state ends[k] at the chunk's last position down to position 0,
// writing the state reached there (first[k]: the chunk's end -> start map) and / or the path.
__global__ __launch_bounds__(256) void viterbi_backtrack_kernel(const short* __restrict__ bp,
                                                                const int* __restrict__ lens,
                                                                const int* __restrict__ ends, long long ntracks,
                                                                int per_chunk, int T, int S, int* __restrict__ first,
                                                                short* __restrict__ path) {
  const long long k = (long long)blockIdx.x * 256 + threadIdx.x;
  if (k >= ntracks) return;
  const long long c = k / per_chunk;
  const int len = min(max(lens[c], 0), T);
  int s = min(max(ends[k], 0), S - 1);
  const short* b = bp + c * (long long)T * S;
  short* p = path ? path + c * (long long)T : nullptr;
  if (p)
    for (int t = len; t < T; ++t) p[t] = -1;
  if (len == 0) {
    if (first) first[k] = -1;
    return;
  }
  if (p) p[len - 1] = (short)s;
  for (int t = len - 1; t > 0; --t) {
    s = b[(long long)t * S + s];
    if (p) p[t - 1] = (short)s;
  }
  if (first) first[k] = s;
}

static bool small_off() {  // AVMI_VITERBI_SMALL=0: one sequence per wavefront at any S (A/B switch)
  const char* e = std::getenv("AVMI_VITERBI_SMALL");
  return e && e[0] == '0';
}

void launch_viterbi(const ViterbiArgs& a, hipStream_t stream) {
  if (a.n <= 0 || a.T <= 0) return;
  if ((size_t)a.S * a.S * sizeof(float) > 160 * 1024) throw std::runtime_error("viterbi: S too large for LDS");
  const unsigned grid = (unsigned)((a.n + 3) / 4);
  const size_t lds = (size_t)a.S * a.S * sizeof(float);
  if (a.S <= 32 && !small_off()) {  // several sequences per wavefront
    const int sp = a.S <= 8 ? 8 : (a.S <= 16 ? 16 : 32);
    const long long per_block = (VT / 64) * (64 / sp);
    const unsigned g2 = (unsigned)((a.n + per_block - 1) / per_block);
    if (sp == 8) viterbi_small_kernel<8><<<g2, VT, lds, stream>>>(a);
    else if (sp == 16) viterbi_small_kernel<16><<<g2, VT, lds, stream>>>(a);
    else viterbi_small_kernel<32><<<g2, VT, lds, stream>>>(a);
  } else if (a.S <= 64)
    viterbi_kernel<1><<<grid, VT, lds, stream>>>(a);
  else if (a.S <= 128)
    viterbi_kernel<2><<<grid, VT, lds, stream>>>(a);
  else if (a.S <= 192)
    viterbi_kernel<3><<<grid, VT, lds, stream>>>(a);
  else
    throw std::runtime_error("viterbi: more than 192 states not supported");
  AV_HIP_CHECK(hipGetLastError());
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

// Tiled variant: 256 sequences' states staged in LDS by coalesced 2-byte loads (row stride L + 1
// shorts), then every thread walks its own sequence from LDS; the plain kernel's per-thread walk
// touched 64 different rows per load instruction.
__global__ __launch_bounds__(256) void markov_logodds_tiled_kernel(const short* __restrict__ st, long long n, int L,
                                                                    const float* __restrict__ lr, int S,
                                                                    float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float sL[];
  short* tile = reinterpret_cast<short*>(sL + S * S);
  const int LP = L + 1;
  for (int i = threadIdx.x; i < S * S; i += 256) sL[i] = lr[i];
  for (long long r0 = (long long)blockIdx.x * 256; r0 < n; r0 += (long long)gridDim.x * 256) {
    const int rows = (int)min(256LL, n - r0);
    __syncthreads();  // lr staged / the previous tile fully walked
    const short* src = st + r0 * L;
    for (int e = threadIdx.x; e < rows * L; e += 256) tile[(e / L) * LP + e % L] = src[e];
    __syncthreads();
    if (threadIdx.x < rows) {
      const short* s = tile + threadIdx.x * LP;
      float acc = 0.f;
      int a = s[0];
      for (int j = 1; j < L; ++j) {
        const int b = s[j];
        if (a < 0 || b < 0 || a >= S || b >= S) break;
        acc += sL[a * S + b];
        a = b;
      }
      out[r0 + threadIdx.x] = acc;
    }
  }
}

}  // namespace

namespace avk {

void viterbi(const short* obs, long long n, int T, int S, int O, const float* logA, const float* logB,
             const float* logpi, int mode, short* bp, short* path, float* score, hipStream_t stream) {
  const ViterbiArgs a{obs, n, 1, 1, T, S, O, mode, logA, logB, logpi,
                      mode == 0 ? bp : nullptr, mode == 0 ? path : nullptr, score, nullptr};
  launch_viterbi(a, stream);
}

void viterbi_chunks(const short* obs, long long n, long long obs_div, int T, int S, int O, const float* logA,
                    const float* logB, const float* logpi, long long pi_mod, short* bp, float* delta_out,
                    hipStream_t stream) {
  const ViterbiArgs a{obs, n, obs_div, pi_mod, T, S, O, 0, logA, logB, logpi, bp, nullptr, nullptr, delta_out};
  launch_viterbi(a, stream);
}

void viterbi_backtrack(const short* bp, const int* lens, const int* ends, long long ntracks, int per_chunk, int T,
                       int S, int* first, short* path, hipStream_t stream) {
  if (ntracks <= 0 || T <= 0) return;
  viterbi_backtrack_kernel<<<(unsigned)((ntracks + 255) / 256), 256, 0, stream>>>(bp, lens, ends, ntracks, per_chunk,
                                                                                  T, S, first, path);
  AV_HIP_CHECK(hipGetLastError());
}

void markov_logodds(const short* states, long long n, int L, const float* lr, int S, float* out,
                    hipStream_t stream) {
  if (n <= 0) return;
  const size_t tiled = (size_t)S * S * sizeof(float) + (size_t)256 * (L + 1) * sizeof(short);
  const char* e = std::getenv("AVMI_LOGODDS_TILED");
  if (tiled <= 64 * 1024 && !(e && e[0] == '0'))
    markov_logodds_tiled_kernel<<<av::stream_grid(n, 256, 1, 4096), 256, tiled, stream>>>(states, n, L, lr, S, out);
  else
    markov_logodds_kernel<<<av::stream_grid(n, 256, 2, 4096), 256, (size_t)S * S * sizeof(float), stream>>>(
        states, n, L, lr, S, out);
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
