// K7 — split scoring with the reference's split semantics (CDNA4, gfx950).
//
// Reference: SplitManager (J/tree/SplitManager.java:256-522) enumerates, per attribute, every
// multi-way numeric split (up to maxSplit segments over the splitScanInterval points) and every
// categorical set partition; DecisionTreeBuilder (J/tree/DecisionTreeBuilder.java:499-616) scores
// each candidate by the population-weighted impurity (entropy / gini, InfoContentStat) of its
// segments, keeps the best (or a random one among the top ``top.split.count``), and creates one
// child per non-empty segment with that segment's class distribution and impurity.
//
// Here every candidate split of every attribute is a row of ONE split table (feature, histogram
// column of its first bin, bin count, segment count, validity, segment map: one byte per bin), so
// binary thresholds, multi-way numeric splits and categorical partitions are scored by the same
// code.  One workgroup per frontier node of the level:
//   1. the node's [C, TB] class histogram is staged in LDS as fp64 (global reads otherwise);
//   2. each thread scores splits: for every segment it sums the class counts of the segment's bins
//      (CM registers), folds the segment's impurity into the weighted average, counts non-empty
//      segments; invalid / non-candidate / one-segment splits score +inf;
//   3. the k best splits (value, then index: deterministic) by k block-wide argmin passes;
//   4. the chosen splits' segment class counts and segment impurities, written for the host, which
//      only creates the node objects.
// Replaces a torch einsum over [A, S, G, C] fp64 tensors plus a host impurity per child.
#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

constexpr int SP_T = 256;
constexpr int SP_LDS_DOUBLES = 12288;  // 96 KiB: node histogram in LDS when C * TB fits
constexpr int SP_LDS_SCORES = 4096;    // split scores in LDS when R fits (else global scratch)

__device__ __forceinline__ double impurity_of(const double* cnt, int C, int algo, double tot) {
  if (tot <= 0.0) return algo == 0 ? 0.0 : 1.0;   // an empty segment: p = 0 (models/tree.py impurity)
  double s = 0.0;
  if (algo == 0) {  // entropy, base 2
    for (int c = 0; c < C; ++c) {
      const double p = cnt[c] / tot;
      if (p > 0.0) s -= p * log2(p);
    }
    return s;
  }
  for (int c = 0; c < C; ++c) {  // gini
    const double p = cnt[c] / tot;
    s += p * p;
  }
  return 1.0 - s;
}

template <int CM>
__global__ __launch_bounds__(SP_T) void ref_split_score_kernel(const long long* __restrict__ hist, int C, int TBt,
                                                               const int* __restrict__ sp,
                                                               const signed char* __restrict__ seg, int R,
                                                               const unsigned char* __restrict__ cand, int F,
                                                               int algo, int k, int G2, long long* __restrict__ top,
                                                               double* __restrict__ topv, double* __restrict__ segc,
                                                               double* __restrict__ cinfo,
                                                               double* __restrict__ scratch) {
  __shared__ double hs[SP_LDS_DOUBLES];
  __shared__ double sc_l[SP_LDS_SCORES];
  __shared__ double red_v[SP_T / 64];
  __shared__ int red_i[SP_T / 64];
  __shared__ int s_pick;
  const int a = blockIdx.x, tid = threadIdx.x;
  const long long* h = hist + (long long)a * C * TBt;
  const bool in_lds = (long long)C * TBt <= SP_LDS_DOUBLES;
  if (in_lds)
    for (int e = tid; e < C * TBt; e += SP_T) hs[e] = (double)h[e];
  __syncthreads();
  double* sc = R <= SP_LDS_SCORES ? sc_l : scratch + (long long)a * R;
  // count of class c in bin column j of this node
  auto hv = [&](int c, int j) -> double { return in_lds ? hs[c * TBt + j] : (double)h[(long long)c * TBt + j]; };
  for (int r = tid; r < R; r += SP_T) {
    const int* q = sp + 6 * r;
    const int f = q[0], col = q[1], nb = q[2], ns = q[3], valid = q[4], soff = q[5];
    double score = INFINITY;
    if (valid && cand[(long long)a * F + f]) {
      double wsum = 0.0, tot = 0.0;
      int nonempty = 0;
      for (int g = 0; g < ns; ++g) {
        double cnt[CM];
#pragma unroll
        for (int c = 0; c < CM; ++c) cnt[c] = 0.0;
        for (int b = 0; b < nb; ++b)
          if (seg[soff + b] == g) {
#pragma unroll
            for (int c = 0; c < CM; ++c)
              if (c < C) cnt[c] += hv(c, col + b);
          }
        double n = 0.0;
#pragma unroll
        for (int c = 0; c < CM; ++c) n += cnt[c];
        if (n > 0.0) {
          ++nonempty;
          wsum += impurity_of(cnt, C, algo, n) * n;
          tot += n;
        }
      }
      if (nonempty >= 2) score = wsum / fmax(tot, 1.0);
    }
    sc[r] = score;
  }
  __syncthreads();
  // k best (value, index) by block argmin passes
  for (int i = 0; i < k; ++i) {
    double bv = INFINITY;
    int bi = 0x7fffffff;
    for (int r = tid; r < R; r += SP_T) {
      const double v = sc[r];
      if (v < bv || (v == bv && r < bi)) { bv = v; bi = r; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double v2 = __shfl_xor(bv, o, 64);
      const int i2 = __shfl_xor(bi, o, 64);
      if (v2 < bv || (v2 == bv && i2 < bi)) { bv = v2; bi = i2; }
    }
    if ((tid & 63) == 0) { red_v[tid >> 6] = bv; red_i[tid >> 6] = bi; }
    __syncthreads();
    if (tid == 0) {
      double v = red_v[0];
      int ix = red_i[0];
      for (int w = 1; w < SP_T / 64; ++w)
        if (red_v[w] < v || (red_v[w] == v && red_i[w] < ix)) { v = red_v[w]; ix = red_i[w]; }
      if (ix >= R) ix = 0;  // R == 0 cannot happen (host); keeps the index in range
      top[(long long)a * k + i] = ix;
      topv[(long long)a * k + i] = v;
      s_pick = ix;
      sc[ix] = INFINITY;   // exclude from the next pass (a non-finite pick stays non-finite)
    }
    __syncthreads();
    // the pick's segment class counts and segment impurities
    const int r = s_pick;
    const int* q = sp + 6 * r;
    const int col = q[1], nb = q[2], ns = q[3], soff = q[5];
    double* outc = segc + (((long long)a * k + i) * G2) * C;
    for (int e = tid; e < G2 * C; e += SP_T) {
      const int g = e / C, c = e % C;
      double s = 0.0;
      if (g < ns)
        for (int b = 0; b < nb; ++b)
          if (seg[soff + b] == g) s += hv(c, col + b);
      outc[e] = s;
    }
    __syncthreads();
    for (int g = tid; g < G2; g += SP_T) {
      double cnt[CM];
      double n = 0.0;
#pragma unroll
      for (int c = 0; c < CM; ++c) {
        cnt[c] = c < C ? outc[g * C + c] : 0.0;
        n += cnt[c];
      }
      cinfo[((long long)a * k + i) * G2 + g] = impurity_of(cnt, C, algo, n);
    }
    __syncthreads();
  }
}

}  // namespace

namespace avk {

void ref_split_score(const long long* hist, int A, int C, int TBt, const int* sp, const signed char* seg, int R,
                     const unsigned char* cand, int F, int algo, int k, int G2, long long* top, double* topv,
                     double* segc, double* cinfo, double* scratch, hipStream_t stream) {
  if (A <= 0) return;
  if (R <= 0 || k <= 0) throw std::runtime_error("ref_split_score: need splits and k >= 1");
  if (R > SP_LDS_SCORES && !scratch) throw std::runtime_error("ref_split_score: scratch required for > 4096 splits");
#define AV_SPS(CM) \
  ref_split_score_kernel<CM><<<A, SP_T, 0, stream>>>(hist, C, TBt, sp, seg, R, cand, F, algo, k, G2, top, topv, segc, cinfo, scratch)
  if (C <= 2) AV_SPS(2);
  else if (C <= 4) AV_SPS(4);
  else if (C <= 8) AV_SPS(8);
  else if (C <= 16) AV_SPS(16);
  else if (C <= 32) AV_SPS(32);
  else throw std::runtime_error("ref_split_score: at most 32 classes");
#undef AV_SPS
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
