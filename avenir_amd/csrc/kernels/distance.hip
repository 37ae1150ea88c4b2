// K9 / K11: pairwise distance + fused top-k on MFMA, and cluster accumulation (CDNA4, gfx950).
//
// Replaces the reference's all-pairs distance stage (the external sifarish SameTypeSimilarity job
// driven by resource/knn.sh, and spark RecordSimilarity's bucket-pair replication,
// S/similarity/RecordSimilarity.scala:80-188) followed by a secondary-sort top-k reducer
// (J/knn/NearestNeighbor.java:317-406, S/similarity/NearestRecords.scala:97-125): the N x M distance
// matrix is never materialised.  k-means assignment (J/cluster/KmeansCluster.java:154-172) is the
// k = 1 case of the same kernel.
//
// Block = 256 threads = 4 waves, a 64-query x 64-reference tile per step.  Each wave computes a
// 32 x 32 block of dot products with the exact f32-input MFMA v_mfma_f32_32x32x2_f32 (bit-exact
// fmaf chain), references as the A operand and queries as the B operand, so each lane's 16
// accumulators are 16 reference distances of ONE query: ||q||^2 + ||r||^2 - 2 q.r goes straight
// from the accumulators into that lane's register-resident sorted top-K (insertion is rare once
// the list has warmed up) — no LDS distance tile, no barrier before the scan.  The query block
// stays in LDS for D <= 256; reference chunks are register-prefetched one step ahead.  The four
// partial lists of a query (2 waves x 2 lane halves) are merged at the end in LDS aliased over the
// tiles.  L1 / Lp metrics run the same tile on the VALU (4 x 4 distances per thread) through an
// LDS distance tile scanned by 4 threads per query.
#include "avenir_common.h"
#include <cmath>
#include "avenir_kernels.h"
#include "avenir_sbf16.h"

namespace {

constexpr int KT = 256;   // threads
constexpr int BQ = 64;    // queries per block
constexpr int BR = 64;    // references per tile
constexpr int KC = 32;    // feature chunk staged in LDS (multiple of 2: MFMA K = 2)

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int N>
__device__ __forceinline__ float sq_norm(const float* __restrict__ row, float acc) {
#pragma unroll
  for (int c = 0; c < N; ++c) acc = fmaf(row[c], row[c], acc);
  return acc;
}

// A[i = lane&31][k = lane>>5] from the query row, B[k = lane>>5][j = lane&31] from the reference row
template <int N>
__device__ __forceinline__ f32x16 mfma_chunk(const float* __restrict__ qrow, const float* __restrict__ rrow, int lk,
                                             f32x16 acc) {
#pragma unroll
  for (int k = 0; k < N; k += 2) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(qrow[k + lk], rrow[k + lk], acc, 0, 0, 0);
  return acc;
}

// the same chunk on the bf16 matrix cores (avenir_sbf16.h): each lane splits its 8 consecutive
// features of the reference row (A) and of the query row (B) into NS bf16 terms per 16 k — the
// fp32 LDS image (and the norms read from it) is unchanged
template <int N, int NS>
__device__ __forceinline__ f32x16 mfma_chunk_sb(const float* __restrict__ rrow, const float* __restrict__ qrow, int lh,
                                                f32x16 acc) {
#pragma unroll
  for (int k = 0; k < N; k += 16) {
    float a[8], b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      a[j] = rrow[k + lh + j];
      b[j] = qrow[k + lh + j];
    }
    sbf::u32x4 ta[NS], tb[NS];
    sbf::split8<NS>(a, ta);
    sbf::split8<NS>(b, tb);
    sbf::bf16x8 fa[NS], fb[NS];
#pragma unroll
    for (int t = 0; t < NS; ++t) {
      fa[t] = sbf::frag(ta[t]);
      fb[t] = sbf::frag(tb[t]);
    }
    sbf::mfma32_terms<NS>(fa, fb, acc);
  }
  return acc;
}

template <int K>
__device__ __forceinline__ void topk_insert(float (&bd)[K], int (&bi)[K], float d, int j) {
  if (d < bd[K - 1]) {
    bd[K - 1] = d;
    bi[K - 1] = j;
#pragma unroll
    for (int s = K - 1; s > 0; --s) {
      if (bd[s] < bd[s - 1]) {
        const float td = bd[s]; bd[s] = bd[s - 1]; bd[s - 1] = td;
        const int ti = bi[s]; bi[s] = bi[s - 1]; bi[s - 1] = ti;
      }
    }
  }
}

// LDS carve (dynamic, 16-byte aligned): the query block (all D features when D <= QRES, so it is
// staged once per block; else one KC chunk), the reference chunk, the distance tile (VALU
// metrics) and the norms, and — aliased over them once the scan is done — the per-query merge
// lists.  qstride = the query rows' LDS stride in floats (padded by one against bank conflicts).
constexpr int QRES = 256;
__host__ __device__ inline int knn_qstride(int D) { return (D <= QRES ? ((D + KC - 1) / KC) * KC : KC) + 1; }
// the distance tile sD exists only for the VALU metrics (MET 1 / 2 scan it for the top-k)
__host__ __device__ inline int knn_off_sr(int qs) { return BQ * qs * 4; }
__host__ __device__ inline int knn_off_sd(int qs) { return knn_off_sr(qs) + BR * (KC + 1) * 4; }
__host__ __device__ inline bool knn_valu(int met) { return met == 1 || met == 2; }
__host__ __device__ inline int knn_off_qn(int qs, int met) { return knn_off_sd(qs) + (knn_valu(met) ? BQ * (BR + 1) * 4 : 0); }
__host__ __device__ inline int knn_off_rn(int qs, int met) { return knn_off_qn(qs, met) + BQ * 4; }
__host__ __device__ inline int knn_lds_bytes(int K, int D, int met) {
  const int main = knn_off_rn(knn_qstride(D), met) + BR * 4;
  return main > BQ * 4 * K * 8 ? main : BQ * 4 * K * 8;
}

// MET: 0 = squared euclidean on MFMA (||q||^2 + ||r||^2 - 2 q.r), 1 = L1 (VALU), 2 = sum |q - r|^p
// (VALU; the caller takes the p-th root of the selected values — the order is the same), 3 / 4 =
// squared euclidean with the dot products in split-bf16 x3 / x6 on the bf16 MFMA.
template <int K, int MET>
__global__ __launch_bounds__(KT) void knn_mfma_kernel(
    const float* __restrict__ Q, long long M, const float* __restrict__ R, long long N, int D,
    long long r_per_split, long long q_index_base, long long r_index_base, int exclude_self,
    float* __restrict__ out_d, long long* __restrict__ out_i, int kk, float pw) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int qs = knn_qstride(D);
  float* sQ = reinterpret_cast<float*>(smem);  // row i at sQ + i * qs
  float(*sR)[KC + 1] = reinterpret_cast<float(*)[KC + 1]>(smem + knn_off_sr(qs));
  float(*sD)[BR + 1] = reinterpret_cast<float(*)[BR + 1]>(smem + knn_off_sd(qs));
  float* sqn = reinterpret_cast<float*>(smem + knn_off_qn(qs, MET));
  float* srn = reinterpret_cast<float*>(smem + knn_off_rn(qs, MET));
  float(*mD)[4][K] = reinterpret_cast<float(*)[4][K]>(smem);
  int(*mI)[4][K] = reinterpret_cast<int(*)[4][K]>(smem + BQ * 4 * K * 4);

  constexpr bool EU = MET == 0 || MET >= 3;  // squared euclidean on the matrix cores
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wq = wave >> 1, wr = wave & 1;
  const long long q0 = (long long)blockIdx.x * BQ;
  const long long rb = (long long)blockIdx.y * r_per_split;
  const long long re = min(N, rb + r_per_split);

  // Norms are accumulated from the LDS-staged chunks (threads 0..63: reference rows, 64..127:
  // query rows on the first reference tile), in the same d order as a plain fmaf loop; a direct
  // per-thread loop over D global loads serialised one memory latency per feature per tile.
  float qn_acc = 0.f;

  float bd[K];
  int bi[K];
#pragma unroll
  for (int s = 0; s < K; ++s) { bd[s] = INFINITY; bi[s] = -1; }
  // top-k owner of each (query, partial list): MET 0 takes candidates straight from the MFMA
  // accumulator (lane = one query column, 16 reference rows), the VALU metrics from the sD tile
  const int my_q = EU ? (wq * 32 + (lane & 31)) : (tid >> 2);
  const int part = EU ? (wr * 2 + (lane >> 5)) : (tid & 3);

  // A query block whose features fit one chunk is staged once; reference chunks are prefetched
  // into registers one step ahead (the global loads of the next chunk / tile are in flight during
  // the MFMAs and the top-k scan of the current one).
  const bool q_once = D <= QRES;  // the whole query block resident in LDS
  const int nchunk = (D + KC - 1) / KC;
  float pr[BR * KC / KT];
  auto load_r = [&](long long rr0, int dd0) {
#pragma unroll
    for (int i = 0; i < BR * KC / KT; ++i) {
      const int e = tid + KT * i, row = e / KC, c = e % KC;
      const long long r = rr0 + row;
      pr[i] = (r < re && dd0 + c < D) ? R[r * D + dd0 + c] : 0.f;
    }
  };
  if (q_once) {
    const int qc = qs - 1;
    for (int e = tid; e < BQ * qc; e += KT) {
      const int row = e / qc, c = e % qc;
      const long long q = q0 + row;
      sQ[row * qs + c] = (q < M && c < D) ? Q[q * D + c] : 0.f;
    }
  }
  if (rb < re) load_r(rb, 0);
  for (long long r0 = rb; r0 < re; r0 += BR) {
    const bool first_tile = r0 == rb;
    float rn_acc = 0.f;
    f32x16 acc;  // MET 0: the wave's 32 x 32 MFMA block; MET 1/2: this thread's 4 x 4 block
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    const int tq = tid >> 4, tr = tid & 15;  // VALU block: queries tq + 16 a, references tr + 16 b
    for (int ci = 0; ci < nchunk; ++ci) {
      const int d0 = ci * KC;
      const int kend = min(KC, D - d0);
      __syncthreads();  // previous chunk's (and tile's) LDS reads are done
      if (!q_once)
        for (int e = tid; e < BQ * KC; e += KT) {
          const int row = e / KC, c = e % KC;
          const long long q = q0 + row;
          sQ[row * qs + c] = (q < M && d0 + c < D) ? Q[q * D + d0 + c] : 0.f;
        }
      const int qo = q_once ? d0 : 0;  // this chunk's column offset in the query rows
#pragma unroll
      for (int i = 0; i < BR * KC / KT; ++i) {
        const int e = tid + KT * i;
        sR[e / KC][e % KC] = pr[i];
      }
      __syncthreads();
      if (ci + 1 < nchunk) load_r(r0, d0 + KC);
      else if (r0 + BR < re) load_r(r0 + BR, 0);
      if constexpr (EU) {
        // norms over a half or a whole chunk; the MFMA chain always covers the whole (zero-padded)
        // chunk: a second, half-length unrolled chain cost more in VGPRs / occupancy than the
        // skipped MFMAs saved (measured at D = 16 and 32)
        const bool half = kend <= KC / 2;
        if (tid < BR) {
          rn_acc = half ? sq_norm<KC / 2>(sR[tid], rn_acc) : sq_norm<KC>(sR[tid], rn_acc);
        } else if (first_tile && tid < BR + BQ) {
          qn_acc = half ? sq_norm<KC / 2>(sQ + (tid - BR) * qs + qo, qn_acc)
                        : sq_norm<KC>(sQ + (tid - BR) * qs + qo, qn_acc);
        }
        const int li = lane & 31, lk = lane >> 5;
        // A = references (rows of the 32 x 32 block), B = queries (columns): each lane's 16
        // accumulators are 16 reference distances of ONE query
        if constexpr (MET == 0) acc = mfma_chunk<KC>(sR[wr * 32 + li], sQ + (wq * 32 + li) * qs + qo, lk, acc);
        else acc = mfma_chunk_sb<KC, MET == 3 ? 2 : 3>(sR[wr * 32 + li], sQ + (wq * 32 + li) * qs + qo, lk * 8, acc);
      } else {
        for (int c = 0; c < kend; ++c) {
          float qa[4], rv[4];
#pragma unroll
          for (int a = 0; a < 4; ++a) qa[a] = sQ[(tq + 16 * a) * qs + qo + c];
#pragma unroll
          for (int b = 0; b < 4; ++b) rv[b] = sR[tr + 16 * b][c];
#pragma unroll
          for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b) {
              const float df = fabsf(qa[a] - rv[b]);
              acc[a * 4 + b] += (MET == 1) ? df : __powf(df, pw);
            }
        }
      }
    }
    if constexpr (EU) {
      if (tid < BR) srn[tid] = rn_acc;
      else if (first_tile && tid < BR + BQ) sqn[tid - BR] = qn_acc;
      __syncthreads();
      // accumulator -> distances -> this lane's top-k, no LDS round trip
      // (C/D map: col = lane&31 = query, row = (r&3) + 8(r>>2) + 4(lane>>5) = reference)
      const long long gq = q0 + my_q;
      const float qn = gq < M ? sqn[my_q] : INFINITY;  // padded query rows never insert
      const int jb = (int)(r0 - rb) + wr * 32 + 4 * (lane >> 5);
      if (r0 + BR <= re && !exclude_self) {
        // full tile, no self exclusion (uniform): the lane's 16 distances, then ONE test of their
        // minimum against the current k-th best — once the lists have filled, a tile rarely holds
        // a better candidate, and the per-candidate compare-and-branch was the kernel's VALU / SALU
        // bound at small D
        float dv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int ro = (r & 3) + 8 * (r >> 2);
          dv[r] = fmaxf(fmaf(-2.f, acc[r], qn + srn[wr * 32 + 4 * (lane >> 5) + ro]), 0.f);
        }
        float mn = dv[0];
#pragma unroll
        for (int r = 1; r < 16; ++r) mn = fminf(mn, dv[r]);
        if (mn < bd[K - 1]) {
#pragma unroll 2
          for (int r = 0; r < 16; ++r) topk_insert<K>(bd, bi, dv[r], jb + (r & 3) + 8 * (r >> 2));
        }
      } else {
#pragma unroll 2
        for (int r = 0; r < 16; ++r) {
          const int ro = (r & 3) + 8 * (r >> 2);
          const int rj = wr * 32 + 4 * (lane >> 5) + ro;
          const long long gr = r0 + rj;
          float dist = fmaxf(fmaf(-2.f, acc[r], qn + srn[rj]), 0.f);
          if (gr >= re) dist = INFINITY;
          if (exclude_self && (q_index_base + gq) == (r_index_base + gr)) dist = INFINITY;
          topk_insert<K>(bd, bi, dist, jb + ro);
        }
      }
    } else {
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int qi = tq + 16 * a, rj = tr + 16 * b;
          const long long gq = q0 + qi, gr = r0 + rj;
          float dist = acc[a * 4 + b];
          if (gr >= re || gq >= M) dist = INFINITY;
          if (exclude_self && (q_index_base + gq) == (r_index_base + gr)) dist = INFINITY;
          sD[qi][rj] = dist;
        }
    }
    if constexpr (!EU) {
      __syncthreads();
#pragma unroll 4
      for (int c = 0; c < 16; ++c) {
        const int j = part * 16 + c;
        topk_insert<K>(bd, bi, sD[my_q][j], (int)(r0 - rb) + j);
      }
    }
  }
  __syncthreads();  // the merge lists alias the tiles
  // merge the 4 partial lists of each query
#pragma unroll
  for (int s = 0; s < K; ++s) {
    mD[my_q][part][s] = bd[s];
    mI[my_q][part][s] = bi[s];
  }
  __syncthreads();
  if (part == 0) {
    const long long gq = q0 + my_q;
    // each reference split writes its own [M][kk] slab (merged by the caller)
    out_d += (long long)blockIdx.y * M * kk;
    out_i += (long long)blockIdx.y * M * kk;
    if (gq < M) {
      int p[4] = {0, 0, 0, 0};
      for (int s = 0; s < kk; ++s) {
        int best = 0;
        float bv = INFINITY;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const float v = p[w] < K ? mD[my_q][w][p[w]] : INFINITY;
          if (v < bv) { bv = v; best = w; }
        }
        const int li = p[best] < K ? mI[my_q][best][p[best]] : -1;
        out_d[gq * kk + s] = bv;
        out_i[gq * kk + s] = (li >= 0 && bv < INFINITY) ? (r_index_base + rb + li) : -1;
        p[best]++;
      }
    }
  }
}

// Cluster accumulation: sums[k][d] (f64) and counts[k] of the rows assigned to cluster k.
// LDS-privatised (K*D doubles per block when it fits), flushed once per block.
__global__ __launch_bounds__(KT) void cluster_accum_kernel(const float* __restrict__ X, long long N, int D,
                                                           const int* __restrict__ assign, int Kc,
                                                           double* __restrict__ sums,
                                                           unsigned long long* __restrict__ counts,
                                                           int use_lds) {
  extern __shared__ __attribute__((aligned(16))) double s_sum[];
  unsigned int* s_cnt = reinterpret_cast<unsigned int*>(s_sum + (use_lds ? Kc * D : 0));
  if (use_lds) {
    for (int i = threadIdx.x; i < Kc * D; i += KT) s_sum[i] = 0.0;
    for (int i = threadIdx.x; i < Kc; i += KT) s_cnt[i] = 0;
    __syncthreads();
  }
  const long long stride = (long long)gridDim.x * KT;
  for (long long r = (long long)blockIdx.x * KT + threadIdx.x; r < N; r += stride) {
    const int k = assign[r];
    if (k < 0 || k >= Kc) continue;
    if (use_lds) {
      atomicAdd(&s_cnt[k], 1u);
      for (int d = 0; d < D; ++d) atomicAdd(&s_sum[k * D + d], (double)X[r * D + d]);
    } else {
      atomicAdd(&counts[k], 1ull);
      for (int d = 0; d < D; ++d) atomicAdd(&sums[(long long)k * D + d], (double)X[r * D + d]);
    }
  }
  if (use_lds) {
    __syncthreads();
    for (int i = threadIdx.x; i < Kc * D; i += KT)
      if (s_sum[i] != 0.0) atomicAdd(&sums[i], s_sum[i]);
    for (int i = threadIdx.x; i < Kc; i += KT)
      if (s_cnt[i]) atomicAdd(&counts[i], (unsigned long long)s_cnt[i]);
  }
}


// ---------------------------------------------------------------------------------------------
// K10: kernel-weighted class vote over each query's k neighbours (J/knn/Neighborhood.java:150-218,
// NearestNeighbor's class-conditional weighting).  One thread per query; the per-class sums live
// in CMAX registers (the class is matched with an unrolled compare, no dynamic register index), so
// scores, percent probabilities and the decision come out of one pass over the [M, k] lists.
// kern: 0 none, 1 linearMultiplicative, 2 linearAdditive, 3 gaussian.  post_mode: 0 none,
// 1 one posterior per training record, 2 [R, C] posterior (the neighbour's own class column).
// ---------------------------------------------------------------------------------------------
constexpr int VOTE_T = 256;

template <int CMAX>
__global__ __launch_bounds__(VOTE_T) void knn_vote_kernel(
    const float* __restrict__ dist, const long long* __restrict__ idx, long long M, int k,
    const long long* __restrict__ ys, const float* __restrict__ post, int post_mode, int C, int kern,
    float kparam, float scale, float kscale, int invdist, float thr, int pos,
    float* __restrict__ scores, float* __restrict__ prob, long long* __restrict__ pred) {
  const long long q = (long long)blockIdx.x * VOTE_T + threadIdx.x;
  if (q >= M) return;
  float acc[CMAX];
#pragma unroll
  for (int c = 0; c < CMAX; ++c) acc[c] = 0.f;
  const float* dq = dist + q * k;
  const long long* iq = idx + q * k;
  for (int j = 0; j < k; ++j) {
    const long long i = iq[j];
    const float d = dq[j];
    if (i < 0 || isinf(d)) continue;
    const float ds = d * scale;
    float s;
    if (kern == 0) s = 1.f;
    else if (kern == 1) s = ds == 0.f ? 2.f * kscale : kscale / fmaxf(ds, 1e-9f);
    else if (kern == 2) s = kscale - ds;
    else { const float t = ds / kparam; s = kscale * __expf(-0.5f * t * t); }
    if (invdist) s = s / fmaxf(ds, 1.f);
    const long long y = ys[i];
    const int c = (int)(y < 0 ? 0 : (y >= C ? C - 1 : y));
    if (post_mode == 1) s *= post[i];
    else if (post_mode == 2) s *= post[i * C + c];
#pragma unroll
    for (int cc = 0; cc < CMAX; ++cc) acc[cc] += (cc == c) ? s : 0.f;
  }
  float total = 0.f;
  int best = 0;
  float bv = acc[0];
#pragma unroll
  for (int c = 0; c < CMAX; ++c) {
    if (c < C) {
      total += acc[c];
      if (acc[c] > bv) { bv = acc[c]; best = c; }
    }
  }
  float* sq = scores + q * C;
  float* pq = prob + q * C;
#pragma unroll
  for (int c = 0; c < CMAX; ++c) {
    if (c < C) {
      sq[c] = acc[c];
      pq[c] = total > 0.f ? acc[c] * 100.f / total : 0.f;
    }
  }
  if (thr > 0.f && C == 2) {
    const float a = pos ? acc[1] : acc[0], b = pos ? acc[0] : acc[1];
    best = a / fmaxf(b, 1e-12f) > thr ? pos : 1 - pos;
  }
  pred[q] = best;
}

// Mixed-type record distance without one-hot expansion: numeric columns
// pre-scaled by sqrt(w) / range contribute squared differences, categorical columns contribute
// w on a code mismatch, w / 2 when exactly one side is missing (-1) and 0 when both are — exactly
// the squared euclidean distance of ops.distance.encode_mixed's scaled one-hot embedding, so
// results match the MFMA path, but the width is the number of columns, not of categorical values.
//
// The categorical part is folded like the one-hot norms: sum_f w_f/2 ([a_f >= 0] + [b_f >= 0])
// - sum_f w_f [a_f == b_f >= 0], i.e. a per-query constant + a per-reference constant (computed
// once per LDS stage) - one compare-and-add per column.  One thread per query (features in
// registers, column counts padded to DN / DC at compile time: padded numerics are 0 on both sides,
// padded codes never match), 256 reference rows per LDS stage read as 16-byte broadcasts, top-k in
// registers.  The references are split over gridDim.y so that a launch has >= 1024 workgroups
// (a few thousand queries alone fill less than a third of the chip); mixed_knn_merge_kernel merges
// the splits' lists (ties to the lower reference index, as within a split).
constexpr int MX_T = 256;
constexpr int MX_MAXD = 32;

template <int K, int DN, int DC>
__global__ __launch_bounds__(MX_T) void mixed_knn_kernel(const float* __restrict__ Qn, const int* __restrict__ Qc,
                                                         long long nq, const float* __restrict__ Rn,
                                                         const int* __restrict__ Rc, long long nr, int Dn, int Dc,
                                                         const float* __restrict__ wc, long long per,
                                                         float* __restrict__ part_d, int* __restrict__ part_i) {
  constexpr int DNS = DN > 0 ? DN : 4, DCS = DC > 0 ? DC : 4;
  __shared__ __attribute__((aligned(16))) float sRn[MX_T][DNS];
  __shared__ __attribute__((aligned(16))) int sRc[MX_T][DCS];
  __shared__ float sK[MX_T];
  const int tid = threadIdx.x;
  const long long q = (long long)blockIdx.x * MX_T + tid;
  const long long rs = (long long)blockIdx.y * per, re = min(nr, rs + per);
  float w[DCS];
#pragma unroll
  for (int f = 0; f < DCS; ++f) w[f] = f < Dc ? wc[f] : 0.f;
  float qn[DNS];
  int qa[DCS];
  float qconst = 0.f;
#pragma unroll
  for (int f = 0; f < DNS; ++f) qn[f] = (q < nq && f < Dn) ? Qn[q * Dn + f] : 0.f;
#pragma unroll
  for (int f = 0; f < DCS; ++f) {
    const int a = (q < nq && f < Dc) ? Qc[q * Dc + f] : -1;
    qconst += a >= 0 ? 0.5f * w[f] : 0.f;
    qa[f] = a >= 0 ? a : -2;  // a missing query code matches nothing
  }
  float bd[K];
  int bi[K];
#pragma unroll
  for (int s = 0; s < K; ++s) { bd[s] = INFINITY; bi[s] = -1; }
  for (long long r0 = rs; r0 < re; r0 += MX_T) {
    const int rows = (int)min((long long)MX_T, re - r0);
    __syncthreads();  // the previous stage's reads are done
    if (DN > 0)
      for (int e = tid; e < MX_T * DN; e += MX_T) {
        const int j = e / DN, f = e % DN;
        sRn[j][f] = (j < rows && f < Dn) ? Rn[(r0 + j) * Dn + f] : 0.f;
      }
    if (DC > 0)
      for (int e = tid; e < MX_T * DC; e += MX_T) {
        const int j = e / DC, f = e % DC;
        sRc[j][f] = (j < rows && f < Dc) ? Rc[(r0 + j) * Dc + f] : -1;
      }
    __syncthreads();
    if (DC > 0) {  // per-reference constant: w/2 per present code
      float c = 0.f;
#pragma unroll
      for (int f = 0; f < DC; ++f) c += sRc[tid][f] >= 0 ? 0.5f * w[f] : 0.f;
      sK[tid] = c;
    } else {
      sK[tid] = 0.f;
    }
    __syncthreads();
    if (q >= nq) continue;
    for (int j = 0; j < rows; ++j) {
      float d = 0.f;
      if (DN > 0) {
#pragma unroll
        for (int f = 0; f < DN; f += 4) {
          const float4 r = *reinterpret_cast<const float4*>(&sRn[j][f]);
          const float t0 = qn[f] - r.x, t1 = qn[f + 1] - r.y, t2 = qn[f + 2] - r.z, t3 = qn[f + 3] - r.w;
          d = fmaf(t0, t0, d);
          d = fmaf(t1, t1, d);
          d = fmaf(t2, t2, d);
          d = fmaf(t3, t3, d);
        }
      }
      if (DC > 0) {
        float m = 0.f;
#pragma unroll
        for (int f = 0; f < DC; f += 4) {
          const int4 r = *reinterpret_cast<const int4*>(&sRc[j][f]);
          m += qa[f] == r.x ? w[f] : 0.f;
          m += qa[f + 1] == r.y ? w[f + 1] : 0.f;
          m += qa[f + 2] == r.z ? w[f + 2] : 0.f;
          m += qa[f + 3] == r.w ? w[f + 3] : 0.f;
        }
        d += (qconst + sK[j]) - m;
      }
      topk_insert<K>(bd, bi, d, (int)(r0 + j));
    }
  }
  if (q >= nq) return;
  const long long o = ((long long)blockIdx.y * nq + q) * K;
#pragma unroll
  for (int s = 0; s < K; ++s) {
    part_d[o + s] = bd[s];
    part_i[o + s] = bi[s];
  }
}

// per query: the splits' sorted lists, in split (= reference index) order, into the final top-k
template <int K>
__global__ __launch_bounds__(MX_T) void mixed_knn_merge_kernel(const float* __restrict__ part_d,
                                                               const int* __restrict__ part_i, long long nq,
                                                               int splits, int k, long long r_base,
                                                               float* __restrict__ out_d,
                                                               long long* __restrict__ out_i) {
  const long long q = (long long)blockIdx.x * MX_T + threadIdx.x;
  if (q >= nq) return;
  float bd[K];
  int bi[K];
#pragma unroll
  for (int s = 0; s < K; ++s) { bd[s] = INFINITY; bi[s] = -1; }
  for (int sp = 0; sp < splits; ++sp) {
    const long long o = ((long long)sp * nq + q) * K;
    for (int s = 0; s < K; ++s) {
      const int i = part_i[o + s];
      if (i < 0) break;  // a split's list is sorted: the rest is empty
      topk_insert<K>(bd, bi, part_d[o + s], i);
    }
  }
  for (int s = 0; s < k; ++s) {
    const bool ok = s < K && bi[s] >= 0;
    out_d[q * k + s] = ok ? sqrtf(fmaxf(bd[s], 0.f)) : INFINITY;
    out_i[q * k + s] = ok ? (long long)bi[s] + r_base : -1;
  }
}


// ---- pairs within a distance threshold (recordSimilarity) ---------------------------
// The job keeps (i, j) pairs whose scaled, rounded euclidean distance round(sqrt(|a-b|^2) / nf *
// scale) is at most ``thr`` (and j > i in global order for a self-join).  Instead of materialising
// [tile, nB] distance blocks and compacting them with a sort / nonzero per tile, each workgroup
// holds AR A rows in LDS (256 for rows of <= 16 floats, else 64), each lane one B row in registers.
// Almost every pair of a selective join is rejected: ``s_max`` (host-computed, an upper bound of
// the squared distance any kept pair can have) rejects them on the squared distance alone, so the
// division, square root and rounding of the exact test run only for candidates.  The A rows are
// broadcast LDS reads (every lane reads the same row: no bank conflicts), 4 floats per read; the
// differences and squares are packed fp32 (v_pk_add_f32 / v_pk_fma_f32) with 4 rows in flight.
// Kept pairs (key i * nB + j, distance) go to an LDS list with LDS atomics; at the end ONE global
// atomic per workgroup reserves its slots in one of PW_SEGS output segments (workgroup id modulo
// PW_SEGS, each segment's counter on its own 128-byte line).  Round 4 appended every pair with a
// global atomic on one counter: ~800 k same-address atomics serialised at ~11 ns each were the
// kernel's 9 ms (VALU busy 0.29 after the packed-math rewrite, the time unchanged).
constexpr int PW_SEGS = 64, PW_CSTRIDE = 32, PW_LIST = 512;
template <int DMAX, int AR>
__global__ __launch_bounds__(256) void pairs_within_kernel(const float* __restrict__ A, int nA,
                                                           const float* __restrict__ B, int nB, int D, float nf,
                                                           float scale, float thr, float s_max, int tri,
                                                           long long a_base, long long b_base, int* __restrict__ cnt,
                                                           long long seg_cap, long long* __restrict__ outK,
                                                           int* __restrict__ outD, int a_row0) {
  __shared__ float4 As[AR][DMAX / 4];
  __shared__ long long s_key[PW_LIST];
  __shared__ int s_d[PW_LIST];
  __shared__ int s_n, s_base;
  const int a0 = a_row0 + blockIdx.y * AR;
  // self-join: a workgroup whose whole j-range lies at or below its first i keeps nothing (about
  // half the grid of a diagonal block): leave before touching memory (uniform per workgroup)
  if (tri) {
    const long long j_last = b_base + min(nB, (int)(blockIdx.x + 1) * 256) - 1;
    if (j_last <= a_base + a0) return;
  }
  const int seg = (int)((blockIdx.y * (long long)gridDim.x + blockIdx.x) % PW_SEGS);
  int* seg_cnt = cnt + seg * PW_CSTRIDE;
  long long* seg_key = outK + seg * seg_cap;
  int* seg_d = outD + seg * seg_cap;
  float* Af = reinterpret_cast<float*>(As);
  for (int e = threadIdx.x; e < AR * DMAX; e += 256) {   // columns D..DMAX-1 zero (b[] is zero there too)
    const int r = e / DMAX, c = e - r * DMAX;
    Af[e] = (a0 + r < nA && c < D) ? A[(long long)(a0 + r) * D + c] : 0.f;
  }
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  const int j = blockIdx.x * 256 + threadIdx.x;
  const bool active = j < nB;
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 b[DMAX / 2];   // packed pairs
#pragma unroll
  for (int c = 0; c < DMAX / 2; ++c)
    b[c] = f2{active && 2 * c < D ? B[(long long)j * D + 2 * c] : 0.f,
              active && 2 * c + 1 < D ? B[(long long)j * D + 2 * c + 1] : 0.f};
  int na = active ? min(AR, nA - a0) : 0;
  const long long gj = b_base + j;
  if (tri && active) {  // rows r with a_base + a0 + r < gj only (j > i in global order)
    const long long lim = gj - a_base - a0;
    na = lim <= 0 ? 0 : (lim < na ? (int)lim : na);
  }
  auto emit = [&](int r, float s2) {
    const float dist = rintf(sqrtf(s2) / nf * scale);   // torch.round: half to even
    if (dist <= thr) {
      const long long key = (long long)(a0 + r) * nB + j;
      const int k = atomicAdd(&s_n, 1);
      if (k < PW_LIST) {
        s_key[k] = key;
        s_d[k] = (int)dist;
      } else {  // the workgroup's list is full: straight to its segment
        const int g = atomicAdd(seg_cnt, 1);
        if ((long long)g < seg_cap) {
          seg_key[g] = key;
          seg_d[g] = (int)dist;
        }
      }
    }
  };
  auto sqd = [&](int r) {
    f2 acc = f2{0.f, 0.f};
#pragma unroll
    for (int c4 = 0; c4 < DMAX / 4; ++c4) {
      const float4 a = As[r][c4];   // zero beyond D on both sides
      const f2 d0 = f2{a.x, a.y} - b[2 * c4], d1 = f2{a.z, a.w} - b[2 * c4 + 1];
      acc = __builtin_elementwise_fma(d0, d0, acc);
      acc = __builtin_elementwise_fma(d1, d1, acc);
    }
    return acc.x + acc.y;
  };
  int r = 0;
  for (; r + 4 <= na; r += 4) {
    const float s0 = sqd(r), s1 = sqd(r + 1), s2 = sqd(r + 2), s3 = sqd(r + 3);
    if (fminf(fminf(s0, s1), fminf(s2, s3)) <= s_max) {  // one branch per 4 pairs (rarely taken)
      if (s0 <= s_max) emit(r, s0);
      if (s1 <= s_max) emit(r + 1, s1);
      if (s2 <= s_max) emit(r + 2, s2);
      if (s3 <= s_max) emit(r + 3, s3);
    }
  }
  for (; r < na; ++r) {
    const float s0 = sqd(r);
    if (s0 <= s_max) emit(r, s0);
  }
  __syncthreads();
  const int n = min(s_n, PW_LIST);
  if (n == 0) return;  // uniform
  if (threadIdx.x == 0) s_base = atomicAdd(seg_cnt, n);
  __syncthreads();
  const long long base = s_base;
  for (int k = threadIdx.x; k < n; k += 256)
    if (base + k < seg_cap) {
      seg_key[base + k] = s_key[k];
      seg_d[base + k] = s_d[k];
    }
}

}  // namespace

namespace avk {

int knn_mode() {
  static const int mode = sbf::env_mode("AVMI_KNN_MFMA", 6);
  return mode;
}

void knn_topk(const float* Q, long long M, const float* R, long long N, int D, int k,
              long long q_index_base, long long r_index_base, int exclude_self, float* out_d,
              long long* out_i, int splits, int metric, float p, hipStream_t stream, int prec) {
  if (M <= 0 || N <= 0) return;
  if (metric == 0) {  // squared euclidean: fp32 MFMA or the split-bf16 dot products
    const int mode = prec >= 0 ? prec : knn_mode();
    metric = mode == 3 ? 3 : mode == 6 ? 4 : 0;
  }
  const long long per = ((N + splits - 1) / splits + BR - 1) / BR * BR;
  dim3 grid((unsigned)((M + BQ - 1) / BQ), (unsigned)splits);
  auto launch = [&](auto kern, int K) {
    const int lds = knn_lds_bytes(K, D, metric);
    if (lds > 160 * 1024) throw std::runtime_error("knn_topk: LDS carve exceeds 160 KiB");
    AV_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    kern<<<grid, KT, lds, stream>>>(Q, M, R, N, D, per, q_index_base, r_index_base, exclude_self, out_d,
                                    reinterpret_cast<long long*>(out_i), k, p);
  };
#define AV_KNN_MET(MET)                                                  \
  if (k <= 1) launch(knn_mfma_kernel<1, MET>, 1);                        \
  else if (k <= 4) launch(knn_mfma_kernel<4, MET>, 4);                   \
  else if (k <= 8) launch(knn_mfma_kernel<8, MET>, 8);                   \
  else if (k <= 10) launch(knn_mfma_kernel<10, MET>, 10);                \
  else if (k <= 16) launch(knn_mfma_kernel<16, MET>, 16);                \
  else if (k <= 32) launch(knn_mfma_kernel<32, MET>, 32);                \
  else if (k <= 64) launch(knn_mfma_kernel<64, MET>, 64);                \
  else throw std::runtime_error("knn_topk: k > 64 not supported by the fused kernel");
  if (metric == 0) { AV_KNN_MET(0) }
  else if (metric == 1) { AV_KNN_MET(1) }
  else if (metric == 2) { AV_KNN_MET(2) }
  else if (metric == 3) { AV_KNN_MET(3) }
  else if (metric == 4) { AV_KNN_MET(4) }
  else throw std::runtime_error("knn_topk: unknown metric");
#undef AV_KNN_MET
  AV_HIP_CHECK(hipGetLastError());
}


void knn_vote(const float* dist, const long long* idx, long long M, int k, const long long* ys,
              const float* post, int post_mode, int C, int kern, float kparam, float scale, float kscale,
              int invdist, float thr, int pos, float* scores, float* prob, long long* pred, hipStream_t stream) {
  if (M <= 0) return;
  const unsigned grid = (unsigned)((M + VOTE_T - 1) / VOTE_T);
#define AV_VOTE(CM) knn_vote_kernel<CM><<<grid, VOTE_T, 0, stream>>>(dist, idx, M, k, ys, post, post_mode, C, kern, \
      kparam, scale, kscale, invdist, thr, pos, scores, prob, pred)
  if (C <= 2) AV_VOTE(2);
  else if (C <= 4) AV_VOTE(4);
  else if (C <= 8) AV_VOTE(8);
  else if (C <= 16) AV_VOTE(16);
  else if (C <= 32) AV_VOTE(32);
  else if (C <= 64) AV_VOTE(64);
  else throw std::runtime_error("knn_vote: more than 64 classes");
#undef AV_VOTE
  AV_HIP_CHECK(hipGetLastError());
}

int mixed_knn_max_dims() { return MX_MAXD; }

// reference splits: enough workgroups for the chip (>= 1024), each split >= 4096 references
int mixed_knn_splits(long long nq, long long nr) {
  const long long gx = (nq + MX_T - 1) / MX_T;
  long long s = (1024 + gx - 1) / gx;
  s = std::min(s, std::max(1LL, nr / 4096));
  return (int)std::max(1LL, std::min(s, 64LL));
}

void mixed_knn(const float* Qn, const int* Qc, long long nq, const float* Rn, const int* Rc, long long nr, int Dn,
               int Dc, const float* wc, int k, long long r_base, float* out_d, long long* out_i, float* part_d,
               int* part_i, int splits, hipStream_t stream) {
  if (nq <= 0) return;
  if (Dn > MX_MAXD || Dc > MX_MAXD || k < 1 || k > 32) throw std::runtime_error("mixed_knn: dims <= 32, 1 <= k <= 32");
  const long long per = std::max(1LL, (nr + splits - 1) / splits);
  const dim3 grid((unsigned)((nq + MX_T - 1) / MX_T), (unsigned)splits);
  const int KK = k <= 4 ? 4 : k <= 8 ? 8 : k <= 16 ? 16 : 32;
  const int DNP = Dn == 0 ? 0 : Dn <= 4 ? 4 : Dn <= 8 ? 8 : Dn <= 16 ? 16 : 32;
  const int DCP = Dc == 0 ? 0 : Dc <= 4 ? 4 : Dc <= 8 ? 8 : Dc <= 16 ? 16 : 32;
#define AV_MX3(KK_, DN_, DC_) \
  if (KK == KK_ && DNP == DN_ && DCP == DC_) \
    mixed_knn_kernel<KK_, DN_, DC_><<<grid, MX_T, 0, stream>>>(Qn, Qc, nq, Rn, Rc, nr, Dn, Dc, wc, per, part_d, part_i);
#define AV_MXD(KK_, DN_) AV_MX3(KK_, DN_, 0) AV_MX3(KK_, DN_, 4) AV_MX3(KK_, DN_, 8) AV_MX3(KK_, DN_, 16) AV_MX3(KK_, DN_, 32)
#define AV_MXK(KK_) AV_MXD(KK_, 0) AV_MXD(KK_, 4) AV_MXD(KK_, 8) AV_MXD(KK_, 16) AV_MXD(KK_, 32)
  AV_MXK(4) AV_MXK(8) AV_MXK(16) AV_MXK(32)
#undef AV_MXK
#undef AV_MXD
#undef AV_MX3
  AV_HIP_CHECK(hipGetLastError());
  const unsigned mg = (unsigned)((nq + MX_T - 1) / MX_T);
#define AV_MM(KK_) \
  if (KK == KK_) mixed_knn_merge_kernel<KK_><<<mg, MX_T, 0, stream>>>(part_d, part_i, nq, splits, k, r_base, out_d, out_i);
  AV_MM(4) AV_MM(8) AV_MM(16) AV_MM(32)
#undef AV_MM
  AV_HIP_CHECK(hipGetLastError());
}

void cluster_accumulate(const float* X, long long N, int D, const int* assign, int K, double* sums,
                        unsigned long long* counts, hipStream_t stream) {
  if (N <= 0) return;
  const size_t lds = (size_t)K * D * sizeof(double) + (size_t)K * sizeof(unsigned);
  const int use_lds = lds <= 64 * 1024 ? 1 : 0;
  cluster_accum_kernel<<<av::stream_grid(N, KT, 8, 2048), KT, use_lds ? lds : 0, stream>>>(
      X, N, D, assign, K, sums, counts, use_lds);
  AV_HIP_CHECK(hipGetLastError());
}


// pairs (i, j) with round(|a_i - b_j| / nf * scale) <= thr, as keys i * nB + j and distances in
// PW_SEGS segments of seg_cap entries; cnt = PW_SEGS counters PW_CSTRIDE ints apart.  Returns the
// largest segment count (the caller re-runs with a larger seg_cap when it exceeds seg_cap) and
// copies the counts to seg_counts[PW_SEGS] (host).
long long pairs_within(const float* A, int nA, const float* B, int nB, int D, float nf, float scale, float thr, int tri,
                       long long a_base, long long b_base, int* cnt, long long seg_cap, long long* outK, int* outD,
                       long long* seg_counts, hipStream_t stream) {
  for (int c = 0; c < PW_SEGS; ++c) seg_counts[c] = 0;
  if (nA <= 0 || nB <= 0) return 0;
  if (D < 1 || D > 64) throw std::runtime_error("pairs_within: 1 <= D <= 64");
  // a kept pair has rint(sqrt(s) / nf * scale) <= thr, so sqrt(s) / nf * scale < thr + 1 and
  // s < ((thr + 1) nf / scale)^2; the factor 1.001 covers the fp32 evaluation of both sides
  float s_max = INFINITY;
  if (std::isfinite(thr) && scale > 0.f && nf > 0.f) {
    const double bound = ((double)thr + 1.0) * (double)nf / (double)scale;
    s_max = bound < 0.0 ? -1.f : (float)(bound * bound * 1.001);
  }
  AV_HIP_CHECK(hipMemsetAsync(cnt, 0, sizeof(int) * PW_SEGS * PW_CSTRIDE, stream));
  // grid.y is capped at 65535 workgroups: A is covered in row chunks of AR x 65535
  auto run = [&](auto kern, int AR) {
    const int CH = AR * 65535;
    for (int a_row0 = 0; a_row0 < nA; a_row0 += CH) {
      const int rows = std::min(CH, nA - a_row0);
      const dim3 grid((unsigned)((nB + 255) / 256), (unsigned)((rows + AR - 1) / AR));
      kern<<<grid, 256, 0, stream>>>(A, nA, B, nB, D, nf, scale, thr, s_max, tri, a_base, b_base, cnt, seg_cap, outK,
                                     outD, a_row0);
    }
  };
  if (D <= 4) run(pairs_within_kernel<4, 256>, 256);
  else if (D <= 8) run(pairs_within_kernel<8, 256>, 256);
  else if (D <= 16) run(pairs_within_kernel<16, 256>, 256);
  else if (D <= 32) run(pairs_within_kernel<32, 64>, 64);
  else run(pairs_within_kernel<64, 64>, 64);
  AV_HIP_CHECK(hipGetLastError());
  int h[PW_SEGS * PW_CSTRIDE];
  AV_HIP_CHECK(hipMemcpyAsync(h, cnt, sizeof(h), hipMemcpyDeviceToHost, stream));
  AV_HIP_CHECK(hipStreamSynchronize(stream));
  long long mx = 0;
  for (int c = 0; c < PW_SEGS; ++c) {
    seg_counts[c] = h[c * PW_CSTRIDE];
    mx = std::max<long long>(mx, h[c * PW_CSTRIDE]);
  }
  return mx;
}

int pairs_within_segments() { return PW_SEGS; }
int pairs_within_counter_ints() { return PW_SEGS * PW_CSTRIDE; }

}  // namespace avk
