// Device-resident random-forest builder for CDNA4 (gfx950): K6 impurity / K7 split argmin /
// row partitioning.
//
// Reference: DecisionTreeBuilder grows ONE tree ONE level per MapReduce job (every mapper re-emits
// each record once per candidate split; a reducer counts classes per child path and picks the
// best split, J/tree/DecisionTreeBuilder.java:209-359, :499-616), and a forest is that job
// repeated per tree (R/rafo.sh).  Here all trees of a forest grow together, level-synchronously,
// with their rows RESIDENT and PARTITIONED in HBM:
//
//   * every tree owns the bootstrap multiset of the training rows (rows with Poisson weight > 0)
//     as a private column-major copy [F][R] of the uint8 fine-bin codes + label + weight; all
//     trees' copies live in one buffer (288 GB of HBM makes T copies of the codes affordable, and
//     it turns every later pass into contiguous streaming reads);
//   * every frontier node owns a CONTIGUOUS segment of its tree's rows, so a node's class
//     histogram reads only its own rows (work per level = rows, independent of the node count),
//     and only the smaller child of each split is histogrammed (the larger is parent - sibling);
//   * forest_split_kernel (K6 + K7) scores every (feature, threshold) of every node from its
//     histogram in one launch: one workgroup per node, one lane per feature scanning the
//     cumulative class counts, Gini or entropy, the random feature subset as a mask, and the best
//     (or a random one of the top-k: randomAmongTop) split per node;
//   * forest_part_count / forest_part_scatter stably partition each splitting node's segment into
//     [left rows | right rows] in a second buffer (wave-ballot ranks, per-chunk bases from a host
//     prefix over the chunk counts — the ONE host copy per level).
//
// Work lists are chunks of <= chunk rows of one segment, so a launch has thousands of equally sized
// workgroups regardless of how unbalanced the frontier is.  All row indices a kernel touches are
// inside the chunk's [start, start + len) which the host derived from segment sizes it computed.
#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

constexpr int FB_THREADS = 256;
constexpr int FB_MAXC = 16;  // classes handled in registers by the split kernel

// ------------------------------------------------------------------------------------------------
// histogram of chunks: hist[slot][c][TB] += w for every (feature bin) + the node total at TB-1
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(FB_THREADS) void forest_hist_kernel(
    const uint8_t* __restrict__ codes, long long ld, const uint8_t* __restrict__ lab, const uint8_t* __restrict__ wt,
    const int* __restrict__ item_slot, const long long* __restrict__ item_start, const int* __restrict__ item_len,
    const int* __restrict__ bins, const int* __restrict__ offs, int nfeat, int TB, int C,
    unsigned long long* __restrict__ hist) {
  extern __shared__ unsigned int s_h[];
  const int item = blockIdx.x;
  const int per = C * TB;
  for (int i = threadIdx.x; i < per; i += FB_THREADS) s_h[i] = 0;
  __syncthreads();
  const long long start = item_start[item];
  const int len = item_len[item];
  for (int i = threadIdx.x; i < len; i += FB_THREADS) {
    const long long r = start + i;
    const unsigned c = lab[r];
    const unsigned w = wt[r];
    if (c >= (unsigned)C || w == 0) continue;
    unsigned int* row = s_h + c * TB;
    for (int f = 0; f < nfeat; ++f) {
      const unsigned v = codes[(long long)f * ld + r];
      if (v < (unsigned)bins[f]) atomicAdd(&row[offs[f] + v], w);
    }
    atomicAdd(&row[TB - 1], w);
  }
  __syncthreads();
  unsigned long long* dst = hist + (long long)item_slot[item] * per;
  for (int i = threadIdx.x; i < per; i += FB_THREADS) {
    const unsigned v = s_h[i];
    if (v) atomicAdd(&dst[i], (unsigned long long)v);
  }
}

// fp64 throughout: the scoring is a few hundred ops per node, and fp64 keeps the choice between
// near-tied splits identical to the CPU oracle (same formula, same order of operations).
__device__ __forceinline__ double impurity(const double* cnt, int C, double tot, int algo) {
  if (tot <= 0.0) return 0.0;
  double s = 0.0;
  if (algo == 0) {  // Gini
    for (int c = 0; c < C; ++c) {
      const double p = cnt[c] / tot;
      s += p * p;
    }
    return 1.0 - s;
  }
  for (int c = 0; c < C; ++c) {  // entropy (log2, like InfoContentStat)
    const double p = cnt[c] / tot;
    if (p > 0.0) s -= p * log2(p);
  }
  return s;
}

// ------------------------------------------------------------------------------------------------
// K6 + K7: best binary split per node.  hist [A][C][TB] (int64), fmask [A][F] (1 = candidate).
// A split at threshold t of feature f sends bins <= t left; bins > t AND missing codes right
// (right = node total - left, the node total being the TB-1 column).  Outputs per node: feature,
// threshold, weighted child impurity (inf = no valid split), node impurity, and the left class
// counts [A][C] of the chosen split.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(FB_THREADS) void forest_split_kernel(
    const long long* __restrict__ hist, const uint8_t* __restrict__ fmask, const int* __restrict__ bins,
    const int* __restrict__ offs, int nfeat, int TB, int C, int algo, int topk, const float* __restrict__ rnd,
    int* __restrict__ out_feat, int* __restrict__ out_thr, float* __restrict__ out_score,
    float* __restrict__ out_imp, long long* __restrict__ out_left) {
  extern __shared__ unsigned char s_raw[];
  double* s_score = reinterpret_cast<double*>(s_raw);             // [nfeat]
  int* s_thr = reinterpret_cast<int*>(s_score + nfeat);            // [nfeat]
  __shared__ double s_tot[FB_MAXC];
  const int a = blockIdx.x;
  const long long* h = hist + (long long)a * C * TB;
  if (threadIdx.x < C) s_tot[threadIdx.x] = (double)h[(long long)threadIdx.x * TB + TB - 1];
  __syncthreads();
  double tot[FB_MAXC];
  double ntot = 0.0;
  for (int c = 0; c < C; ++c) {
    tot[c] = s_tot[c];
    ntot += tot[c];
  }
  for (int f = threadIdx.x; f < nfeat; f += FB_THREADS) {
    double best = INFINITY;
    int bthr = -1;
    if (fmask[(long long)a * nfeat + f]) {
      double left[FB_MAXC], right[FB_MAXC];
      for (int c = 0; c < C; ++c) left[c] = 0.0;
      const int B = bins[f], o = offs[f];
      for (int b = 0; b + 1 < B; ++b) {
        double nl = 0.0;
        for (int c = 0; c < C; ++c) {
          left[c] += (double)h[(long long)c * TB + o + b];
          nl += left[c];
        }
        const double nr = ntot - nl;
        if (nl <= 0.0 || nr <= 0.0) continue;
        for (int c = 0; c < C; ++c) right[c] = tot[c] - left[c];
        const double s = (nl * impurity(left, C, nl, algo) + nr * impurity(right, C, nr, algo)) / ntot;
        if (s < best) {
          best = s;
          bthr = b;
        }
      }
    }
    s_score[f] = best;
    s_thr[f] = bthr;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    // best, or a uniformly random one of the top-k per-feature bests (randomAmongTop)
    int pick = -1;
    if (topk <= 1) {
      double bv = INFINITY;
      for (int f = 0; f < nfeat; ++f)
        if (s_score[f] < bv) {
          bv = s_score[f];
          pick = f;
        }
    } else {
      int chosen[32];
      int nk = 0;
      const int K = topk < 32 ? topk : 32;
      for (int k = 0; k < K; ++k) {
        double bv = INFINITY;
        int bf = -1;
        for (int f = 0; f < nfeat; ++f) {
          bool used = false;
          for (int j = 0; j < nk; ++j) used |= chosen[j] == f;
          if (!used && s_score[f] < bv) {
            bv = s_score[f];
            bf = f;
          }
        }
        if (bf < 0) break;
        chosen[nk++] = bf;
      }
      if (nk > 0) {
        int j = (int)(rnd[a] * nk);
        pick = chosen[j < nk ? j : nk - 1];
      }
    }
    out_imp[a] = (float)impurity(tot, C, ntot, algo);
    if (pick >= 0) {
      out_feat[a] = pick;
      out_thr[a] = s_thr[pick];
      out_score[a] = (float)s_score[pick];
      const int o = offs[pick];
      for (int c = 0; c < C; ++c) {
        long long l = 0;
        for (int b = 0; b <= s_thr[pick]; ++b) l += h[(long long)c * TB + o + b];
        out_left[(long long)a * C + c] = l;
      }
    } else {
      out_feat[a] = -1;
      out_thr[a] = -1;
      out_score[a] = INFINITY;
      for (int c = 0; c < C; ++c) out_left[(long long)a * C + c] = 0;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// partition: count rows going left / right per chunk of a splitting node's segment
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ bool goes_left(const uint8_t* codes, long long ld, long long r, int f, int thr) {
  return (int)codes[(long long)f * ld + r] <= thr;  // missing codes (>= bins) are > thr: right
}

__global__ __launch_bounds__(FB_THREADS) void forest_part_count_kernel(
    const uint8_t* __restrict__ codes, long long ld, const int* __restrict__ item_node,
    const long long* __restrict__ item_start, const int* __restrict__ item_len, const int* __restrict__ feat,
    const int* __restrict__ thr, int* __restrict__ item_left) {
  __shared__ int s_cnt;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  const int item = blockIdx.x;
  const int a = item_node[item];
  const int f = feat[a];
  const int t = thr[a];
  const long long start = item_start[item];
  const int len = item_len[item];
  int cnt = 0;
  if (f >= 0)
    for (int i = threadIdx.x; i < len; i += FB_THREADS) cnt += goes_left(codes, ld, start + i, f, t) ? 1 : 0;
  cnt = av::wave_sum(cnt);
  if (av::lane_id() == 0 && cnt) atomicAdd(&s_cnt, cnt);
  __syncthreads();
  if (threadIdx.x == 0) item_left[item] = s_cnt;
}

// Stable scatter: rows of a chunk keep their order within the left / right part.
//
// A tile of 1024 rows (4 per lane, strided so every wave load is 64 contiguous bytes) is ranked
// with wave ballots (4 sub-passes of 256 rows, LDS prefix over the 4 waves), then every column of
// the tile is STAGED in LDS in partitioned order ([left rows | right rows], F + 2 columns x 1 KiB),
// and written out as two contiguous runs per column with aligned dword stores (byte stores only
// for the unaligned head / tail of a run).  The first version stored every byte of every row at its
// destination individually (~1.1 TB/s); the runs of consecutive tiles abut, and a dword is only
// written when the run owns all four of its bytes, so tiles never clobber each other.
constexpr int PT = 4;
constexpr int TILE = FB_THREADS * PT;

__device__ __forceinline__ void write_run(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, int n) {
  const int head = min(n, (int)((4 - (reinterpret_cast<uintptr_t>(dst) & 3)) & 3));
  for (int i = threadIdx.x; i < head; i += FB_THREADS) dst[i] = src[i];
  const int nd = (n - head) >> 2;
  unsigned int* d32 = reinterpret_cast<unsigned int*>(dst + head);
  for (int w = threadIdx.x; w < nd; w += FB_THREADS) {
    const uint8_t* q = src + head + 4 * w;
    d32[w] = (unsigned)q[0] | ((unsigned)q[1] << 8) | ((unsigned)q[2] << 16) | ((unsigned)q[3] << 24);
  }
  for (int i = head + 4 * nd + threadIdx.x; i < n; i += FB_THREADS) dst[i] = src[i];
}

__global__ __launch_bounds__(FB_THREADS) void forest_part_scatter_kernel(
    const uint8_t* __restrict__ codes, const uint8_t* __restrict__ lab, const uint8_t* __restrict__ wt,
    uint8_t* __restrict__ dcodes, uint8_t* __restrict__ dlab, uint8_t* __restrict__ dwt, long long ld, int nfeat,
    const int* __restrict__ item_node, const long long* __restrict__ item_start, const int* __restrict__ item_len,
    const long long* __restrict__ left_base, const long long* __restrict__ right_base, const int* __restrict__ feat,
    const int* __restrict__ thr) {
  extern __shared__ uint8_t s_stage[];  // [(nfeat + 2)][TILE]
  __shared__ int s_wl[FB_THREADS / AV_WAVE], s_wr[FB_THREADS / AV_WAVE];
  const int item = blockIdx.x;
  const int a = item_node[item];
  const int f = feat[a];
  if (f < 0) return;  // uniform over the block: no barrier is skipped by part of it
  const int t = thr[a];
  const long long start = item_start[item];
  const int len = item_len[item];
  const int ncol = nfeat + 2;
  long long lb = left_base[item], rb = right_base[item];
  const int lane = av::lane_id(), wave = av::wave_id();
  const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int t0 = 0; t0 < len; t0 += TILE) {
    int pos[PT];
    bool isl[PT];
    int nl = 0, nr = 0;
#pragma unroll
    for (int j = 0; j < PT; ++j) {
      const int i = t0 + j * FB_THREADS + threadIdx.x;
      const bool valid = i < len;
      const bool left = valid && goes_left(codes, ld, start + i, f, t);
      const bool right = valid && !left;
      const unsigned long long bl = __ballot(left), br = __ballot(right);
      if (lane == 0) {
        s_wl[wave] = __popcll(bl);
        s_wr[wave] = __popcll(br);
      }
      __syncthreads();
      int ol = 0, orr = 0, tl = 0, tr = 0;
      for (int w = 0; w < FB_THREADS / AV_WAVE; ++w) {
        if (w < wave) {
          ol += s_wl[w];
          orr += s_wr[w];
        }
        tl += s_wl[w];
        tr += s_wr[w];
      }
      isl[j] = left;
      pos[j] = !valid ? -1 : (left ? nl + ol + __popcll(bl & below) : nr + orr + __popcll(br & below));
      nl += tl;
      nr += tr;
      __syncthreads();  // s_wl / s_wr are rewritten by the next sub-pass
    }
    // stage every column in partitioned order: [0, nl) left rows, [nl, nl + nr) right rows
    for (int k = 0; k < ncol; ++k) {
      const uint8_t* src = k < nfeat ? codes + (long long)k * ld : (k == nfeat ? lab : wt);
      uint8_t* st = s_stage + k * TILE;
#pragma unroll
      for (int j = 0; j < PT; ++j)
        if (pos[j] >= 0) st[isl[j] ? pos[j] : nl + pos[j]] = src[start + t0 + j * FB_THREADS + threadIdx.x];
    }
    __syncthreads();
    for (int k = 0; k < ncol; ++k) {
      uint8_t* dst = k < nfeat ? dcodes + (long long)k * ld : (k == nfeat ? dlab : dwt);
      write_run(dst + lb, s_stage + k * TILE, nl);
      write_run(dst + rb, s_stage + k * TILE + nl, nr);
    }
    lb += nl;
    rb += nr;
    __syncthreads();  // the stage is rewritten by the next tile
  }
}

// ------------------------------------------------------------------------------------------------
// Fused fine-bin encoding of all numeric columns: out[f][r] = #{edges of f < x} (bin b covers
// (P[b-1], P[b]]), 255 for NaN.  One launch for every feature instead of one torch.bucketize
// (int64 intermediates) per feature.  grid = (row blocks, F); the feature's edges sit in LDS.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(FB_THREADS) void bucketize_u8_kernel(const float* __restrict__ X, long long ldx,
                                                                  long long n, const float* __restrict__ edges,
                                                                  const int* __restrict__ eoff,
                                                                  uint8_t* __restrict__ out, long long ldo) {
  __shared__ float s_e[256];
  const int f = blockIdx.y;
  const int e0 = eoff[f], ne = eoff[f + 1] - e0;  // ne <= 254 (checked on the host)
  for (int i = threadIdx.x; i < ne; i += FB_THREADS) s_e[i] = edges[e0 + i];
  __syncthreads();
  const float* x = X + (long long)f * ldx;
  uint8_t* o = out + (long long)f * ldo;
  const long long stride = (long long)gridDim.x * FB_THREADS;
  for (long long r = (long long)blockIdx.x * FB_THREADS + threadIdx.x; r < n; r += stride) {
    const float v = x[r];
    int lo = 0, hi = ne;  // first edge >= v
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if (s_e[m] < v) lo = m + 1; else hi = m;
    }
    o[r] = (v != v) ? (uint8_t)255 : (uint8_t)lo;
  }
}

}  // namespace

namespace avk {

void bucketize_u8(const float* X, long long ldx, long long n, int F, const float* edges, const int* eoff, uint8_t* out,
                  long long ldo, hipStream_t stream) {
  if (n <= 0 || F <= 0) return;
  const int gx = av::stream_grid(n, FB_THREADS, 2, 4096);
  bucketize_u8_kernel<<<dim3(gx, F), FB_THREADS, 0, stream>>>(X, ldx, n, edges, eoff, out, ldo);
  AV_HIP_CHECK(hipGetLastError());
}

void forest_hist(const uint8_t* codes, long long ld, const uint8_t* lab, const uint8_t* wt, const int* item_slot,
                 const long long* item_start, const int* item_len, int n_items, const int* bins, const int* offs,
                 int nfeat, int TB, int C, unsigned long long* hist, hipStream_t stream) {
  if (n_items <= 0) return;
  const size_t lds = sizeof(unsigned) * (size_t)C * TB;
  if (lds > 64 * 1024) throw std::runtime_error("forest_hist: class x bin table exceeds LDS");
  forest_hist_kernel<<<n_items, FB_THREADS, lds, stream>>>(codes, ld, lab, wt, item_slot, item_start, item_len, bins,
                                                            offs, nfeat, TB, C, hist);
  AV_HIP_CHECK(hipGetLastError());
}

void forest_split(const long long* hist, const uint8_t* fmask, const int* bins, const int* offs, int nfeat, int TB,
                  int C, int algo, int topk, const float* rnd, int A, int* feat, int* thr, float* score, float* imp,
                  long long* left, hipStream_t stream) {
  if (A <= 0) return;
  if (C > FB_MAXC) throw std::runtime_error("forest_split: more than 16 classes");
  const size_t lds = (sizeof(double) + sizeof(int)) * (size_t)nfeat;
  forest_split_kernel<<<A, FB_THREADS, lds, stream>>>(hist, fmask, bins, offs, nfeat, TB, C, algo, topk, rnd, feat,
                                                       thr, score, imp, left);
  AV_HIP_CHECK(hipGetLastError());
}

void forest_part_count(const uint8_t* codes, long long ld, const int* item_node, const long long* item_start,
                       const int* item_len, int n_items, const int* feat, const int* thr, int* item_left,
                       hipStream_t stream) {
  if (n_items <= 0) return;
  forest_part_count_kernel<<<n_items, FB_THREADS, 0, stream>>>(codes, ld, item_node, item_start, item_len, feat, thr,
                                                                item_left);
  AV_HIP_CHECK(hipGetLastError());
}

void forest_part_scatter(const uint8_t* codes, const uint8_t* lab, const uint8_t* wt, uint8_t* dcodes, uint8_t* dlab,
                         uint8_t* dwt, long long ld, int nfeat, const int* item_node, const long long* item_start,
                         const int* item_len, int n_items, const long long* left_base, const long long* right_base,
                         const int* feat, const int* thr, hipStream_t stream) {
  if (n_items <= 0) return;
  const size_t lds = (size_t)(nfeat + 2) * TILE;
  if (lds > 64 * 1024) throw std::runtime_error("forest_part_scatter: more than 62 features");
  forest_part_scatter_kernel<<<n_items, FB_THREADS, lds, stream>>>(codes, lab, wt, dcodes, dlab, dwt, ld, nfeat,
                                                                  item_node, item_start, item_len, left_base,
                                                                  right_base, feat, thr);
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
