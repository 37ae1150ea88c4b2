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
// Row-buffer access pattern shared by the three streaming kernels: a chunk [start, start + len) is
// walked in tiles of 8 * 256 rows starting at start rounded DOWN to 8; lane t owns the 8
// consecutive rows [base + 8t, base + 8t + 8) and fetches every column of them with one aligned
// 8-byte load (a wave reads 512 contiguous bytes per column per instruction instead of 64); rows
// outside the chunk are masked.  The buffers are padded to a multiple of 16 rows (checked by the
// binding), so the rounded-up tail of the last chunk stays inside them.
// ------------------------------------------------------------------------------------------------
constexpr int RPT = 8;                    // rows per lane per tile
constexpr int RTILE = RPT * FB_THREADS;   // 2048 rows per tile

__device__ __forceinline__ unsigned valid_mask(long long r0, long long start, long long end) {
  unsigned m = 0;
#pragma unroll
  for (int j = 0; j < RPT; ++j) m |= (unsigned)(r0 + j >= start && r0 + j < end) << j;
  return m;
}

__device__ __forceinline__ unsigned byte_of(const uint2& v, int j) {
  return ((j < 4 ? v.x : v.y) >> (8 * (j & 3))) & 0xFFu;
}

// histogram of chunks: hist[slot][c][TB] += w for every (feature bin) + the node total at TB-1.
// The node total is NOT a per-row atomic (every row of a class hit the same LDS word: the main
// source of LDS conflicts): feature 0's missing codes go to the TB-1 word, and at the flush each
// class adds its feature-0 bins to it (every counted row is in exactly one of those words).
// The LDS table is replicated `rep` times (1..8, as many as fit): lane l adds into replica
// l % rep, so lanes of one wave whose rows share a (class, bin) word — the common case with few
// classes and skewed bins — hit different words; the replica stride is odd, so the copies of a
// word sit in different banks.  The replicas are summed before the flush.
__global__ __launch_bounds__(FB_THREADS) void forest_hist_kernel(
    const uint8_t* __restrict__ codes, long long ld, const uint8_t* __restrict__ lab, const uint8_t* __restrict__ wt,
    const int* __restrict__ item_slot, const long long* __restrict__ item_start, const int* __restrict__ item_len,
    const int* __restrict__ bins, const int* __restrict__ offs, int nfeat, int TB, int C,
    unsigned long long* __restrict__ hist, int rep) {
  extern __shared__ unsigned int s_all[];
  const int item = blockIdx.x;
  const int per = C * TB, stride = per | 1;
  for (int i = threadIdx.x; i < rep * stride; i += FB_THREADS) s_all[i] = 0;
  __syncthreads();
  unsigned* s_h = s_all + (threadIdx.x & (rep - 1)) * stride;  // this lane's replica
  const long long start = item_start[item];
  const long long end = start + item_len[item];
  for (long long base = start & ~7LL; base < end; base += RTILE) {
    const long long r0 = base + RPT * threadIdx.x;
    unsigned m = valid_mask(r0, start, end);
    if (!m) continue;
    const uint2 lv = *reinterpret_cast<const uint2*>(lab + r0);
    const uint2 wv = *reinterpret_cast<const uint2*>(wt + r0);
    unsigned c8[RPT], w8[RPT];
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      c8[j] = byte_of(lv, j);
      w8[j] = byte_of(wv, j);
      if (c8[j] >= (unsigned)C || w8[j] == 0) m &= ~(1u << j);
    }
    if (!m) continue;
    if (nfeat == 0) {
#pragma unroll
      for (int j = 0; j < RPT; ++j)
        if (m >> j & 1) atomicAdd(&s_h[c8[j] * TB + TB - 1], w8[j]);
    }
    for (int f = 0; f < nfeat; ++f) {
      const uint2 cv = *reinterpret_cast<const uint2*>(codes + (long long)f * ld + r0);
      const unsigned B = (unsigned)bins[f], o = (unsigned)offs[f];
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        const unsigned v = byte_of(cv, j);
        if (m >> j & 1) {
          if (v < B) atomicAdd(&s_h[c8[j] * TB + o + v], w8[j]);
          else if (f == 0) atomicAdd(&s_h[c8[j] * TB + TB - 1], w8[j]);  // missing: total word
        }
      }
    }
  }
  __syncthreads();
  s_h = s_all;
  if (rep > 1) {  // replicas -> replica 0
    for (int i = threadIdx.x; i < per; i += FB_THREADS) {
      unsigned t = s_all[i];
      for (int r = 1; r < rep; ++r) t += s_all[r * stride + i];
      s_all[i] = t;
    }
    __syncthreads();
  }
  if (nfeat > 0 && threadIdx.x < C) {  // node total = feature 0's bins + its missing rows
    const int c = threadIdx.x, B0 = bins[0], o0 = offs[0];
    unsigned t = s_h[c * TB + TB - 1];
    for (int v = 0; v < B0; ++v) t += s_h[c * TB + o0 + v];
    s_h[c * TB + TB - 1] = t;
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
        int j = (int)((double)rnd[a] * nk);  // fp64 product, as the host twin
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
// partition: count rows going left per chunk of a splitting node's segment
// ------------------------------------------------------------------------------------------------
// left bits of the 8 rows (code <= thr; missing codes >= bins are > thr: right)
__device__ __forceinline__ unsigned left_bits(const uint2& cv, int thr) {
  unsigned b = 0;
#pragma unroll
  for (int j = 0; j < RPT; ++j) b |= (unsigned)((int)byte_of(cv, j) <= thr) << j;
  return b;
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
  const long long end = start + item_len[item];
  int cnt = 0;
  if (f >= 0) {
    const uint8_t* col = codes + (long long)f * ld;
    for (long long base = start & ~7LL; base < end; base += RTILE) {
      const long long r0 = base + RPT * threadIdx.x;
      const unsigned m = valid_mask(r0, start, end);
      if (m) cnt += __popc(left_bits(*reinterpret_cast<const uint2*>(col + r0), t) & m);
    }
  }
  cnt = av::wave_sum(cnt);
  if (av::lane_id() == 0 && cnt) atomicAdd(&s_cnt, cnt);
  __syncthreads();
  if (threadIdx.x == 0) item_left[item] = s_cnt;
}

// Stable scatter of a splitting node's rows into [left rows | right rows] (order kept within each).
//
// Per 2048-row tile: every lane ranks its 8 rows (popcounts of the left / right bits), one wave
// inclusive scan of the packed (left | right << 16) counts + an LDS prefix over the 4 waves gives
// each row its position in the tile's partitioned order; then the columns are moved in groups of
// SG: aligned 8-byte loads, bytes dropped into an LDS stage at their partitioned position, and the
// stage written out as two contiguous runs per column (left run at lb, right run at rb) with
// aligned dword stores (byte stores only for a run's unaligned head / tail; a dword is written
// only when the run owns all 4 of its bytes, so abutting runs of consecutive tiles never clobber
// each other).
constexpr int SG = 6;  // columns staged per group: SG * 2 KiB of LDS

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
  __shared__ uint8_t s_stage[SG][RTILE];
  __shared__ int s_wtot[FB_THREADS / AV_WAVE];
  const int item = blockIdx.x;
  const int a = item_node[item];
  const int f = feat[a];
  if (f < 0) return;  // uniform over the block: no barrier is skipped by part of it
  const int t = thr[a];
  const long long start = item_start[item];
  const long long end = start + item_len[item];
  const int ncol = nfeat + 2;
  long long lb = left_base[item], rb = right_base[item];
  const int lane = av::lane_id(), wave = av::wave_id();
  const uint8_t* scol = codes + (long long)f * ld;
  for (long long base = start & ~7LL; base < end; base += RTILE) {
    const long long r0 = base + RPT * threadIdx.x;
    const unsigned m = valid_mask(r0, start, end);
    const unsigned lbits = m ? (left_bits(*reinterpret_cast<const uint2*>(scol + r0), t) & m) : 0u;
    const unsigned rbits = m & ~lbits;
    // packed inclusive scan over the wave: low 16 bits left counts, high 16 bits right counts
    const int mine = __popc(lbits) | (__popc(rbits) << 16);
    int inc = mine;
#pragma unroll
    for (int o = 1; o < AV_WAVE; o <<= 1) {
      const int y = __shfl_up(inc, o, AV_WAVE);
      if (lane >= o) inc += y;
    }
    if (lane == AV_WAVE - 1) s_wtot[wave] = inc;
    __syncthreads();
    int before = 0, tot = 0;
    for (int w = 0; w < FB_THREADS / AV_WAVE; ++w) {
      if (w < wave) before += s_wtot[w];
      tot += s_wtot[w];
    }
    const int excl = before + inc - mine;
    const int nl = tot & 0xFFFF, nr = tot >> 16;
    int pl = excl & 0xFFFF, pr = nl + (excl >> 16);
    short pos[RPT];
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      pos[j] = -1;
      if (lbits >> j & 1) pos[j] = (short)(pl++);
      else if (rbits >> j & 1) pos[j] = (short)(pr++);
    }
    for (int g0 = 0; g0 < ncol; g0 += SG) {
      const int ng = min(SG, ncol - g0);
      for (int g = 0; g < ng; ++g) {
        const int k = g0 + g;
        const uint8_t* src = k < nfeat ? codes + (long long)k * ld : (k == nfeat ? lab : wt);
        if (m) {
          const uint2 v = *reinterpret_cast<const uint2*>(src + r0);
#pragma unroll
          for (int j = 0; j < RPT; ++j)
            if (pos[j] >= 0) s_stage[g][pos[j]] = (uint8_t)byte_of(v, j);
        }
      }
      __syncthreads();
      for (int g = 0; g < ng; ++g) {
        const int k = g0 + g;
        uint8_t* dst = k < nfeat ? dcodes + (long long)k * ld : (k == nfeat ? dlab : dwt);
        write_run(dst + lb, s_stage[g], nl);
        write_run(dst + rb, s_stage[g] + nl, nr);
      }
      __syncthreads();  // the stage (and s_wtot, on the last group) is rewritten next
    }
    lb += nl;
    rb += nr;
  }
}

// ------------------------------------------------------------------------------------------------
// Bootstrap row buffers.  The multiplicity of (tree, global row) is a pure function of the tree key
// and the row index (splitmix64 -> 32 uniform bits -> Poisson(1) by inverse CDF, Bernoulli(rate) or
// 1), so the sample is the same on any device and any number of ranks (rows are keyed by their
// GLOBAL index).  Two passes over grid (row tiles, trees): count the kept rows per tile, then, after
// a scan of the tile counts, write every kept row's codes / label / weight compacted into the
// tree-major buffers through the same LDS stage + aligned run writes as the partition.
// ------------------------------------------------------------------------------------------------
__constant__ unsigned kPoisson1Cdf[12] = {1580030168u, 3160060337u, 3950075421u, 4213413783u,
                                          4279248373u, 4292415291u, 4294609777u, 4294923276u,
                                          4294962463u, 4294966817u, 4294967252u, 4294967292u};

__device__ __forceinline__ unsigned boot_weight(unsigned long long key, unsigned long long row, int mode,
                                                unsigned rate32) {
  if (mode == 0) return 1u;
  unsigned long long z = key + row * 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  z ^= z >> 31;
  const unsigned u = (unsigned)(z >> 32);
  if (mode == 2) return u < rate32 ? 1u : 0u;
  unsigned k = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) k += u >= kPoisson1Cdf[i] ? 1u : 0u;
  return k;
}

// weights of this lane's 8 rows packed one byte each (rows >= n weigh 0)
__device__ __forceinline__ unsigned long long boot_weights8(unsigned long long key, long long row_off, long long r0,
                                                            long long n, int mode, unsigned rate32) {
  unsigned long long w = 0;
#pragma unroll
  for (int j = 0; j < RPT; ++j)
    if (r0 + j < n) w |= (unsigned long long)boot_weight(key, (unsigned long long)(row_off + r0 + j), mode, rate32)
                         << (8 * j);
  return w;
}

__device__ __forceinline__ unsigned nonzero_bytes(unsigned long long w) {
  unsigned b = 0;
#pragma unroll
  for (int j = 0; j < RPT; ++j) b |= (unsigned)((w >> (8 * j) & 0xFF) != 0) << j;
  return b;
}

__device__ __forceinline__ int block_excl_scan(int mine, int* s_wtot, int& tot) {
  const int lane = av::lane_id(), wave = av::wave_id();
  int inc = mine;
#pragma unroll
  for (int o = 1; o < AV_WAVE; o <<= 1) {
    const int y = __shfl_up(inc, o, AV_WAVE);
    if (lane >= o) inc += y;
  }
  if (lane == AV_WAVE - 1) s_wtot[wave] = inc;
  __syncthreads();
  int before = 0;
  tot = 0;
  for (int w = 0; w < FB_THREADS / AV_WAVE; ++w) {
    if (w < wave) before += s_wtot[w];
    tot += s_wtot[w];
  }
  return before + inc - mine;
}

__global__ __launch_bounds__(FB_THREADS) void forest_boot_count_kernel(const unsigned long long* __restrict__ keys,
                                                                       long long n, long long row_off, int mode,
                                                                       unsigned rate32, int* __restrict__ tile_cnt) {
  __shared__ int s_wtot[FB_THREADS / AV_WAVE];
  const int tree = blockIdx.y;
  const long long r0 = (long long)blockIdx.x * RTILE + RPT * threadIdx.x;
  const unsigned long long w = boot_weights8(keys[tree], row_off, r0, n, mode, rate32);
  int tot;
  block_excl_scan(__popc(nonzero_bytes(w)), s_wtot, tot);
  if (threadIdx.x == 0) tile_cnt[(long long)tree * gridDim.x + blockIdx.x] = tot;
}

__global__ __launch_bounds__(FB_THREADS) void forest_boot_scatter_kernel(
    const uint8_t* __restrict__ codes, long long ld, int nfeat, const uint8_t* __restrict__ lab,
    const unsigned long long* __restrict__ keys, long long n, long long row_off, int mode, unsigned rate32,
    const long long* __restrict__ tile_off, uint8_t* __restrict__ dcodes, uint8_t* __restrict__ dlab,
    uint8_t* __restrict__ dwt, long long ldb) {
  __shared__ uint8_t s_stage[SG][RTILE];
  __shared__ int s_wtot[FB_THREADS / AV_WAVE];
  const int tree = blockIdx.y;
  const long long r0 = (long long)blockIdx.x * RTILE + RPT * threadIdx.x;
  const unsigned long long w = boot_weights8(keys[tree], row_off, r0, n, mode, rate32);
  const unsigned keep = nonzero_bytes(w);
  int tot;
  int p = block_excl_scan(__popc(keep), s_wtot, tot);
  if (tot == 0) return;  // uniform over the block
  short pos[RPT];
#pragma unroll
  for (int j = 0; j < RPT; ++j) pos[j] = (keep >> j & 1) ? (short)(p++) : (short)-1;
  const long long out = tile_off[(long long)tree * gridDim.x + blockIdx.x];
  const bool any = r0 < n;
  const int ncol = nfeat + 2;
  for (int g0 = 0; g0 < ncol; g0 += SG) {
    const int ng = min(SG, ncol - g0);
    for (int g = 0; g < ng; ++g) {
      const int k = g0 + g;
      if (!any || !keep) continue;
      unsigned long long v;
      if (k < nfeat) {
        const uint2 x = *reinterpret_cast<const uint2*>(codes + (long long)k * ld + r0);
        v = (unsigned long long)x.x | ((unsigned long long)x.y << 32);
      } else if (k == nfeat) {
        const uint2 x = *reinterpret_cast<const uint2*>(lab + r0);
        v = (unsigned long long)x.x | ((unsigned long long)x.y << 32);
      } else {
        v = w;
      }
#pragma unroll
      for (int j = 0; j < RPT; ++j)
        if (pos[j] >= 0) s_stage[g][pos[j]] = (uint8_t)(v >> (8 * j));
    }
    __syncthreads();
    for (int g = 0; g < ng; ++g) {
      const int k = g0 + g;
      uint8_t* dst = k < nfeat ? dcodes + (long long)k * ldb : (k == nfeat ? dlab : dwt);
      write_run(dst + out, s_stage[g], tot);
    }
    __syncthreads();
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
  const size_t stride = ((size_t)C * TB) | 1;
  if (sizeof(unsigned) * stride > 64 * 1024) throw std::runtime_error("forest_hist: class x bin table exceeds LDS");
  int rep = 8;  // replicas that fit 32 KB (keeps several workgroups per CU)
  while (rep > 1 && sizeof(unsigned) * stride * rep > 32 * 1024) rep >>= 1;
  const char* e = std::getenv("AVMI_FOREST_HIST_REP");
  if (e && *e) {
    const int r = std::atoi(e);
    if (r == 1 || r == 2 || r == 4 || r == 8) rep = r;
  }
  if (sizeof(unsigned) * stride * rep > 64 * 1024) rep = 1;
  const size_t lds = sizeof(unsigned) * stride * rep;
  forest_hist_kernel<<<n_items, FB_THREADS, lds, stream>>>(codes, ld, lab, wt, item_slot, item_start, item_len, bins,
                                                            offs, nfeat, TB, C, hist, rep);
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
  forest_part_scatter_kernel<<<n_items, FB_THREADS, 0, stream>>>(codes, lab, wt, dcodes, dlab, dwt, ld, nfeat,
                                                                  item_node, item_start, item_len, left_base,
                                                                  right_base, feat, thr);
  AV_HIP_CHECK(hipGetLastError());
}


void forest_boot_count(const unsigned long long* keys, int ntrees, long long n, long long row_off, int mode,
                       unsigned rate32, int* tile_cnt, hipStream_t stream) {
  if (n <= 0 || ntrees <= 0) return;
  const long long tiles = (n + RTILE - 1) / RTILE;
  forest_boot_count_kernel<<<dim3((unsigned)tiles, ntrees), FB_THREADS, 0, stream>>>(keys, n, row_off, mode, rate32,
                                                                                    tile_cnt);
  AV_HIP_CHECK(hipGetLastError());
}

void forest_boot_scatter(const uint8_t* codes, long long ld, int nfeat, const uint8_t* lab,
                         const unsigned long long* keys, int ntrees, long long n, long long row_off, int mode,
                         unsigned rate32, const long long* tile_off, uint8_t* dcodes, uint8_t* dlab, uint8_t* dwt,
                         long long ldb, hipStream_t stream) {
  if (n <= 0 || ntrees <= 0) return;
  const long long tiles = (n + RTILE - 1) / RTILE;
  forest_boot_scatter_kernel<<<dim3((unsigned)tiles, ntrees), FB_THREADS, 0, stream>>>(
      codes, ld, nfeat, lab, keys, n, row_off, mode, rate32, tile_off, dcodes, dlab, dwt, ldb);
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
