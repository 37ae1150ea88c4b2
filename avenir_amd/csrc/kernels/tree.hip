// K7 / K8: GPU decision-tree building blocks for CDNA4 (gfx950).
//
// The reference grows a tree one MapReduce job per level: every mapper re-emits each record once
// per (candidate attribute x candidate split predicate) and a reducer counts classes per child
// path (J/tree/DecisionTreeBuilder.java:209-359, :499-616, :730-767).  Here a level is:
//   1. node_hist      : ONE pass over the device-resident columns -> class counts
//                       hist[node][c][off_f + fine_bin]  (every candidate split of every attribute
//                       is a grouping of fine bins, so one histogram answers all of them),
//   2. split scoring  : batched on device from the histogram (host code, torch),
//   3. tree_assign    : one pass moving each row to its child node.
// node_grad_hist is the gradient-boosting variant (sum of g and h per bin, exact fixed point so
// results are bitwise reproducible across grid shapes and world sizes), and tree_predict is the
// batched inference kernel (ModelPredictor / DecisionTreeModel / EnsemblePredictiveModel).
#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

constexpr int TB_THREADS = 256;

// Both histogram kernels give each lane 4 consecutive rows per step: the node ids / labels / weights
// / gradients of the 4 rows and, for a chunk of 8 features, the 8 x 4 codes are fetched with wide
// loads before any LDS atomic is issued, so the HBM latency of a step is paid once instead of once
// per feature (the first version loaded one byte per feature and waited on each).
constexpr int FCH = 8;  // features whose codes are in flight together

// hist layout: [A][C][TB] uint64; node ids are LOCAL indices of the active frontier (-1 = skip).
// Each block owns a contiguous range of nodes [a0, a0 + na) held in LDS (uint32), so rows of other
// nodes are skipped; grid.y walks node chunks.
__global__ __launch_bounds__(TB_THREADS) void node_hist_kernel(
    const uint8_t* __restrict__ codes, long long ld, long long n, const uint8_t* __restrict__ labels,
    const int* __restrict__ node, const uint8_t* __restrict__ weight, const int* __restrict__ bins,
    const int* __restrict__ offs, int nfeat, int total_bins, int n_classes, int nodes_per_chunk,
    int n_nodes, const long long* __restrict__ node_rows, unsigned long long* __restrict__ hist) {
  extern __shared__ __attribute__((aligned(16))) unsigned int s_h[];
  const int a0 = blockIdx.y * nodes_per_chunk;
  const int na = min(nodes_per_chunk, n_nodes - a0);
  const int per_node = n_classes * total_bins;
  for (int i = threadIdx.x; i < na * per_node; i += TB_THREADS) s_h[i] = 0;
  // rows a chunk can hold: the union of its nodes' row ranges (a forest's trees are contiguous
  // row blocks, so a chunk of one tree's nodes scans that tree's rows only)
  long long lo = 0, hi = n;
  if (node_rows) {
    lo = n;
    hi = 0;
    for (int i = 0; i < na; ++i) {
      lo = min(lo, node_rows[2 * (a0 + i)]);
      hi = max(hi, node_rows[2 * (a0 + i) + 1]);
    }
    lo = max(lo, 0LL);
    hi = min(hi, n);
  }
  __syncthreads();
  const long long q1 = lo < hi ? (hi + 3) >> 2 : 0;  // 4-row quads (ld is a multiple of 16: quads never cross it)
  const long long stride = (long long)gridDim.x * TB_THREADS;
  for (long long q = (lo >> 2) + (long long)blockIdx.x * TB_THREADS + threadIdx.x; q < q1; q += stride) {
    const long long r0 = q * 4;
    const int4 nd4 = *reinterpret_cast<const int4*>(node + r0);
    const uchar4 lb4 = *reinterpret_cast<const uchar4*>(labels + r0);
    const uchar4 w4 = weight ? *reinterpret_cast<const uchar4*>(weight + r0) : make_uchar4(1, 1, 1, 1);
    int a[4] = {nd4.x - a0, nd4.y - a0, nd4.z - a0, nd4.w - a0};
    const unsigned c[4] = {lb4.x, lb4.y, lb4.z, lb4.w};
    const unsigned w[4] = {w4.x, w4.y, w4.z, w4.w};
    bool any = false;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool ok = r0 + j < n && a[j] >= 0 && a[j] < na && c[j] < (unsigned)n_classes && w[j] != 0;
      if (!ok) a[j] = -1;
      any |= ok;
    }
    if (!any) continue;
    for (int f0 = 0; f0 < nfeat; f0 += FCH) {
      uchar4 v4[FCH];
#pragma unroll
      for (int k = 0; k < FCH; ++k)
        if (f0 + k < nfeat) v4[k] = *reinterpret_cast<const uchar4*>(codes + (long long)(f0 + k) * ld + r0);
#pragma unroll
      for (int k = 0; k < FCH; ++k) {
        if (f0 + k >= nfeat) break;
        const unsigned B = (unsigned)bins[f0 + k], o = (unsigned)offs[f0 + k];
        const unsigned v[4] = {v4[k].x, v4[k].y, v4[k].z, v4[k].w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (a[j] >= 0 && v[j] < B) atomicAdd(&s_h[a[j] * per_node + c[j] * total_bins + o + v[j]], w[j]);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < na * per_node; i += TB_THREADS) {
    const unsigned v = s_h[i];
    if (v) atomicAdd(&hist[(long long)a0 * per_node + i], (unsigned long long)v);
  }
}

// Gradient-boosting histogram: per (node, bin) exact fixed-point sums of g and h (scale S = 2^16 per
// row, round to nearest; inputs |g| <= 1, 0 <= h <= 1 — deviance gradients / hessians).  ONE 64-bit LDS atomic per (row, feature): the slot holds
// (h_q << 32) + g_q (g_q sign-extended), whose wrapping 64-bit sum is (sum h_q << 32) + sum g_q as
// long as |sum g_q| < 2^31 — guaranteed because a block scans at most 2^14 rows (the host sizes
// the grid) and |g_q| <= 2^16; sum h_q < 2^32 likewise (h <= 1/4).  The flush splits the two sums
// and adds them to the int64 output [A][TB][2] (exact, order-independent).
// tot_slot >= 0: rows whose feature-0 code is missing (>= bins[0]) go to that slot, so feature 0's
// bins + tot_slot hold the node total (no separate all-rows feature).
constexpr long long GH_MAX_ROWS_PER_BLOCK = 1LL << 14;

__global__ __launch_bounds__(TB_THREADS) void node_grad_hist_kernel(
    const uint8_t* __restrict__ codes, long long ld, long long n, const int* __restrict__ node,
    const float* __restrict__ g, const float* __restrict__ h, const int* __restrict__ bins,
    const int* __restrict__ offs, int nfeat, int total_bins, int nodes_per_chunk, int n_nodes, int even_only,
    int tot_slot, float S, long long* __restrict__ out, int rep) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long s_all[];
  const int a0 = blockIdx.y * nodes_per_chunk;
  const int na = min(nodes_per_chunk, n_nodes - a0);
  const int per_node = total_bins;
  // rep replicas of the table (lane l adds into replica l % rep; odd stride: a word's copies sit in
  // different banks), summed before the flush — fewer same-word atomics from one wave
  const int rstride = (nodes_per_chunk * per_node) | 1;
  for (int i = threadIdx.x; i < rep * rstride; i += TB_THREADS) s_all[i] = 0ull;
  __syncthreads();
  unsigned long long* s_p = s_all + (threadIdx.x & (rep - 1)) * rstride;
  const long long nq = (n + 3) >> 2;
  const long long stride = (long long)gridDim.x * TB_THREADS;
  for (long long q = (long long)blockIdx.x * TB_THREADS + threadIdx.x; q < nq; q += stride) {
    const long long r0 = q * 4;
    const int4 nd4 = *reinterpret_cast<const int4*>(node + r0);
    int a[4] = {nd4.x, nd4.y, nd4.z, nd4.w};
    bool any = false;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      // even_only (GBT sibling subtraction): only rows of even (left) slots, counted at slot / 2
      if (even_only) a[j] = (a[j] < 0 || (a[j] & 1)) ? -1 : (a[j] >> 1);
      a[j] = a[j] < 0 ? -1 : a[j] - a0;
      const bool ok = r0 + j < n && a[j] >= 0 && a[j] < na;
      if (!ok) a[j] = -1;
      any |= ok;
    }
    if (!any) continue;
    const float4 g4 = *reinterpret_cast<const float4*>(g + r0);
    const float4 h4 = *reinterpret_cast<const float4*>(h + r0);
    const float gv[4] = {g4.x, g4.y, g4.z, g4.w}, hv[4] = {h4.x, h4.y, h4.z, h4.w};
    unsigned long long pk[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long long gq = __float2ll_rn(gv[j] * S), hq = __float2ll_rn(hv[j] * S);
      pk[j] = ((unsigned long long)hq << 32) + (unsigned long long)gq;
    }
    for (int f0 = 0; f0 < nfeat; f0 += FCH) {
      uchar4 v4[FCH];
#pragma unroll
      for (int k = 0; k < FCH; ++k)
        if (f0 + k < nfeat) v4[k] = *reinterpret_cast<const uchar4*>(codes + (long long)(f0 + k) * ld + r0);
#pragma unroll
      for (int k = 0; k < FCH; ++k) {
        if (f0 + k >= nfeat) break;
        const unsigned B = (unsigned)bins[f0 + k], o = (unsigned)offs[f0 + k];
        const unsigned v[4] = {v4[k].x, v4[k].y, v4[k].z, v4[k].w};
        const bool tot_here = f0 + k == 0 && tot_slot >= 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (a[j] < 0) continue;
          const int slot = v[j] < B ? (int)(o + v[j]) : (tot_here ? tot_slot : -1);
          if (slot >= 0) atomicAdd(&s_p[a[j] * per_node + slot], pk[j]);
        }
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < na * per_node; i += TB_THREADS) {
    unsigned long long v = s_all[i];
    for (int r = 1; r < rep; ++r) v += s_all[r * rstride + i];  // wrapping packed sums add exactly
    if (v) {
      const long long gs = (long long)(int)(unsigned)(v & 0xFFFFFFFFull);
      const long long hs = (long long)((v - (unsigned long long)gs) >> 32);
      long long* o = out + ((long long)a0 * per_node + i) * 2;
      if (gs) atomicAdd((unsigned long long*)&o[0], (unsigned long long)gs);
      if (hs) atomicAdd((unsigned long long*)&o[1], (unsigned long long)hs);
    }
  }
}

// Move every row of an expanding node to its child: child = child_of[a * max_seg + segmap[a][code]]
// (-1 = leaf / stopped: the row leaves the frontier).  Rows of non-expanding nodes (feat < 0) go -1.
__global__ __launch_bounds__(TB_THREADS) void tree_assign_kernel(
    const uint8_t* __restrict__ codes, long long ld, long long n, int* __restrict__ node,
    const int* __restrict__ split_feat, const short* __restrict__ segmap, int max_bins,
    const int* __restrict__ child_of, int max_seg) {
  const long long stride = (long long)gridDim.x * TB_THREADS;
  for (long long r = (long long)blockIdx.x * TB_THREADS + threadIdx.x; r < n; r += stride) {
    const int a = node[r];
    if (a < 0) continue;
    const int f = split_feat[a];
    int nxt = -1;
    if (f >= 0) {
      const unsigned v = codes[(long long)f * ld + r];
      if (v < (unsigned)max_bins) {
        const int seg = segmap[(long long)a * max_bins + v];
        if (seg >= 0) nxt = child_of[(long long)a * max_seg + seg];
      }
    }
    node[r] = nxt;
  }
}

// Batched inference over a forest of flattened trees.
//   node arrays (all trees concatenated): feat[k] (-1 = leaf), seg_base[k] (row into segmap),
//   child_base[k] (index into child), leaf value row leaf_idx[k] into values [L][V].
//   tree_root[t] = index of tree t's root.
// mode 0: out[r][V] += values[leaf]            (probability / regression sums)
// mode 1: out[r][argmax(values[leaf])] += w_t  (weighted majority vote, V = C)
__global__ __launch_bounds__(TB_THREADS) void tree_predict_kernel(
    const uint8_t* __restrict__ codes, long long ld, long long n, const int* __restrict__ feat,
    const int* __restrict__ seg_base, const short* __restrict__ segmap, int max_bins,
    const int* __restrict__ child_base, const int* __restrict__ child, const int* __restrict__ leaf_idx,
    const float* __restrict__ values, int V, const int* __restrict__ tree_root,
    const float* __restrict__ tree_w, int n_trees, int mode, float* __restrict__ out) {
  const long long stride = (long long)gridDim.x * TB_THREADS;
  for (long long r = (long long)blockIdx.x * TB_THREADS + threadIdx.x; r < n; r += stride) {
    for (int t = 0; t < n_trees; ++t) {
      int k = tree_root[t];
      int guard = 0;
      while (feat[k] >= 0 && guard++ < 4096) {
        const unsigned v = codes[(long long)feat[k] * ld + r];
        const int seg = v < (unsigned)max_bins ? segmap[(long long)seg_base[k] * max_bins + v] : -1;
        if (seg < 0) break;  // unseen value: predict from this internal node's distribution
        const int nk = child[child_base[k] + seg];
        if (nk < 0) break;
        k = nk;
      }
      const float* val = values + (long long)leaf_idx[k] * V;
      const float w = tree_w ? tree_w[t] : 1.f;
      if (mode == 0) {
        for (int j = 0; j < V; ++j) out[r * V + j] += w * val[j];
      } else {
        int best = 0;
        for (int j = 1; j < V; ++j)
          if (val[j] > val[best]) best = j;
        out[r * V + best] += w;
      }
    }
  }
}


// Binary-split forests (every internal node: code <= thr -> left, else right; the ForestBuilder /
// binary DecisionTreeBuilder output): the node table of ALL trees sits in LDS as 8-byte records
//   x = feat | thr << 8 | n_bins << 16   (feat 255 = leaf),   y = left | right << 16  (global ids)
// and every thread first copies its row's F codes (coalesced column loads) into an LDS row slot,
// so the traversal is LDS-only; per-tree node values (read once per tree at the stopping node)
// come from global memory and the V outputs accumulate in registers, written once per row.
// A code >= n_bins (missing / unseen) stops the walk at that node, as in tree_predict_kernel.
constexpr int FPB_MAXV = 8;
__global__ __launch_bounds__(TB_THREADS) void forest_predict_bin_kernel(
    const uint8_t* __restrict__ codes, long long ld, long long n, int nfeat, const uint2* __restrict__ nodes,
    int n_nodes, const float* __restrict__ values, int V, const int* __restrict__ tree_root,
    const float* __restrict__ tree_w, int n_trees, int mode, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char fp_smem[];
  uint2* s_nodes = reinterpret_cast<uint2*>(fp_smem);
  uint8_t* s_row = fp_smem + (size_t)n_nodes * sizeof(uint2) + threadIdx.x * nfeat;
  for (int i = threadIdx.x; i < n_nodes; i += TB_THREADS) s_nodes[i] = nodes[i];
  __syncthreads();
  const long long stride = (long long)gridDim.x * TB_THREADS;
  for (long long r = (long long)blockIdx.x * TB_THREADS + threadIdx.x; r < n; r += stride) {
    for (int f = 0; f < nfeat; ++f) s_row[f] = codes[(long long)f * ld + r];
    float acc[FPB_MAXV];
#pragma unroll
    for (int j = 0; j < FPB_MAXV; ++j) acc[j] = 0.f;
    for (int t = 0; t < n_trees; ++t) {
      int k = tree_root[t];
      for (int guard = 0; guard < 256; ++guard) {
        const uint2 nd = s_nodes[k];
        const unsigned f = nd.x & 0xFF;
        if (f == 0xFF) break;
        const unsigned v = s_row[f];
        if (v >= ((nd.x >> 16) & 0xFF)) break;
        k = (int)(v <= ((nd.x >> 8) & 0xFF) ? (nd.y & 0xFFFF) : (nd.y >> 16));
      }
      const float* val = values + (long long)k * V;
      const float w = tree_w ? tree_w[t] : 1.f;
      if (mode == 0) {
#pragma unroll
        for (int j = 0; j < FPB_MAXV; ++j)
          if (j < V) acc[j] += w * val[j];
      } else {
        int best = 0;
        float bv = val[0];
        for (int j = 1; j < V; ++j)
          if (val[j] > bv) { bv = val[j]; best = j; }
#pragma unroll
        for (int j = 0; j < FPB_MAXV; ++j)
          if (j == best) acc[j] += w;
      }
    }
#pragma unroll
    for (int j = 0; j < FPB_MAXV; ++j)
      if (j < V) out[r * V + j] += acc[j];
  }
}

}  // namespace

namespace avk {

// LDS per workgroup for the node tables: 32 KiB keeps 4+ workgroups per CU (measured better than
// 64 KiB even though more node chunks re-read the rows).
static long long tree_lds_budget() { return 32 * 1024; }

void node_histogram(const uint8_t* codes, long long ld, long long n, const uint8_t* labels,
                    const int* node, const uint8_t* weight, const int* bins, const int* offs,
                    int nfeat, int total_bins, int n_classes, int n_nodes, const long long* node_rows,
                    unsigned long long* hist, hipStream_t stream) {
  if (n <= 0 || n_nodes <= 0) return;
  const long long per_node_bytes = 4LL * n_classes * total_bins;
  if (per_node_bytes > 64 * 1024) throw std::runtime_error("node_histogram: per-node table exceeds LDS");
  const int npc = (int)std::max<long long>(1, std::min<long long>(n_nodes, tree_lds_budget() / per_node_bytes));
  const int chunks = (n_nodes + npc - 1) / npc;
  const int gx = std::max(1, std::min(av::stream_grid((n + 3) / 4, TB_THREADS, 2, 2048), std::max(64, 4096 / chunks)));
  dim3 grid(gx, chunks);
  node_hist_kernel<<<grid, TB_THREADS, per_node_bytes * npc, stream>>>(
      codes, ld, n, labels, node, weight, bins, offs, nfeat, total_bins, n_classes, npc, n_nodes, node_rows, hist);
  AV_HIP_CHECK(hipGetLastError());
}

void node_grad_histogram(const uint8_t* codes, long long ld, long long n, const int* node,
                         const float* g, const float* h, const int* bins, const int* offs, int nfeat,
                         int total_bins, int n_nodes, int even_only, int tot_slot, float scale, long long* out,
                         hipStream_t stream) {
  if (n <= 0 || n_nodes <= 0) return;
  if (scale > 65536.0f) throw std::runtime_error("node_grad_histogram: scale must be <= 2^16 (packed sums)");
  const long long per_node_bytes = 8LL * total_bins;
  if (per_node_bytes > 64 * 1024) throw std::runtime_error("node_grad_histogram: table exceeds LDS");
  const int npc = (int)std::max<long long>(1, std::min<long long>(n_nodes, tree_lds_budget() / per_node_bytes));
  const int chunks = (n_nodes + npc - 1) / npc;
  long long gx = std::max(1, std::min(av::stream_grid((n + 3) / 4, TB_THREADS, 2, 2048), std::max(64, 4096 / chunks)));
  // packed 32-bit partial sums: at most GH_MAX_ROWS_PER_BLOCK rows scanned per block
  const long long quads_per_block = GH_MAX_ROWS_PER_BLOCK / 4;
  const long long min_gx = ((n + 3) / 4 + quads_per_block - 1) / quads_per_block;
  gx = std::max(gx, min_gx);
  if (gx > 0x7fffffffLL) throw std::runtime_error("node_grad_histogram: too many rows");
  dim3 grid((unsigned)gx, chunks);
  // table replicas (opt-in, AVMI_GBT_HIST_REP=2|4): unlike the forest's 32-bit class counts they
  // do not pay for the 64-bit packed sums — GBT 120 x depth 3 at 16.7 M rows: 137 ms with one
  // table, 139-140 ms with 2 or 4 (profiles/r3_gbt_hist_replicas_ab.txt)
  const long long rbytes = 8LL * ((npc * (long long)total_bins) | 1);
  int rep = 1;
  const char* e = std::getenv("AVMI_GBT_HIST_REP");
  if (e && *e) {
    const int r = std::atoi(e);
    if ((r == 1 || r == 2 || r == 4) && rbytes * r <= 64 * 1024) rep = r;
  }
  node_grad_hist_kernel<<<grid, TB_THREADS, rbytes * rep, stream>>>(
      codes, ld, n, node, g, h, bins, offs, nfeat, total_bins, npc, n_nodes, even_only, tot_slot, scale, out, rep);
  AV_HIP_CHECK(hipGetLastError());
}

void tree_assign(const uint8_t* codes, long long ld, long long n, int* node, const int* split_feat,
                 const short* segmap, int max_bins, const int* child_of, int max_seg,
                 hipStream_t stream) {
  if (n <= 0) return;
  tree_assign_kernel<<<av::stream_grid(n, TB_THREADS, 4, 4096), TB_THREADS, 0, stream>>>(
      codes, ld, n, node, split_feat, segmap, max_bins, child_of, max_seg);
  AV_HIP_CHECK(hipGetLastError());
}

void tree_predict(const uint8_t* codes, long long ld, long long n, const int* feat, const int* seg_base,
                  const short* segmap, int max_bins, const int* child_base, const int* child,
                  const int* leaf_idx, const float* values, int V, const int* tree_root,
                  const float* tree_w, int n_trees, int mode, float* out, hipStream_t stream) {
  if (n <= 0 || n_trees <= 0) return;
  tree_predict_kernel<<<av::stream_grid(n, TB_THREADS, 2, 8192), TB_THREADS, 0, stream>>>(
      codes, ld, n, feat, seg_base, segmap, max_bins, child_base, child, leaf_idx, values, V,
      tree_root, tree_w, n_trees, mode, out);
  AV_HIP_CHECK(hipGetLastError());
}


long long forest_predict_bin_lds(int n_nodes, int nfeat) {
  return (long long)n_nodes * 8 + (long long)TB_THREADS * nfeat;
}

void forest_predict_bin(const uint8_t* codes, long long ld, long long n, int nfeat, const uint2* nodes, int n_nodes,
                        const float* values, int V, const int* tree_root, const float* tree_w, int n_trees, int mode,
                        float* out, hipStream_t stream) {
  if (n <= 0 || n_trees <= 0) return;
  const long long lds = forest_predict_bin_lds(n_nodes, nfeat);
  if (lds > 160 * 1024 || V > FPB_MAXV) throw std::runtime_error("forest_predict_bin: forest too large for LDS");
  AV_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(forest_predict_bin_kernel),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  forest_predict_bin_kernel<<<av::stream_grid(n, TB_THREADS, 1, 4096), TB_THREADS, (size_t)lds, stream>>>(
      codes, ld, n, nfeat, nodes, n_nodes, values, V, tree_root, tree_w, n_trees, mode, out);
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
