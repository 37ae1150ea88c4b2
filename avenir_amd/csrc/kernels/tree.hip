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

// hist layout: [A][C][TB] uint64; node ids are LOCAL indices of the active frontier (-1 = skip).
// Each block owns a contiguous range of nodes [a0, a0 + na) held in LDS (uint32), so rows of other
// nodes are skipped; grid.y walks node chunks.
__global__ __launch_bounds__(TB_THREADS) void node_hist_kernel(
    const uint8_t* __restrict__ codes, long long ld, long long n, const uint8_t* __restrict__ labels,
    const int* __restrict__ node, const uint8_t* __restrict__ weight, const int* __restrict__ bins,
    const int* __restrict__ offs, int nfeat, int total_bins, int n_classes, int nodes_per_chunk,
    int n_nodes, unsigned long long* __restrict__ hist) {
  extern __shared__ __attribute__((aligned(16))) unsigned int s_h[];
  const int a0 = blockIdx.y * nodes_per_chunk;
  const int na = min(nodes_per_chunk, n_nodes - a0);
  const int per_node = n_classes * total_bins;
  for (int i = threadIdx.x; i < na * per_node; i += TB_THREADS) s_h[i] = 0;
  __syncthreads();
  const long long stride = (long long)gridDim.x * TB_THREADS;
  for (long long r = (long long)blockIdx.x * TB_THREADS + threadIdx.x; r < n; r += stride) {
    const int a = node[r] - a0;
    if (a < 0 || a >= na) continue;
    const unsigned c = labels[r];
    if (c >= (unsigned)n_classes) continue;
    const unsigned w = weight ? weight[r] : 1u;
    if (w == 0) continue;
    unsigned int* h = s_h + a * per_node + c * total_bins;
    for (int f = 0; f < nfeat; ++f) {
      const unsigned v = codes[(long long)f * ld + r];
      if (v < (unsigned)bins[f]) atomicAdd(&h[offs[f] + v], w);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < na * per_node; i += TB_THREADS) {
    const unsigned v = s_h[i];
    if (v) atomicAdd(&hist[(long long)a0 * per_node + i], (unsigned long long)v);
  }
}

// Gradient-boosting histogram: per (node, bin) exact fixed-point sums of g and h (scale 2^24),
// accumulated as int64 in LDS (ds_add_u64 is exact and order-independent).  out: [A][TB][2].
__global__ __launch_bounds__(TB_THREADS) void node_grad_hist_kernel(
    const uint8_t* __restrict__ codes, long long ld, long long n, const int* __restrict__ node,
    const float* __restrict__ g, const float* __restrict__ h, const int* __restrict__ bins,
    const int* __restrict__ offs, int nfeat, int total_bins, int nodes_per_chunk, int n_nodes,
    long long* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) long long s_g[];
  const int a0 = blockIdx.y * nodes_per_chunk;
  const int na = min(nodes_per_chunk, n_nodes - a0);
  const int per_node = total_bins * 2;
  for (int i = threadIdx.x; i < na * per_node; i += TB_THREADS) s_g[i] = 0;
  __syncthreads();
  const long long stride = (long long)gridDim.x * TB_THREADS;
  const float S = 16777216.0f;
  for (long long r = (long long)blockIdx.x * TB_THREADS + threadIdx.x; r < n; r += stride) {
    const int a = node[r] - a0;
    if (a < 0 || a >= na) continue;
    const long long gi = __float2ll_rn(g[r] * S);
    const long long hi = __float2ll_rn(h[r] * S);
    long long* base = s_g + a * per_node;
    for (int f = 0; f < nfeat; ++f) {
      const unsigned v = codes[(long long)f * ld + r];
      if (v < (unsigned)bins[f]) {
        const int b = offs[f] + v;
        atomicAdd((unsigned long long*)&base[2 * b], (unsigned long long)gi);
        atomicAdd((unsigned long long*)&base[2 * b + 1], (unsigned long long)hi);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < na * per_node; i += TB_THREADS) {
    const long long v = s_g[i];
    if (v) atomicAdd((unsigned long long*)&out[(long long)a0 * per_node + i], (unsigned long long)v);
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

}  // namespace

namespace avk {

void node_histogram(const uint8_t* codes, long long ld, long long n, const uint8_t* labels,
                    const int* node, const uint8_t* weight, const int* bins, const int* offs,
                    int nfeat, int total_bins, int n_classes, int n_nodes, unsigned long long* hist,
                    hipStream_t stream) {
  if (n <= 0 || n_nodes <= 0) return;
  const long long per_node_bytes = 4LL * n_classes * total_bins;
  if (per_node_bytes > 64 * 1024) throw std::runtime_error("node_histogram: per-node table exceeds LDS");
  const int npc = (int)std::max<long long>(1, std::min<long long>(n_nodes, (64 * 1024) / per_node_bytes));
  const int chunks = (n_nodes + npc - 1) / npc;
  const int gx = std::max(1, std::min(av::stream_grid(n, TB_THREADS, 8, 2048), std::max(64, 4096 / chunks)));
  dim3 grid(gx, chunks);
  node_hist_kernel<<<grid, TB_THREADS, per_node_bytes * npc, stream>>>(
      codes, ld, n, labels, node, weight, bins, offs, nfeat, total_bins, n_classes, npc, n_nodes, hist);
  AV_HIP_CHECK(hipGetLastError());
}

void node_grad_histogram(const uint8_t* codes, long long ld, long long n, const int* node,
                         const float* g, const float* h, const int* bins, const int* offs, int nfeat,
                         int total_bins, int n_nodes, long long* out, hipStream_t stream) {
  if (n <= 0 || n_nodes <= 0) return;
  const long long per_node_bytes = 16LL * total_bins;
  if (per_node_bytes > 64 * 1024) throw std::runtime_error("node_grad_histogram: table exceeds LDS");
  const int npc = (int)std::max<long long>(1, std::min<long long>(n_nodes, (64 * 1024) / per_node_bytes));
  const int chunks = (n_nodes + npc - 1) / npc;
  const int gx = std::max(1, std::min(av::stream_grid(n, TB_THREADS, 8, 2048), std::max(64, 4096 / chunks)));
  dim3 grid(gx, chunks);
  node_grad_hist_kernel<<<grid, TB_THREADS, per_node_bytes * npc, stream>>>(
      codes, ld, n, node, g, h, bins, offs, nfeat, total_bins, npc, n_nodes, out);
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

}  // namespace avk
