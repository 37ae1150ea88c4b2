// K17: Apriori support counting on transaction bitsets (CDNA4, gfx950).
//
// The reference re-scans transactions in every mapper and emits (itemset -> transId/1) for each
// candidate contained in a transaction (J/association/FrequentItemsApriori.java:133-196,
// S/association/FrequentItemsApriori.scala:222-276).  Here every item is a bit row over
// transactions ([I][W] uint64, W = T/64) and every frequent (k-1)-itemset keeps its tid bitset from
// the previous level, so a k-candidate = (prefix bitset p, extension item j) and its support is
// popcount(P[p] & items[j]) — pure streaming AND + v_bcnt, 32 candidates per block with per-lane
// 32-bit partials and one wave reduction per candidate.
#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

constexpr int AT = 256;
constexpr int CPB = 32;   // candidates per block
constexpr int WPT = 16;   // words per thread

__global__ __launch_bounds__(AT) void support_kernel(const unsigned long long* __restrict__ P, int W,
                                                     const unsigned long long* __restrict__ items,
                                                     const int* __restrict__ cand_prefix,
                                                     const int* __restrict__ cand_item, int M,
                                                     unsigned long long* __restrict__ support) {
  const int c0 = blockIdx.x * CPB;
  const long long w0 = (long long)blockIdx.y * AT * WPT;
  __shared__ unsigned int s_red[AT / 64][CPB];
  const int ncand = min(CPB, M - c0);
  for (int c = 0; c < ncand; ++c) {  // block-uniform trip count
    const unsigned long long* pr = P + (long long)cand_prefix[c0 + c] * W;
    const unsigned long long* it = items + (long long)cand_item[c0 + c] * W;
    unsigned int s = 0;
#pragma unroll
    for (int q = 0; q < WPT; ++q) {
      const long long w = w0 + (long long)q * AT + threadIdx.x;  // coalesced across the block
      if (w < W) s += __popcll(pr[w] & it[w]);
    }
    s = av::wave_sum(s);
    if (av::lane_id() == 0) s_red[av::wave_id()][c] = s;
  }
  __syncthreads();
  if (threadIdx.x < CPB && c0 + threadIdx.x < M) {
    unsigned long long t = 0;
#pragma unroll
    for (int w = 0; w < AT / 64; ++w) t += s_red[w][threadIdx.x];
    if (t) atomicAdd(&support[c0 + threadIdx.x], t);
  }
}

// bits[item][t >> 6] |= 1 << (t & 63) for every (transaction, item) pair
__global__ __launch_bounds__(AT) void build_bitsets_kernel(const long long* __restrict__ tx,
                                                           const int* __restrict__ item, long long n,
                                                           int W, int n_items,
                                                           unsigned long long* __restrict__ bits) {
  const long long stride = (long long)gridDim.x * AT;
  for (long long i = (long long)blockIdx.x * AT + threadIdx.x; i < n; i += stride) {
    const long long t = tx[i];
    const int it = item[i];
    if (it < 0 || it >= n_items || t < 0 || (t >> 6) >= W) continue;
    atomicOr(&bits[(long long)it * W + (t >> 6)], 1ull << (t & 63));
  }
}

}  // namespace

namespace avk {

void itemset_support(const unsigned long long* P, int W, const unsigned long long* items,
                     const int* cand_prefix, const int* cand_item, int M, unsigned long long* support,
                     hipStream_t stream) {
  if (M <= 0 || W <= 0) return;
  dim3 grid((M + CPB - 1) / CPB, (unsigned)((W + AT * WPT - 1) / (AT * WPT)));
  support_kernel<<<grid, AT, 0, stream>>>(P, W, items, cand_prefix, cand_item, M, support);
  AV_HIP_CHECK(hipGetLastError());
}

void build_bitsets(const long long* tx, const int* item, long long n, int W, int n_items,
                   unsigned long long* bits, hipStream_t stream) {
  if (n <= 0) return;
  build_bitsets_kernel<<<av::stream_grid(n, AT, 4, 4096), AT, 0, stream>>>(tx, item, n, W, n_items, bits);
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
