// K18 GSP candidate self-join for CDNA4 (gfx950).
//
// Reference: CandidateGenerationWithSelfJoin replicates every frequent k-sequence to all hash
// bucket pairs and joins pairs in the reducer on a slide-by-1 overlap
// (J/sequence/CandidateGenerationWithSelfJoin.java:116-144, 175-276).  Here the k-sequences are
// rows of a lexicographically SORTED int32 matrix X [N, k] (dense token ids), so all rows b with
// the same (k-1)-prefix b[0:k-1] are contiguous.  For a left row a the partners are exactly the
// rows whose prefix equals a's suffix a[1:k]: two binary searches (lower/upper bound) give the
// segment, and the candidates a ++ b[k-1] are written to a compacted output.
//
//   gsp_count_kernel: one lane per left row -> segment start and length (the comparisons read
//                     k-1 ints per probe; X is small and L2-resident, lanes of a wave walk
//                     neighbouring a's whose suffixes are close, so probes coalesce well);
//   (host)            exclusive scan of the lengths -> output offsets;
//   gsp_emit_kernel:  one WAVE per left row: its lanes stride over the row's segment, each lane
//                     writes one candidate (k+1 ints), so a long segment is written by 64 lanes.
//
// Every lane that reads X does so with row indices inside [0, N) and every candidate slot lies
// inside [offset[a], offset[a] + len[a]), which the host sized from the same lengths.
#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

// lexicographic compare of X[row, 0:k-1] against key[0:k-1] (key = a's suffix)
__device__ __forceinline__ int cmp_prefix(const int* __restrict__ X, int k, int row, const int* __restrict__ key) {
  const int* r = X + (long long)row * k;
  for (int j = 0; j < k - 1; ++j) {
    const int x = r[j], y = key[j];
    if (x != y) return x < y ? -1 : 1;
  }
  return 0;
}

__global__ __launch_bounds__(256) void gsp_count_kernel(const int* __restrict__ X, int N, int k, int lo, int hi,
                                                          int* __restrict__ seg_start, int* __restrict__ seg_len) {
  const int a = lo + blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= hi) return;
  const int* key = X + (long long)a * k + 1;  // suffix a[1:k]
  int l = 0, h = N;                            // first row with prefix >= key
  while (l < h) {
    const int m = (l + h) >> 1;
    if (cmp_prefix(X, k, m, key) < 0) l = m + 1; else h = m;
  }
  int l2 = l, h2 = N;                          // first row with prefix > key
  while (l2 < h2) {
    const int m = (l2 + h2) >> 1;
    if (cmp_prefix(X, k, m, key) <= 0) l2 = m + 1; else h2 = m;
  }
  seg_start[a - lo] = l;
  seg_len[a - lo] = l2 - l;
}

__global__ __launch_bounds__(256) void gsp_emit_kernel(const int* __restrict__ X, int k, int lo, int hi,
                                                         const int* __restrict__ seg_start,
                                                         const int* __restrict__ seg_len,
                                                         const long long* __restrict__ offs, int* __restrict__ out) {
  const int waves = blockDim.x >> 6;
  const int a_rel = blockIdx.x * waves + av::wave_id();
  if (a_rel >= hi - lo) return;
  const int a = lo + a_rel;
  const int s = seg_start[a_rel], n = seg_len[a_rel];
  const long long o = offs[a_rel];
  const int* ra = X + (long long)a * k;
  for (int i = av::lane_id(); i < n; i += AV_WAVE) {
    int* dst = out + (o + i) * (long long)(k + 1);
    for (int j = 0; j < k; ++j) dst[j] = ra[j];
    dst[k] = X[(long long)(s + i) * k + (k - 1)];
  }
}

}  // namespace

namespace avk {

void gsp_count(const int* X, int N, int k, int lo, int hi, int* seg_start, int* seg_len, hipStream_t stream) {
  const int n = hi - lo;
  if (n <= 0) return;
  gsp_count_kernel<<<(n + 255) / 256, 256, 0, stream>>>(X, N, k, lo, hi, seg_start, seg_len);
  AV_HIP_CHECK(hipGetLastError());
}

void gsp_emit(const int* X, int k, int lo, int hi, const int* seg_start, const int* seg_len, const long long* offs,
              int* out, hipStream_t stream) {
  const int n = hi - lo;
  if (n <= 0) return;
  gsp_emit_kernel<<<(n + 3) / 4, 256, 0, stream>>>(X, k, lo, hi, seg_start, seg_len, offs, out);
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
