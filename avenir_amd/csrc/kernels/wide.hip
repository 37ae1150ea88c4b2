// K2w: class-conditional histogram over 16-bit dictionary codes (high-cardinality categoricals).
//
// The reference keys every categorical by its raw string, so a field may hold any number of
// values (e.g. the supplier / product ids of the high-cardinality `hica` driver,
// J/explore/CategoricalContinuousEncoding.java:116-137, S/explore/CategoricalLeaveOneOutEncoding.scala:80).
// Tables whose binned fields exceed 255 values carry uint16 codes [F, ld] (65535 = missing), and
// beyond 65,534 values int32 codes (INT32_MAX = missing); these kernels count both (templated on the
// code type; the unsigned compare against bins[f] skips missing codes).
//
// Layout: counters are u32 slots c * TB + off_f + code.  When the whole [C, TB] table fits in LDS
// (<= 36 K counters = 144 KiB of the 160 KiB per CU) each workgroup privatises it: one 1024-thread
// block per CU, rows grid-strided so every block amortises its zero + flush over many records, and
// the flush adds only non-zero slots to the int64 output (global atomics).  Larger tables
// (e.g. 10^5-value fields x many classes) use direct 64-bit global atomics; their slots are spread
// over so many cache lines that contention stays low.
#include <algorithm>

#include "avenir_common.h"

namespace {

constexpr int kWideThreads = 1024;
constexpr int kLdsSlots = 36 * 1024;

template <typename CT>
__global__ __launch_bounds__(kWideThreads) void hist_wide_lds_kernel(
    const CT* __restrict__ codes, long long ld, long long n, const uint8_t* __restrict__ labels,
    const int* __restrict__ bins, const int* __restrict__ offs, int nfeat, int total_bins, int n_classes,
    int count_labels, unsigned long long* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned int s_tab[];
  const int slots = n_classes * total_bins;
  for (int i = threadIdx.x; i < slots; i += kWideThreads) s_tab[i] = 0u;
  __syncthreads();
  const long long stride = (long long)gridDim.x * kWideThreads;
  for (long long r = (long long)blockIdx.x * kWideThreads + threadIdx.x; r < n; r += stride) {
    const int c = labels ? (int)labels[r] : 0;
    if (c >= n_classes) continue;
    unsigned int* row = s_tab + c * total_bins;
    if (count_labels) atomicAdd(&row[total_bins - 1], 1u);
    for (int f = 0; f < nfeat; ++f) {
      // coalesced: consecutive lanes, consecutive rows; unsigned compare skips the missing code
      const unsigned v = (unsigned)codes[(long long)f * ld + r];
      if (v < (unsigned)bins[f]) atomicAdd(&row[offs[f] + v], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < slots; i += kWideThreads) {
    const unsigned int v = s_tab[i];
    if (v) atomicAdd(&out[i], (unsigned long long)v);
  }
}

template <typename CT>
__global__ __launch_bounds__(256) void hist_wide_global_kernel(
    const CT* __restrict__ codes, long long ld, long long n, const uint8_t* __restrict__ labels,
    const int* __restrict__ bins, const int* __restrict__ offs, int nfeat, int total_bins, int n_classes,
    int count_labels, unsigned long long* __restrict__ out) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long r = (long long)blockIdx.x * 256 + threadIdx.x; r < n; r += stride) {
    const int c = labels ? (int)labels[r] : 0;
    if (c >= n_classes) continue;
    unsigned long long* row = out + (long long)c * total_bins;
    if (count_labels) atomicAdd(&row[total_bins - 1], 1ull);
    for (int f = 0; f < nfeat; ++f) {
      const unsigned v = (unsigned)codes[(long long)f * ld + r];
      if (v < (unsigned)bins[f]) atomicAdd(&row[(long long)offs[f] + v], 1ull);
    }
  }
}

int num_cus() {  // of the current device, queried per call (a host attribute read)
  int dev = 0, cus = 0;
  AV_HIP_CHECK(hipGetDevice(&dev));
  AV_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  return cus;
}

}  // namespace

namespace avk {

template <typename CT>
void hist_wide(const CT* codes, long long ld, long long n, const uint8_t* labels, const int* d_bins, const int* d_offs,
               int nfeat, int total_bins, int n_classes, int count_labels, unsigned long long* out, int mode,
               hipStream_t stream) {
  if (n <= 0) return;
  const long long slots = (long long)n_classes * total_bins;
  if (mode != 2 && slots <= kLdsSlots) {
    const size_t lds = (size_t)slots * sizeof(unsigned int);
    // set on every call: the attribute belongs to the current device (no process-wide cache)
    AV_HIP_CHECK(hipFuncSetAttribute((const void*)hist_wide_lds_kernel<CT>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, kLdsSlots * 4));
    // one block per CU (the table takes most of the LDS), never more blocks than row tiles
    const long long tiles = (n + kWideThreads - 1) / kWideThreads;
    const int grid = (int)std::min<long long>(tiles, (long long)num_cus());
    hist_wide_lds_kernel<CT><<<grid, kWideThreads, lds, stream>>>(codes, ld, n, labels, d_bins, d_offs, nfeat,
                                                                  total_bins, n_classes, count_labels, out);
  } else {
    const long long tiles = (n + 255) / 256;
    const int grid = (int)std::min<long long>(tiles, (long long)num_cus() * 8);
    hist_wide_global_kernel<CT><<<grid, 256, 0, stream>>>(codes, ld, n, labels, d_bins, d_offs, nfeat, total_bins,
                                                          n_classes, count_labels, out);
  }
  AV_HIP_CHECK(hipGetLastError());
}

void class_histogram_wide(const uint16_t* codes, long long ld, long long n, const uint8_t* labels, const int* d_bins,
                          const int* d_offs, int nfeat, int total_bins, int n_classes, int count_labels,
                          unsigned long long* out, int mode, hipStream_t stream) {
  hist_wide<uint16_t>(codes, ld, n, labels, d_bins, d_offs, nfeat, total_bins, n_classes, count_labels, out, mode,
                      stream);
}

// int32 codes (categoricals beyond 65,534 values; missing = INT32_MAX)
void class_histogram_i32(const int* codes, long long ld, long long n, const uint8_t* labels, const int* d_bins,
                         const int* d_offs, int nfeat, int total_bins, int n_classes, int count_labels,
                         unsigned long long* out, int mode, hipStream_t stream) {
  hist_wide<int>(codes, ld, n, labels, d_bins, d_offs, nfeat, total_bins, n_classes, count_labels, out, mode, stream);
}

}  // namespace avk
