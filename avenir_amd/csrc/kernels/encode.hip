// K23 encoding transforms + K26 column statistics for CDNA4 (gfx950).
//
// K26 col_moments_kernel: per-column count / sum / min / max (pass 0) and central power sums
//   sum d^2, d^3, d^4 about the pass-0 mean (pass 1) of a column-major [F, ld] matrix.  Two
//   passes instead of a one-pass Welford merge: both are HBM-bound streams, and the two-pass
//   central sums are exact to fp64 rounding, which the skew / kurtosis of P/mlextra/daexp.py
//   getStats (and NumericalCorrelation's moments) need.  Grid (nblk, F): every block streams one
//   column slice with 16-byte loads (fp32) and fp64 accumulators, reduces wave -> block in a
//   fixed order and writes ONE partial row; the host sums the [F, nblk] partials with a
//   fixed-shape reduction, so the result is bit-reproducible run to run (no float atomics).
//   NaN entries are skipped (the reference's null handling).
//
// K23 leave-one-out target encoding.  The kernel formula is a superset: with gmean = 0, amp = 1 and
//   u = (z + 1) / 2 it is S/explore/CategoricalLeaveOneOutEncoding.scala:110-125
//   ((posSum - y) / (count - 1 + reg) * (1 + z), z truncated Gaussian; models/explore.py
//   leave_one_out_encoding(formula="reference")); gmean != 0 is the "smoothed" variant, not in the
//   reference.
//   loo_stats_kernel: per (column, code) target sum and count.  uint8 codes: a block privatises
//     the 256-slot table in LDS (fp64 ds_add + u32 counters), then flushes the touched slots with
//     global atomics; uint16 ("wide", > 255 values) and int32 (> 65,534 values) codes go to global
//     atomics directly.
//   loo_apply_kernel: out[i, j] = (sum[c] - y_i + reg * gmean) / max(cnt[c] - 1 + reg, 1e-12)
//     (x (1 + amp * (2u - 1)) with the caller's uniforms u [F, n], one stream per column), fused gather + formula + layout
//     change: a block stages a [Fc, 256] code tile (columns contiguous, coalesced reads) in LDS and
//     writes the row-major [256, Fc] output tile with consecutive lanes on consecutive floats.
//
// Index safety: every load is inside [0, n) of its column; code values index tables of m slots
// with m = 256 (uint8) or 65536 (uint16), so any code value is in range by construction; int32
// codes (> 65,534 values) are clamped to the last slot m - 1 (missing / out of range).
#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

constexpr int MOM_THREADS = 256;

__device__ __forceinline__ void mom_acc0(double x, double& c, double& s, double& lo, double& hi) {
  if (x == x) {  // skip NaN
    c += 1.0;
    s += x;
    lo = fmin(lo, x);
    hi = fmax(hi, x);
  }
}

__device__ __forceinline__ void mom_acc1(double x, double m, double& a2, double& a3, double& a4) {
  if (x == x) {
    const double d = x - m, d2 = d * d;
    a2 += d2;
    a3 += d2 * d;
    a4 += d2 * d2;
  }
}

template <typename T, int PASS>
__global__ __launch_bounds__(MOM_THREADS) void col_moments_kernel(const T* __restrict__ X, long long n, long long ld,
                                                                  const double* __restrict__ mean,
                                                                  double* __restrict__ part) {
  const int f = blockIdx.y, nblk = gridDim.x;
  const T* col = X + (long long)f * ld;
  double r0 = 0.0, r1 = 0.0, r2, r3;
  double m = 0.0;
  if (PASS == 0) {
    r2 = __builtin_inf();
    r3 = -__builtin_inf();
  } else {
    r2 = r3 = 0.0;
    m = mean[f];
  }
  const long long stride = (long long)nblk * MOM_THREADS;
  if constexpr (sizeof(T) == 4) {
    // 16-byte loads over the aligned body; the binding guarantees ld % 4 == 0 and alignment
    const long long n4 = n >> 2;
    const float4* c4 = reinterpret_cast<const float4*>(col);
    for (long long i = (long long)blockIdx.x * MOM_THREADS + threadIdx.x; i < n4; i += stride) {
      const float4 v = c4[i];
      if (PASS == 0) {
        mom_acc0(v.x, r0, r1, r2, r3); mom_acc0(v.y, r0, r1, r2, r3);
        mom_acc0(v.z, r0, r1, r2, r3); mom_acc0(v.w, r0, r1, r2, r3);
      } else {
        mom_acc1(v.x, m, r0, r1, r2); mom_acc1(v.y, m, r0, r1, r2);
        mom_acc1(v.z, m, r0, r1, r2); mom_acc1(v.w, m, r0, r1, r2);
      }
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
      const double x = col[(n4 << 2) + threadIdx.x];
      if (PASS == 0) mom_acc0(x, r0, r1, r2, r3); else mom_acc1(x, m, r0, r1, r2);
    }
  } else {
    for (long long i = (long long)blockIdx.x * MOM_THREADS + threadIdx.x; i < n; i += stride) {
      const double x = col[i];
      if (PASS == 0) mom_acc0(x, r0, r1, r2, r3); else mom_acc1(x, m, r0, r1, r2);
    }
  }
  r0 = av::wave_sum(r0);
  r1 = av::wave_sum(r1);
  if (PASS == 0) {
    r2 = av::wave_min(r2);
    r3 = av::wave_max(r3);
  } else {
    r2 = av::wave_sum(r2);
  }
  __shared__ double red[MOM_THREADS / AV_WAVE][4];
  const int w = av::wave_id();
  if (av::lane_id() == 0) {
    red[w][0] = r0; red[w][1] = r1; red[w][2] = r2; red[w][3] = r3;
  }
  __syncthreads();
  if (threadIdx.x < 4) {  // fixed-order combine of the 4 waves: deterministic
    const int q = threadIdx.x;
    double a = red[0][q];
    for (int k = 1; k < MOM_THREADS / AV_WAVE; ++k) {
      const double b = red[k][q];
      if (PASS == 0 && q == 2) a = fmin(a, b);
      else if (PASS == 0 && q == 3) a = fmax(a, b);
      else a += b;
    }
    part[((long long)f * nblk + blockIdx.x) * 4 + q] = a;
  }
}

// ---- K23 leave-one-out -------------------------------------------------------------------------
constexpr int LOO_THREADS = 256;

template <typename CT>
__global__ __launch_bounds__(LOO_THREADS) void loo_stats_kernel(const CT* __restrict__ codes, long long ld, long long n,
                                                                const double* __restrict__ y, double* __restrict__ sum,
                                                                unsigned* __restrict__ cnt, int m) {
  const int f = blockIdx.y;
  const CT* col = codes + (long long)f * ld;
  const long long stride = (long long)gridDim.x * LOO_THREADS;
  if constexpr (sizeof(CT) == 1) {
    __shared__ double s_sum[256];
    __shared__ unsigned s_cnt[256];
    s_sum[threadIdx.x] = 0.0;
    s_cnt[threadIdx.x] = 0u;
    __syncthreads();
    for (long long i = (long long)blockIdx.x * LOO_THREADS + threadIdx.x; i < n; i += stride) {
      const int c = col[i];
      atomicAdd(&s_sum[c], y[i]);
      atomicAdd(&s_cnt[c], 1u);
    }
    __syncthreads();
    const unsigned k = s_cnt[threadIdx.x];
    if (k) {
      atomicAdd(&sum[(long long)f * 256 + threadIdx.x], s_sum[threadIdx.x]);
      atomicAdd(&cnt[(long long)f * 256 + threadIdx.x], k);
    }
  } else {
    const unsigned top = (unsigned)(m - 1);  // the missing / out-of-range slot
    for (long long i = (long long)blockIdx.x * LOO_THREADS + threadIdx.x; i < n; i += stride) {
      const unsigned v = (unsigned)col[i];
      const long long c = (long long)f * m + (v < top ? v : top);
      atomicAdd(&sum[c], y[i]);
      atomicAdd(&cnt[c], 1u);
    }
  }
}

// Wide codes (uint16 / int32) whose per-column table fits LDS (m slots x (fp64 sum + u32 count)
// <= 144 KiB, i.e. up to ~12 k values): 1024-thread blocks privatise the column's table in LDS
// (native ds_add_f64), then flush only the touched slots with global atomics — one atomic pair
// per (block, value) instead of per row.
constexpr int LOO_WIDE_T = 1024;
constexpr size_t LOO_WIDE_LDS = 144 * 1024;

template <typename CT>
__global__ __launch_bounds__(LOO_WIDE_T) void loo_stats_lds_kernel(const CT* __restrict__ codes, long long ld,
                                                                   long long n, const double* __restrict__ y,
                                                                   double* __restrict__ sum,
                                                                   unsigned* __restrict__ cnt, int m) {
  extern __shared__ double s_dyn[];
  double* s_sum = s_dyn;
  unsigned* s_cnt = reinterpret_cast<unsigned*>(s_dyn + m);
  const int f = blockIdx.y;
  const CT* col = codes + (long long)f * ld;
  for (int i = threadIdx.x; i < m; i += LOO_WIDE_T) {
    s_sum[i] = 0.0;
    s_cnt[i] = 0u;
  }
  __syncthreads();
  const unsigned top = (unsigned)(m - 1);
  const long long stride = (long long)gridDim.x * LOO_WIDE_T;
  for (long long i = (long long)blockIdx.x * LOO_WIDE_T + threadIdx.x; i < n; i += stride) {
    const unsigned v = (unsigned)col[i];
    const unsigned c = v < top ? v : top;
    atomicAdd(&s_sum[c], y[i]);
    atomicAdd(&s_cnt[c], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < m; i += LOO_WIDE_T) {
    const unsigned k = s_cnt[i];
    if (k) {
      atomicAdd(&sum[(long long)f * m + i], s_sum[i]);
      atomicAdd(&cnt[(long long)f * m + i], k);
    }
  }
}

constexpr int LOO_TILE_F = 32;  // columns per tile -> [32][256] u32 = 32 KB of LDS

template <typename CT>
__global__ __launch_bounds__(LOO_THREADS) void loo_apply_kernel(const CT* __restrict__ codes, long long ld, long long n,
                                                                int F, const double* __restrict__ y,
                                                                const double* __restrict__ sum,
                                                                const unsigned* __restrict__ cnt, int m,
                                                                const double* __restrict__ gmean, double reg,
                                                                const double* __restrict__ noise, double amp,
                                                                float* __restrict__ out) {
  __shared__ unsigned tile[LOO_TILE_F][LOO_THREADS];
  __shared__ double ys[LOO_THREADS];
  const long long r0 = (long long)blockIdx.x * LOO_THREADS;
  const int f0 = blockIdx.y * LOO_TILE_F;
  const int fc = min(LOO_TILE_F, F - f0);
  const int rows = (int)min((long long)LOO_THREADS, n - r0);
  const int t = threadIdx.x;
  if (t < rows) {
    ys[t] = y[r0 + t];
    const unsigned top = (unsigned)(m - 1);
    for (int j = 0; j < fc; ++j) {
      const unsigned v = (unsigned)codes[(long long)(f0 + j) * ld + r0 + t];
      tile[j][t] = v < top ? v : top;
    }
  }
  __syncthreads();
  const double gm = reg * gmean[0];
  for (int e = t; e < rows * fc; e += LOO_THREADS) {
    const int r = e / fc, j = e - r * fc;
    const long long slot = (long long)(f0 + j) * m + tile[j][r];
    double v = (sum[slot] - ys[r] + gm) / fmax((double)cnt[slot] - 1.0 + reg, 1e-12);
    if (noise) v *= 1.0 + amp * (2.0 * noise[(long long)(f0 + j) * n + r0 + r] - 1.0);
    out[(r0 + r) * F + f0 + j] = (float)v;
  }
}

int mom_blocks(long long n, int F) {
  const long long per = (long long)MOM_THREADS * 16;  // >= 16 elements per thread
  long long b = (n + per - 1) / per;
  const long long want = (2048 + F - 1) / F;           // fill 256 CUs x 8 blocks
  if (b > want) b = want;
  return (int)(b < 1 ? 1 : b);
}

}  // namespace

namespace avk {

int col_moments_blocks(long long n, int F) { return mom_blocks(n, F); }

void col_moments_f32(const float* X, long long n, long long ld, int F, int pass, const double* mean, double* part,
                     hipStream_t stream) {
  const dim3 grid(mom_blocks(n, F), F);
  if (pass == 0) col_moments_kernel<float, 0><<<grid, MOM_THREADS, 0, stream>>>(X, n, ld, mean, part);
  else col_moments_kernel<float, 1><<<grid, MOM_THREADS, 0, stream>>>(X, n, ld, mean, part);
  AV_HIP_CHECK(hipGetLastError());
}

void col_moments_f64(const double* X, long long n, long long ld, int F, int pass, const double* mean, double* part,
                     hipStream_t stream) {
  const dim3 grid(mom_blocks(n, F), F);
  if (pass == 0) col_moments_kernel<double, 0><<<grid, MOM_THREADS, 0, stream>>>(X, n, ld, mean, part);
  else col_moments_kernel<double, 1><<<grid, MOM_THREADS, 0, stream>>>(X, n, ld, mean, part);
  AV_HIP_CHECK(hipGetLastError());
}

static int loo_blocks(long long n, int F) {
  long long b = (n + LOO_THREADS * 64 - 1) / (LOO_THREADS * 64);  // >= 64 rows per thread: LDS flush amortised
  const long long want = (2048 + F - 1) / F;
  if (b > want) b = want;
  return (int)(b < 1 ? 1 : b);
}

void loo_stats(const void* codes, int code_bytes, int m, long long ld, long long n, int F, const double* y, double* sum,
               unsigned* cnt, hipStream_t stream) {
  const size_t wide_lds = (size_t)m * (sizeof(double) + sizeof(unsigned));
  if (code_bytes >= 2 && wide_lds <= LOO_WIDE_LDS) {
    // set on every call: the attribute belongs to the current device (no process-wide cache)
    AV_HIP_CHECK(hipFuncSetAttribute((const void*)loo_stats_lds_kernel<int>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)LOO_WIDE_LDS));
    AV_HIP_CHECK(hipFuncSetAttribute((const void*)loo_stats_lds_kernel<unsigned short>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)LOO_WIDE_LDS));
    // >= 16 rows per thread so the table zero + flush is amortised; <= 256 blocks per column
    long long gx = n / (LOO_WIDE_T * 16);
    gx = gx < 1 ? 1 : (gx > 256 ? 256 : gx);
    const dim3 wgrid((unsigned)gx, F);
    if (code_bytes == 4)
      loo_stats_lds_kernel<int><<<wgrid, LOO_WIDE_T, wide_lds, stream>>>(static_cast<const int*>(codes), ld, n, y, sum,
                                                                        cnt, m);
    else
      loo_stats_lds_kernel<unsigned short><<<wgrid, LOO_WIDE_T, wide_lds, stream>>>(
          static_cast<const unsigned short*>(codes), ld, n, y, sum, cnt, m);
    AV_HIP_CHECK(hipGetLastError());
    return;
  }
  const dim3 grid(loo_blocks(n, F), F);
  if (code_bytes == 4)
    loo_stats_kernel<int><<<grid, LOO_THREADS, 0, stream>>>(static_cast<const int*>(codes), ld, n, y, sum, cnt, m);
  else if (code_bytes == 2)
    loo_stats_kernel<unsigned short><<<grid, LOO_THREADS, 0, stream>>>(static_cast<const unsigned short*>(codes), ld, n,
                                                                       y, sum, cnt, m);
  else
    loo_stats_kernel<unsigned char><<<grid, LOO_THREADS, 0, stream>>>(static_cast<const unsigned char*>(codes), ld, n,
                                                                      y, sum, cnt, m);
  AV_HIP_CHECK(hipGetLastError());
}

void loo_apply(const void* codes, int code_bytes, int m, long long ld, long long n, int F, const double* y,
               const double* sum, const unsigned* cnt, const double* gmean, double reg, const double* noise, double amp,
               float* out, hipStream_t stream) {
  const dim3 grid((unsigned)((n + LOO_THREADS - 1) / LOO_THREADS), (F + LOO_TILE_F - 1) / LOO_TILE_F);
  if (code_bytes == 4)
    loo_apply_kernel<int><<<grid, LOO_THREADS, 0, stream>>>(static_cast<const int*>(codes), ld, n, F, y, sum, cnt, m,
                                                            gmean, reg, noise, amp, out);
  else if (code_bytes == 2)
    loo_apply_kernel<unsigned short><<<grid, LOO_THREADS, 0, stream>>>(
        static_cast<const unsigned short*>(codes), ld, n, F, y, sum, cnt, m, gmean, reg, noise, amp, out);
  else
    loo_apply_kernel<unsigned char><<<grid, LOO_THREADS, 0, stream>>>(
        static_cast<const unsigned char*>(codes), ld, n, F, y, sum, cnt, m, gmean, reg, noise, amp, out);
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
