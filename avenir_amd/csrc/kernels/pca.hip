// K24 streaming PCA (SPIRIT / Sanger-style deflation updates) for CDNA4 (gfx950).
//
// Reference: S/explore/IncrementalPrincipalComponent.scala:83-167 updates, per key and per record,
// every live hidden unit i: y = w_i . x, E_i = lam E_i + y^2, w_i += (x - y w_i) y / E_i, x -= y w_i,
// then tracks the visible / hidden energy and grows or shrinks the number of hidden units.  The
// recurrence is strictly sequential in time, so the torch formulation costs ~15 launches per
// (record, hidden unit) plus host syncs.  Here ONE WAVE owns one key for its whole stream:
//   lane d holds dimension d of x and of every w_i (W lives in LDS, each lane touching only its
//   own column, so no barriers are needed), the dot products are wave reductions, and lane i holds
//   the per-unit scalars E_i / hidden energy / y_i (read wave-wide with a lane broadcast).
// One launch replaces T x H x ~15 launches.  Limits: D <= 64, H <= D (the binding checks).
#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

__device__ __forceinline__ double bcast(double v, int l) { return __shfl(v, l, 64); }

__global__ __launch_bounds__(64) void spirit_kernel(const double* __restrict__ X, int T, int D, int H,
                                                    const int* __restrict__ lens, double* __restrict__ W,
                                                    double* __restrict__ E, double* __restrict__ he,
                                                    double* __restrict__ ve, double* __restrict__ cnt,
                                                    int* __restrict__ nh_io, double lam, double lo, double hi) {
  __shared__ double Ws[64 * 64];
  const int k = blockIdx.x, lane = threadIdx.x;
  const bool on = lane < D;
  double* Wk = W + (long long)k * H * D;
  for (int i = 0; i < H; ++i) Ws[i * 64 + lane] = on ? Wk[i * D + lane] : 0.0;
  double e_l = lane < H ? E[(long long)k * H + lane] : 1.0;   // lane i: E_i
  double h_l = lane < H ? he[(long long)k * H + lane] : 0.0;  // lane i: hidden energy of unit i
  double v = ve[k], c = cnt[k];
  int nh = nh_io[k];
  const int len = lens[k];
  const double* Xk = X + (long long)k * T * D;
  for (int t = 0; t < len; ++t) {
    const double xin = on ? Xk[(long long)t * D + lane] : 0.0;
    double x = xin, y_l = 0.0;
    for (int i = 0; i < nh; ++i) {
      const double w = Ws[i * 64 + lane];
      const double y = av::wave_sum(w * x);
      const double Ei = lam * bcast(e_l, i) + y * y;
      const double wn = w + (x - y * w) * (y / fmax(Ei, 1e-300));
      Ws[i * 64 + lane] = wn;
      if (lane == i) {
        e_l = Ei;
        y_l = y;
      }
      x -= wn * y;
    }
    const double vn = av::wave_sum(xin * xin);
    v = (c * v + vn) / (c + 1.0);
    if (lane < nh) h_l = (c * h_l + y_l * y_l) / (c + 1.0);
    const double tot = av::wave_sum(lane < nh ? h_l : 0.0);
    if (tot < lo * v && nh < H) {  // grow: the new unit starts as the next basis vector
      Ws[nh * 64 + lane] = lane == nh ? 1.0 : 0.0;
      if (lane == nh) {
        e_l = 1.0;
        h_l = 0.0;
      }
      ++nh;
    } else if (tot > hi * v && nh > 1) {
      --nh;
    }
    c += 1.0;
  }
  for (int i = 0; i < H; ++i)
    if (on) Wk[i * D + lane] = Ws[i * 64 + lane];
  if (lane < H) {
    E[(long long)k * H + lane] = e_l;
    he[(long long)k * H + lane] = h_l;
  }
  if (lane == 0) {
    ve[k] = v;
    cnt[k] = c;
    nh_io[k] = nh;
  }
}

}  // namespace

namespace avk {

void spirit_update(const double* X, int K, int T, int D, int H, const int* lens, double* W, double* E, double* he,
                   double* ve, double* cnt, int* nh, double lam, double lo, double hi, hipStream_t stream) {
  if (K <= 0) return;
  spirit_kernel<<<K, 64, 0, stream>>>(X, T, D, H, lens, W, E, he, ve, cnt, nh, lam, lo, hi);
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
