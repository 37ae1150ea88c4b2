// avenir_amd — shared CDNA4 (gfx950) device helpers.
//
// Everything here is written for 64-lane wavefronts: lane = threadIdx.x & 63, ballots are 64-bit,
// reductions use __shfl_xor over offsets 32..1.  No CUDA shims, no warp-32 idioms.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define AV_WAVE 64

#define AV_HIP_CHECK(expr)                                                                 \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess) {                                                                 \
      av_report_hip_error(_e, #expr, __FILE__, __LINE__);                                   \
    }                                                                                       \
  } while (0)

// defined in host/runtime.cpp — throws std::runtime_error (turned into a Python exception)
void av_report_hip_error(hipError_t e, const char* expr, const char* file, int line);

namespace av {

// ---- XCD-aware tile order ------------------------------------------------------------------------
// The dispatcher hands workgroup i of a launch to XCD i % 8 (round robin over the 8 XCDs, each with
// its own L2).  xcd_remap turns the flat dispatch id into a logical id such that every XCD runs a
// CONTIGUOUS range of logical ids (XCD x: ids [x q + min(x, r), ... + q + (x < r)) for total = 8 q
// + r) — a bijection, so neighbouring tiles in the logical order share one L2.
constexpr int AV_NUM_XCD = 8;
__device__ __forceinline__ int xcd_remap(int pid, int total) {
  const int q = total / AV_NUM_XCD, r = total % AV_NUM_XCD;
  const int x = pid % AV_NUM_XCD, i = pid / AV_NUM_XCD;
  return x * q + (x < r ? x : r) + i;
}
// logical id -> (tile row, tile col) in groups of G tile rows: consecutive ids walk the G rows of
// a group for one tile column, then the next column — a column's operand tile is reused by G
// neighbours and a group's row operands by every column.
__device__ __forceinline__ void grouped_tile(int lid, int ntm, int ntn, int G, int& tm, int& tn) {
  const int per = G * ntn, g = lid / per, first = g * G;
  const int gs = (ntm - first) < G ? (ntm - first) : G;
  const int in = lid - g * per;
  tm = first + in % gs;
  tn = in / gs;
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

// ---- wave-wide reductions on DPP + v_readlane (no LDS traffic) ---------------------------------
// Steps 1 and 2 are quad_perm swaps, 4 and 8 are row rotations inside each 16-lane row (all VALU
// DPP moves, a few cycles each); the four row results are then combined from v_readlane into a
// wave-uniform value.  __shfl_xor lowers to ds_bpermute (an LDS-pipe round trip per step), which
// dominated latency-bound loops such as the SMO step (smo_ws_kernel).
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) { return __builtin_amdgcn_update_dpp(v, v, CTRL, 0xF, 0xF, false); }
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) { return __int_as_float(dpp_i<CTRL>(__float_as_int(v))); }
__device__ __forceinline__ float lane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

template <typename Op>
__device__ __forceinline__ float wave_reduce_f(float v, Op op) {
  v = op(v, dpp_f<0xB1>(v));   // quad_perm [1,0,3,2]
  v = op(v, dpp_f<0x4E>(v));   // quad_perm [2,3,0,1]
  v = op(v, dpp_f<0x124>(v));  // row_ror:4
  v = op(v, dpp_f<0x128>(v));  // row_ror:8
  return op(op(lane_f(v, 0), lane_f(v, 16)), op(lane_f(v, 32), lane_f(v, 48)));
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
template <>
__device__ __forceinline__ float wave_sum<float>(float v) {
  return wave_reduce_f(v, [](float a, float b) { return a + b; });
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    T w = __shfl_xor(v, o, 64);
    v = v > w ? v : w;
  }
  return v;
}
template <>
__device__ __forceinline__ float wave_max<float>(float v) {
  return wave_reduce_f(v, [](float a, float b) { return fmaxf(a, b); });
}

template <typename T>
__device__ __forceinline__ T wave_min(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    T w = __shfl_xor(v, o, 64);
    v = v < w ? v : w;
  }
  return v;
}
template <>
__device__ __forceinline__ float wave_min<float>(float v) {
  return wave_reduce_f(v, [](float a, float b) { return fminf(a, b); });
}

// (value, index) argmax / argmin over the wave; ties -> lowest index (deterministic).  The result
// is wave-uniform.
template <bool MAX>
__device__ __forceinline__ void wave_arg_step(float& v, int& i, float v2, int i2) {
  if ((MAX ? v2 > v : v2 < v) || (v2 == v && i2 < i)) { v = v2; i = i2; }
}
template <bool MAX>
__device__ __forceinline__ void wave_arg(float& v, int& idx) {
  wave_arg_step<MAX>(v, idx, dpp_f<0xB1>(v), dpp_i<0xB1>(idx));
  wave_arg_step<MAX>(v, idx, dpp_f<0x4E>(v), dpp_i<0x4E>(idx));
  wave_arg_step<MAX>(v, idx, dpp_f<0x124>(v), dpp_i<0x124>(idx));
  wave_arg_step<MAX>(v, idx, dpp_f<0x128>(v), dpp_i<0x128>(idx));
  float r = lane_f(v, 0);
  int ri = __builtin_amdgcn_readlane(idx, 0);
#pragma unroll
  for (int l = 16; l < 64; l += 16) wave_arg_step<MAX>(r, ri, lane_f(v, l), __builtin_amdgcn_readlane(idx, l));
  v = r;
  idx = ri;
}
__device__ __forceinline__ void wave_argmax(float& v, int& idx) { wave_arg<true>(v, idx); }
__device__ __forceinline__ void wave_argmin(float& v, int& idx) { wave_arg<false>(v, idx); }

// 64-bit wave sum built from two 32-bit shuffles per step.
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    unsigned lo = __shfl_xor((unsigned)(v & 0xffffffffu), o, 64);
    unsigned hi = __shfl_xor((unsigned)(v >> 32), o, 64);
    v += ((unsigned long long)hi << 32) | lo;
  }
  return v;
}

// ---------------------------------------------------------------------------------------------
// Philox4x32-10 counter-based RNG (Salmon et al. 2011).  Stateless: (key, counter) -> 4 x u32.
// Every device sampler in avenir_amd draws from this so results are reproducible for a given
// (seed, offset) independent of grid shape and world size.
// ---------------------------------------------------------------------------------------------
struct u4 { uint32_t x, y, z, w; };

__host__ __device__ __forceinline__ u4 philox4x32_10(u4 ctr, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint64_t p0 = (uint64_t)M0 * ctr.x;
    uint64_t p1 = (uint64_t)M1 * ctr.z;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    u4 n;
    n.x = hi1 ^ ctr.y ^ k0;
    n.y = lo1;
    n.z = hi0 ^ ctr.w ^ k1;
    n.w = lo0;
    ctr = n;
    k0 += W0;
    k1 += W1;
  }
  return ctr;
}

// uniform in (0, 1]  (never 0: safe for log)
__host__ __device__ __forceinline__ float u32_to_unit(uint32_t x) {
  return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f);
}

__device__ __forceinline__ u4 philox_draw(uint64_t seed, uint64_t offset, uint64_t idx) {
  u4 c;
  c.x = (uint32_t)idx;
  c.y = (uint32_t)(idx >> 32);
  c.z = (uint32_t)offset;
  c.w = (uint32_t)(offset >> 32);
  return philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}

// Workgroups of `kernel` (block threads, lds dynamic bytes) resident on the whole device at once
// (occupancy x CUs).  A grid-stride kernel launched with more workgroups than this runs a second,
// partial round at lower occupancy; host/runtime.cpp.
int resident_blocks(const void* kernel, int block, size_t lds);

// Grid sizing for memory-bound streaming kernels: enough waves to fill 256 CUs several times
// over, capped so the tail is short (Guideline 11).
inline int stream_grid(long long work_items, int block, int per_thread = 1, int cap = 2048) {
  long long g = (work_items + (long long)block * per_thread - 1) / ((long long)block * per_thread);
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

}  // namespace av
