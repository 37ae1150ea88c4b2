// hand-written small-message all-reduce over peer-mapped device memory.
//
// Replaces the combiner + reducer shuffle of every counting model (e.g. the reference's
// src/main/java/org/avenir/bayesian/BayesianDistribution.java:72-79: per-key partial counts sent
// through the shuffle to one reducer) by ONE kernel per rank that reads every peer's staged
// buffer directly — over xGMI on a multi-GPU node, through the same HBM when several ranks share
// one device — instead of a library ring / tree with its proxy thread.
//
// Memory (per rank, exported once through hipIpcGetMemHandle and mapped by every peer with
// hipIpcOpenMemHandle; parallel/p2p.py exchanges the handles over the process group):
//   data  : 2 parities x [input staging cap | result staging cap] bytes (plain hipMalloc)
//   flags : u32 [P2P_MAX_RANKS][P2P_MAX_BLOCKS] written ONLY by peers (flags[src][block]),
//           uncached (hipDeviceMallocUncached), so a poll always sees the HBM value
//   status: i32, set by this rank's kernel when a wait timed out
//
// Protocol of call `epoch` e (e >= 1, every rank calls in the same order with the same size):
//   parity = e & 1; flag values 2e-1 (phase A) and 2e (phase B) are monotone in e.
//   one-shot (small): block b copies its chunk of the operand into its own input staging, releases
//     it (system-scope release fence: waits for the stores and writes the L2 back), raises
//     flags[me][b] = 2e in every peer's flag array, waits until every peer raised flags[p][b] >= 2e
//     in its own array, acquires (L2 / L1 invalidate), then sums chunk b of all W stagings IN RANK
//     ORDER into the operand.  Every rank reads the same staged bits in the same order, so the
//     result is bit-identical on every rank and every run (fp32 / fp64 included).
//   two-shot (larger): the operand is cut into W slices; block b of rank r stages sub-chunk b of
//     every slice (phase A, 2e-1), reduces sub-chunk b of slice r in rank order into its result
//     staging (phase B, 2e), then copies sub-chunk b of slice s from rank s's result staging —
//     each element is reduced by exactly one rank, again in rank order: deterministic, and each
//     rank reads 2 (W-1)/W of the message instead of W-1 times it.
// Reuse safety: parity e & 1 is rewritten at e + 2 only.  A rank can reach e + 2 only after its
//   e + 1 kernel observed every peer's e + 1 flag, and a peer raises that only after its own
//   e kernel (which read our parity-(e & 1) buffers) completed in stream order.  So no end
//   barrier is needed, and flags never need resetting.
// Termination and failure reporting: every wait has a wall-clock bound (s_memrealtime, 100 MHz;
//   the communicator's timeout, 600 s by default like the process group's); on expiry the kernel
//   records status = 1 — in its uncached device word AND in a pinned host-mapped word the host
//   reads without synchronising — stops waiting and drains.  The result is then garbage, and
//   parallel/comm.py raises P2PError at the rank's next collective or status check, before any
//   job writes output.  A kernel that finds status already set waits for nothing and raises its
//   flags with the poison bit (P2P_POISON), so a peer's wait on it ends at once with status 2 —
//   the failure propagates through the flags themselves instead of a cascade of timeouts (the
//   host's p2p_poison launch does the same for every block before a failing rank raises).
// Index safety: all indices are < units(n) (checked per unit against n for the operand); the
//   staging buffers hold cap >= n * sizeof(T) bytes (checked by the binding), flag indices are
//   src < P2P_MAX_RANKS, b < gridDim.x <= P2P_MAX_BLOCKS (checked by the launcher).
#include <stdexcept>

#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

constexpr int P2P_T = 256;

struct PeerPtrs {
  char* data[avk::P2P_MAX_RANKS];       // base of every rank's data region (own included)
  unsigned* flags[avk::P2P_MAX_RANKS];  // base of every rank's flag array (own included)
};

// 16-byte unit of the operand: K elements.  Units fully inside [0, n) of a 16-byte aligned array
// move as one dwordx4; the (at most one) partial unit element by element.
template <typename T>
struct Unit {
  static constexpr int K = 16 / sizeof(T);
  T v[K];
};

template <typename T>
__device__ __forceinline__ Unit<T> load_unit(const T* p, long long u, long long n) {
  Unit<T> r;
  const long long e0 = u * Unit<T>::K;
  if (e0 + Unit<T>::K <= n) {
    *reinterpret_cast<uint4*>(r.v) = *reinterpret_cast<const uint4*>(p + e0);
  } else {
#pragma unroll
    for (int j = 0; j < Unit<T>::K; ++j) r.v[j] = e0 + j < n ? p[e0 + j] : T(0);
  }
  return r;
}

template <typename T>
__device__ __forceinline__ void store_unit(T* p, long long u, long long n, const Unit<T>& r) {
  const long long e0 = u * Unit<T>::K;
  if (e0 + Unit<T>::K <= n) {
    *reinterpret_cast<uint4*>(p + e0) = *reinterpret_cast<const uint4*>(r.v);
  } else {
#pragma unroll
    for (int j = 0; j < Unit<T>::K; ++j)
      if (e0 + j < n) p[e0 + j] = r.v[j];
  }
}

// staging buffers always hold whole units: no bound check
template <typename T>
__device__ __forceinline__ Unit<T> load_full(const T* p, long long u) {
  Unit<T> r;
  *reinterpret_cast<uint4*>(r.v) = *reinterpret_cast<const uint4*>(p + u * Unit<T>::K);
  return r;
}
template <typename T>
__device__ __forceinline__ void store_full(T* p, long long u, const Unit<T>& r) {
  *reinterpret_cast<uint4*>(p + u * Unit<T>::K) = *reinterpret_cast<const uint4*>(r.v);
}

// Publish this block's stores to every peer: each wave waits for its own stores and writes the L2
// back (system-scope release fence), then one lane per peer raises the flag in that peer's array.
// Then lanes 0..W-1 of wave 0 wait for the peers' flags in our own array; everyone acquires.
__device__ __forceinline__ void fail(int* status, int* host_status, int code) {
  __hip_atomic_store(status, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(host_status, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void block_exchange(const PeerPtrs& P, int rank, int world, int b, unsigned sig,
                                               int* status, int* host_status, long long timeout,
                                               bool failed) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __syncthreads();
  const int t = threadIdx.x;
  if (t < world && t != rank) {
    __hip_atomic_store(P.flags[t] + rank * avk::P2P_MAX_BLOCKS + b, failed ? (sig | avk::P2P_POISON) : sig,
                       __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (!failed) {
      unsigned* f = P.flags[rank] + t * avk::P2P_MAX_BLOCKS + b;
      const long long t0 = wall_clock64();
      for (;;) {
        const unsigned v = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (v >= sig) {
          if (v & avk::P2P_POISON) fail(status, host_status, 2);   // the peer failed before us
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        if (wall_clock64() - t0 > timeout) {
          fail(status, host_status, 1);
          // overwrite the flag we raised for the late peer with the poisoned one: when its kernel
          // arrives it fails too (status 2) instead of completing against our abandoned call
          __hip_atomic_store(P.flags[t] + rank * avk::P2P_MAX_BLOCKS + b, sig | avk::P2P_POISON,
                             __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
      }
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

// every peer's flag slots for this rank, every block: poisoned (one thread per slot)
__global__ __launch_bounds__(P2P_T) void p2p_poison_kernel(PeerPtrs P, int rank, int world) {
  for (int i = threadIdx.x; i < world * avk::P2P_MAX_BLOCKS; i += P2P_T) {
    const int peer = i / avk::P2P_MAX_BLOCKS;
    if (peer == rank) continue;
    __hip_atomic_store(P.flags[peer] + rank * avk::P2P_MAX_BLOCKS + i % avk::P2P_MAX_BLOCKS, 0xFFFFFFFFu,
                       __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

template <typename T>
__device__ __forceinline__ void add_unit(Unit<T>& a, const Unit<T>& b) {
#pragma unroll
  for (int j = 0; j < Unit<T>::K; ++j) a.v[j] += b.v[j];
}

// one-shot: grid = B blocks, block b owns units [b * per, min((b + 1) * per, nu))
template <typename T>
__global__ __launch_bounds__(P2P_T) void p2p_oneshot_kernel(T* __restrict__ x, long long n, PeerPtrs P, int rank,
                                                            int world, unsigned epoch, long long cap_elems,
                                                            long long per, int* status, int* host_status,
                                                            long long timeout) {
  const int b = blockIdx.x;
  const long long nu = (n + Unit<T>::K - 1) / Unit<T>::K;
  const long long lo = (long long)b * per;
  const long long hi = lo + per < nu ? lo + per : nu;
  const long long poff = (long long)(epoch & 1u) * 2 * cap_elems;  // input staging of this parity
  T* mine = reinterpret_cast<T*>(P.data[rank]) + poff;
  for (long long u = lo + threadIdx.x; u < hi; u += P2P_T) store_full(mine, u, load_unit(x, u, n));
  const bool failed = __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  block_exchange(P, rank, world, b, 2u * epoch, status, host_status, timeout, failed);
  for (long long u = lo + threadIdx.x; u < hi; u += P2P_T) {
    Unit<T> acc = load_full(reinterpret_cast<const T*>(P.data[0]) + poff, u);
    for (int k = 1; k < world; ++k) add_unit(acc, load_full(reinterpret_cast<const T*>(P.data[k]) + poff, u));
    store_unit(x, u, n, acc);
  }
}

// two-shot: the nu units are cut into W slices of S units; block b owns sub-chunk b (C units) of
// every slice.  Phase A stages them, phase B reduces slice `rank` into the result staging, phase C
// gathers every other slice's reduced sub-chunk from its owner.
template <typename T>
__global__ __launch_bounds__(P2P_T) void p2p_twoshot_kernel(T* __restrict__ x, long long n, PeerPtrs P, int rank,
                                                            int world, unsigned epoch, long long cap_elems,
                                                            long long S, long long C, int* status,
                                                            int* host_status, long long timeout) {
  const int b = blockIdx.x;
  const long long nu = (n + Unit<T>::K - 1) / Unit<T>::K;
  const long long poff = (long long)(epoch & 1u) * 2 * cap_elems;
  const long long roff = poff + cap_elems;                          // result staging of this parity
  T* mine = reinterpret_cast<T*>(P.data[rank]) + poff;
  for (int s = 0; s < world; ++s) {
    const long long lo = s * S + (long long)b * C;
    long long hi = lo + C < (s + 1) * S ? lo + C : (s + 1) * S;
    hi = hi < nu ? hi : nu;
    for (long long u = lo + threadIdx.x; u < hi; u += P2P_T) store_full(mine, u, load_unit(x, u, n));
  }
  const bool failed = __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  block_exchange(P, rank, world, b, 2u * epoch - 1u, status, host_status, timeout, failed);
  {
    const long long lo = rank * S + (long long)b * C;
    long long hi = lo + C < (rank + 1) * S ? lo + C : (rank + 1) * S;
    hi = hi < nu ? hi : nu;
    T* res = reinterpret_cast<T*>(P.data[rank]) + roff;
    for (long long u = lo + threadIdx.x; u < hi; u += P2P_T) {
      Unit<T> acc = load_full(reinterpret_cast<const T*>(P.data[0]) + poff, u);
      for (int k = 1; k < world; ++k) add_unit(acc, load_full(reinterpret_cast<const T*>(P.data[k]) + poff, u));
      store_full(res, u, acc);
      store_unit(x, u, n, acc);
    }
  }
  // a wait of phase A that failed poisons phase B's flags too
  block_exchange(P, rank, world, b, 2u * epoch, status, host_status, timeout,
                 failed || __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0);
  for (int s = 0; s < world; ++s) {
    if (s == rank) continue;
    const long long lo = s * S + (long long)b * C;
    long long hi = lo + C < (s + 1) * S ? lo + C : (s + 1) * S;
    hi = hi < nu ? hi : nu;
    const T* res = reinterpret_cast<const T*>(P.data[s]) + roff;
    for (long long u = lo + threadIdx.x; u < hi; u += P2P_T) store_unit(x, u, n, load_full(res, u));
  }
}

template <typename T>
void launch(void* x, long long n, const avk::P2PView& v, unsigned epoch, int two_shot, long long timeout,
            hipStream_t st) {
  PeerPtrs P{};
  for (int k = 0; k < v.world; ++k) {
    P.data[k] = reinterpret_cast<char*>(v.data[k]);
    P.flags[k] = v.flags[k];
  }
  const long long cap_elems = v.cap_bytes / (long long)sizeof(T);
  const long long nu = (n + Unit<T>::K - 1) / Unit<T>::K;
  if (two_shot) {
    const long long S = (nu + v.world - 1) / v.world;
    int B = (int)std::min<long long>(avk::P2P_MAX_BLOCKS, std::max<long long>(1, (S + 4 * P2P_T - 1) / (4 * P2P_T)));
    const long long C = (S + B - 1) / B;
    hipLaunchKernelGGL(p2p_twoshot_kernel<T>, dim3(B), dim3(P2P_T), 0, st, reinterpret_cast<T*>(x), n, P, v.rank,
                       v.world, epoch, cap_elems, S, C, v.status, v.host_status, timeout);
  } else {
    int B = (int)std::min<long long>(avk::P2P_MAX_BLOCKS, std::max<long long>(1, (nu + 4 * P2P_T - 1) / (4 * P2P_T)));
    const long long per = (nu + B - 1) / B;
    hipLaunchKernelGGL(p2p_oneshot_kernel<T>, dim3(B), dim3(P2P_T), 0, st, reinterpret_cast<T*>(x), n, P, v.rank,
                       v.world, epoch, cap_elems, per, v.status, v.host_status, timeout);
  }
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace

namespace avk {

void p2p_all_reduce(void* x, long long n, int dtype, const P2PView& v, unsigned epoch, int two_shot,
                    long long timeout_ticks, hipStream_t st) {
  if (v.world < 1 || v.world > P2P_MAX_RANKS || v.rank < 0 || v.rank >= v.world)
    throw std::invalid_argument("p2p_all_reduce: bad rank / world");
  if (epoch == 0 || epoch > P2P_MAX_EPOCH) throw std::invalid_argument("p2p_all_reduce: epoch out of range");
  if (v.status == nullptr || v.host_status == nullptr) throw std::invalid_argument("p2p_all_reduce: no status words");
  if (n <= 0) return;
  switch (dtype) {
    case P2P_F32: launch<float>(x, n, v, epoch, two_shot, timeout_ticks, st); break;
    case P2P_F64: launch<double>(x, n, v, epoch, two_shot, timeout_ticks, st); break;
    case P2P_I32: launch<int>(x, n, v, epoch, two_shot, timeout_ticks, st); break;
    case P2P_I64: launch<long long>(x, n, v, epoch, two_shot, timeout_ticks, st); break;
    default: throw std::invalid_argument("p2p_all_reduce: unsupported dtype");
  }
}

void p2p_poison(const P2PView& v, hipStream_t st) {
  if (v.world < 1 || v.world > P2P_MAX_RANKS || v.rank < 0 || v.rank >= v.world)
    throw std::invalid_argument("p2p_poison: bad rank / world");
  PeerPtrs P{};
  for (int k = 0; k < v.world; ++k) {
    P.data[k] = reinterpret_cast<char*>(v.data[k]);
    P.flags[k] = v.flags[k];
  }
  hipLaunchKernelGGL(p2p_poison_kernel, dim3(1), dim3(P2P_T), 0, st, P, v.rank, v.world);
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
