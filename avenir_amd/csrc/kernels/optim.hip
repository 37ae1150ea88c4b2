// K22: many simulated-annealing chains in one persistent launch (CDNA4, gfx950).
//
// Reference: one SA chain per Spark partition, mutating string-encoded solutions through the
// BasicSearchDomain SPI (S/optimize/SimulatedAnnealing.scala:111-187,
// J/optimize/BasicSearchDomain.java:272-394, cost J/examples/TaskScheduleSearch.java:169-305).
// Here an assignment-type domain (solution s[L] with s[i] in [0, V); total cost = mean_i C[i][s[i]];
// a solution is invalid when two positions with a conflict share a value) is compiled into a
// [L][V] cost table and an [L][L] conflict table, and every lane runs one chain for `iters`
// Metropolis steps: O(1) cost delta per move, O(L) validity check, Philox randomness, geometric or
// linear cooling — the whole optimisation is one kernel launch for thousands of chains.
#include "avenir_common.h"
#include "avenir_kernels.h"

namespace {

// true when position i conflicts with no other position holding the same value
__device__ __forceinline__ bool position_ok(const short* s, int L, int i, const uint8_t* __restrict__ conflict) {
  const short v = s[i * 64];
  const uint8_t* row = conflict + (long long)i * L;
  for (int j = 0; j < L; ++j)
    if (j != i && s[j * 64] == v && row[j]) return false;
  return true;
}

// One chain per lane, 64-lane workgroups (one wave): the chain's current solution lives in LDS as
// column `lane` of an [L][64] short tile (lane-private, conflict-free), the best solution is written
// to global memory only on improvement.  Move = reassign one position to a different value; with
// `swap` set, the position that already held the new value takes the old one (the reference's
// replaceSolutionComponent, J/examples/TaskScheduleSearch.java:140-166).
__global__ __launch_bounds__(64) void sa_assign_kernel(
    const float* __restrict__ cost, int L, int V, const uint8_t* __restrict__ conflict, int swap,
    short* __restrict__ sol, float* __restrict__ cur_cost, short* __restrict__ best_sol,
    float* __restrict__ best_cost, int P, int iters, float t0, float cool, int interval, int geometric,
    int max_retry, unsigned long long seed, unsigned long long offset, int it_begin, float temp_start,
    unsigned long long* __restrict__ stats, long long chain_base) {
  extern __shared__ short lds_sol[];
  const int lane = threadIdx.x;
  const int p = blockIdx.x * 64 + lane;
  const bool live = p < P;
  // Philox stream of GLOBAL chain chain_base + p: a chain draws the same moves whichever rank
  // (and launch) runs it, so chains can be re-dealt over a different world size on resume
  const unsigned long long gp = (unsigned long long)(chain_base + p);
  short* s = lds_sol + lane;  // element j at s[j * 64]
  if (live)
    for (int j = 0; j < L; ++j) s[j * 64] = sol[(long long)p * L + j];
  if (!live) return;
  short* bs = best_sol + (long long)p * L;
  float c = cur_cost[p];
  float bc = best_cost[p];
  // resumable: a run split into segments [it_begin, it_begin + iters) draws the same Philox counters
  // and follows the same cooling schedule as one uninterrupted launch
  float temp = temp_start;
  unsigned long long acc_better = 0, acc_worse = 0, rejected = 0;
  const float invL = 1.f / (float)L;
  for (int it = it_begin; it < it_begin + iters; ++it) {
    int pos = -1, nv = 0, old = 0, j2 = -1;
    for (int tr = 0; tr <= max_retry; ++tr) {
      const av::u4 r = av::philox_draw(seed, offset + (unsigned long long)it * (max_retry + 1) + tr, gp);
      const int cp = min((int)(av::u32_to_unit(r.x) * (float)L), L - 1);
      int cv = min((int)(av::u32_to_unit(r.y) * (float)(V - 1)), V - 2);
      const int ov = s[cp * 64];
      if (cv >= ov) ++cv;  // a different value
      int sw = -1;
      if (swap)
        for (int j = 0; j < L; ++j)
          if (j != cp && s[j * 64] == cv) { sw = j; break; }
      s[cp * 64] = (short)cv;
      if (sw >= 0) s[sw * 64] = (short)ov;
      const bool ok = !conflict || (position_ok(s, L, cp, conflict) && (sw < 0 || position_ok(s, L, sw, conflict)));
      if (ok) { pos = cp; nv = cv; old = ov; j2 = sw; break; }
      s[cp * 64] = (short)ov;
      if (sw >= 0) s[sw * 64] = (short)cv;
    }
    if (pos >= 0) {
      float delta = cost[(long long)pos * V + nv] - cost[(long long)pos * V + old];
      if (j2 >= 0) delta += cost[(long long)j2 * V + old] - cost[(long long)j2 * V + nv];
      delta *= invL;
      const av::u4 r2 = av::philox_draw(seed ^ 0x9e3779b97f4a7c15ull, offset + it, gp);
      const bool accept = delta <= 0.f || av::u32_to_unit(r2.x) < __expf(-delta / fmaxf(temp, 1e-12f));
      if (accept) {
        c += delta;
        if (delta <= 0.f) ++acc_better; else ++acc_worse;
        if (c < bc) {
          bc = c;
          for (int j = 0; j < L; ++j) bs[j] = s[j * 64];
        }
      } else {
        s[pos * 64] = (short)old;
        if (j2 >= 0) s[j2 * 64] = (short)nv;
        ++rejected;
      }
    }
    // cooling every `interval` moves: geometric, or linear T0 - it * rate (the Python optimiser's
    // form, P/mlextra/optsolo.py:84-88; the Scala linear branch subtracts T0 each time, a bug)
    if (interval > 0 && (it + 1) % interval == 0)
      temp = geometric ? temp * cool : fmaxf(t0 - (float)(it + 1) * cool, 1e-12f);
  }
  for (int j = 0; j < L; ++j) sol[(long long)p * L + j] = s[j * 64];
  cur_cost[p] = c;
  best_cost[p] = bc;
  if (stats) {
    if (p == 0) stats[3] = (unsigned long long)__float_as_uint(temp);  // segment hand-off temperature
    atomicAdd(&stats[0], acc_better);
    atomicAdd(&stats[1], acc_worse);
    atomicAdd(&stats[2], rejected);
  }
}

}  // namespace

namespace avk {

void sa_assign(const float* cost, int L, int V, const uint8_t* conflict, int swap, short* sol, float* cur_cost,
               short* best_sol, float* best_cost, int P, int iters, float t0, float cool, int interval,
               int geometric, int max_retry, unsigned long long seed, unsigned long long offset,
               int it_begin, float temp_start, unsigned long long* stats, long long chain_base, hipStream_t stream) {
  if (P <= 0 || iters <= 0) return;
  const size_t lds = (size_t)L * 64 * sizeof(short);
  sa_assign_kernel<<<(P + 63) / 64, 64, lds, stream>>>(cost, L, V, conflict, swap, sol, cur_cost, best_sol,
                                                       best_cost, P, iters, t0, cool, interval, geometric, max_retry,
                                                       seed, offset, it_begin, temp_start, stats, chain_base);
  AV_HIP_CHECK(hipGetLastError());
}

}  // namespace avk
