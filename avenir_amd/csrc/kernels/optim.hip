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
#include <stdexcept>

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

// ---- island genetic algorithm: one workgroup (one wave) per island, G generations per launch ----
// Reference: Spark GA — an independent GA per partition (S/optimize/GeneticAlgorithm.scala:70-163) —
// and the Python GeneticAlgorithmOptimizer (P/mlextra/optpopu.py:98-187: pool, mating list,
// replacement, purge).  An island's pool [P][L], its costs and the children of a generation live in
// LDS; per generation, one lane per member / pair / child:
//   1. rank the pool by (cost, index) (lane j counts the members ahead of member j) -> ord[];
//      hist[g] = the best cost at the generation's start;
//   2. pair k < r draws Philox(seed, 256 (gen_base + g) + k, island): parents ord[a], ord[b] (a != b) from the
//      m best, crossover point x in [1, L), children a[:x] b[x:] and b[:x] a[x:]; with `mutate`,
//      Philox(seed ^ M, 16 ctr + try, island) moves one position of each child to a different
//      value (a swap move with `swap`), retried until the child is valid (<= 10 tries);
//   3. lane c < 2r prices child c: fp32 sum of C[l][s_l] in position order times 1/L, or
//      `invalid` when two conflicting positions share a value;
//   4. the best r children by (cost, index) replace the worst r members (purge_first) or join the
//      pool, whose best P by (cost, index; members before children) survive — written to the other
//      pool buffer in rank order.
// The island's stream is keyed by its GLOBAL index (island_base + blockIdx.x), so any world size
// yields the same islands; optimize/ga.py::ga_assign_reference is the bit-exact host twin.
constexpr int GA_MAX_TRY = 10;

__device__ __forceinline__ bool ga_valid(const short* s, int L, const uint8_t* __restrict__ conflict) {
  if (conflict)
    for (int i = 0; i < L; ++i)
      for (int j = i + 1; j < L; ++j)
        if (s[i] == s[j] && conflict[(long long)i * L + j]) return false;
  return true;
}

__device__ __forceinline__ float ga_price(const short* s, int L, int V, const float* __restrict__ cost,
                                          const uint8_t* __restrict__ conflict, float invL, float invalid) {
  float acc = 0.f;
  for (int l = 0; l < L; ++l) acc += cost[(long long)l * V + s[l]];
  return ga_valid(s, L, conflict) ? acc * invL : invalid;
}

__global__ __launch_bounds__(64) void ga_assign_kernel(
    const float* __restrict__ cost, int L, int V, const uint8_t* __restrict__ conflict, float invalid,
    short* __restrict__ pop, float* __restrict__ pop_cost, float* __restrict__ hist, int P, int G, int m, int r,
    int purge_first, int mutate, int swap, unsigned long long seed, long long island_base, int gen_base) {
  extern __shared__ unsigned char ga_lds[];
  short* pa = reinterpret_cast<short*>(ga_lds);   // [P][L] current pool
  short* pb = pa + (size_t)P * L;                 // [P][L] next pool
  short* kid = pb + (size_t)P * L;                // [2r][L] children
  float* pc = reinterpret_cast<float*>(kid + (size_t)2 * r * L);  // [P] pool costs
  float* pc2 = pc + P;                            // [P] next pool costs
  float* kc = pc2 + P;                            // [2r] child costs
  int* ord = reinterpret_cast<int*>(kc + 2 * r);  // [P] pool order
  int* kord = ord + P;                            // [2r] child order
  int* nsrc = kord + 2 * r;                       // [P] source of next pool slot (>= P: child)
  const int lane = threadIdx.x;
  const long long isl = blockIdx.x;
  const unsigned long long gi = (unsigned long long)(island_base + isl);
  const float invL = 1.f / (float)L;
  short* gpop = pop + isl * P * L;
  for (int e = lane; e < P * L; e += 64) pa[e] = gpop[e];
  if (lane < P) pc[lane] = pop_cost[isl * P + lane];
  __syncthreads();
  for (int g = 0; g < G; ++g) {
    // 1. rank
    if (lane < P) {
      const float c = pc[lane];
      int rk = 0;
      for (int j = 0; j < P; ++j) rk += (pc[j] < c) || (pc[j] == c && j < lane);
      ord[rk] = lane;
    }
    __syncthreads();
    if (lane == 0) hist[isl * G + g] = pc[ord[0]];
    // 2. children
    if (lane < r) {
      const unsigned long long ctr = 256ull * (unsigned long long)(gen_base + g) + lane;
      const av::u4 R = av::philox_draw(seed, ctr, gi);
      const int a = min((int)(av::u32_to_unit(R.x) * (float)m), m - 1);
      int b = 0;
      if (m > 1) {
        b = min((int)(av::u32_to_unit(R.y) * (float)(m - 1)), m - 2);
        b += b >= a;
      }
      const int x = L > 1 ? 1 + min((int)(av::u32_to_unit(R.z) * (float)(L - 1)), L - 2) : 0;
      const short* A = pa + (size_t)ord[a] * L;
      const short* B = pa + (size_t)ord[b] * L;
      short* c1 = kid + (size_t)(2 * lane) * L;
      short* c2 = c1 + L;
      for (int l = 0; l < L; ++l) {
        c1[l] = l < x ? A[l] : B[l];
        c2[l] = l < x ? B[l] : A[l];
      }
      if (mutate) {
        // one position to a different value (with `swap`, the first other position holding that
        // value takes the old one: the domain's swap move), redrawn up to GA_MAX_TRY times until
        // the child is valid; the last attempt stays otherwise (BasicSearchDomain.mutateSolution)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          short* c = h == 0 ? c1 : c2;
          for (int t = 0; t < GA_MAX_TRY; ++t) {
            const av::u4 Q = av::philox_draw(seed ^ 0xD1B54A32D192ED03ull, ctr * 16ull + t, gi);
            const unsigned qp = h == 0 ? Q.x : Q.z, qv = h == 0 ? Q.y : Q.w;
            const int pos = min((int)(av::u32_to_unit(qp) * (float)L), L - 1);
            const int old = c[pos];
            int v = min((int)(av::u32_to_unit(qv) * (float)(V - 1)), V - 2);
            v += v >= old;
            int holder = -1;
            if (swap)
              for (int j = 0; j < L; ++j)
                if (j != pos && c[j] == v) { holder = j; break; }
            if (holder >= 0) c[holder] = (short)old;
            c[pos] = (short)v;
            if (t == GA_MAX_TRY - 1 || ga_valid(c, L, conflict)) break;
            c[pos] = (short)old;
            if (holder >= 0) c[holder] = (short)v;
          }
        }
      }
    }
    __syncthreads();
    // 3. price the children
    if (lane < 2 * r) kc[lane] = ga_price(kid + (size_t)lane * L, L, V, cost, conflict, invL, invalid);
    __syncthreads();
    if (lane < 2 * r) {
      const float c = kc[lane];
      int rk = 0;
      for (int j = 0; j < 2 * r; ++j) rk += (kc[j] < c) || (kc[j] == c && j < lane);
      kord[rk] = lane;
    }
    __syncthreads();
    // 4. replacement: the source of every next-pool slot
    if (purge_first) {
      if (lane < P) nsrc[lane] = lane < P - r ? ord[lane] : P + kord[lane - (P - r)];
    } else if (lane < P + r) {
      // candidate lane: member ord-independent index (lane < P) or child kord[lane - P]; its rank
      // among all candidates by (cost, candidate index)
      const int src = lane < P ? lane : P + kord[lane - P];
      const float c = lane < P ? pc[lane] : kc[src - P];
      int rk = 0;
      for (int j = 0; j < P + r; ++j) {
        const int sj = j < P ? j : P + kord[j - P];
        const float cj = j < P ? pc[j] : kc[sj - P];
        rk += (cj < c) || (cj == c && j < lane);
      }
      if (rk < P) nsrc[rk] = src;
    }
    __syncthreads();
    for (int e = lane; e < P * L; e += 64) {
      const int slot = e / L, l = e - slot * L;
      const int src = nsrc[slot];
      pb[e] = src < P ? pa[(size_t)src * L + l] : kid[(size_t)(src - P) * L + l];
    }
    if (lane < P) {
      const int src = nsrc[lane];
      pc2[lane] = src < P ? pc[src] : kc[src - P];
    }
    __syncthreads();
    short* t = pa; pa = pb; pb = t;
    float* tc = pc; pc = pc2; pc2 = tc;
  }
  for (int e = lane; e < P * L; e += 64) gpop[e] = pa[e];
  if (lane < P) pop_cost[isl * P + lane] = pc[lane];
}

}  // namespace

namespace avk {

size_t ga_assign_lds(int P, int L, int r) {
  return (size_t)(2 * P + 2 * r) * L * sizeof(short) + (size_t)(2 * P + 2 * r) * sizeof(float) +
         (size_t)(2 * P + 2 * r) * sizeof(int);
}

void ga_assign(const float* cost, int L, int V, const uint8_t* conflict, float invalid, short* pop, float* pop_cost,
               float* hist, int islands, int P, int G, int m, int r, int purge_first, int mutate, int swap,
               unsigned long long seed, long long island_base, int gen_base, hipStream_t stream) {
  if (islands <= 0 || G <= 0) return;
  if (P < 2 || P > 64 || r < 1 || 2 * r > 64 || r > P || m < 1 || m > P || L < 1 || V < 2)
    throw std::invalid_argument("ga_assign: 2 <= P <= 64, 1 <= r <= min(P, 32), 1 <= m <= P, L >= 1, V >= 2");
  if (!purge_first && P + r > 64) throw std::invalid_argument("ga_assign: P + r <= 64 when children join the pool");
  const size_t lds = ga_assign_lds(P, L, r);
  if (lds > 64 * 1024) throw std::invalid_argument("ga_assign: pool, children and costs exceed 64 KiB of LDS");
  ga_assign_kernel<<<islands, 64, lds, stream>>>(cost, L, V, conflict, invalid, pop, pop_cost, hist, P, G, m, r,
                                                 purge_first, mutate, swap, seed, island_base, gen_base);
  AV_HIP_CHECK(hipGetLastError());
}

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
