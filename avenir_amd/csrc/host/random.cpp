// Host-side counter-based Gaussian draws (Philox4x32-10, the generator of avenir_common.h and
// ops/random.py): value i = normal(seed, offset, index_base + i), fp64 Box-Muller over two 53-bit
// uniforms, filled by several threads.  Keyed by a GLOBAL row index, the draws of a row do not
// depend on which rank reads it or how the file is split; and one host array feeds both the CPU
// and the GPU path of a job, so the two write the same output.
#include <cmath>
#include <cstdint>
#include <thread>
#include <vector>

#include "avenir_host.h"

namespace {

struct U4 {
  uint32_t x, y, z, w;
};

inline U4 philox(uint64_t seed, uint64_t offset, uint64_t idx) {
  uint32_t c0 = (uint32_t)idx, c1 = (uint32_t)(idx >> 32), c2 = (uint32_t)offset, c3 = (uint32_t)(offset >> 32);
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0, hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return {c0, c1, c2, c3};
}

inline double unit53(uint32_t a, uint32_t b) {  // (0, 1]
  const uint64_t m = ((uint64_t)a << 21) ^ (uint64_t)(b >> 11);
  return ((double)(m & ((1ull << 53) - 1)) + 1.0) * (1.0 / 9007199254740992.0);
}

}  // namespace

namespace avh {

void philox_normal(uint64_t seed, uint64_t offset, uint64_t index_base, int64_t n, double* out, int nthreads,
                   int pairs) {
  if (n <= 0) return;
  const int T = std::max(1, std::min<int>(nthreads, (int)((n + 65535) / 65536)));
  auto work = [&](int t) {
    const int64_t lo = n * t / T, hi = n * (t + 1) / T;
    for (int64_t i = lo; i < hi; ++i) {
      const U4 r = philox(seed, offset, index_base + (uint64_t)i);
      const double u1 = unit53(r.x, r.y), u2 = unit53(r.z, r.w);
      const double rad = std::sqrt(-2.0 * std::log(u1)), a = 6.283185307179586476925 * u2;
      if (pairs) {               // both Box-Muller outputs: out[2 i] (cos), out[2 i + 1] (sin)
        out[2 * i] = rad * std::cos(a);
        out[2 * i + 1] = rad * std::sin(a);
      } else {
        out[i] = rad * std::cos(a);
      }
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < T; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
}

}  // namespace avh
