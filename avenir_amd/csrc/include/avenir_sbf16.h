// Split-bf16 ("bf16xN") arithmetic for fp32 GEMM-shaped kernels on the bf16 matrix cores (gfx950).
//
// An fp32 value x is carried as NS bf16 terms x = x_0 + x_1 (+ x_2), each term the RNE bf16 of what
// the previous ones left (v_cvt_pk_bf16_f32, exact subtraction in fp32).  A product x w is then the
// sum of the term products of order <= NS - 1:
//   NS = 2 ("bf16x3"): x_0 w_0 + x_1 w_0 + x_0 w_1 — ~16 significand bits per input, ~2^-17 relative
//                      error per product;
//   NS = 3 ("bf16x6"): + x_2 w_0 + x_1 w_1 + x_0 w_2 — ~24 bits, fp32-level error.
// Every term product is one bf16 MFMA with fp32 accumulation (16x the fp32 MFMA rate on CDNA4), so a
// bf16x3 tile spends ~3/16 and a bf16x6 tile ~6/16 of the matrix-core time of the fp32 MFMA tile.
// bf16 has fp32's exponent range: no scaling (an input of +-inf yields NaN).
//
// mlp.hip (K27) and cluster.hip (k-means) carry their own copies specialised to their LDS layouts;
// gemm.hip (gemm_tn) and distance.hip (knn) use these.
#pragma once

#include <cstdlib>
#include <string>

namespace sbf {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned pack(float a, float b) {  // v_cvt_pk_bf16_f32 (RNE)
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){a, b}, bf16x2));
}
__device__ __forceinline__ float lo(unsigned p) { return __builtin_bit_cast(float, p << 16); }
__device__ __forceinline__ float hi(unsigned p) { return __builtin_bit_cast(float, p & 0xffff0000u); }

// 8 fp32 values (consecutive k of one operand row) -> NS bf16x8 terms, as packed u32 quads
template <int NS>
__device__ __forceinline__ void split8(float (&r)[8], u32x4 (&t)[NS]) {
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    u32x4 u;
#pragma unroll
    for (int q = 0; q < 4; ++q) u[q] = pack(r[2 * q], r[2 * q + 1]);
    t[s] = u;
    if (s + 1 < NS) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        r[2 * q] -= lo(u[q]);
        r[2 * q + 1] -= hi(u[q]);
      }
    }
  }
}

__device__ __forceinline__ bf16x8 frag(u32x4 u) { return __builtin_bit_cast(bf16x8, u); }

// acc += sum of the term products of order <= NS - 1 on v_mfma_f32_32x32x16_bf16, smallest order
// first (a[t] / b[t]: the operands' terms as that MFMA's A / B fragments)
template <int NS>
__device__ __forceinline__ void mfma32_terms(const bf16x8 (&a)[NS], const bf16x8 (&b)[NS],
                                             float __attribute__((ext_vector_type(16))) & acc) {
#pragma unroll
  for (int ord = NS - 1; ord >= 0; --ord)
#pragma unroll
    for (int ta = ord; ta >= 0; --ta) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ta], b[ord - ta], acc, 0, 0, 0);
}

// Arithmetic mode from an environment variable: "f32" -> 0, "bf16x3" -> 3, "bf16x6" -> 6; unset or
// anything else -> `dflt`.
inline int env_mode(const char* var, int dflt) {
  const char* e = std::getenv(var);
  if (e == nullptr) return dflt;
  const std::string v(e);
  if (v == "f32") return 0;
  if (v == "bf16x3") return 3;
  if (v == "bf16x6") return 6;
  return dflt;
}

}  // namespace sbf
