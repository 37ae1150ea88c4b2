// Host-side launcher declarations for every avenir_amd HIP kernel family.
// Implemented in csrc/kernels/*.hip; bound to Python in csrc/bindings.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include <stdexcept>

namespace avk {

// ---- histogram.hip (K2/K3/K4) -------------------------------------------------------------
void class_histogram(const uint8_t* codes, long long ld, long long n, const uint8_t* labels,
                     const int* d_bins, const int* d_offs, const int* h_bins, int nfeat,
                     int total_bins, int n_classes, int count_labels, unsigned long long* out,
                     int mode, hipStream_t stream);
void pair_histogram(const uint8_t* codes, long long ld, long long n, const uint8_t* labels,
                    const int* d_bins, const int* d_pairs, const long long* d_poff, int n_pairs,
                    int max_tab, int n_classes, unsigned long long* out, hipStream_t stream);
void bigram_histogram(const int16_t* states, long long n, int L, const uint8_t* labels,
                      int n_classes, int S, unsigned long long* out, hipStream_t stream);
void class_moments(const float* x, long long ld, long long n, int nfeat, const uint8_t* labels,
                   int n_classes, double* part, int nblocks, double* out, hipStream_t stream);
int moments_blocks(long long n);

// ---- bayes.hip ----------------------------------------------------------------------------
void nb_predict(const uint8_t* codes, long long ld, long long n, int nfeat, const int* offs,
                const float* logp, const float* logfp, int total_bins, const float* x, long long ldx,
                int ncont, const float* gmean, const float* ginvstd, const float* glognorm,
                const float* pmean, const float* pinvstd, const float* plognorm,
                const float* logprior, int C, int ref_scale, float* post, int* pred,
                const uint8_t* labels, unsigned long long* confusion, hipStream_t stream);

}  // namespace avk
