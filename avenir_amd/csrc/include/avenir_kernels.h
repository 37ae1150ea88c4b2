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
// ---- wide.hip: uint16 codes (> 255 values per field) -------------------------------------------
void class_histogram_wide(const uint16_t* codes, long long ld, long long n, const uint8_t* labels, const int* d_bins,
                          const int* d_offs, int nfeat, int total_bins, int n_classes, int count_labels,
                          unsigned long long* out, int mode, hipStream_t stream);
void class_histogram_i32(const int* codes, long long ld, long long n, const uint8_t* labels, const int* d_bins,
                          const int* d_offs, int nfeat, int total_bins, int n_classes, int count_labels,
                          unsigned long long* out, int mode, hipStream_t stream);
void pair_histogram(const uint8_t* codes, long long ld, long long n, const uint8_t* labels,
                    const int* d_bins, const int* d_pairs, const long long* d_poff, int n_pairs,
                    int max_tab, int n_classes, unsigned long long* out, hipStream_t stream);
void bigram_histogram(const int16_t* states, long long n, int L, const uint8_t* labels,
                      int n_classes, int S, unsigned long long* out, hipStream_t stream);
void class_moments(const float* x, long long ld, long long n, int nfeat, const uint8_t* labels,
                   int n_classes, double* part, int nblocks, double* out, hipStream_t stream);
int moments_blocks(long long n);
// K2 on row-packed records: one uint16 word per record, field k at bit h_shift[k] (1..3 bits,
// all-ones = missing), class at label_shift.
void class_histogram_rowpacked(const uint16_t* words, long long n, const int* h_shift, const int* h_width, int nfeat,
                               int label_shift, int label_width, const int* d_bins, const int* d_offs, int total_bins,
                               int n_classes, int count_labels, unsigned long long* out, hipStream_t stream);

// ---- bayes.hip ----------------------------------------------------------------------------
int nb_predict_wide_max_classes();
void nb_predict_wide(const void* codes, int code_bytes, long long ld, long long n, int nfeat, const int* offs,
                     const int* bins, const float* logpT, const float* logfp, const float* x, long long ldx, int ncont,
                     const float* gmean, const float* ginvstd, const float* glognorm, const float* pmean,
                     const float* pinvstd, const float* plognorm, const float* logprior, int C, int ref_scale,
                     float* post, int* pred, const uint8_t* labels, unsigned long long* confusion, hipStream_t stream);
void nb_predict(const uint8_t* codes, long long ld, long long n, int nfeat, const int* offs,
                const float* logp, const float* logfp, int total_bins, const float* x, long long ldx,
                int ncont, const float* gmean, const float* ginvstd, const float* glognorm,
                const float* pmean, const float* pinvstd, const float* plognorm,
                const float* logprior, int C, int ref_scale, float* post, int* pred,
                const uint8_t* labels, unsigned long long* confusion, hipStream_t stream);

// ---- tree.hip (K7/K8) -----------------------------------------------------------------------
void node_histogram(const uint8_t* codes, long long ld, long long n, const uint8_t* labels,
                    const int* node, const uint8_t* weight, const int* bins, const int* offs,
                    int nfeat, int total_bins, int n_classes, int n_nodes, const long long* node_rows,
                    unsigned long long* hist, hipStream_t stream);
void node_grad_histogram(const uint8_t* codes, long long ld, long long n, const int* node,
                         const float* g, const float* h, const int* bins, const int* offs, int nfeat,
                         int total_bins, int n_nodes, int even_only, int tot_slot, float scale, long long* out, hipStream_t stream);
void tree_assign(const uint8_t* codes, long long ld, long long n, int* node, const int* split_feat,
                 const short* segmap, int max_bins, const int* child_of, int max_seg,
                 hipStream_t stream);
void tree_predict(const uint8_t* codes, long long ld, long long n, const int* feat, const int* seg_base,
                  const short* segmap, int max_bins, const int* child_base, const int* child,
                  const int* leaf_idx, const float* values, int V, const int* tree_root,
                  const float* tree_w, int n_trees, int mode, float* out, hipStream_t stream);

// ---- distance.hip (K9/K11) -----------------------------------------------------------------
void knn_topk(const float* Q, long long M, const float* R, long long N, int D, int k,
              long long q_index_base, long long r_index_base, int exclude_self, float* out_d,
              long long* out_i, int splits, int metric, float p, hipStream_t stream, int prec = -1);
// squared-euclidean dot products: 0 fp32 MFMA, 3 / 6 split-bf16 (AVMI_KNN_MFMA; default bf16x6)
int knn_mode();
void knn_vote(const float* dist, const long long* idx, long long M, int k, const long long* ys,
              const float* post, int post_mode, int C, int kern, float kparam, float scale, float kscale,
              int invdist, float thr, int pos, float* scores, float* prob, long long* pred, hipStream_t stream);
void cluster_accumulate(const float* X, long long N, int D, const int* assign, int K, double* sums,
                        unsigned long long* counts, hipStream_t stream);

// ---- sequence.hip (K14/K15) ----------------------------------------------------------------
void viterbi(const short* obs, long long n, int T, int S, int O, const float* logA, const float* logB,
             const float* logpi, int mode, short* bp, short* path, float* score, hipStream_t stream);
// chunked Viterbi pieces: n runs (run k reads observation row k / obs_div, starts from logpi row
// k % pi_mod), optional back-pointers [n, T, S], final delta vectors [n, S]
void viterbi_chunks(const short* obs, long long n, long long obs_div, int T, int S, int O, const float* logA,
                    const float* logB, const float* logpi, long long pi_mod, short* bp, float* delta_out,
                    hipStream_t stream);
void viterbi_backtrack(const short* bp, const int* lens, const int* ends, long long ntracks, int per_chunk, int T,
                       int S, int* first, short* path, hipStream_t stream);
void markov_logodds(const short* states, long long n, int L, const float* lr, int S, float* out,
                    hipStream_t stream);

// ---- assoc.hip (K17) -----------------------------------------------------------------------
void itemset_support(const unsigned long long* P, int W, const unsigned long long* items,
                     const int* cand_prefix, const int* cand_item, int M, unsigned long long* support,
                     hipStream_t stream);
void build_bitsets(const long long* tx, const int* item, long long n, int W, int n_items,
                   unsigned long long* bits, hipStream_t stream);

// ---- bandit.hip (K20) ----------------------------------------------------------------------
void bandit_select(int algo, int G, int A, int batch, const int* trials, const float* rsum, const float* probs,
                   const unsigned* hist, int nb, float bin_width, const float* fparam, const int* iparam,
                   float* gstate, int* istate, int* epochs, unsigned long long seed, unsigned long long round,
                   int* out, hipStream_t stream);

// ---- sampler.hip (K21) ---------------------------------------------------------------------
// fp64 N(0,1) of Philox(seed, offset, index_base + i) (pairs: both Box-Muller outputs, out [n][2]);
// the device twin of avh::philox_normal (sampler.hip)
void philox_normal(unsigned long long seed, unsigned long long offset, unsigned long long index_base, long long n,
                   double* out, int pairs, hipStream_t stream);
void sample(int dist, long long n, const float* params, const float* table, int nbins, unsigned long long seed,
            unsigned long long offset, float* out, hipStream_t stream);

// ---- optim.hip (K22) -----------------------------------------------------------------------
// island GA over an assignment domain: pop [islands][P][L] and pop_cost [islands][P] in / out,
// hist [islands][G] the best cost at each generation's start (optim.hip)
size_t ga_assign_lds(int P, int L, int r);
void ga_assign(const float* cost, int L, int V, const uint8_t* conflict, float invalid, short* pop, float* pop_cost,
               float* hist, int islands, int P, int G, int m, int r, int purge_first, int mutate, int swap,
               unsigned long long seed, long long island_base, int gen_base, hipStream_t stream);
void sa_assign(const float* cost, int L, int V, const uint8_t* conflict, int swap, short* sol, float* cur_cost,
               short* best_sol, float* best_cost, int P, int iters, float t0, float cool, int interval,
               int geometric, int max_retry, unsigned long long seed, unsigned long long offset,
               int it_begin, float temp_start, unsigned long long* stats, long long chain_base,
               hipStream_t stream);

// ---- linear.hip (K13) ----------------------------------------------------------------------
int glm_grid(long long n);
void glm_grad(const float* X, long long ld, long long n, int D, const float* y, const float* sw, const float* w,
              int mode, double* partial, int grid, float* hw, hipStream_t stream);

// ---- svm.hip (K12) -------------------------------------------------------------------------
void smo_solve(const float* K, const float* y, const float* diag, float* alpha, float* G, int B, int N, float C,
               float eps, int max_iter, int* iters, hipStream_t stream);
// working-set selection (gap, top-h up / low violators, duplicate mask) and gradient update
void smo_ws_select(const float* alpha, const float* G, const float* y, int B, int N, int ldag, float C, int h,
                   long long* ws, bool* ok, float* gap, int* cand, int* cnt, float skip, hipStream_t stream);
int smo_ws_select_parts(int N);
void smo_ws_update(const float* K, const long long* ws, const float* dA, const bool* ok, const float* y, float* G,
                   int B, int N, int ldag, int Q, const float* gap, float skip, long long kbs, hipStream_t stream);
// Implicit kernel source of the working-set solver: k(x_i, x_j) recomputed from the rows of X instead
// of read from an N x N matrix (O(N D) memory).  Problem b uses rows X + b * xbs (xbs = 0: shared).
struct SvmKerX {
  const float* X;   // [B or 1][N][D] row-major
  const float* xn;  // [B or 1][N] squared norms
  long long xbs;    // problem stride in rows (0 or N)
  int D;
  int kind;         // 0 linear, 1 poly, 2 rbf, 3 sigmoid
  int degree;
  float gamma, coef0;
};
void smo_ws_gather_x(const SvmKerX& k, const long long* ws, const bool* ok, float* Kws, int B, int N, const float* gap,
                     float skip, hipStream_t stream);
// HBM cache of kernel rows K[r, 0..N) for the implicit-kernel solver (one problem, shared X):
// S slots in sets of `ways`, LRU within a set by last-used step; slots S..S+Q-1 are transient rows
// for misses a full set cannot take.  All state lives on the device (graph-capturable).
struct SvmCache {
  float* rows;                // [S + Q][N]
  int* tag;                   // [S] cached row or -1
  int* stamp;                 // [S] step of last use
  int* slot_of;               // [N] slot of a row or -1 (validated against tag)
  int* step;                  // [1] step counter (advanced by the lookup kernel)
  long long* ws_slot;         // [Q] row of the cache holding K[ws[q], :] this step
  int* miss_q;                // [Q] working-set positions whose row must be computed this step
  int* miss_cnt;              // [1]
  unsigned long long* stats;  // [2] hits, misses (cumulative)
  int S, ways;
};
// one outer step's gradient update through the cache: lookup / LRU replacement, the missing rows
// computed from X into their slots, then G[n] += y[n] sum_q dA_q rows[slot_q][n] (dense update)
void smo_ws_update_cached(const SvmKerX& k, const SvmCache& c, const long long* ws, const float* dA, const bool* ok,
                          const float* y, float* G, int N, int ldag, int Q, const float* gap, float skip,
                          hipStream_t stream);
void smo_ws_update_x(const SvmKerX& k, const long long* ws, const float* dA, const bool* ok, const float* y, float* G,
                     int B, int N, int ldag, int Q, const float* gap, float skip, hipStream_t stream);
// K [na, nb] = k(a_i, b_j) through f32 MFMA (v_mfma_f32_16x16x4_f32) for any d; a.X / a.xn are the
// rows of A, Bx / bn those of B
void svm_kernel_matrix_mfma(const SvmKerX& a, const float* Bx, const float* bn, int na, int nb, float* K,
                            hipStream_t stream);
// kx == nullptr: explicit K (kbs = problem stride); else the implicit source (K unused)
long long smo_ws_run(const float* K, int N, float* alpha, float* G, const float* y, int B, int ldag, float C,
                     float eps, int inner_iter, float rel_tol, long long max_outer, int check_every, long long* ws,
                     bool* ok, float* dA, long long* inner_total, float* gap, int* cand, int* cnt, float* Kws,
                     float* host_gap, long long kbs, hipStream_t stream, const SvmKerX* kx = nullptr,
                     float* gap_next = nullptr, const SvmCache* cache = nullptr);
void smo_ws_solve_fused(const float* K, int N, const long long* ws, const bool* ok, float* alpha, const float* G,
                        const float* y, int ldag, const float* gap, int B, float C, float eps, int max_iter, float* dA,
                        long long* inner_total, float* Kws, float rel_tol, long long kbs, hipStream_t stream);
int smo_ws_size();
void rbf_matrix(const float* A, const float* B, int na, int nb, int d, float gamma, float* K, hipStream_t stream);
void smo_ws_solve(const float* Kws, const float* yws, float* aws, const float* gws, const float* gap, int B, float C,
                  float eps, int max_iter, int* iters, hipStream_t stream);

// ---- split.hip (K7 reference-semantics split scoring) ------------------------------------------
void ref_split_score(const long long* hist, int A, int C, int TBt, const int* sp, const signed char* seg, int R,
                     const unsigned char* cand, int F, int algo, int k, int G2, long long* top, double* topv,
                     double* segc, double* cinfo, double* scratch, hipStream_t stream);

// ---- transformer.hip: encoder epilogues (BERT for semantic search) -----------------------------
void add_layernorm(const float* x, const float* res, const float* gamma, const float* beta, float* out, long long rows,
                   int H, float eps, hipStream_t stream);
// out = LN(sum_{s < S} partial[s] + bias + res) (transformer.hip; S = 1, bias = null: LN(x + res))
void add_layernorm_slices(const float* partial, int S, long long sstride, const float* bias, const float* res,
                          const float* gamma, const float* beta, float* out, long long rows, int H, float eps,
                          hipStream_t stream);
// multi-head attention, head dim 64: qkv [B*S, 3H] (Q | K | V, heads of 64), kbias [B, S] additive or null
void attention_f32(const float* qkv, const float* kbias, float* out, int B, int S, int nh, float scale,
                   hipStream_t stream);
void embed_layernorm(const long long* ids, const long long* tt, const float* word, const float* pos, const float* type,
                     const float* gamma, const float* beta, float* out, long long rows, int S, int H, float eps,
                     long long nword, int ntype, hipStream_t stream);

// ---- gemm.hip: split-K fp32 A^T B (weight gradients over a long row dimension) ---------------
int gemm_tn_slices(int K, int M, int N);
// prec: -1 the process default (gemm_tn_mode(): AVMI_GEMM_TN, else f32_gemm_mode()), 0 fp32 MFMA,
// 3 split-bf16 x3, 6 split-bf16 x6 (avenir_sbf16.h)
void gemm_tn(const float* A, const float* B, float* C, float* partial, int K, int M, int N, int S, hipStream_t stream,
             int prec = -1);
int gemm_tn_mode();

// ---- rnn_f32.hip (K27 fp32) ------------------------------------------------------------------
void lstm_fwd_f32(const float* xw, const float* x, const float* wxfrag, const float* biask, const float* wfrag,
                  const float* h0, const float* c0, int B, int T, int H, int I, int KS, float* hseq, float* cseq,
                  float* gates, float* hx, hipStream_t s);
void lstm_pack_f32(const float* w_ih, const float* w_hh, const float* b_ih, const float* b_hh, int H, int I, int KS,
                   float* wfrag, float* wfragT, float* wihk, float* biask, float* wxfrag, hipStream_t s);
void lstm_bwd_f32(const float* dhseq, const float* gates, const float* cseq, const float* c0, const float* dhn,
                  const float* dcn, const float* wfragT, int B, int T, int H, int KS, float* dz, float* dh0,
                  float* dc0, hipStream_t s);

// ---- bayes.hip: model finalisation -----------------------------------------------------------
void nb_finalize(const long long* counts, int C, int TB, const int* offs, const int* bins, int F, float laplace,
                 float log_floor, float* logp, float* logfp, float* logprior, hipStream_t stream);

int gram_grid(long long n);
void weighted_gram(const float* X, long long ld, long long n, int D, const float* h, float* partial, int grid,
                   hipStream_t stream);

// ---- cluster.hip (K16) ---------------------------------------------------------------------
int kmeans_grid(long long n, int D, int K, int R);
void kmeans_assign(const float* X, long long n, int D, const float* C2, const float* Cn, const int* roff, int R, int K,
                   int* assign, float* partial, double* sse_partial, int grid, hipStream_t stream);
void kmeans_reduce(const float* partial, const double* sse_partial, int grid, int K, int D, int R, double* out,
                   hipStream_t stream);
void kmeans_update(const double* flat, int K, int D, int R, const int* run_of, const unsigned char* frozen, float* C2,
                   float* Cn, float* moves, hipStream_t stream);

// seqmine.hip (K5 n-gram hash counts, K16 uniformisation, K19 dot-matrix matching)
void ngram_count(const short* st, long long n, int L, int S, int min_len, int max_len, const int* group,
                 unsigned long long group_mul, unsigned long long* keys, unsigned* counts, unsigned long long cap,
                 int* overflow, hipStream_t stream);
void hash_compact(const unsigned long long* keys, const unsigned* counts, unsigned long long cap, long long* out_keys,
                  long long* out_counts, unsigned long long* n_out, hipStream_t stream);
void uniformization(const double* P, int S, const double* w1, const double* w2, const int* steps, int ldw, int B,
                    double* out, hipStream_t stream);
void dot_matrix(const int* A, int n, int Wa, const int* B, int m, int Wb, int* hits, hipStream_t stream);

// forest.hip (device-resident forest builder: chunk histograms, K6/K7 split scoring, partitioning)
void bucketize_u8(const float* X, long long ldx, long long n, int F, const float* edges, const int* eoff, uint8_t* out,
                  long long ldo, hipStream_t stream);
void forest_hist(const uint8_t* codes, long long ld, const uint8_t* lab, const uint8_t* wt, const int* item_slot,
                 const long long* item_start, const int* item_len, int n_items, const int* bins, const int* offs,
                 int nfeat, int TB, int C, unsigned long long* hist, hipStream_t stream);
void forest_split(const long long* hist, const uint8_t* fmask, const int* bins, const int* offs, int nfeat, int TB,
                  int C, int algo, int topk, const float* rnd, int A, int* feat, int* thr, float* score, float* imp,
                  long long* left, hipStream_t stream);
void forest_part_count(const uint8_t* codes, long long ld, const int* item_node, const long long* item_start,
                       const int* item_len, int n_items, const int* feat, const int* thr, int* item_left,
                       hipStream_t stream);
// K27 fused Linear + bias + activation (mlp.hip); with S > 1 and a partial buffer of S*M*N floats
// the K range is split over S slices (linear_act_fwd_slices picks S for few output tiles over a long K)
int linear_act_fwd_slices(int M, int N, int K);
// arithmetic of the fp32 GEMM tiles: 0 exact-f32 MFMA, 3 split-bf16 x3 (~2^-16 per product), 6
// split-bf16 x6 (fp32-level error); f32_gemm_mode() is the process default (AVMI_F32_GEMM = f32 |
// bf16x3 | bf16x6, default bf16x6), a call's prec < 0 takes it
int f32_gemm_mode();
// the raw split-K partial products [S_eff][M][N] of X W^T (no bias / activation); returns S_eff
int linear_splitk_partial(const float* X, const float* W, float* partial, int M, int N, int K, int S,
                          hipStream_t stream, int prec = -1);
// bytes of bf16 term-plane scratch the large-shape split-bf16 path of linear_act_fwd takes (its
// `planes` argument); 0 when that path is not taken for this shape / mode (AVMI_SBF16_PLANES=0: never)
long long linear_act_fwd_planes_bytes(int M, int N, int K, int prec = -1);
// bf16 term planes of a weight W [N, K] in the planes path's layout (reusable for any X while W and
// the mode are unchanged: linear_act_fwd's w_planes skips W's split); 0 bytes = path off for prec
long long sbf16_weight_planes_bytes(int N, int K, int prec = -1);
void sbf16_weight_planes(const float* W, int N, int K, int prec, void* out, hipStream_t stream);
void linear_act_fwd(const float* X, const float* W, const float* b, float* Y, int M, int N, int K, int act,
                    hipStream_t stream, float* partial = nullptr, int S = 1, int prec = -1, void* planes = nullptr,
                    const void* w_planes = nullptr);
int linear_act_bwd_rows(int M, int N);
int linear_act_bwd_blocks(int M, int N);
void linear_act_bwd(const float* dY, const float* Y, float* dZ, float* partial, int M, int N, int act,
                    hipStream_t stream);
// out [N*K + N] = (dW = dZ^T X row-major [N, K], db = colsum dZ) with dZ = dY * act'(Y) fused (dZ
// written when non-null); pW [S, N*K + N] slice partials, tmp [ceil(S / 64), N*K + N],
// S = linear_act_wgrad_slices(M, N, K)
int linear_act_wgrad_slices(int M, int N, int K);
void linear_act_wgrad(const float* dY, const float* Y, const float* X, float* dZ, float* pW, float* tmp, float* out,
                      int M, int N, int K, int act, hipStream_t stream);
long long forest_predict_bin_lds(int n_nodes, int nfeat);
void forest_predict_bin(const uint8_t* codes, long long ld, long long n, int nfeat, const uint2* nodes, int n_nodes,
                        const float* values, int V, const int* tree_root, const float* tree_w, int n_trees, int mode,
                        float* out, hipStream_t stream);
// dense B-bit record streams (histogram.hip)
long long dense_words(long long n, int B);
void pack_dense(const uint16_t* words, long long n, int B, uint32_t* dense, hipStream_t stream);
void class_histogram_dense(const uint32_t* dense, long long n, int B, const int* h_shift, const int* h_width,
                           int nfeat, int label_shift, int label_width, const int* d_bins, const int* d_offs,
                           int total_bins, int n_classes, int count_labels, unsigned long long* out,
                           hipStream_t stream);
// K1 device CSV parse (csv.hip)
long long csv_chunks(long long size);
// tokens parsed since the last call whose rounding the device could not settle (then re-parse on the
// host); synchronises the stream
unsigned long long csv_slow_tokens_take(hipStream_t stream);
unsigned long long rec_slow_tokens_take(hipStream_t stream);
void csv_newline_counts(const uint8_t* bytes, long long size, unsigned* counts, hipStream_t stream);
void csv_newline_positions(const uint8_t* bytes, long long size, const long long* offsets, long long* pos,
                           hipStream_t stream);
// per line: starts / ends (line i ends at pos[i]), keep = not blank (CR-only lines are blank),
// *blank += blank lines
void csv_line_bounds(const uint8_t* bytes, const long long* pos, long long nl, long long* starts, long long* ends,
                     uint8_t* keep, unsigned long long* blank, hipStream_t stream);
void csv_parse_rows(const uint8_t* bytes, long long size_padded, const long long* starts, const long long* ends,
                    long long n, char delim, const void* specs, int nspecs, int max_ord, const int* tabs,
                    const int* voff, const int* vlen, const uint8_t* vbytes, int ntab, int nvoc, int nvb,
                    unsigned long long* short_rows, hipStream_t stream);
int csv_devspec_bytes();
// K25 re-sampling (resample.hip)
void resample_uniform(unsigned long long seed, unsigned long long stream, long long base, long long n, float* out,
                      hipStream_t st);
void smote(const float* X, const float* Xn, const int* nn, const int* Cs, const int* Cn, long long m, int k, int D,
           int Dc, int mult, long long gbase, unsigned long long seed, int exponential, float exp_mean, float* outX,
           int* outC, int* outPick, hipStream_t st);
// device GBT round (gbt.hip)
void gbt_grad(const float* F, int K, int k, const uint8_t* y, long long n, long long row_off, unsigned long long seed,
              unsigned rate32, float* g, float* h, double* loss, hipStream_t stream);
void gbt_split(const long long* hist, const long long* parent, const long long* left, long long* out_hist, int A,
               int TB, int tot, const int* pfeat, const int* pthr, const int* pstart, const int* pend,
               const unsigned char* pvalid, int nb, double l2, double invS, int hb, int hc, int level0, int* feat,
               int* thr, double* val, hipStream_t stream);
void gbt_assign(const uint8_t* codes, long long ld, long long n, int* node, const int* feat, const int* thr,
                const double* value, const int* bins, int level, int last, float lr, float* F, int K, int k,
                hipStream_t stream);
// K1 device tokenizer for non-schema record layouts (records.hip)
void rec_lines(const uint8_t* bytes, const long long* nlpos, long long nraw, const char* delims, int ndelims,
               long long* lstart, long long* lend, int* ntok, hipStream_t stream);
void rec_tokens(const uint8_t* bytes, const long long* lstart, const long long* lend, const long long* off, long long L,
                const char* delims, int ndelims, const char* modes, int nmodes, char tail_mode, char sub_delim,
                bool trim, char last_mode, unsigned long long* keys, unsigned* h2tab, unsigned long long* first,
                unsigned long long mask, int* tslot, unsigned* th2, int* tsub, unsigned* th2sub, double* nums,
                unsigned* inserted, unsigned* overflow, hipStream_t stream);
void rec_codes(const int* tslot, const unsigned* th2, long long T, const int* slot_code, const unsigned* h2tab,
               int* codes, unsigned* mismatch, hipStream_t stream);
void rec_vocab(const uint8_t* bytes, const long long* lstart, const long long* lend, const long long* off, long long L,
               const unsigned long long* occ, long long D, const char* delims, int ndelims, char sub_delim, bool trim,
               long long* vstart, int* vlen, hipStream_t stream);
void rec_gather(const uint8_t* bytes, const long long* vstart, const int* vlen, const long long* vout, long long D,
                uint8_t* out, hipStream_t stream);
void forest_boot_count(const unsigned long long* keys, int ntrees, long long n, long long row_off, int mode,
                       unsigned rate32, int* tile_cnt, hipStream_t stream);
void forest_boot_scatter(const uint8_t* codes, long long ld, int nfeat, const uint8_t* lab,
                         const unsigned long long* keys, int ntrees, long long n, long long row_off, int mode,
                         unsigned rate32, const long long* tile_off, uint8_t* dcodes, uint8_t* dlab, uint8_t* dwt,
                         long long ldb, hipStream_t stream);
void forest_part_scatter(const uint8_t* codes, const uint8_t* lab, const uint8_t* wt, uint8_t* dcodes, uint8_t* dlab,
                         uint8_t* dwt, long long ld, int nfeat, const int* item_node, const long long* item_start,
                         const int* item_len, int n_items, const long long* left_base, const long long* right_base,
                         const int* feat, const int* thr, hipStream_t stream);

// gsp.hip (K18 GSP candidate self-join over a lexicographically sorted [N, k] sequence matrix)
void gsp_count(const int* X, int N, int k, int lo, int hi, int* seg_start, int* seg_len, hipStream_t stream);
void gsp_emit(const int* X, int k, int lo, int hi, const int* seg_start, const int* seg_len, const long long* offs,
              int* out, hipStream_t stream);

// encode.hip (K26 column moments, K23 leave-one-out target encoding)
int col_moments_blocks(long long n, int F);
void col_moments_f32(const float* X, long long n, long long ld, int F, int pass, const double* mean, double* part,
                     hipStream_t stream);
void col_moments_f64(const double* X, long long n, long long ld, int F, int pass, const double* mean, double* part,
                     hipStream_t stream);
void loo_stats(const void* codes, int code_bytes, int m, long long ld, long long n, int F, const double* y, double* sum,
               unsigned* cnt, hipStream_t stream);
void loo_apply(const void* codes, int code_bytes, int m, long long ld, long long n, int F, const double* y, const double* sum,
               const unsigned* cnt, const double* gmean, double reg, const double* noise, double amp, float* out,
               hipStream_t stream);

// pca.hip (K24 streaming PCA, one wave per key; D <= 64, H <= D)
void spirit_update(const double* X, int K, int T, int D, int H, const int* lens, double* W, double* E, double* he,
                   double* ve, double* cnt, int* nh, double lam, double lo, double hi, hipStream_t stream);

// ---- rnn.hip (K27 persistent LSTM recurrence, bf16 MFMA) -------------------------------------
// KS = HP / 32 (HP = hidden size padded to 32, 64 or 128), IS = IP / 32 likewise for the layer
// input size, RT = 16-sequence tiles per workgroup.
int lstm_row_tiles(long long B, int KS);
void lstm_fwd(const float* x, int I, int IS, const void* wfrag, const float* bias, const float* h0, const float* c0,
              int B, int T, int H, int KS, int RT, float* hseq, float* cseq, unsigned short* gates, unsigned short* hx,
              hipStream_t stream);
void lstm_bwd(const float* dhseq, const unsigned short* gates, const float* cseq, const float* c0, const float* dhn,
              const float* dcn, const void* wfragT, int B, int T, int H, int KS, int RT, unsigned short* dz,
              float* dh0, float* dc0, hipStream_t stream);

// distance.hip: mixed-type kNN without one-hot expansion
int mixed_knn_max_dims();
int mixed_knn_splits(long long nq, long long nr);
void mixed_knn(const float* Qn, const int* Qc, long long nq, const float* Rn, const int* Rc, long long nr, int Dn,
               int Dc, const float* wc, int k, long long r_base, float* out_d, long long* out_i, float* part_d,
               int* part_i, int splits, hipStream_t stream);

// stats.hip (K26 rank statistics)
void rank_avg(const double* sorted, const long long* perm, long long n, const int* group, int n_groups, double* ranks,
              double* tie, double* gsum, hipStream_t stream);
void kendall_pairs(const double* x, const double* y, long long n, unsigned long long* out, hipStream_t stream);
// strict inversions of a[0, m) by merge-path merges (m a power of two >= inv_merge_block(), pad
// with +inf); a / tmp clobbered, returns the one holding the sorted values; inv (u64) += count
int inv_merge_block();
double* inversions(double* a, double* tmp, long long m, unsigned long long* inv, hipStream_t stream);

// text.hip (K28)
// TF-IDF of a CSR count matrix in place: document frequencies (df, V zeroed ints) then the
// weighted, normalised rows; status bit 1 = column id out of range, 2 = bad row pointers
void tfidf_csr(const long long* crow, const long long* col, float* val, long long n_rows, long long nnz, long long V,
               int smooth, int sublinear, int norm, int* df, int* status, hipStream_t stream);
// multi-workgroup power iteration (any n): see text.hip; result in buf[state[1] & 1]
int pagerank_multi_rows();
void pagerank_multi(const double* P, int n, double d, int k0, int k1, double tol, double* buf, double* partial,
                    double* dpart, int* state, hipStream_t stream);
int pagerank_max_n();
void pagerank(const double* P, int n, double d, int iters, double tol, double* r, int* it, hipStream_t stream);
int sgns_hot_replicas();
void sgns_step(float* Win, float* Wout, float* gIn, float* gOut, float* cIn, float* cOut, int dim, long long rows_in,
               const int* centre, const int* context, long long n_pairs, const float* aprob, const int* alias, int V,
               int neg, float lr, int mean_in, unsigned long long seed, unsigned long long step, const int* hot, int H,
               float* gOutHot, float* gInHot, float* cIn_next, long long n_cin, float* cOut_next, long long n_cout,
               hipStream_t stream);

// ---- distance.hip: threshold pairs (recordSimilarity) ----------------------------------------
long long pairs_within(const float* A, int nA, const float* B, int nB, int D, float nf, float scale, float thr, int tri,
                       long long a_base, long long b_base, int* cnt, long long seg_cap, long long* outK, int* outD,
                       long long* seg_counts, hipStream_t stream);
int pairs_within_segments();
int pairs_within_counter_ints();
// ---- format.hip: output rows formatted on the device ------------------------------------------
struct DevFmtCol {
  enum Kind : int { STR = 0, F64 = 1, I64 = 2, LIT = 3, LIST = 4, GLUE = 5, RAW = 6, FIELD = 7, TAIL = 8,
                    PAIRS = 9 };
  int kind = STR;
  int prec = 0;              // F64: fraction digits 0..9
  int field = 0;             // FIELD / TAIL
  int same = 0;              // RAW: the separators are the output delimiter (copy as is)
  const int32_t* idx = nullptr;
  const int64_t* off = nullptr;
  const double* dv = nullptr;
  const int64_t* iv = nullptr;
  const uint8_t* tbytes = nullptr;  // string table bytes / offsets [tV + 1]
  const int64_t* toff = nullptr;
  int64_t tV = 0;
  const uint8_t* lbytes = nullptr;  // line bytes, per-row start and length
  const int64_t* lstart = nullptr;
  const int64_t* llen = nullptr;
  const uint8_t* lit = nullptr;
  int litlen = 0;
  uint32_t sep[8] = {0, 0, 0, 0, 0, 0, 0, 0};
};
void format_rows_len(const DevFmtCol* cols, int ncols, int64_t n, const uint8_t* delim, int dl, int64_t* len, int* bad,
                     hipStream_t stream);
void format_rows_write(const DevFmtCol* cols, int ncols, int64_t n, const uint8_t* delim, int dl, const int64_t* start,
                       char* out, hipStream_t stream);

// ---- comm.hip: peer-mapped small-message all-reduce (one-shot / two-shot) --------------------
constexpr int P2P_MAX_RANKS = 16;
constexpr int P2P_MAX_BLOCKS = 64;
enum P2PDtype { P2P_F32 = 0, P2P_F64 = 1, P2P_I32 = 2, P2P_I64 = 3 };
struct P2PView {
  void* data[P2P_MAX_RANKS];       // every rank's data region as mapped in this process
  unsigned* flags[P2P_MAX_RANKS];  // every rank's flag array as mapped in this process
  int* status;                     // this rank's status word (device, uncached: the kernels' own check)
  int* host_status;                // its host-visible copy (pinned, coherent, mapped): 1 = a wait
                                   // timed out here, 2 = a peer reported a failure
  long long cap_bytes;             // bytes of ONE staging buffer (4 per data region)
  int rank, world;
};
constexpr unsigned P2P_POISON = 0x80000000u;   // flag bit: "the rank that raised this has failed"
constexpr unsigned P2P_MAX_EPOCH = 0x3FFFFFFFu;  // so 2 * epoch never reaches the poison bit
void p2p_all_reduce(void* x, long long n, int dtype, const P2PView& v, unsigned epoch, int two_shot,
                    long long timeout_ticks, hipStream_t st);
// raise the poison flag in every peer's array for every block: their next wait on this rank ends
// at once and records status 2 (the failing rank's last act before it raises on the host)
void p2p_poison(const P2PView& v, hipStream_t st);

}  // namespace avk
