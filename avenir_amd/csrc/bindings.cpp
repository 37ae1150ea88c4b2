#include <atomic>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <chrono>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <unistd.h>
#include <sys/stat.h>
#include <sys/mman.h>
#include <fcntl.h>
// pybind11 bindings for avenir_amd._C — the only translation unit that includes torch.
//
// Each binding validates device / dtype / contiguity / shape on the host BEFORE launching (a bad
// shape must never reach a hand-written kernel), fetches the current HIP stream of the tensor's
// device, and calls the torch-free launcher in csrc/kernels/*.hip.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "avenir_kernels.h"
#include "avenir_host.h"

namespace {

// PyTorch-ROCm exposes HIP devices as device type "cuda": use its masquerading guard/stream.
using DevGuard = c10::hip::HIPGuardMasqueradingAsCUDA;

hipStream_t cur_stream(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

#define CHECK_CUDA(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_DTYPE(t, d) TORCH_CHECK((t).scalar_type() == (d), #t " must be " #d)
#define CHECK_DEV(t) \
  CHECK_CUDA(t);     \
  CHECK_CONTIG(t)

// vector loads in the kernels need the base address aligned (a sliced view may not be)
bool aligned(const at::Tensor& t, int bytes) { return reinterpret_cast<uintptr_t>(t.data_ptr()) % bytes == 0; }

template <typename T>
T* ptr_or_null(const c10::optional<at::Tensor>& t) {
  return t.has_value() && t->defined() ? t->data_ptr<T>() : nullptr;
}

// ---------------------------------------------------------------------------------------------
// K2 class-conditional histogram.  codes uint8 [F][ld] (ld >= n), labels uint8 [>=n] or None,
// bins/offs int32 [F] (device), h_bins list[int]; out int64 [C][TB] (accumulated into).
void class_histogram(const at::Tensor& codes, int64_t n, const c10::optional<at::Tensor>& labels,
                     const at::Tensor& bins, const at::Tensor& offs, std::vector<int64_t> h_bins,
                     int64_t total_bins, int64_t n_classes, at::Tensor& out, int64_t mode,
                     bool count_labels) {
  CHECK_DEV(codes);
  const bool huge = codes.scalar_type() == at::kInt;
  const bool wide = huge || codes.scalar_type() == at::kUInt16;
  TORCH_CHECK(wide || codes.scalar_type() == at::kByte, "codes must be uint8, uint16 or int32");
  TORCH_CHECK(codes.dim() == 2, "codes must be [F, ld]");
  const int64_t F = codes.size(0), ld = codes.size(1);
  TORCH_CHECK(n <= ld, "n exceeds codes leading dimension");
  TORCH_CHECK((int64_t)h_bins.size() == F, "h_bins length != F");
  CHECK_DEV(bins);
  CHECK_DTYPE(bins, at::kInt);
  CHECK_DEV(offs);
  CHECK_DTYPE(offs, at::kInt);
  TORCH_CHECK(bins.numel() == F && offs.numel() == F, "bins/offs must have F entries");
  CHECK_DEV(out);
  CHECK_DTYPE(out, at::kLong);
  TORCH_CHECK(out.numel() == n_classes * total_bins, "out must be [C*TB]");
  int64_t sum_bins = 0;
  std::vector<int> hb(F);
  for (int64_t f = 0; f < F; ++f) {
    const int64_t cap = huge ? 0x7FFFFFFE : (wide ? 65535 : 255);
    TORCH_CHECK(h_bins[f] > 0 && h_bins[f] <= cap, "bins per feature must be in [1, ", cap, "]");
    hb[f] = (int)h_bins[f];
    sum_bins += h_bins[f];
  }
  TORCH_CHECK(sum_bins + (count_labels ? 1 : 0) <= total_bins, "sum(bins) > total_bins");
  TORCH_CHECK(n_classes * total_bins < (1LL << 31), "histogram table exceeds 2^31 slots");
  TORCH_CHECK(n_classes >= 1 && n_classes <= 255, "n_classes must be in [1,255]");
  const uint8_t* lab = nullptr;
  if (labels.has_value() && labels->defined()) {
    CHECK_DEV((*labels));
    CHECK_DTYPE((*labels), at::kByte);
    TORCH_CHECK(labels->numel() >= n, "labels shorter than n");
    lab = labels->data_ptr<uint8_t>();
  }
  DevGuard g(codes.device());
  if (huge) {
    avk::class_histogram_i32(codes.data_ptr<int>(), ld, n, lab, bins.data_ptr<int>(), offs.data_ptr<int>(), (int)F,
                             (int)total_bins, (int)n_classes, count_labels ? 1 : 0,
                             reinterpret_cast<unsigned long long*>(out.data_ptr<int64_t>()), (int)mode,
                             cur_stream(codes));
    return;
  }
  if (wide) {
    avk::class_histogram_wide(reinterpret_cast<const uint16_t*>(codes.data_ptr()), ld, n, lab, bins.data_ptr<int>(),
                              offs.data_ptr<int>(), (int)F, (int)total_bins, (int)n_classes, count_labels ? 1 : 0,
                              reinterpret_cast<unsigned long long*>(out.data_ptr<int64_t>()), (int)mode,
                              cur_stream(codes));
    return;
  }
  avk::class_histogram(codes.data_ptr<uint8_t>(), ld, n, lab, bins.data_ptr<int>(),
                       offs.data_ptr<int>(), hb.data(), (int)F, (int)total_bins, (int)n_classes,
                       count_labels ? 1 : 0,
                       reinterpret_cast<unsigned long long*>(out.data_ptr<int64_t>()), (int)mode,
                       cur_stream(codes));
}

// K2 over row-packed records: words int16 [>= n] (bit layout from shifts / widths), bins / offs
// int32 [F] (device), out int64 [C][TB] (accumulated into).
void class_histogram_rowpacked(const at::Tensor& words, int64_t n, std::vector<int64_t> shifts,
                               std::vector<int64_t> widths, int64_t label_shift, int64_t label_width,
                               const at::Tensor& bins, const at::Tensor& offs, int64_t total_bins, int64_t n_classes,
                               at::Tensor& out, bool count_labels) {
  CHECK_DEV(words);
  CHECK_DTYPE(words, at::kShort);
  TORCH_CHECK(words.dim() == 1 && n >= 0 && n <= words.numel(), "words must be [>= n]");
  TORCH_CHECK(aligned(words, 16), "words must be 16-byte aligned");
  const int64_t F = (int64_t)shifts.size();
  TORCH_CHECK(F >= 1 && F <= 8 && (int64_t)widths.size() == F, "1..8 packed fields");
  std::vector<int> sh(F), wd(F);
  int64_t used = 0;
  for (int64_t k = 0; k < F; ++k) {
    TORCH_CHECK(widths[k] >= 1 && widths[k] <= 3 && shifts[k] >= 0 && shifts[k] + widths[k] <= 16,
                "packed field must be 1..3 bits inside 16");
    sh[k] = (int)shifts[k];
    wd[k] = (int)widths[k];
    used = std::max<int64_t>(used, shifts[k] + widths[k]);
  }
  TORCH_CHECK(n_classes >= 1 && n_classes <= 2, "row-packed histogram supports 1 or 2 classes");
  TORCH_CHECK(n_classes == 1 || (label_width == n_classes && label_shift >= 0 && label_shift + label_width <= 16),
              "the class must be C one-hot bits inside the 16-bit record");
  CHECK_DEV(bins);
  CHECK_DTYPE(bins, at::kInt);
  CHECK_DEV(offs);
  CHECK_DTYPE(offs, at::kInt);
  TORCH_CHECK(bins.numel() == F && offs.numel() == F, "bins / offs must have F entries");
  CHECK_DEV(out);
  CHECK_DTYPE(out, at::kLong);
  TORCH_CHECK(out.numel() == n_classes * total_bins, "out must be [C * TB]");
  DevGuard g(words.device());
  avk::class_histogram_rowpacked(reinterpret_cast<const uint16_t*>(words.data_ptr()), n, sh.data(), wd.data(), (int)F,
                                 (int)label_shift, (int)label_width, bins.data_ptr<int>(), offs.data_ptr<int>(),
                                 (int)total_bins, (int)n_classes, count_labels ? 1 : 0,
                                 reinterpret_cast<unsigned long long*>(out.data_ptr<int64_t>()), cur_stream(words));
}

// Dense B-bit record stream from the 16-bit row-packed words (32 records per B dwords).
at::Tensor pack_dense(const at::Tensor& words, int64_t n, int64_t B) {
  CHECK_DEV(words);
  CHECK_DTYPE(words, at::kShort);
  TORCH_CHECK(words.dim() == 1 && n >= 0 && n <= words.numel(), "words must be [>= n]");
  TORCH_CHECK(B >= 4 && B <= 15, "4..15 bits per record");
  auto dense = at::zeros({std::max<int64_t>(1, avk::dense_words(n, (int)B))}, words.options().dtype(at::kInt));
  DevGuard g(words.device());
  avk::pack_dense(reinterpret_cast<const uint16_t*>(words.data_ptr()), n, (int)B,
                  reinterpret_cast<uint32_t*>(dense.data_ptr<int>()), cur_stream(words));
  return dense;
}

void class_histogram_dense(const at::Tensor& dense, int64_t n, int64_t B, std::vector<int64_t> shifts,
                           std::vector<int64_t> widths, int64_t label_shift, int64_t label_width, const at::Tensor& bins,
                           const at::Tensor& offs, int64_t total_bins, int64_t n_classes, at::Tensor& out,
                           bool count_labels, std::vector<int64_t> bins_host, std::vector<int64_t> offs_host) {
  CHECK_DEV(dense);
  CHECK_DTYPE(dense, at::kInt);
  TORCH_CHECK(B >= 4 && B <= 15 && n >= 0 && dense.numel() >= avk::dense_words(n, (int)B), "dense stream too short");
  const int64_t F = (int64_t)shifts.size();
  TORCH_CHECK(F >= 1 && F <= 8 && (int64_t)widths.size() == F, "1..8 packed fields");
  std::vector<int> sh(F), wd(F);
  for (int64_t k = 0; k < F; ++k) {
    TORCH_CHECK(widths[k] >= 1 && widths[k] <= 8 && shifts[k] >= 0 && shifts[k] + widths[k] <= B,
                "packed field outside the record");
    sh[k] = (int)shifts[k];
    wd[k] = (int)widths[k];
  }
  TORCH_CHECK(n_classes >= 1 && n_classes <= 2, "1 or 2 classes");
  CHECK_DEV(bins); CHECK_DTYPE(bins, at::kInt);
  CHECK_DEV(offs); CHECK_DTYPE(offs, at::kInt);
  TORCH_CHECK(bins.numel() == F && offs.numel() == F, "bins / offs must have F entries");
  // the table bounds are checked on the host copies of bins / offs (the caller's cached device
  // tensors hold the same values): reading the device tensors back here would be a blocking
  // copy that drains the stream and serialises every training step with the host
  TORCH_CHECK((int64_t)bins_host.size() == F && (int64_t)offs_host.size() == F, "bins_host / offs_host: F entries");
  for (int64_t k = 0; k < F; ++k)
    TORCH_CHECK(offs_host[k] >= 0 && bins_host[k] >= 1 && offs_host[k] + bins_host[k] <= total_bins,
                "feature bins outside the table");
  CHECK_DEV(out); CHECK_DTYPE(out, at::kLong);
  TORCH_CHECK(out.numel() == n_classes * total_bins, "out must be [C * TB]");
  DevGuard g(dense.device());
  avk::class_histogram_dense(reinterpret_cast<const uint32_t*>(dense.data_ptr<int>()), n, (int)B, sh.data(), wd.data(),
                             (int)F, (int)label_shift, (int)label_width, bins.data_ptr<int>(), offs.data_ptr<int>(),
                             (int)total_bins, (int)n_classes, count_labels ? 1 : 0,
                             reinterpret_cast<unsigned long long*>(out.data_ptr<int64_t>()), cur_stream(dense));
}

void pair_histogram(const at::Tensor& codes, int64_t n, const c10::optional<at::Tensor>& labels,
                    const at::Tensor& bins, const at::Tensor& pairs, const at::Tensor& poff,
                    int64_t max_tab, int64_t n_classes, at::Tensor& out) {
  CHECK_DEV(codes);
  CHECK_DTYPE(codes, at::kByte);
  TORCH_CHECK(codes.dim() == 2 && n <= codes.size(1), "codes must be [F, ld>=n]");
  CHECK_DEV(bins);
  CHECK_DTYPE(bins, at::kInt);
  CHECK_DEV(pairs);
  CHECK_DTYPE(pairs, at::kInt);
  CHECK_DEV(poff);
  CHECK_DTYPE(poff, at::kLong);
  CHECK_DEV(out);
  CHECK_DTYPE(out, at::kLong);
  TORCH_CHECK(pairs.dim() == 2 && pairs.size(1) == 2, "pairs must be [P,2]");
  TORCH_CHECK(poff.numel() == pairs.size(0), "poff must be [P]");
  const uint8_t* lab = nullptr;
  if (labels.has_value() && labels->defined()) {
    CHECK_DEV((*labels));
    CHECK_DTYPE((*labels), at::kByte);
    TORCH_CHECK(labels->numel() >= n, "labels shorter than n");
    lab = labels->data_ptr<uint8_t>();
  }
  DevGuard g(codes.device());
  avk::pair_histogram(codes.data_ptr<uint8_t>(), codes.size(1), n, lab, bins.data_ptr<int>(),
                      pairs.data_ptr<int>(), reinterpret_cast<const long long*>(poff.data_ptr<int64_t>()), (int)pairs.size(0),
                      (int)max_tab, (int)n_classes,
                      reinterpret_cast<unsigned long long*>(out.data_ptr<int64_t>()),
                      cur_stream(codes));
}

void bigram_histogram(const at::Tensor& states, const c10::optional<at::Tensor>& labels,
                      int64_t n_classes, int64_t S, at::Tensor& out) {
  CHECK_DEV(states);
  CHECK_DTYPE(states, at::kShort);
  TORCH_CHECK(states.dim() == 2, "states must be [N, L]");
  CHECK_DEV(out);
  CHECK_DTYPE(out, at::kLong);
  TORCH_CHECK(out.numel() == n_classes * S * S, "out must be [C*S*S]");
  TORCH_CHECK(S >= 1 && S <= 32767, "bad S");
  const uint8_t* lab = nullptr;
  if (labels.has_value() && labels->defined()) {
    CHECK_DEV((*labels));
    CHECK_DTYPE((*labels), at::kByte);
    TORCH_CHECK(labels->numel() >= states.size(0), "labels shorter than N");
    lab = labels->data_ptr<uint8_t>();
  }
  DevGuard g(states.device());
  avk::bigram_histogram(states.data_ptr<int16_t>(), states.size(0), (int)states.size(1), lab,
                        (int)n_classes, (int)S,
                        reinterpret_cast<unsigned long long*>(out.data_ptr<int64_t>()),
                        cur_stream(states));
}

at::Tensor class_moments(const at::Tensor& x, int64_t n, const c10::optional<at::Tensor>& labels,
                         int64_t n_classes) {
  CHECK_DEV(x);
  CHECK_DTYPE(x, at::kFloat);
  TORCH_CHECK(x.dim() == 2 && n <= x.size(1), "x must be [F, ld>=n]");
  const uint8_t* lab = nullptr;
  if (labels.has_value() && labels->defined()) {
    CHECK_DEV((*labels));
    CHECK_DTYPE((*labels), at::kByte);
    TORCH_CHECK(labels->numel() >= n, "labels shorter than n");
    lab = labels->data_ptr<uint8_t>();
  }
  const int64_t F = x.size(0);
  DevGuard g(x.device());
  auto opts = x.options().dtype(at::kDouble);
  auto out = at::zeros({n_classes, F, 3}, opts);
  const int nb = avk::moments_blocks(n);
  auto part = at::empty({nb, n_classes, F, 3}, opts);
  avk::class_moments(x.data_ptr<float>(), x.size(1), n, (int)F, lab, (int)n_classes,
                     part.data_ptr<double>(), nb, out.data_ptr<double>(), cur_stream(x));
  return out;
}

// ---------------------------------------------------------------------------------------------
void nb_predict(const at::Tensor& codes, int64_t n, const at::Tensor& offs, const at::Tensor& logp,
                const c10::optional<at::Tensor>& logfp, const c10::optional<at::Tensor>& x,
                const c10::optional<at::Tensor>& gmean, const c10::optional<at::Tensor>& ginvstd,
                const c10::optional<at::Tensor>& glognorm, const c10::optional<at::Tensor>& pmean,
                const c10::optional<at::Tensor>& pinvstd, const c10::optional<at::Tensor>& plognorm,
                const at::Tensor& logprior, bool ref_scale, const c10::optional<at::Tensor>& post,
                at::Tensor& pred, const c10::optional<at::Tensor>& labels,
                const c10::optional<at::Tensor>& confusion) {
  CHECK_DEV(codes);
  CHECK_DTYPE(codes, at::kByte);
  TORCH_CHECK(codes.dim() == 2 && n <= codes.size(1), "codes must be [F, ld>=n]");
  CHECK_DEV(logp);
  CHECK_DTYPE(logp, at::kFloat);
  TORCH_CHECK(logp.dim() == 2, "logp must be [C, TB]");
  const int C = (int)logp.size(0), TB = (int)logp.size(1);
  CHECK_DEV(offs);
  CHECK_DTYPE(offs, at::kInt);
  TORCH_CHECK(offs.numel() == codes.size(0), "offs must be [F]");
  CHECK_DEV(logprior);
  CHECK_DTYPE(logprior, at::kFloat);
  TORCH_CHECK(logprior.numel() == C, "logprior must be [C]");
  CHECK_DEV(pred);
  CHECK_DTYPE(pred, at::kInt);
  TORCH_CHECK(pred.numel() >= n, "pred too short");
  int ncont = 0;
  long long ldx = 0;
  if (x.has_value() && x->defined()) {
    CHECK_DEV((*x));
    CHECK_DTYPE((*x), at::kFloat);
    TORCH_CHECK(x->dim() == 2 && n <= x->size(1), "x must be [Fc, ld>=n]");
    ncont = (int)x->size(0);
    ldx = x->size(1);
    TORCH_CHECK(gmean.has_value() && gmean->numel() == (int64_t)C * ncont, "gmean must be [C,Fc]");
    TORCH_CHECK(ginvstd.has_value() && ginvstd->numel() == (int64_t)C * ncont, "ginvstd");
    TORCH_CHECK(glognorm.has_value() && glognorm->numel() == (int64_t)C * ncont, "glognorm");
    if (ref_scale)
      TORCH_CHECK(pmean.has_value() && pinvstd.has_value() && plognorm.has_value(),
                  "feature-prior Gaussian params required with ref_scale");
  }
  if (ref_scale) TORCH_CHECK(logfp.has_value() && logfp->numel() == TB, "logfp must be [TB]");
  if (post.has_value() && post->defined()) {
    CHECK_DEV((*post));
    TORCH_CHECK(post->numel() >= n * C, "post too short");
  }
  const uint8_t* lab = nullptr;
  unsigned long long* conf = nullptr;
  if (confusion.has_value() && confusion->defined()) {
    TORCH_CHECK(labels.has_value() && labels->defined(), "confusion requires labels");
    CHECK_DEV((*labels));
    CHECK_DTYPE((*labels), at::kByte);
    TORCH_CHECK(labels->numel() >= n, "labels too short");
    CHECK_DEV((*confusion));
    CHECK_DTYPE((*confusion), at::kLong);
    TORCH_CHECK(confusion->numel() == (int64_t)C * C, "confusion must be [C,C]");
    lab = labels->data_ptr<uint8_t>();
    conf = reinterpret_cast<unsigned long long*>(confusion->data_ptr<int64_t>());
  }
  DevGuard g(codes.device());
  avk::nb_predict(codes.data_ptr<uint8_t>(), codes.size(1), n, (int)codes.size(0),
                  offs.data_ptr<int>(), logp.data_ptr<float>(), ptr_or_null<float>(logfp), TB,
                  ptr_or_null<float>(x), ldx, ncont, ptr_or_null<float>(gmean),
                  ptr_or_null<float>(ginvstd), ptr_or_null<float>(glognorm),
                  ptr_or_null<float>(pmean), ptr_or_null<float>(pinvstd),
                  ptr_or_null<float>(plognorm), logprior.data_ptr<float>(), C, ref_scale ? 1 : 0,
                  ptr_or_null<float>(post), pred.data_ptr<int>(), lab, conf, cur_stream(codes));
}

// Wide tables: codes uint8 / uint16 / int32 [F, ld], bins int32 [F] (device), logpT [TB, C] (transposed).
void nb_predict_wide(const at::Tensor& codes, int64_t n, const at::Tensor& offs, const at::Tensor& bins,
                     const at::Tensor& logpT,
                const c10::optional<at::Tensor>& logfp, const c10::optional<at::Tensor>& x,
                const c10::optional<at::Tensor>& gmean, const c10::optional<at::Tensor>& ginvstd,
                const c10::optional<at::Tensor>& glognorm, const c10::optional<at::Tensor>& pmean,
                const c10::optional<at::Tensor>& pinvstd, const c10::optional<at::Tensor>& plognorm,
                const at::Tensor& logprior, bool ref_scale, const c10::optional<at::Tensor>& post,
                at::Tensor& pred, const c10::optional<at::Tensor>& labels,
                const c10::optional<at::Tensor>& confusion) {
  CHECK_DEV(codes);
  TORCH_CHECK(codes.scalar_type() == at::kByte || codes.scalar_type() == at::kUInt16 ||
                  codes.scalar_type() == at::kInt, "codes must be uint8, uint16 or int32");
  TORCH_CHECK(codes.dim() == 2 && n <= codes.size(1) && codes.is_contiguous(), "codes must be [F, ld>=n]");
  CHECK_DEV(logpT);
  CHECK_DTYPE(logpT, at::kFloat);
  TORCH_CHECK(logpT.dim() == 2 && logpT.is_contiguous(), "logpT must be [TB, C]");
  const int TB = (int)logpT.size(0), C = (int)logpT.size(1);
  TORCH_CHECK(C >= 1 && C <= avk::nb_predict_wide_max_classes(), "nb_predict_wide: 1..32 classes");
  CHECK_DEV(bins);
  CHECK_DTYPE(bins, at::kInt);
  TORCH_CHECK(bins.numel() == codes.size(0), "bins must be [F]");
  {
    // every valid code indexes inside the table: offs[f] + bins[f] <= TB
    auto hb = bins.cpu(), ho = offs.cpu();
    for (int64_t f = 0; f < codes.size(0); ++f)
      TORCH_CHECK(ho.data_ptr<int>()[f] >= 0 && hb.data_ptr<int>()[f] >= 0 &&
                      (int64_t)ho.data_ptr<int>()[f] + hb.data_ptr<int>()[f] <= TB, "offs/bins exceed the table");
  }
  CHECK_DEV(offs);
  CHECK_DTYPE(offs, at::kInt);
  TORCH_CHECK(offs.numel() == codes.size(0), "offs must be [F]");
  CHECK_DEV(logprior);
  CHECK_DTYPE(logprior, at::kFloat);
  TORCH_CHECK(logprior.numel() == C, "logprior must be [C]");
  CHECK_DEV(pred);
  CHECK_DTYPE(pred, at::kInt);
  TORCH_CHECK(pred.numel() >= n, "pred too short");
  int ncont = 0;
  long long ldx = 0;
  if (x.has_value() && x->defined()) {
    CHECK_DEV((*x));
    CHECK_DTYPE((*x), at::kFloat);
    TORCH_CHECK(x->dim() == 2 && n <= x->size(1), "x must be [Fc, ld>=n]");
    ncont = (int)x->size(0);
    ldx = x->size(1);
    TORCH_CHECK(gmean.has_value() && gmean->numel() == (int64_t)C * ncont, "gmean must be [C,Fc]");
    TORCH_CHECK(ginvstd.has_value() && ginvstd->numel() == (int64_t)C * ncont, "ginvstd");
    TORCH_CHECK(glognorm.has_value() && glognorm->numel() == (int64_t)C * ncont, "glognorm");
    if (ref_scale)
      TORCH_CHECK(pmean.has_value() && pinvstd.has_value() && plognorm.has_value(),
                  "feature-prior Gaussian params required with ref_scale");
  }
  if (ref_scale) TORCH_CHECK(logfp.has_value() && logfp->numel() == TB, "logfp must be [TB]");
  if (post.has_value() && post->defined()) {
    CHECK_DEV((*post));
    TORCH_CHECK(post->numel() >= n * C, "post too short");
  }
  const uint8_t* lab = nullptr;
  unsigned long long* conf = nullptr;
  if (confusion.has_value() && confusion->defined()) {
    TORCH_CHECK(labels.has_value() && labels->defined(), "confusion requires labels");
    CHECK_DEV((*labels));
    CHECK_DTYPE((*labels), at::kByte);
    TORCH_CHECK(labels->numel() >= n, "labels too short");
    CHECK_DEV((*confusion));
    CHECK_DTYPE((*confusion), at::kLong);
    TORCH_CHECK(confusion->numel() == (int64_t)C * C, "confusion must be [C,C]");
    lab = labels->data_ptr<uint8_t>();
    conf = reinterpret_cast<unsigned long long*>(confusion->data_ptr<int64_t>());
  }
  DevGuard g(codes.device());
  avk::nb_predict_wide(codes.data_ptr(), (int)codes.element_size(), codes.size(1), n, (int)codes.size(0),
                       offs.data_ptr<int>(), bins.data_ptr<int>(), logpT.data_ptr<float>(), ptr_or_null<float>(logfp),
                       ptr_or_null<float>(x), ldx, ncont, ptr_or_null<float>(gmean),
                  ptr_or_null<float>(ginvstd), ptr_or_null<float>(glognorm),
                  ptr_or_null<float>(pmean), ptr_or_null<float>(pinvstd),
                  ptr_or_null<float>(plognorm), logprior.data_ptr<float>(), C, ref_scale ? 1 : 0,
                  ptr_or_null<float>(post), pred.data_ptr<int>(), lab, conf, cur_stream(codes));
}


// ---------------------------------------------------------------------------------------------
// trees (K7/K8)
// ---------------------------------------------------------------------------------------------
static void check_codes(const at::Tensor& codes, int64_t n) {
  CHECK_DEV(codes);
  CHECK_DTYPE(codes, at::kByte);
  TORCH_CHECK(codes.dim() == 2 && n <= codes.size(1), "codes must be [F, ld>=n]");
}

void node_histogram(const at::Tensor& codes, int64_t n, const at::Tensor& labels,
                    const at::Tensor& node, const c10::optional<at::Tensor>& weight,
                    const at::Tensor& bins, const at::Tensor& offs, int64_t total_bins,
                    int64_t n_classes, int64_t n_nodes, at::Tensor& hist,
                    const c10::optional<at::Tensor>& node_rows) {
  check_codes(codes, n);
  CHECK_DEV(labels);
  CHECK_DTYPE(labels, at::kByte);
  CHECK_DEV(node);
  CHECK_DTYPE(node, at::kInt);
  const int64_t n4 = (n + 3) / 4 * 4;  // the kernels read whole 4-row quads
  TORCH_CHECK(labels.numel() >= n4 && node.numel() >= n4, "labels/node must cover n rounded up to 4");
  TORCH_CHECK(codes.size(1) % 4 == 0, "codes leading dimension must be a multiple of 4");
  TORCH_CHECK(aligned(node, 16) && aligned(labels, 4) && aligned(codes, 4), "node / labels / codes misaligned");
  CHECK_DEV(bins);
  CHECK_DEV(offs);
  TORCH_CHECK(bins.numel() == codes.size(0) && offs.numel() == codes.size(0), "bins/offs != F");
  CHECK_DEV(hist);
  CHECK_DTYPE(hist, at::kLong);
  TORCH_CHECK(hist.numel() == n_nodes * n_classes * total_bins, "hist must be [A, C, TB]");
  const uint8_t* w = nullptr;
  if (weight.has_value() && weight->defined()) {
    CHECK_DEV((*weight));
    CHECK_DTYPE((*weight), at::kByte);
    TORCH_CHECK(weight->numel() >= n4 && aligned(*weight, 4), "weight must cover n rounded up to 4, 4-byte aligned");
    w = weight->data_ptr<uint8_t>();
  }
  const long long* nr = nullptr;  // per node [lo, hi) row range (the kernel clamps it to [0, n))
  if (node_rows.has_value() && node_rows->defined()) {
    CHECK_DEV((*node_rows));
    CHECK_DTYPE((*node_rows), at::kLong);
    TORCH_CHECK(node_rows->is_contiguous() && node_rows->numel() == 2 * n_nodes, "node_rows must be [A, 2]");
    nr = reinterpret_cast<const long long*>(node_rows->data_ptr<int64_t>());
  }
  DevGuard g(codes.device());
  avk::node_histogram(codes.data_ptr<uint8_t>(), codes.size(1), n, labels.data_ptr<uint8_t>(),
                      node.data_ptr<int>(), w, bins.data_ptr<int>(), offs.data_ptr<int>(),
                      (int)codes.size(0), (int)total_bins, (int)n_classes, (int)n_nodes, nr,
                      reinterpret_cast<unsigned long long*>(hist.data_ptr<int64_t>()), cur_stream(codes));
}

void node_grad_histogram(const at::Tensor& codes, int64_t n, const at::Tensor& node,
                         const at::Tensor& g, const at::Tensor& h, const at::Tensor& bins,
                         const at::Tensor& offs, int64_t total_bins, int64_t n_nodes, at::Tensor& out,
                         bool even_only, int64_t tot_slot, double scale) {
  check_codes(codes, n);
  CHECK_DEV(node);
  CHECK_DTYPE(node, at::kInt);
  CHECK_DEV(g);
  CHECK_DTYPE(g, at::kFloat);
  CHECK_DEV(h);
  CHECK_DTYPE(h, at::kFloat);
  const int64_t n4 = (n + 3) / 4 * 4;  // the kernel reads whole 4-row quads
  TORCH_CHECK(node.numel() >= n4 && g.numel() >= n4 && h.numel() >= n4, "node/g/h must cover n rounded up to 4");
  TORCH_CHECK(codes.size(1) % 4 == 0, "codes leading dimension must be a multiple of 4");
  TORCH_CHECK(aligned(node, 16) && aligned(g, 16) && aligned(h, 16) && aligned(codes, 4), "node / g / h / codes misaligned");
  CHECK_DEV(out);
  CHECK_DTYPE(out, at::kLong);
  TORCH_CHECK(out.numel() == n_nodes * total_bins * 2, "out must be [A, TB, 2]");
  TORCH_CHECK(tot_slot >= -1 && tot_slot < total_bins, "tot_slot out of range");
  TORCH_CHECK(scale > 0 && scale <= 65536.0, "scale must be in (0, 2^16]");
  DevGuard gd(codes.device());
  avk::node_grad_histogram(codes.data_ptr<uint8_t>(), codes.size(1), n, node.data_ptr<int>(),
                           g.data_ptr<float>(), h.data_ptr<float>(), bins.data_ptr<int>(),
                           offs.data_ptr<int>(), (int)codes.size(0), (int)total_bins, (int)n_nodes,
                           even_only ? 1 : 0, (int)tot_slot, (float)scale,
                           reinterpret_cast<long long*>(out.data_ptr<int64_t>()), cur_stream(codes));
}

// K25 re-sampling (resample.hip)
at::Tensor resample_uniform(int64_t seed, int64_t stream, int64_t base, int64_t n, const at::Tensor& like) {
  CHECK_DEV(like);
  TORCH_CHECK(n >= 0 && base >= 0, "bad range");
  auto out = at::empty({n}, like.options().dtype(at::kFloat));
  DevGuard gd(like.device());
  avk::resample_uniform((unsigned long long)seed, (unsigned long long)stream, base, n, out.data_ptr<float>(),
                        cur_stream(like));
  return out;
}

std::vector<at::Tensor> smote(const at::Tensor& X, const at::Tensor& Xn, const at::Tensor& nn,
                              const c10::optional<at::Tensor>& Cs, const c10::optional<at::Tensor>& Cn, int64_t mult,
                              int64_t gbase, int64_t seed, bool exponential, double exp_mean) {
  CHECK_DEV(X); CHECK_DTYPE(X, at::kFloat);
  CHECK_DEV(Xn); CHECK_DTYPE(Xn, at::kFloat);
  CHECK_DEV(nn); CHECK_DTYPE(nn, at::kInt);
  TORCH_CHECK(X.dim() == 2 && Xn.dim() == 3 && X.is_contiguous() && Xn.is_contiguous() && nn.is_contiguous(),
              "X [m, D], Xn [m, k, D] contiguous");
  const int64_t m = X.size(0), D = X.size(1), k = Xn.size(1);
  TORCH_CHECK(Xn.size(0) == m && Xn.size(2) == D && nn.numel() == m && mult >= 0 && k >= 1, "shape mismatch");
  TORCH_CHECK(m * std::max<int64_t>(mult, 1) < (1LL << 40), "too many synthetic rows");
  // every neighbour count must be <= k (the kernel indexes Xn[r, pick < nn[r]])
  if (m) TORCH_CHECK(nn.max().item<int>() <= k && nn.min().item<int>() >= 0, "neighbour counts must be in [0, k]");
  int64_t Dc = 0;
  const int* cs = nullptr;
  const int* cn = nullptr;
  if (Cs.has_value() && Cs->defined()) {
    TORCH_CHECK(Cn.has_value() && Cn->defined(), "categorical neighbours missing");
    CHECK_DEV((*Cs)); CHECK_DTYPE((*Cs), at::kInt);
    CHECK_DEV((*Cn)); CHECK_DTYPE((*Cn), at::kInt);
    Dc = Cs->size(1);
    TORCH_CHECK(Cs->dim() == 2 && Cs->size(0) == m && Cn->dim() == 3 && Cn->size(0) == m && Cn->size(1) == k &&
                Cn->size(2) == Dc && Cs->is_contiguous() && Cn->is_contiguous(), "Cs [m, Dc], Cn [m, k, Dc]");
    cs = Cs->data_ptr<int>();
    cn = Cn->data_ptr<int>();
  }
  auto outX = at::empty({m * mult, D}, X.options());
  auto outC = at::empty({m * mult, Dc}, X.options().dtype(at::kInt));
  auto pick = at::empty({m * mult}, X.options().dtype(at::kInt));
  DevGuard gd(X.device());
  avk::smote(X.data_ptr<float>(), Xn.data_ptr<float>(), nn.data_ptr<int>(), cs, cn, m, (int)k, (int)D, (int)Dc,
             (int)mult, gbase, (unsigned long long)seed, exponential ? 1 : 0, (float)exp_mean, outX.data_ptr<float>(),
             Dc ? outC.data_ptr<int>() : nullptr, pick.data_ptr<int>(), cur_stream(X));
  return {outX, outC, pick};
}

// Device GBT round pieces (gbt.hip).  F: [ld, K] float32 raw scores (row-major), y uint8 labels.
void gbt_grad(const at::Tensor& F, int64_t k, const at::Tensor& y, int64_t n, int64_t row_off, int64_t seed,
              int64_t rate32, at::Tensor& g, at::Tensor& h, const c10::optional<at::Tensor>& loss) {
  CHECK_DEV(F); CHECK_DTYPE(F, at::kFloat);
  CHECK_DEV(y); CHECK_DTYPE(y, at::kByte);
  CHECK_DEV(g); CHECK_DTYPE(g, at::kFloat);
  CHECK_DEV(h); CHECK_DTYPE(h, at::kFloat);
  TORCH_CHECK(F.dim() == 2 && F.is_contiguous() && F.size(0) >= n, "F must be a contiguous [>= n, K] tensor");
  const int64_t K = F.size(1);
  TORCH_CHECK(k >= 0 && k < K && K >= 1 && K <= 255, "bad class index");
  TORCH_CHECK(y.numel() >= n && g.numel() >= n && h.numel() >= n, "y / g / h shorter than n");
  TORCH_CHECK(rate32 >= 0 && rate32 <= 0xFFFFFFFFLL, "rate32 is a uint32");
  double* lp = nullptr;
  if (loss.has_value() && loss->defined()) {
    CHECK_DEV((*loss)); CHECK_DTYPE((*loss), at::kDouble);
    TORCH_CHECK(loss->numel() >= 1, "loss slot");
    lp = loss->data_ptr<double>();
  }
  DevGuard gd(F.device());
  avk::gbt_grad(F.data_ptr<float>(), (int)K, (int)k, y.data_ptr<uint8_t>(), n, row_off, (unsigned long long)seed,
                (unsigned)rate32, g.data_ptr<float>(), h.data_ptr<float>(), lp, cur_stream(F));
}

void gbt_assign(const at::Tensor& codes, int64_t n, at::Tensor& node, const at::Tensor& feat, const at::Tensor& thr,
                const at::Tensor& value, const at::Tensor& bins, int64_t level, bool last, double lr, at::Tensor& F,
                int64_t k) {
  check_codes(codes, n);
  CHECK_DEV(node); CHECK_DTYPE(node, at::kInt);
  CHECK_DEV(feat); CHECK_DTYPE(feat, at::kInt);
  CHECK_DEV(thr); CHECK_DTYPE(thr, at::kInt);
  CHECK_DEV(value); CHECK_DTYPE(value, at::kDouble);
  CHECK_DEV(bins); CHECK_DTYPE(bins, at::kInt);
  CHECK_DEV(F); CHECK_DTYPE(F, at::kFloat);
  TORCH_CHECK(level >= 0 && level < 24, "level out of range");
  const int64_t H = (2LL << level) - 1 + (2LL << level);   // heap entries up to the next level
  TORCH_CHECK(feat.numel() >= H && thr.numel() >= H && value.numel() >= H, "heap arrays too short for the level");
  TORCH_CHECK(node.numel() >= n && F.dim() == 2 && F.is_contiguous() && F.size(0) >= n, "node / F shapes");
  TORCH_CHECK(k >= 0 && k < F.size(1), "bad class index");
  TORCH_CHECK(bins.numel() >= codes.size(0) - 1, "bins per feature");
  DevGuard gd(codes.device());
  avk::gbt_assign(codes.data_ptr<uint8_t>(), codes.size(1), n, node.data_ptr<int>(), feat.data_ptr<int>(),
                  thr.data_ptr<int>(), value.data_ptr<double>(), bins.data_ptr<int>(), (int)level, last ? 1 : 0,
                  (float)lr, F.data_ptr<float>(), (int)F.size(1), (int)k, cur_stream(codes));
}

// One GBT level's split scoring (gbt.hip gbt_split_kernel).  Either `hist` [A, TB, 2] int64, or
// `parent` / `left` [A / 2, TB, 2] (sibling subtraction); `out_hist` [A, TB, 2] or None receives the
// level's histogram.  Scan tables: int32 [nb] (pvalid uint8).  Heap arrays feat / thr int32, val f64.
void gbt_split(const c10::optional<at::Tensor>& hist, const c10::optional<at::Tensor>& parent,
               const c10::optional<at::Tensor>& left, const c10::optional<at::Tensor>& out_hist, int64_t A,
               int64_t tot, const at::Tensor& pfeat, const at::Tensor& pthr, const at::Tensor& pstart,
               const at::Tensor& pend, const at::Tensor& pvalid, double l2, double scale, int64_t level,
               at::Tensor& feat, at::Tensor& thr, at::Tensor& val) {
  const bool has_h = hist.has_value() && hist->defined();
  const at::Tensor& ref = has_h ? *hist : *left;
  TORCH_CHECK(has_h || (parent.has_value() && parent->defined() && left.has_value() && left->defined()),
              "gbt_split: hist, or parent + left");
  CHECK_DEV(ref);
  CHECK_DTYPE(ref, at::kLong);
  TORCH_CHECK(ref.dim() == 3 && ref.size(2) == 2 && ref.is_contiguous(), "histograms must be [nodes, TB, 2]");
  const int64_t TB = ref.size(1);
  if (has_h) {
    TORCH_CHECK(hist->size(0) == A, "hist must have A nodes");
  } else {
    TORCH_CHECK(A % 2 == 0 && left->size(0) == A / 2 && parent->sizes() == left->sizes() && parent->is_contiguous() &&
                    parent->scalar_type() == at::kLong,
                "parent / left must be [A / 2, TB, 2] int64");
  }
  long long* oh = nullptr;
  if (out_hist.has_value() && out_hist->defined()) {
    TORCH_CHECK(out_hist->scalar_type() == at::kLong && out_hist->is_contiguous() && out_hist->size(0) == A &&
                    out_hist->size(1) == TB && out_hist->size(2) == 2,
                "out_hist must be [A, TB, 2] int64");
    oh = reinterpret_cast<long long*>(out_hist->data_ptr<int64_t>());
  }
  const int64_t nb = pfeat.numel();
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&pfeat, &pthr, &pstart, &pend}) {
    CHECK_DEV((*t));
    CHECK_DTYPE((*t), at::kInt);
    TORCH_CHECK(t->numel() == nb, "scan tables must have nb entries");
  }
  CHECK_DTYPE(pvalid, at::kByte);
  TORCH_CHECK(pvalid.numel() == nb && nb < TB && tot >= 0 && tot < TB, "scan tables / total bin");
  // (no host read-back of the scan tables: this runs inside captured graphs; the kernel clamps
  // every table-derived index into [p, nb))
  CHECK_DTYPE(feat, at::kInt);
  CHECK_DTYPE(thr, at::kInt);
  CHECK_DTYPE(val, at::kDouble);
  TORCH_CHECK(level >= 0 && level < 24 && A == (1LL << level), "A must be 2^level");
  const int64_t hb = A - 1, hc = 2 * A - 1;
  TORCH_CHECK(feat.numel() >= hc && thr.numel() >= hc && val.numel() >= hc + 2 * A, "heap arrays too short");
  DevGuard gd(ref.device());
  using ll = const long long*;
  avk::gbt_split(has_h ? reinterpret_cast<ll>(hist->data_ptr<int64_t>()) : nullptr,
                 has_h ? nullptr : reinterpret_cast<ll>(parent->data_ptr<int64_t>()),
                 has_h ? nullptr : reinterpret_cast<ll>(left->data_ptr<int64_t>()), oh, (int)A, (int)TB, (int)tot, pfeat.data_ptr<int>(),
                 pthr.data_ptr<int>(), pstart.data_ptr<int>(), pend.data_ptr<int>(), pvalid.data_ptr<uint8_t>(),
                 (int)nb, l2, 1.0 / scale, (int)hb, (int)hc, level == 0 ? 1 : 0, feat.data_ptr<int>(),
                 thr.data_ptr<int>(), val.data_ptr<double>(), cur_stream(ref));
}

// K26 rank statistics (stats.hip).  sorted / perm: torch.sort of the sample (ascending);
// group int32 [n] (original order) or None.  Returns (ranks f64 [n], tie terms f64 [4], group rank
// sums f64 [n_groups]).
py::tuple rank_avg(const at::Tensor& sorted, const at::Tensor& perm, const c10::optional<at::Tensor>& group,
                   int64_t n_groups) {
  CHECK_DEV(sorted);
  CHECK_DTYPE(sorted, at::kDouble);
  CHECK_DEV(perm);
  CHECK_DTYPE(perm, at::kLong);
  TORCH_CHECK(sorted.dim() == 1 && sorted.is_contiguous() && perm.sizes() == sorted.sizes() && perm.is_contiguous(),
              "sorted / perm must be contiguous [n]");
  const int64_t n = sorted.numel();
  const int* gp = nullptr;
  if (group.has_value() && group->defined()) {
    CHECK_DEV((*group));
    CHECK_DTYPE((*group), at::kInt);
    TORCH_CHECK(group->numel() == n && group->is_contiguous(), "group must be [n]");
    TORCH_CHECK(n_groups >= 1 && n_groups < (1 << 20), "n_groups in [1, 2^20)");
    gp = group->data_ptr<int>();
  }
  auto o = sorted.options();
  auto ranks = at::empty({n}, o), tie = at::zeros({4}, o), gsum = at::zeros({std::max<int64_t>(n_groups, 1)}, o);
  DevGuard gd(sorted.device());
  avk::rank_avg(sorted.data_ptr<double>(), reinterpret_cast<const long long*>(perm.data_ptr<int64_t>()), n, gp,
                (int)n_groups, ranks.data_ptr<double>(), tie.data_ptr<double>(), gsum.data_ptr<double>(),
                cur_stream(sorted));
  return py::make_tuple(ranks, tie, gsum);
}

// Kendall pair counts of (x, y) f64 [n]: int64 [5] = concordant, discordant, x-only ties, y-only
// ties, ties in both.
at::Tensor kendall_pairs(const at::Tensor& x, const at::Tensor& y) {
  CHECK_DEV(x);
  CHECK_DTYPE(x, at::kDouble);
  CHECK_DEV(y);
  CHECK_DTYPE(y, at::kDouble);
  TORCH_CHECK(x.dim() == 1 && x.is_contiguous() && y.sizes() == x.sizes() && y.is_contiguous(), "x, y must be [n]");
  TORCH_CHECK(x.numel() <= (1LL << 24), "kendall_pairs: n <= 2^24");
  auto out = at::zeros({5}, x.options().dtype(at::kLong));
  DevGuard gd(x.device());
  avk::kendall_pairs(x.data_ptr<double>(), y.data_ptr<double>(), x.numel(),
                     reinterpret_cast<unsigned long long*>(out.data_ptr<int64_t>()), cur_stream(x));
  return out;
}

// Strict inversions of y f64 [n] (Knight's Kendall discordant count when y is ordered by (x, y)):
// int64 [1] on the device, no host synchronisation.
at::Tensor inversion_count(const at::Tensor& y) {
  CHECK_DEV(y);
  CHECK_DTYPE(y, at::kDouble);
  TORCH_CHECK(y.dim() == 1, "y must be [n]");
  DevGuard gd(y.device());
  const int64_t n = y.numel();
  auto out = at::zeros({1}, y.options().dtype(at::kLong));
  if (n <= 1) return out;
  int64_t m = avk::inv_merge_block();
  while (m < n) m <<= 1;
  auto a = at::full({m}, std::numeric_limits<double>::infinity(), y.options());
  a.narrow(0, 0, n).copy_(y);
  auto tmp = at::empty({m}, y.options());
  avk::inversions(a.data_ptr<double>(), tmp.data_ptr<double>(), m,
                  reinterpret_cast<unsigned long long*>(out.data_ptr<int64_t>()), cur_stream(y));
  return out;
}

// Mixed-type kNN (distance.hip): Qn [nq, Dn] / Rn [nr, Dn] f32 scaled numerics, Qc / Rc int32 codes
// (-1 = missing), wc f32 [Dc].  Returns (dist f32 [nq, k], idx int64 [nq, k]).
py::tuple mixed_knn(const at::Tensor& Qn, const at::Tensor& Qc, const at::Tensor& Rn, const at::Tensor& Rc,
                    const at::Tensor& wc, int64_t k, int64_t r_base) {
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&Qn, &Rn, &wc}) {
    CHECK_DEV((*t));
    CHECK_DTYPE((*t), at::kFloat);
    TORCH_CHECK(t->is_contiguous(), "contiguous tensors required");
  }
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&Qc, &Rc}) {
    CHECK_DEV((*t));
    CHECK_DTYPE((*t), at::kInt);
    TORCH_CHECK(t->is_contiguous(), "contiguous tensors required");
  }
  TORCH_CHECK(Qn.dim() == 2 && Rn.dim() == 2 && Qc.dim() == 2 && Rc.dim() == 2, "2-D inputs");
  const int64_t nq = Qn.size(0), nr = Rn.size(0), Dn = Qn.size(1), Dc = Qc.size(1);
  TORCH_CHECK(Qc.size(0) == nq && Rc.size(0) == nr && Rn.size(1) == Dn && Rc.size(1) == Dc && wc.numel() == Dc,
              "shape mismatch");
  TORCH_CHECK(Dn <= avk::mixed_knn_max_dims() && Dc <= avk::mixed_knn_max_dims() && k >= 1 && k <= 32,
              "mixed_knn: <= 32 numeric and <= 32 categorical columns, 1 <= k <= 32");
  TORCH_CHECK(nr < (1LL << 31), "too many reference rows");
  auto d = at::empty({nq, k}, Qn.options());
  auto i = at::empty({nq, k}, Qn.options().dtype(at::kLong));
  DevGuard gd(Qn.device());
  const int splits = avk::mixed_knn_splits(nq, nr);
  const int64_t KK = k <= 4 ? 4 : k <= 8 ? 8 : k <= 16 ? 16 : 32;
  auto pd = at::empty({splits, nq, KK}, Qn.options());
  auto pi = at::empty({splits, nq, KK}, Qn.options().dtype(at::kInt));
  avk::mixed_knn(Qn.data_ptr<float>(), Qc.data_ptr<int>(), nq, Rn.data_ptr<float>(), Rc.data_ptr<int>(), nr, (int)Dn,
                 (int)Dc, wc.data_ptr<float>(), (int)k, r_base, d.data_ptr<float>(),
                 reinterpret_cast<long long*>(i.data_ptr<int64_t>()), pd.data_ptr<float>(), pi.data_ptr<int>(), splits,
                 cur_stream(Qn));
  return py::make_tuple(d, i);
}

// K28 text kernels (text.hip)
// K28 TF-IDF (text.hip): val (float counts, contiguous) is weighted and normalised in place;
// returns the document frequencies.  Index checks run on the device; one status read per call.
at::Tensor tfidf_csr(const at::Tensor& crow, const at::Tensor& col, at::Tensor& val, int64_t V, bool smooth,
                     bool sublinear, int64_t norm) {
  CHECK_DEV(crow); CHECK_DTYPE(crow, at::kLong);
  CHECK_DEV(col); CHECK_DTYPE(col, at::kLong);
  CHECK_DEV(val); CHECK_DTYPE(val, at::kFloat);
  TORCH_CHECK(crow.dim() == 1 && crow.numel() >= 1 && col.numel() == val.numel() && val.is_contiguous() &&
                  col.is_contiguous() && crow.is_contiguous(), "CSR arrays");
  TORCH_CHECK(norm >= 0 && norm <= 2, "norm: 0 none, 1 l1, 2 l2");
  TORCH_CHECK(V >= 1, "vocabulary size >= 1");
  DevGuard gd(val.device());
  auto df = at::zeros({V}, val.options().dtype(at::kInt));
  auto status = at::zeros({1}, val.options().dtype(at::kInt));
  avk::tfidf_csr(reinterpret_cast<const long long*>(crow.data_ptr<int64_t>()),
                 reinterpret_cast<const long long*>(col.data_ptr<int64_t>()), val.data_ptr<float>(),
                 crow.numel() - 1, col.numel(), V, smooth ? 1 : 0, sublinear ? 1 : 0, (int)norm,
                 df.data_ptr<int>(), status.data_ptr<int>(), cur_stream(val));
  const int st = status.item<int>();
  TORCH_CHECK(!(st & 1), "tfidf: column id out of range [0, ", V, ")");
  TORCH_CHECK(!(st & 2), "tfidf: row pointers must be monotone within [0, nnz]");
  return df;
}

py::tuple pagerank(const at::Tensor& P, double d, int64_t iters, double tol) {
  CHECK_DEV(P);
  CHECK_DTYPE(P, at::kDouble);
  TORCH_CHECK(P.dim() == 2 && P.size(0) == P.size(1) && P.is_contiguous(), "P must be contiguous [n, n]");
  TORCH_CHECK(P.size(0) <= avk::pagerank_max_n(), "pagerank: n <= ", avk::pagerank_max_n());
  const int n = (int)P.size(0);
  auto r = at::empty({n}, P.options());
  auto it = at::zeros({1}, P.options().dtype(at::kInt));
  DevGuard gd(P.device());
  avk::pagerank(P.data_ptr<double>(), n, d, (int)iters, tol, r.data_ptr<double>(), it.data_ptr<int>(), cur_stream(P));
  return py::make_tuple(r, it);
}

// Weighted pagerank for any n on several workgroups per iteration (no host sync per iteration):
// (r [n], iterations [1]).
py::tuple pagerank_multi(const at::Tensor& P, double d, int64_t iters, double tol) {
  CHECK_DEV(P);
  CHECK_DTYPE(P, at::kDouble);
  TORCH_CHECK(P.dim() == 2 && P.size(0) == P.size(1) && P.is_contiguous(), "P must be contiguous [n, n]");
  TORCH_CHECK(P.size(0) < (1LL << 31) && iters >= 0 && iters < (1LL << 30), "pagerank: n < 2^31");
  const int64_t n = P.size(0);
  DevGuard gd(P.device());
  auto buf = at::empty({2, n}, P.options());
  buf[0].fill_(1.0 / (double)std::max<int64_t>(n, 1));
  auto partial = at::empty({(n + avk::pagerank_multi_rows() - 1) / avk::pagerank_multi_rows(), n}, P.options());
  auto dpart = at::empty({(n + 255) / 256}, P.options());
  auto state = at::zeros({2}, P.options().dtype(at::kInt));
  // batches of 8 iterations, one host read of the flag per batch: a converged run stops enqueueing
  // (the early-exit launches of a whole up-front enqueue cost more than the work at small n)
  auto state_h = at::empty({2}, at::TensorOptions().dtype(at::kInt).pinned_memory(true));
  int it = 0;
  for (int64_t k0 = 0; k0 < iters; k0 += 8) {
    const int64_t k1 = std::min<int64_t>(iters, k0 + 8);
    avk::pagerank_multi(P.data_ptr<double>(), (int)n, d, (int)k0, (int)k1, tol, buf.data_ptr<double>(),
                        partial.data_ptr<double>(), dpart.data_ptr<double>(), state.data_ptr<int>(), cur_stream(P));
    state_h.copy_(state);
    it = state_h[1].item<int>();
    if (state_h[0].item<int>()) break;
  }
  return py::make_tuple(buf[it & 1].clone(), state.narrow(0, 1, 1).clone());
}

// One SGNS mini-batch: gradients of every pair into gIn / gOut (+ per-row counts cIn / cOut), then
// the rows move by their mean update (gIn for the centre table summed when mean_in is false).
// The caller checks id ranges once per fit (pairs / alias are built from the vocabulary).
void sgns_step(at::Tensor& Win, at::Tensor& Wout, at::Tensor& gIn, at::Tensor& gOut, at::Tensor& cIn, at::Tensor& cOut,
               const at::Tensor& centre, const at::Tensor& context, const at::Tensor& aprob, const at::Tensor& alias,
               int64_t neg, double lr, bool mean_in, int64_t seed, int64_t step, const c10::optional<at::Tensor>& hot,
               const c10::optional<at::Tensor>& gOutHot, const c10::optional<at::Tensor>& gInHot,
               const c10::optional<at::Tensor>& cIn_next, const c10::optional<at::Tensor>& cOut_next) {
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&Win, &Wout, &gIn, &gOut, &cIn, &cOut, &aprob}) {
    CHECK_DEV((*t));
    CHECK_DTYPE((*t), at::kFloat);
    TORCH_CHECK(t->is_contiguous(), "contiguous tensors required");
  }
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&centre, &context, &alias}) {
    CHECK_DEV((*t));
    CHECK_DTYPE((*t), at::kInt);
    TORCH_CHECK(t->is_contiguous(), "contiguous tensors required");
  }
  TORCH_CHECK(Win.dim() == 2 && Wout.dim() == 2 && Win.size(1) == Wout.size(1), "Win [Rin, d], Wout [V, d]");
  const int64_t V = Wout.size(0), dim = Win.size(1), R = avk::sgns_hot_replicas();
  // hot rows: hot int32 [V] (slot in [0, H) or -1), gOutHot [R, H, d]; gInHot [R, H, d] or None (the
  // centre table shares the word ids: word2vec); the counts carry R x H extra entries after the rows
  int64_t H = 0;
  if (hot) {
    CHECK_DEV((*hot));
    CHECK_DTYPE((*hot), at::kInt);
    TORCH_CHECK(hot->numel() == V && gOutHot && gOutHot->dim() == 3 && gOutHot->size(0) == R &&
                    gOutHot->size(2) == dim && gOutHot->is_contiguous(), "hot [V], gOutHot [R, H, d]");
    CHECK_DTYPE((*gOutHot), at::kFloat);
    H = gOutHot->size(1);  // slots outside [0, H) are treated as cold by the kernels (no host sync here)
    if (gInHot) {
      CHECK_DTYPE((*gInHot), at::kFloat);
      TORCH_CHECK(gInHot->sizes() == gOutHot->sizes() && gInHot->is_contiguous() && Win.size(0) == V,
                  "gInHot like gOutHot, centre table over the same ids");
    }
  }
  const int64_t extra_in = (hot && gInHot) ? R * H : 0, extra_out = hot ? R * H : 0;
  // ping-pong counts: the buffers of the next batch, cleared by this batch's apply pass
  const at::Tensor* cin_n = cIn_next ? &*cIn_next : nullptr;
  const at::Tensor* cout_n = cOut_next ? &*cOut_next : nullptr;
  for (const at::Tensor* t : {cin_n, cout_n})
    if (t) {
      CHECK_DEV((*t));
      CHECK_DTYPE((*t), at::kFloat);
      TORCH_CHECK(t->is_contiguous(), "contiguous tensors required");
    }
  TORCH_CHECK((!cin_n || cin_n->numel() == cIn.numel()) && (!cout_n || cout_n->numel() == cOut.numel()),
              "next count buffers must match the current ones");
  TORCH_CHECK(gIn.sizes() == Win.sizes() && gOut.sizes() == Wout.sizes() && cIn.numel() == Win.size(0) + extra_in &&
                  cOut.numel() == Wout.size(0) + extra_out, "gradient / count buffers must match the tables");
  TORCH_CHECK(aprob.numel() == V && alias.numel() == V, "alias table must have V entries");
  TORCH_CHECK(centre.numel() == context.numel(), "centre / context lengths");
  TORCH_CHECK(neg >= 0 && neg <= 64, "0 <= neg <= 64");
  DevGuard gd(Win.device());
  avk::sgns_step(Win.data_ptr<float>(), Wout.data_ptr<float>(), gIn.data_ptr<float>(), gOut.data_ptr<float>(),
                 cIn.data_ptr<float>(), cOut.data_ptr<float>(), (int)dim, Win.size(0), centre.data_ptr<int>(),
                 context.data_ptr<int>(), centre.numel(), aprob.data_ptr<float>(), alias.data_ptr<int>(), (int)V,
                 (int)neg, (float)lr, mean_in ? 1 : 0, (unsigned long long)seed, (unsigned long long)step,
                 hot ? hot->data_ptr<int>() : nullptr, (int)H, hot ? gOutHot->data_ptr<float>() : nullptr,
                 (hot && gInHot) ? gInHot->data_ptr<float>() : nullptr, cin_n ? cin_n->data_ptr<float>() : nullptr,
                 cin_n ? cin_n->numel() : 0, cout_n ? cout_n->data_ptr<float>() : nullptr, cout_n ? cout_n->numel() : 0,
                 cur_stream(Win));
}

void tree_assign(const at::Tensor& codes, int64_t n, at::Tensor& node, const at::Tensor& split_feat,
                 const at::Tensor& segmap, const at::Tensor& child_of) {
  check_codes(codes, n);
  CHECK_DEV(node);
  CHECK_DTYPE(node, at::kInt);
  TORCH_CHECK(node.numel() >= n, "node too short");
  CHECK_DEV(split_feat);
  CHECK_DTYPE(split_feat, at::kInt);
  CHECK_DEV(segmap);
  CHECK_DTYPE(segmap, at::kShort);
  CHECK_DEV(child_of);
  CHECK_DTYPE(child_of, at::kInt);
  const int64_t A = split_feat.numel();
  TORCH_CHECK(segmap.dim() == 2 && segmap.size(0) == A, "segmap must be [A, max_bins]");
  TORCH_CHECK(child_of.dim() == 2 && child_of.size(0) == A, "child_of must be [A, max_seg]");
  auto sf = split_feat.cpu();
  for (int64_t a = 0; a < A; ++a)
    TORCH_CHECK(sf.data_ptr<int>()[a] < codes.size(0), "split feature out of range");
  DevGuard g(codes.device());
  avk::tree_assign(codes.data_ptr<uint8_t>(), codes.size(1), n, node.data_ptr<int>(),
                   split_feat.data_ptr<int>(), segmap.data_ptr<int16_t>(), (int)segmap.size(1),
                   child_of.data_ptr<int>(), (int)child_of.size(1), cur_stream(codes));
}

void tree_predict(const at::Tensor& codes, int64_t n, const at::Tensor& feat, const at::Tensor& seg_base,
                  const at::Tensor& segmap, const at::Tensor& child_base, const at::Tensor& child,
                  const at::Tensor& leaf_idx, const at::Tensor& values, const at::Tensor& tree_root,
                  const c10::optional<at::Tensor>& tree_w, int64_t mode, at::Tensor& out) {
  check_codes(codes, n);
  for (const at::Tensor* t : {&feat, &seg_base, &child_base, &child, &leaf_idx, &tree_root}) {
    CHECK_DEV((*t));
    CHECK_DTYPE((*t), at::kInt);
  }
  CHECK_DEV(segmap);
  CHECK_DTYPE(segmap, at::kShort);
  CHECK_DEV(values);
  CHECK_DTYPE(values, at::kFloat);
  CHECK_DEV(out);
  CHECK_DTYPE(out, at::kFloat);
  TORCH_CHECK(values.dim() == 2, "values must be [L, V]");
  const int V = (int)values.size(1);
  TORCH_CHECK(out.numel() >= n * V, "out too short");
  const int K = (int)feat.numel();
  TORCH_CHECK(seg_base.numel() == K && child_base.numel() == K && leaf_idx.numel() == K,
              "node arrays must have equal length");
  // host-side structural validation (the kernel trusts these indices)
  auto fc = feat.cpu(), sc = seg_base.cpu(), cb = child_base.cpu(), lc = leaf_idx.cpu(), ch = child.cpu(),
       tr = tree_root.cpu();
  for (int k = 0; k < K; ++k) {
    const int f = fc.data_ptr<int>()[k];
    TORCH_CHECK(f < codes.size(0), "tree feature out of range");
    TORCH_CHECK(lc.data_ptr<int>()[k] >= 0 && lc.data_ptr<int>()[k] < values.size(0), "leaf idx range");
    if (f >= 0) {
      TORCH_CHECK(sc.data_ptr<int>()[k] >= 0 && sc.data_ptr<int>()[k] < segmap.size(0), "seg_base range");
      TORCH_CHECK(cb.data_ptr<int>()[k] >= 0 && cb.data_ptr<int>()[k] < ch.numel(), "child_base range");
    }
  }
  for (int64_t i = 0; i < ch.numel(); ++i) TORCH_CHECK(ch.data_ptr<int>()[i] < K, "child index range");
  for (int64_t i = 0; i < tr.numel(); ++i)
    TORCH_CHECK(tr.data_ptr<int>()[i] >= 0 && tr.data_ptr<int>()[i] < K, "tree root range");
  const float* tw = nullptr;
  if (tree_w.has_value() && tree_w->defined()) {
    CHECK_DEV((*tree_w));
    TORCH_CHECK(tree_w->numel() == tree_root.numel(), "tree_w length");
    tw = tree_w->data_ptr<float>();
  }
  DevGuard g(codes.device());
  avk::tree_predict(codes.data_ptr<uint8_t>(), codes.size(1), n, feat.data_ptr<int>(),
                    seg_base.data_ptr<int>(), segmap.data_ptr<int16_t>(), (int)segmap.size(1),
                    child_base.data_ptr<int>(), child.data_ptr<int>(), leaf_idx.data_ptr<int>(),
                    values.data_ptr<float>(), V, tree_root.data_ptr<int>(), tw, (int)tree_root.numel(),
                    (int)mode, out.data_ptr<float>(), cur_stream(codes));
}

// Binary-split forest inference from LDS (forest_predict_bin_kernel).  nodes int32 [K, 2] packed
// records (see tree.hip); validated on the host: feature / child ranges, leaves marked 255.
void forest_predict_bin(const at::Tensor& codes, int64_t n, const at::Tensor& nodes, const at::Tensor& values,
                        const at::Tensor& tree_root, const c10::optional<at::Tensor>& tree_w, int64_t mode,
                        at::Tensor& out) {
  check_codes(codes, n);
  CHECK_DEV(nodes); CHECK_DTYPE(nodes, at::kInt);
  CHECK_DEV(values); CHECK_DTYPE(values, at::kFloat);
  CHECK_DEV(tree_root); CHECK_DTYPE(tree_root, at::kInt);
  CHECK_DEV(out); CHECK_DTYPE(out, at::kFloat);
  TORCH_CHECK(nodes.dim() == 2 && nodes.size(1) == 2 && nodes.is_contiguous(), "nodes [K, 2] int32");
  const int64_t K = nodes.size(0);
  TORCH_CHECK(K > 0 && K <= 65535 && values.dim() == 2 && values.size(0) == K, "values [K, V], K <= 65535");
  const int V = (int)values.size(1);
  TORCH_CHECK(V >= 1 && V <= 8 && out.numel() >= n * V, "1..8 outputs per row");
  const int F = (int)codes.size(0);
  TORCH_CHECK(F <= 255, "at most 255 features");
  TORCH_CHECK(avk::forest_predict_bin_lds((int)K, F) <= 160 * 1024, "forest too large for the LDS kernel");
  auto nc = nodes.cpu(), rc = tree_root.cpu();
  const int* nd = nc.data_ptr<int>();
  for (int64_t k = 0; k < K; ++k) {
    const unsigned x = (unsigned)nd[2 * k], y = (unsigned)nd[2 * k + 1];
    const unsigned f = x & 0xFF;
    if (f == 0xFF) continue;
    TORCH_CHECK((int)f < F && (y & 0xFFFF) < K && (y >> 16) < K, "forest node out of range");
  }
  for (int64_t t = 0; t < rc.numel(); ++t)
    TORCH_CHECK(rc.data_ptr<int>()[t] >= 0 && rc.data_ptr<int>()[t] < K, "tree root out of range");
  const float* tw = nullptr;
  if (tree_w.has_value() && tree_w->defined()) {
    CHECK_DEV((*tree_w)); CHECK_DTYPE((*tree_w), at::kFloat);
    TORCH_CHECK(tree_w->numel() == tree_root.numel(), "one weight per tree");
    tw = tree_w->data_ptr<float>();
  }
  auto vc = values.contiguous();
  DevGuard g(codes.device());
  avk::forest_predict_bin(codes.data_ptr<uint8_t>(), codes.size(1), n, F,
                          reinterpret_cast<const uint2*>(nodes.data_ptr<int>()), (int)K, vc.data_ptr<float>(), V,
                          tree_root.data_ptr<int>(), tw, (int)tree_root.numel(), (int)mode, out.data_ptr<float>(),
                          cur_stream(codes));
}

// ---------------------------------------------------------------------------------------------
// distance / kNN / clustering (K9/K11)
// ---------------------------------------------------------------------------------------------
py::tuple knn_topk(const at::Tensor& Q, const at::Tensor& R, int64_t k, int64_t q_base, int64_t r_base,
                   bool exclude_self, int64_t splits, int64_t metric, double p, int64_t prec) {
  CHECK_DEV(Q);
  CHECK_DTYPE(Q, at::kFloat);
  CHECK_DEV(R);
  CHECK_DTYPE(R, at::kFloat);
  TORCH_CHECK(Q.dim() == 2 && R.dim() == 2 && Q.size(1) == R.size(1), "Q [M,D], R [N,D] required");
  TORCH_CHECK(k >= 1 && k <= 64, "k must be in [1,64]");
  TORCH_CHECK(metric >= 0 && metric <= 2 && (metric != 2 || p > 0), "metric 0 (sq euclidean), 1 (L1), 2 (Lp, p > 0)");
  const int64_t M = Q.size(0), N = R.size(0), D = Q.size(1);
  TORCH_CHECK(D >= 1, "D must be >= 1");
  if (splits <= 0) {
    const int64_t qb = (M + 63) / 64;
    splits = std::max<int64_t>(1, std::min<int64_t>((N + 63) / 64, (2048 + qb - 1) / qb));
  }
  auto od = at::empty({splits, M, k}, Q.options());
  auto oi = at::empty({splits, M, k}, Q.options().dtype(at::kLong));
  DevGuard g(Q.device());
  avk::knn_topk(Q.data_ptr<float>(), M, R.data_ptr<float>(), N, (int)D, (int)k, q_base, r_base,
                exclude_self ? 1 : 0, od.data_ptr<float>(), reinterpret_cast<long long*>(oi.data_ptr<int64_t>()),
                (int)splits, (int)metric, (float)p, cur_stream(Q), (int)prec);
  return py::make_tuple(od, oi, splits);
}


py::tuple knn_vote(const at::Tensor& d, const at::Tensor& idx, const at::Tensor& ys,
                   const c10::optional<at::Tensor>& post, int64_t C, int64_t kern, double kparam, double scale,
                   double kscale, bool invdist, double thr, int64_t pos) {
  CHECK_DEV(d);
  CHECK_DTYPE(d, at::kFloat);
  CHECK_DEV(idx);
  CHECK_DTYPE(idx, at::kLong);
  CHECK_DEV(ys);
  CHECK_DTYPE(ys, at::kLong);
  TORCH_CHECK(d.dim() == 2 && idx.sizes() == d.sizes() && d.is_contiguous() && idx.is_contiguous(),
              "d / idx must be contiguous [M, k]");
  TORCH_CHECK(ys.dim() == 1 && ys.is_contiguous(), "ys must be contiguous [R]");
  TORCH_CHECK(C >= 1 && C <= 64, "knn_vote: 1 <= C <= 64");
  TORCH_CHECK(kern >= 0 && kern <= 3, "kern 0 none, 1 linearMultiplicative, 2 linearAdditive, 3 gaussian");
  int post_mode = 0;
  const float* pp = nullptr;
  if (post.has_value() && post->defined()) {
    CHECK_DEV((*post));
    CHECK_DTYPE((*post), at::kFloat);
    TORCH_CHECK(post->is_contiguous() && post->size(0) == ys.size(0) &&
                (post->dim() == 1 || (post->dim() == 2 && post->size(1) == C)), "post must be [R] or [R, C]");
    post_mode = post->dim() == 1 ? 1 : 2;
    pp = post->data_ptr<float>();
  }
  // every neighbour index must address ys / post (the kernel reads them unchecked)
  const int64_t M = d.size(0), k = d.size(1);
  if (M > 0 && k > 0) {
    TORCH_CHECK(idx.max().item<int64_t>() < ys.size(0), "knn_vote: neighbour index outside the label vector");
  }
  auto scores = at::empty({M, C}, d.options());
  auto prob = at::empty({M, C}, d.options());
  auto pred = at::empty({M}, d.options().dtype(at::kLong));
  DevGuard g(d.device());
  avk::knn_vote(d.data_ptr<float>(), reinterpret_cast<const long long*>(idx.data_ptr<int64_t>()), M, (int)k,
                reinterpret_cast<const long long*>(ys.data_ptr<int64_t>()), pp, post_mode, (int)C, (int)kern,
                (float)kparam, (float)scale, (float)kscale, invdist ? 1 : 0, (float)thr, (int)pos,
                scores.data_ptr<float>(), prob.data_ptr<float>(), reinterpret_cast<long long*>(pred.data_ptr<int64_t>()),
                cur_stream(d));
  return py::make_tuple(scores, prob, pred);
}

py::tuple cluster_accumulate(const at::Tensor& X, const at::Tensor& assign, int64_t K) {
  CHECK_DEV(X);
  CHECK_DTYPE(X, at::kFloat);
  CHECK_DEV(assign);
  CHECK_DTYPE(assign, at::kInt);
  TORCH_CHECK(X.dim() == 2 && assign.numel() == X.size(0), "X [N,D], assign [N]");
  auto sums = at::zeros({K, X.size(1)}, X.options().dtype(at::kDouble));
  auto counts = at::zeros({K}, X.options().dtype(at::kLong));
  DevGuard g(X.device());
  avk::cluster_accumulate(X.data_ptr<float>(), X.size(0), (int)X.size(1), assign.data_ptr<int>(), (int)K,
                          sums.data_ptr<double>(),
                          reinterpret_cast<unsigned long long*>(counts.data_ptr<int64_t>()), cur_stream(X));
  return py::make_tuple(sums, counts);
}

// ---------------------------------------------------------------------------------------------
// sequences (K14/K15)
// ---------------------------------------------------------------------------------------------
py::tuple viterbi(const at::Tensor& obs, const at::Tensor& logA, const at::Tensor& logB,
                  const at::Tensor& logpi, int64_t mode) {
  CHECK_DEV(obs);
  CHECK_DTYPE(obs, at::kShort);
  TORCH_CHECK(obs.dim() == 2, "obs must be [N, T]");
  for (const at::Tensor* t : {&logA, &logB, &logpi}) {
    CHECK_DEV((*t));
    CHECK_DTYPE((*t), at::kFloat);
  }
  const int64_t S = logA.size(0), O = logB.size(1);
  TORCH_CHECK(logA.dim() == 2 && logA.size(1) == S, "logA must be [S, S]");
  TORCH_CHECK(logB.dim() == 2 && logB.size(0) == S, "logB must be [S, O]");
  TORCH_CHECK(logpi.numel() == S, "logpi must be [S]");
  TORCH_CHECK(S >= 1 && S <= 192, "1 <= S <= 192");
  const int64_t N = obs.size(0), T = obs.size(1);
  auto opts = obs.options();
  auto path = at::empty({N, T}, opts);
  auto score = at::empty({N}, logA.options());
  at::Tensor bp = mode == 0 ? at::empty({N, T, S}, opts) : at::empty({1}, opts);
  DevGuard g(obs.device());
  avk::viterbi(obs.data_ptr<int16_t>(), N, (int)T, (int)S, (int)O, logA.data_ptr<float>(),
               logB.data_ptr<float>(), logpi.data_ptr<float>(), (int)mode, bp.data_ptr<int16_t>(),
               path.data_ptr<int16_t>(), score.data_ptr<float>(), cur_stream(obs));
  return py::make_tuple(path, score);
}

at::Tensor viterbi_chunks(const at::Tensor& obs, const at::Tensor& logA, const at::Tensor& logB,
                          const at::Tensor& logpi, int64_t n, int64_t obs_div, const c10::optional<at::Tensor>& bp) {
  CHECK_DEV(obs);
  CHECK_DTYPE(obs, at::kShort);
  TORCH_CHECK(obs.dim() == 2, "obs must be [rows, T]");
  for (const at::Tensor* t : {&logA, &logB, &logpi}) {
    CHECK_DEV((*t));
    CHECK_DTYPE((*t), at::kFloat);
  }
  const int64_t S = logA.size(0), O = logB.size(1), T = obs.size(1);
  TORCH_CHECK(logA.dim() == 2 && logA.size(1) == S, "logA must be [S, S]");
  TORCH_CHECK(logB.dim() == 2 && logB.size(0) == S, "logB must be [S, O]");
  TORCH_CHECK(logpi.dim() == 2 && logpi.size(1) == S && logpi.size(0) >= 1, "logpi must be [rows, S]");
  TORCH_CHECK(S >= 1 && S <= 192, "1 <= S <= 192");
  TORCH_CHECK(n >= 0 && obs_div >= 1 && (n == 0 || (n - 1) / obs_div < obs.size(0)),
              "obs has fewer rows than n / obs_div");
  auto delta = at::empty({n, S}, logA.options());
  short* bpp = nullptr;
  if (bp.has_value() && bp->defined()) {
    CHECK_DEV((*bp));
    CHECK_DTYPE((*bp), at::kShort);
    TORCH_CHECK(bp->numel() == n * T * S, "bp must be [n, T, S]");
    bpp = bp->data_ptr<int16_t>();
  }
  DevGuard g(obs.device());
  avk::viterbi_chunks(obs.data_ptr<int16_t>(), n, obs_div, (int)T, (int)S, (int)O, logA.data_ptr<float>(),
                      logB.data_ptr<float>(), logpi.data_ptr<float>(), logpi.size(0), bpp, delta.data_ptr<float>(),
                      cur_stream(obs));
  return delta;
}

void viterbi_backtrack(const at::Tensor& bp, const at::Tensor& lens, const at::Tensor& ends, int64_t per_chunk,
                       const c10::optional<at::Tensor>& first, const c10::optional<at::Tensor>& path) {
  CHECK_DEV(bp);
  CHECK_DTYPE(bp, at::kShort);
  TORCH_CHECK(bp.dim() == 3, "bp must be [P, T, S]");
  const int64_t P = bp.size(0), T = bp.size(1), S = bp.size(2);
  CHECK_DEV(lens);
  CHECK_DTYPE(lens, at::kInt);
  CHECK_DEV(ends);
  CHECK_DTYPE(ends, at::kInt);
  TORCH_CHECK(lens.numel() == P, "lens must be [P]");
  TORCH_CHECK(per_chunk >= 1 && ends.numel() == P * per_chunk, "ends must be [P * per_chunk]");
  int* fp = nullptr;
  short* pp = nullptr;
  if (first.has_value() && first->defined()) {
    CHECK_DEV((*first));
    CHECK_DTYPE((*first), at::kInt);
    TORCH_CHECK(first->numel() == P * per_chunk, "first must be [P * per_chunk]");
    fp = first->data_ptr<int>();
  }
  if (path.has_value() && path->defined()) {
    CHECK_DEV((*path));
    CHECK_DTYPE((*path), at::kShort);
    TORCH_CHECK(per_chunk == 1 && path->numel() == P * T, "path needs one track per chunk and [P, T]");
    pp = path->data_ptr<int16_t>();
  }
  DevGuard g(bp.device());
  avk::viterbi_backtrack(bp.data_ptr<int16_t>(), lens.data_ptr<int>(), ends.data_ptr<int>(), P * per_chunk,
                         (int)per_chunk, (int)T, (int)S, fp, pp, cur_stream(bp));
}

at::Tensor markov_logodds(const at::Tensor& states, const at::Tensor& lr) {
  CHECK_DEV(states);
  CHECK_DTYPE(states, at::kShort);
  TORCH_CHECK(states.dim() == 2, "states must be [N, L]");
  CHECK_DEV(lr);
  CHECK_DTYPE(lr, at::kFloat);
  TORCH_CHECK(lr.dim() == 2 && lr.size(0) == lr.size(1), "lr must be [S, S]");
  TORCH_CHECK(lr.size(0) <= 200, "S <= 200");
  auto out = at::empty({states.size(0)}, lr.options());
  DevGuard g(states.device());
  avk::markov_logodds(states.data_ptr<int16_t>(), states.size(0), (int)states.size(1), lr.data_ptr<float>(),
                      (int)lr.size(0), out.data_ptr<float>(), cur_stream(states));
  return out;
}

// ---------------------------------------------------------------------------------------------
// association mining (K17)
// ---------------------------------------------------------------------------------------------
at::Tensor itemset_support(const at::Tensor& P, const at::Tensor& items, const at::Tensor& cand_prefix,
                           const at::Tensor& cand_item) {
  CHECK_DEV(P);
  CHECK_DTYPE(P, at::kLong);
  CHECK_DEV(items);
  CHECK_DTYPE(items, at::kLong);
  CHECK_DEV(cand_prefix);
  CHECK_DTYPE(cand_prefix, at::kInt);
  CHECK_DEV(cand_item);
  CHECK_DTYPE(cand_item, at::kInt);
  TORCH_CHECK(P.dim() == 2 && items.dim() == 2 && P.size(1) == items.size(1), "P [F,W], items [I,W]");
  TORCH_CHECK(cand_prefix.numel() == cand_item.numel(), "candidate arrays differ in length");
  const int64_t M = cand_prefix.numel();
  if (M) {
    TORCH_CHECK(cand_prefix.min().item<int>() >= 0 && cand_prefix.max().item<int>() < P.size(0),
                "cand_prefix out of range");
    TORCH_CHECK(cand_item.min().item<int>() >= 0 && cand_item.max().item<int>() < items.size(0),
                "cand_item out of range");
  }
  auto sup = at::zeros({M}, P.options());
  DevGuard g(P.device());
  avk::itemset_support(reinterpret_cast<const unsigned long long*>(P.data_ptr<int64_t>()), (int)P.size(1),
                       reinterpret_cast<const unsigned long long*>(items.data_ptr<int64_t>()),
                       cand_prefix.data_ptr<int>(), cand_item.data_ptr<int>(), (int)M,
                       reinterpret_cast<unsigned long long*>(sup.data_ptr<int64_t>()), cur_stream(P));
  return sup;
}

at::Tensor build_bitsets(const at::Tensor& tx, const at::Tensor& item, int64_t n_tx, int64_t n_items) {
  CHECK_DEV(tx);
  CHECK_DTYPE(tx, at::kLong);
  CHECK_DEV(item);
  CHECK_DTYPE(item, at::kInt);
  TORCH_CHECK(tx.numel() == item.numel(), "tx/item length mismatch");
  const int64_t W = (n_tx + 63) / 64;
  auto bits = at::zeros({n_items, std::max<int64_t>(W, 1)}, tx.options());
  DevGuard g(tx.device());
  avk::build_bitsets(reinterpret_cast<const long long*>(tx.data_ptr<int64_t>()), item.data_ptr<int>(),
                     tx.numel(), (int)std::max<int64_t>(W, 1), (int)n_items,
                     reinterpret_cast<unsigned long long*>(bits.data_ptr<int64_t>()), cur_stream(tx));
  return bits;
}

// ---------------------------------------------------------------------------------------------
// bandits (K20)
// ---------------------------------------------------------------------------------------------
at::Tensor bandit_select(int64_t algo, int64_t batch, const at::Tensor& trials, const at::Tensor& rsum,
                         const at::Tensor& probs, const at::Tensor& hist, double bin_width,
                         const at::Tensor& fparam, const at::Tensor& iparam, at::Tensor& gstate,
                         at::Tensor& istate, at::Tensor& epochs, int64_t seed, int64_t round) {
  CHECK_DEV(trials);
  CHECK_DTYPE(trials, at::kInt);
  TORCH_CHECK(trials.dim() == 2, "trials must be [G, A]");
  const int64_t G = trials.size(0), A = trials.size(1);
  TORCH_CHECK(A >= 1 && A <= 1024, "1 <= arms <= 1024");
  CHECK_DEV(rsum);
  CHECK_DTYPE(rsum, at::kFloat);
  CHECK_DEV(probs);
  CHECK_DTYPE(probs, at::kFloat);
  CHECK_DEV(hist);
  CHECK_DTYPE(hist, at::kInt);
  TORCH_CHECK(rsum.sizes() == trials.sizes() && probs.sizes() == trials.sizes(), "rsum/probs shape");
  TORCH_CHECK(hist.dim() == 3 && hist.size(0) == G && hist.size(1) == A, "hist must be [G, A, NB]");
  CHECK_DEV(fparam);
  CHECK_DTYPE(fparam, at::kFloat);
  CHECK_DEV(iparam);
  CHECK_DTYPE(iparam, at::kInt);
  TORCH_CHECK(fparam.numel() >= 8 && iparam.numel() >= 8, "param vectors need 8 entries");
  CHECK_DEV(gstate);
  CHECK_DTYPE(gstate, at::kFloat);
  CHECK_DEV(istate);
  CHECK_DTYPE(istate, at::kInt);
  CHECK_DEV(epochs);
  CHECK_DTYPE(epochs, at::kInt);
  TORCH_CHECK(gstate.numel() == G * 4 && istate.numel() == G * 4 && epochs.sizes() == trials.sizes(),
              "state shapes");
  TORCH_CHECK(batch >= 1, "batch >= 1");
  auto out = at::empty({G, batch}, trials.options());
  DevGuard g(trials.device());
  avk::bandit_select((int)algo, (int)G, (int)A, (int)batch, trials.data_ptr<int>(), rsum.data_ptr<float>(),
                     probs.data_ptr<float>(), reinterpret_cast<const unsigned*>(hist.data_ptr<int>()),
                     (int)hist.size(2), (float)bin_width, fparam.data_ptr<float>(), iparam.data_ptr<int>(),
                     gstate.data_ptr<float>(), istate.data_ptr<int>(), epochs.data_ptr<int>(),
                     (unsigned long long)seed, (unsigned long long)round, out.data_ptr<int>(), cur_stream(trials));
  return out;
}

// ---------------------------------------------------------------------------------------------
// samplers (K21)
// ---------------------------------------------------------------------------------------------
at::Tensor sample(int64_t dist, int64_t n, const at::Tensor& params, const c10::optional<at::Tensor>& table,
                  int64_t seed, int64_t offset) {
  CHECK_DEV(params);
  CHECK_DTYPE(params, at::kFloat);
  TORCH_CHECK(params.numel() >= 3, "params needs 3 entries");
  TORCH_CHECK(n >= 0, "n >= 0");
  const float* tp = nullptr;
  int nb = 0;
  if (table.has_value() && table->defined()) {
    CHECK_DEV((*table));
    CHECK_DTYPE((*table), at::kFloat);
    TORCH_CHECK(table->numel() >= 1, "empty CDF table");
    tp = table->data_ptr<float>();
    nb = (int)table->numel();
  }
  TORCH_CHECK(dist != 9 || tp != nullptr, "table sampler needs a CDF");
  auto out = at::empty({n}, params.options());
  DevGuard g(params.device());
  avk::sample((int)dist, n, params.data_ptr<float>(), tp, nb, (unsigned long long)seed, (unsigned long long)offset,
              out.data_ptr<float>(), cur_stream(params));
  return out;
}

// ---------------------------------------------------------------------------------------------
// optimisation (K22)
// ---------------------------------------------------------------------------------------------
void sa_assign(const at::Tensor& cost, const c10::optional<at::Tensor>& conflict, bool swap, at::Tensor& sol,
               at::Tensor& cur_cost, at::Tensor& best_sol, at::Tensor& best_cost, int64_t iters, double t0,
               double cool, int64_t interval, bool geometric, int64_t max_retry, int64_t seed, int64_t offset,
               at::Tensor& stats, int64_t it_begin, double temp_start, int64_t chain_base) {
  CHECK_DEV(cost);
  CHECK_DTYPE(cost, at::kFloat);
  TORCH_CHECK(cost.dim() == 2 && cost.size(1) >= 2, "cost must be [L, V>=2]");
  const int64_t L = cost.size(0), V = cost.size(1);
  TORCH_CHECK(V <= 32767 && L <= 512, "V or L too large (L <= 512: the [L][64] solution tile lives in LDS)");
  CHECK_DEV(sol);
  CHECK_DTYPE(sol, at::kShort);
  TORCH_CHECK(sol.dim() == 2 && sol.size(1) == L, "sol must be [P, L]");
  const int64_t P = sol.size(0);
  TORCH_CHECK(sol.min().item<int>() >= 0 && sol.max().item<int>() < V, "solution values out of range");
  CHECK_DEV(best_sol);
  CHECK_DTYPE(best_sol, at::kShort);
  TORCH_CHECK(best_sol.sizes() == sol.sizes(), "best_sol shape");
  for (at::Tensor* t : {&cur_cost, &best_cost}) {
    CHECK_DEV((*t));
    CHECK_DTYPE((*t), at::kFloat);
    TORCH_CHECK(t->numel() == P, "cost vectors must be [P]");
  }
  CHECK_DEV(stats);
  CHECK_DTYPE(stats, at::kLong);
  TORCH_CHECK(stats.numel() >= 4, "stats needs 4 entries (3 counters + hand-off temperature)");
  const uint8_t* cf = nullptr;
  if (conflict.has_value() && conflict->defined()) {
    CHECK_DEV((*conflict));
    CHECK_DTYPE((*conflict), at::kByte);
    TORCH_CHECK(conflict->dim() == 2 && conflict->size(0) == L && conflict->size(1) == L, "conflict [L, L]");
    cf = conflict->data_ptr<uint8_t>();
  }
  DevGuard g(cost.device());
  avk::sa_assign(cost.data_ptr<float>(), (int)L, (int)V, cf, swap ? 1 : 0, sol.data_ptr<int16_t>(), cur_cost.data_ptr<float>(),
                 best_sol.data_ptr<int16_t>(), best_cost.data_ptr<float>(), (int)P, (int)iters, (float)t0,
                 (float)cool, (int)interval, geometric ? 1 : 0, (int)max_retry, (unsigned long long)seed,
                 (unsigned long long)offset, (int)it_begin, (float)temp_start,
                 reinterpret_cast<unsigned long long*>(stats.data_ptr<int64_t>()), (long long)chain_base,
                 cur_stream(cost));
}

void ga_assign(const at::Tensor& cost, const c10::optional<at::Tensor>& conflict, double invalid, at::Tensor& pop,
               at::Tensor& pop_cost, at::Tensor& hist, int64_t G, int64_t m, int64_t r, bool purge_first, bool mutate,
               bool swap, int64_t seed, int64_t island_base, int64_t gen_base) {
  CHECK_DEV(cost);
  CHECK_DTYPE(cost, at::kFloat);
  TORCH_CHECK(cost.dim() == 2 && cost.size(1) >= 2 && cost.is_contiguous(), "cost must be contiguous [L, V>=2]");
  TORCH_CHECK(gen_base >= 0 && gen_base + G < (1LL << 40), "generation counter out of range");
  const int64_t L = cost.size(0), V = cost.size(1);
  TORCH_CHECK(V <= 32767, "V too large");
  CHECK_DEV(pop);
  CHECK_DTYPE(pop, at::kShort);
  TORCH_CHECK(pop.dim() == 3 && pop.size(2) == L && pop.is_contiguous(), "pop must be contiguous [islands, P, L]");
  const int64_t I = pop.size(0), P = pop.size(1);
  if (pop.numel())
    TORCH_CHECK(pop.min().item<int>() >= 0 && pop.max().item<int>() < V, "solution values out of range");
  CHECK_DEV(pop_cost);
  CHECK_DTYPE(pop_cost, at::kFloat);
  TORCH_CHECK(pop_cost.is_contiguous() && pop_cost.numel() == I * P, "pop_cost must be [islands, P]");
  CHECK_DEV(hist);
  CHECK_DTYPE(hist, at::kFloat);
  TORCH_CHECK(hist.is_contiguous() && hist.numel() == I * G, "hist must be [islands, G]");
  const uint8_t* cf = nullptr;
  if (conflict.has_value() && conflict->defined()) {
    CHECK_DEV((*conflict));
    CHECK_DTYPE((*conflict), at::kByte);
    TORCH_CHECK(conflict->dim() == 2 && conflict->size(0) == L && conflict->size(1) == L && conflict->is_contiguous(),
                "conflict [L, L]");
    cf = conflict->data_ptr<uint8_t>();
  }
  DevGuard g(cost.device());
  avk::ga_assign(cost.data_ptr<float>(), (int)L, (int)V, cf, (float)invalid, pop.data_ptr<int16_t>(),
                 pop_cost.data_ptr<float>(), hist.data_ptr<float>(), (int)I, (int)P, (int)G, (int)m, (int)r,
                 purge_first ? 1 : 0, mutate ? 1 : 0, swap ? 1 : 0, (unsigned long long)seed, (long long)island_base,
                 (int)gen_base,
                 cur_stream(cost));
}

// ---------------------------------------------------------------------------------------------
// generalised linear models (K13)
// ---------------------------------------------------------------------------------------------
at::Tensor glm_gradient(const at::Tensor& X, int64_t n, const at::Tensor& y, const c10::optional<at::Tensor>& sw,
                        const at::Tensor& w, int64_t mode, const c10::optional<at::Tensor>& hw) {
  CHECK_DEV(X);
  CHECK_DTYPE(X, at::kFloat);
  TORCH_CHECK(X.dim() == 2 && X.is_contiguous(), "X must be contiguous [D, ld]");
  const int64_t D = X.size(0), ld = X.size(1);
  TORCH_CHECK(D == 4 || D == 8 || D == 16 || D == 32 || (D > 32 && D <= 256),
              "D must be padded to 4/8/16/32 or lie in (32, 256]");
  TORCH_CHECK(ld % 16 == 0 && n >= 0 && n <= ld, "ld must be a multiple of 16 and >= n");
  TORCH_CHECK(mode >= 0 && mode <= 2, "mode: 0 logistic, 1 squared, 2 hinge");
  CHECK_DEV(y);
  CHECK_DTYPE(y, at::kFloat);
  TORCH_CHECK(y.is_contiguous() && y.numel() >= ld, "y must cover ld rows");
  CHECK_DEV(w);
  CHECK_DTYPE(w, at::kFloat);
  TORCH_CHECK(w.is_contiguous() && w.numel() == D, "w must be [D]");
  const float* swp = nullptr;
  if (sw.has_value() && sw->defined()) {
    CHECK_DEV((*sw));
    CHECK_DTYPE((*sw), at::kFloat);
    TORCH_CHECK(sw->is_contiguous() && sw->numel() >= ld, "sw must cover ld rows");
    swp = sw->data_ptr<float>();
  }
  float* hwp = nullptr;
  if (hw.has_value() && hw->defined()) {
    CHECK_DEV((*hw));
    CHECK_DTYPE((*hw), at::kFloat);
    TORCH_CHECK(hw->is_contiguous() && hw->numel() >= n, "hw must cover n rows");
    hwp = hw->data_ptr<float>();
  }
  DevGuard g(X.device());
  const int grid = avk::glm_grid(n);
  auto partial = at::empty({grid, D + 1}, X.options().dtype(at::kDouble));
  avk::glm_grad(X.data_ptr<float>(), ld, n, (int)D, y.data_ptr<float>(), swp, w.data_ptr<float>(), (int)mode,
                partial.data_ptr<double>(), grid, hwp, cur_stream(X));
  return partial.sum(0);
}

// ---------------------------------------------------------------------------------------------
// SMO kernel SVM (K12)
// ---------------------------------------------------------------------------------------------
at::Tensor smo_solve(const at::Tensor& K, const at::Tensor& y, const at::Tensor& diag, at::Tensor& alpha,
                     at::Tensor& G, double C, double eps, int64_t max_iter) {
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&K, &y, &diag, &alpha, &G}) {
    CHECK_DEV((*t));
    CHECK_DTYPE((*t), at::kFloat);
    TORCH_CHECK(t->is_contiguous(), "SMO tensors must be contiguous");
  }
  TORCH_CHECK(K.dim() == 3 && K.size(1) == K.size(2), "K must be [B, N, N]");
  const int64_t B = K.size(0), N = K.size(1);
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&y, &diag, &alpha, &G})
    TORCH_CHECK(t->dim() == 2 && t->size(0) == B && t->size(1) == N, "SMO vectors must be [B, N]");
  TORCH_CHECK(N < (1LL << 31) / 2, "N too large");
  TORCH_CHECK(C > 0 && eps > 0 && max_iter >= 0, "bad SMO parameters");
  DevGuard g(K.device());
  auto iters = at::zeros({B}, K.options().dtype(at::kInt));
  avk::smo_solve(K.data_ptr<float>(), y.data_ptr<float>(), diag.data_ptr<float>(), alpha.data_ptr<float>(),
                 G.data_ptr<float>(), (int)B, (int)N, (float)C, (float)eps, (int)max_iter, iters.data_ptr<int>(),
                 cur_stream(K));
  return iters;
}

// Working-set sub-problems: Kws [B, Q, Q], yws / aws / gws [B, Q], gap [B]; aws updated in place.
at::Tensor smo_ws_solve(const at::Tensor& Kws, const at::Tensor& yws, at::Tensor& aws, const at::Tensor& gws,
                        const at::Tensor& gap, double C, double eps, int64_t max_iter) {
  const int64_t Q = avk::smo_ws_size();
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&Kws, &yws, &aws, &gws, &gap}) {
    CHECK_DEV((*t));
    CHECK_DTYPE((*t), at::kFloat);
  }
  TORCH_CHECK(Kws.dim() == 3 && Kws.size(1) == Q && Kws.size(2) == Q, "Kws must be [B, Q, Q] with Q = ", Q);
  const int64_t B = Kws.size(0);
  TORCH_CHECK(aligned(Kws, 16), "Kws must be 16-byte aligned");
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&yws, &aws, &gws})
    TORCH_CHECK(t->dim() == 2 && t->size(0) == B && t->size(1) == Q, "working-set vectors must be [B, Q]");
  TORCH_CHECK(gap.numel() == B, "gap must be [B]");
  TORCH_CHECK(C > 0 && eps > 0 && max_iter >= 0, "bad SMO parameters");
  DevGuard g(Kws.device());
  auto iters = at::zeros({B}, Kws.options().dtype(at::kInt));
  avk::smo_ws_solve(Kws.data_ptr<float>(), yws.data_ptr<float>(), aws.data_ptr<float>(), gws.data_ptr<float>(),
                    gap.data_ptr<float>(), (int)B, (float)C, (float)eps, (int)max_iter, iters.data_ptr<int>(),
                    cur_stream(Kws));
  return iters;
}

void smo_ws_select(const at::Tensor& alpha, const at::Tensor& G, const at::Tensor& y, double C, int64_t h,
                   at::Tensor& ws, at::Tensor& ok, at::Tensor& gap) {
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&alpha, &G, &y, &gap}) {
    CHECK_DEV((*t));
    CHECK_DTYPE((*t), at::kFloat);
  }
  TORCH_CHECK(y.dim() == 2, "y must be [B, N]");
  const int64_t B = y.size(0), N = y.size(1);
  TORCH_CHECK(alpha.dim() == 2 && alpha.size(0) == B && alpha.size(1) >= N && G.sizes() == alpha.sizes(),
              "alpha / G must be [B, >= N]");
  TORCH_CHECK(h >= 1 && h <= 64 && N >= 1 && N <= (1 << 26) && (N <= (1 << 18) || h == 64),
              "1 <= h <= 64, 1 <= N <= 2^26 (h = 64 above 2^18)");
  CHECK_DEV(ws);
  CHECK_DTYPE(ws, at::kLong);
  CHECK_DEV(ok);
  CHECK_DTYPE(ok, at::kBool);
  TORCH_CHECK(ws.numel() == B * 2 * h && ok.numel() == B * 2 * h && gap.numel() == B, "ws / ok [B, 2h], gap [B]");
  DevGuard g(y.device());
  // two-level selection scratch: per (problem, part, side) local candidates and counts (inside a
  // graph capture these come from the capture's private pool)
  const int64_t parts = avk::smo_ws_select_parts((int)N);
  auto cand = at::empty({2, B, parts, 2, h}, y.options().dtype(at::kInt));  // rows, then float values
  auto cnt = at::empty({B, std::max<int64_t>(parts, 64), 2}, y.options().dtype(at::kInt));  // <= 64 streaming parts
  avk::smo_ws_select(alpha.data_ptr<float>(), G.data_ptr<float>(), y.data_ptr<float>(), (int)B, (int)N,
                     (int)alpha.size(1), (float)C, (int)h, reinterpret_cast<long long*>(ws.data_ptr<int64_t>()),
                     ok.data_ptr<bool>(), gap.data_ptr<float>(), cand.data_ptr<int>(), cnt.data_ptr<int>(),
                     -INFINITY, cur_stream(y));
}

void smo_ws_solve_fused(const at::Tensor& K, const at::Tensor& ws, const at::Tensor& ok, at::Tensor& alpha,
                        const at::Tensor& G, const at::Tensor& y, const at::Tensor& gap, double C, double eps,
                        int64_t max_iter, at::Tensor& dA, at::Tensor& inner_total, double rel_tol) {
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&K, &alpha, &G, &y, &gap, &dA}) {
    CHECK_DEV((*t));
    CHECK_DTYPE((*t), at::kFloat);
  }
  TORCH_CHECK(y.dim() == 2, "y must be [B, N]");
  const int64_t B = y.size(0), N = y.size(1), Q = avk::smo_ws_size();
  TORCH_CHECK(K.dim() == 3 && (K.size(0) == B || K.size(0) == 1) && K.size(1) == N && K.size(2) == N,
              "K must be [B or 1 (shared by all problems), N, N]");
  const long long kbs = K.size(0) == 1 ? 0LL : (long long)N * N;
  TORCH_CHECK(alpha.dim() == 2 && alpha.size(0) == B && alpha.size(1) >= N && G.sizes() == alpha.sizes(),
              "alpha / G must be [B, >= N]");
  CHECK_DEV(ws);
  CHECK_DTYPE(ws, at::kLong);
  CHECK_DEV(ok);
  CHECK_DTYPE(ok, at::kBool);
  CHECK_DEV(inner_total);
  CHECK_DTYPE(inner_total, at::kLong);
  TORCH_CHECK(ws.numel() == B * Q && ok.numel() == B * Q && dA.numel() == B * Q, "ws / ok / dA must be [B, ", Q, "]");
  TORCH_CHECK(gap.numel() == B && inner_total.numel() == B, "gap / inner_total must be [B]");
  TORCH_CHECK(C > 0 && eps > 0 && max_iter >= 0, "bad SMO parameters");
  DevGuard g(y.device());
  // gathered K[ws, ws] blocks (graph capture: from the capture's private pool)
  auto Kws = at::empty({B, Q, Q}, K.options());
  avk::smo_ws_solve_fused(K.data_ptr<float>(), (int)N, reinterpret_cast<const long long*>(ws.data_ptr<int64_t>()),
                          ok.data_ptr<bool>(), alpha.data_ptr<float>(), G.data_ptr<float>(), y.data_ptr<float>(),
                          (int)alpha.size(1), gap.data_ptr<float>(), (int)B, (float)C, (float)eps, (int)max_iter,
                          dA.data_ptr<float>(), reinterpret_cast<long long*>(inner_total.data_ptr<int64_t>()),
                          Kws.data_ptr<float>(), (float)rel_tol, kbs, cur_stream(y));
}

void smo_ws_update(const at::Tensor& K, const at::Tensor& ws, const at::Tensor& dA, const at::Tensor& ok,
                   const at::Tensor& y, at::Tensor& G) {
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&K, &dA, &y, &G}) {
    CHECK_DEV((*t));
    CHECK_DTYPE((*t), at::kFloat);
  }
  TORCH_CHECK(y.dim() == 2, "y must be [B, N]");
  const int64_t B = y.size(0), N = y.size(1);
  TORCH_CHECK(K.dim() == 3 && (K.size(0) == B || K.size(0) == 1) && K.size(1) == N && K.size(2) == N,
              "K must be [B or 1 (shared by all problems), N, N]");
  const long long kbs = K.size(0) == 1 ? 0LL : (long long)N * N;
  TORCH_CHECK(G.dim() == 2 && G.size(0) == B && G.size(1) >= N, "G must be [B, >= N]");
  CHECK_DEV(ws);
  CHECK_DTYPE(ws, at::kLong);
  CHECK_DEV(ok);
  CHECK_DTYPE(ok, at::kBool);
  TORCH_CHECK(ws.dim() == 2 && ws.size(0) == B && ws.size(1) <= avk::smo_ws_size() && dA.sizes() == ws.sizes() &&
                  ok.sizes() == ws.sizes(),
              "ws / dA / ok must be [B, Q <= ", avk::smo_ws_size(), "]");
  DevGuard g(y.device());
  avk::smo_ws_update(K.data_ptr<float>(), reinterpret_cast<const long long*>(ws.data_ptr<int64_t>()),
                     dA.data_ptr<float>(), ok.data_ptr<bool>(), y.data_ptr<float>(), G.data_ptr<float>(), (int)B,
                     (int)N, (int)G.size(1), (int)ws.size(1), nullptr, -INFINITY, kbs, cur_stream(y));
}

// exp(-gamma |a_i - b_j|^2) [na, nb] float32 in one pass (d <= 64)
at::Tensor rbf_matrix(const at::Tensor& A, const at::Tensor& B, double gamma) {
  CHECK_DEV(A);
  CHECK_DEV(B);
  CHECK_DTYPE(A, at::kFloat);
  CHECK_DTYPE(B, at::kFloat);
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.size(1) == B.size(1) && A.size(1) >= 1 && A.size(1) <= 64,
              "A [na, d], B [nb, d], 1 <= d <= 64");
  TORCH_CHECK(A.size(0) < (1LL << 31) / 64 && B.size(0) < (1LL << 31) / 64, "too many rows");
  DevGuard g(A.device());
  const auto Ac = A.contiguous(), Bc = B.contiguous();
  auto K = at::empty({A.size(0), B.size(0)}, A.options());
  avk::rbf_matrix(Ac.data_ptr<float>(), Bc.data_ptr<float>(), (int)A.size(0), (int)B.size(0), (int)A.size(1),
                  (float)gamma, K.data_ptr<float>(), cur_stream(A));
  return K;
}

// The whole working-set solve in one call (avk::smo_ws_run): state tensors as in the per-step
// bindings above; returns the number of outer steps enqueued.
int64_t smo_ws_run(const at::Tensor& K, at::Tensor& alpha, at::Tensor& G, const at::Tensor& y, double C, double eps,
                   int64_t inner_iter, double rel_tol, int64_t max_outer, int64_t check_every, at::Tensor& ws,
                   at::Tensor& ok, at::Tensor& dA, at::Tensor& inner_total, at::Tensor& gap) {
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&K, &alpha, &G, &y, &gap, &dA}) {
    CHECK_DEV((*t));
    CHECK_DTYPE((*t), at::kFloat);
  }
  TORCH_CHECK(y.dim() == 2, "y must be [B, N]");
  const int64_t B = y.size(0), N = y.size(1), Q = avk::smo_ws_size();
  TORCH_CHECK(N >= 1 && N <= (1 << 26), "1 <= N <= 2^26");
  TORCH_CHECK(K.dim() == 3 && (K.size(0) == B || K.size(0) == 1) && K.size(1) == N && K.size(2) == N,
              "K must be [B or 1 (shared by all problems), N, N]");
  const long long kbs = K.size(0) == 1 ? 0LL : (long long)N * N;
  TORCH_CHECK(alpha.dim() == 2 && alpha.size(0) == B && alpha.size(1) >= N && G.sizes() == alpha.sizes(),
              "alpha / G must be [B, >= N]");
  CHECK_DEV(ws);
  CHECK_DTYPE(ws, at::kLong);
  CHECK_DEV(ok);
  CHECK_DTYPE(ok, at::kBool);
  CHECK_DEV(inner_total);
  CHECK_DTYPE(inner_total, at::kLong);
  TORCH_CHECK(ws.numel() == B * Q && ok.numel() == B * Q && dA.numel() == B * Q, "ws / ok / dA must be [B, ", Q, "]");
  TORCH_CHECK(gap.numel() == B && inner_total.numel() == B, "gap / inner_total must be [B]");
  TORCH_CHECK(C > 0 && eps > 0 && inner_iter >= 0, "bad SMO parameters");
  DevGuard g(y.device());
  const int64_t parts = avk::smo_ws_select_parts((int)N);
  auto cand = at::empty({2, B, parts, 2, Q / 2}, y.options().dtype(at::kInt));  // rows, then float values
  auto cnt = at::empty({B, std::max<int64_t>(parts, 64), 2}, y.options().dtype(at::kInt));  // <= 64 streaming parts
  auto Kws = at::empty({B, Q, Q}, K.options());
  auto host_gap = at::empty({2 * B}, at::TensorOptions().dtype(at::kFloat).pinned_memory(true));
  auto gap_next = at::empty({B}, y.options());
  return avk::smo_ws_run(K.data_ptr<float>(), (int)N, alpha.data_ptr<float>(), G.data_ptr<float>(),
                         y.data_ptr<float>(), (int)B, (int)alpha.size(1), (float)C, (float)eps, (int)inner_iter,
                         (float)rel_tol, max_outer, (int)check_every,
                         reinterpret_cast<long long*>(ws.data_ptr<int64_t>()), ok.data_ptr<bool>(),
                         dA.data_ptr<float>(), reinterpret_cast<long long*>(inner_total.data_ptr<int64_t>()),
                         gap.data_ptr<float>(), cand.data_ptr<int>(), cnt.data_ptr<int>(), Kws.data_ptr<float>(),
                         host_gap.data_ptr<float>(), kbs, cur_stream(y), nullptr, gap_next.data_ptr<float>());
}

// implicit kernel source from X [B or 1, N, D] (or [N, D]) and its squared norms
static avk::SvmKerX make_kerx(const at::Tensor& X, const at::Tensor& xn, int64_t B, int64_t N, int64_t kind,
                              double gamma, double coef0, int64_t degree) {
  CHECK_DEV(X);
  CHECK_DTYPE(X, at::kFloat);
  CHECK_DEV(xn);
  CHECK_DTYPE(xn, at::kFloat);
  TORCH_CHECK(X.is_contiguous() && xn.is_contiguous(), "X / xn must be contiguous");
  const bool batched = X.dim() == 3;
  TORCH_CHECK((X.dim() == 2 && X.size(0) == N) || (batched && (X.size(0) == B || X.size(0) == 1) && X.size(1) == N),
              "X must be [N, D] or [B or 1, N, D]");
  const int64_t D = X.size(X.dim() - 1);
  TORCH_CHECK(D >= 1 && D <= 65536, "1 <= D <= 65536");
  TORCH_CHECK(xn.numel() == (batched ? X.size(0) : 1) * N, "xn must hold the squared norms of X's rows");
  TORCH_CHECK(kind >= 0 && kind <= 3 && degree >= 0 && degree <= 16, "kernel kind 0..3, degree 0..16");
  avk::SvmKerX k;
  k.X = X.data_ptr<float>();
  k.xn = xn.data_ptr<float>();
  k.xbs = (batched && X.size(0) == B && B > 1) ? N : 0;
  k.D = (int)D;
  k.kind = (int)kind;
  k.degree = (int)degree;
  k.gamma = (float)gamma;
  k.coef0 = (float)coef0;
  return k;
}

// The working-set solve with the implicit kernel (no N x N matrix): K[ws, ws] and the gradient
// updates are recomputed from X each outer step (avk::smo_ws_run with kx).
int64_t smo_ws_run_x(const at::Tensor& X, const at::Tensor& xn, int64_t kind, double gamma, double coef0,
                     int64_t degree, at::Tensor& alpha, at::Tensor& G, const at::Tensor& y, double C, double eps,
                     int64_t inner_iter, double rel_tol, int64_t max_outer, int64_t check_every, at::Tensor& ws,
                     at::Tensor& ok, at::Tensor& dA, at::Tensor& inner_total, at::Tensor& gap, int64_t cache_slots,
                     const c10::optional<at::Tensor>& cache_stats) {
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&alpha, &G, &y, &gap, &dA}) {
    CHECK_DEV((*t));
    CHECK_DTYPE((*t), at::kFloat);
  }
  TORCH_CHECK(y.dim() == 2, "y must be [B, N]");
  const int64_t B = y.size(0), N = y.size(1), Q = avk::smo_ws_size();
  TORCH_CHECK(N >= 1 && N <= (1 << 26), "1 <= N <= 2^26");
  const avk::SvmKerX k = make_kerx(X, xn, B, N, kind, gamma, coef0, degree);
  // kernel-row cache (one problem on a shared X): S slots in sets of 8 + Q transient rows
  constexpr int kWays = 8;
  const int64_t S = cache_slots > 0 ? std::max<int64_t>(kWays, cache_slots / kWays * kWays) : 0;
  TORCH_CHECK(S == 0 || (B == 1 && k.xbs == 0), "the row cache needs one problem on a shared X");
  TORCH_CHECK(S <= 16384, "at most 16384 cache slots");
  at::Tensor c_rows, c_tag, c_stamp, c_slot_of, c_step, c_ws_slot, c_miss_q, c_miss_cnt, c_stats;
  avk::SvmCache cache{};
  if (S > 0) {
    auto iopt = y.options().dtype(at::kInt);
    c_rows = at::empty({(S + Q) * N}, y.options());
    c_tag = at::full({S}, -1, iopt);
    c_stamp = at::zeros({S}, iopt);
    c_slot_of = at::full({N}, -1, iopt);
    c_step = at::zeros({1}, iopt);
    c_ws_slot = at::zeros({Q}, y.options().dtype(at::kLong));
    c_miss_q = at::zeros({Q}, iopt);
    c_miss_cnt = at::zeros({1}, iopt);
    if (cache_stats.has_value() && cache_stats->defined()) {
      CHECK_DEV((*cache_stats));
      CHECK_DTYPE((*cache_stats), at::kLong);
      TORCH_CHECK(cache_stats->numel() == 2, "cache_stats must be int64 [2]");
      c_stats = *cache_stats;
    } else {
      c_stats = at::zeros({2}, y.options().dtype(at::kLong));
    }
    cache = avk::SvmCache{c_rows.data_ptr<float>(), c_tag.data_ptr<int>(), c_stamp.data_ptr<int>(),
                          c_slot_of.data_ptr<int>(), c_step.data_ptr<int>(),
                          reinterpret_cast<long long*>(c_ws_slot.data_ptr<int64_t>()), c_miss_q.data_ptr<int>(),
                          c_miss_cnt.data_ptr<int>(), reinterpret_cast<unsigned long long*>(c_stats.data_ptr<int64_t>()),
                          (int)S, kWays};
  }
  TORCH_CHECK(alpha.dim() == 2 && alpha.size(0) == B && alpha.size(1) >= N && G.sizes() == alpha.sizes(),
              "alpha / G must be [B, >= N]");
  CHECK_DEV(ws);
  CHECK_DTYPE(ws, at::kLong);
  CHECK_DEV(ok);
  CHECK_DTYPE(ok, at::kBool);
  CHECK_DEV(inner_total);
  CHECK_DTYPE(inner_total, at::kLong);
  TORCH_CHECK(ws.numel() == B * Q && ok.numel() == B * Q && dA.numel() == B * Q, "ws / ok / dA must be [B, ", Q, "]");
  TORCH_CHECK(gap.numel() == B && inner_total.numel() == B, "gap / inner_total must be [B]");
  TORCH_CHECK(C > 0 && eps > 0 && inner_iter >= 0, "bad SMO parameters");
  DevGuard g(y.device());
  const int64_t parts = avk::smo_ws_select_parts((int)N);
  auto cand = at::empty({2, B, parts, 2, Q / 2}, y.options().dtype(at::kInt));
  auto cnt = at::empty({B, std::max<int64_t>(parts, 64), 2}, y.options().dtype(at::kInt));  // <= 64 streaming parts
  auto Kws = at::empty({B, Q, Q}, y.options());
  auto host_gap = at::empty({2 * B}, at::TensorOptions().dtype(at::kFloat).pinned_memory(true));
  return avk::smo_ws_run(nullptr, (int)N, alpha.data_ptr<float>(), G.data_ptr<float>(), y.data_ptr<float>(), (int)B,
                         (int)alpha.size(1), (float)C, (float)eps, (int)inner_iter, (float)rel_tol, max_outer,
                         (int)check_every, reinterpret_cast<long long*>(ws.data_ptr<int64_t>()), ok.data_ptr<bool>(),
                         dA.data_ptr<float>(), reinterpret_cast<long long*>(inner_total.data_ptr<int64_t>()),
                         gap.data_ptr<float>(), cand.data_ptr<int>(), cnt.data_ptr<int>(), Kws.data_ptr<float>(),
                         host_gap.data_ptr<float>(), 0, cur_stream(y), &k, nullptr, S > 0 ? &cache : nullptr);
}

// one implicit-kernel gather (K[ws, ws] -> [B, Q, Q]) and one gradient update (tests / oracles)
at::Tensor smo_ws_gather_x(const at::Tensor& X, const at::Tensor& xn, int64_t kind, double gamma, double coef0,
                           int64_t degree, const at::Tensor& ws, const at::Tensor& ok, int64_t N) {
  CHECK_DEV(ws);
  CHECK_DTYPE(ws, at::kLong);
  CHECK_DTYPE(ok, at::kBool);
  const int64_t Q = avk::smo_ws_size(), B = ws.size(0);
  TORCH_CHECK(ws.dim() == 2 && ws.size(1) == Q && ok.sizes() == ws.sizes(), "ws / ok must be [B, ", Q, "]");
  TORCH_CHECK(ws.numel() == 0 || (ws.min().item<int64_t>() >= 0 && ws.max().item<int64_t>() < N), "ws out of range");
  const avk::SvmKerX k = make_kerx(X, xn, B, N, kind, gamma, coef0, degree);
  DevGuard g(ws.device());
  auto Kws = at::zeros({B, Q, Q}, X.options());
  avk::smo_ws_gather_x(k, reinterpret_cast<const long long*>(ws.data_ptr<int64_t>()), ok.data_ptr<bool>(),
                       Kws.data_ptr<float>(), (int)B, (int)N, nullptr, -INFINITY, cur_stream(ws));
  return Kws;
}

void smo_ws_update_x(const at::Tensor& X, const at::Tensor& xn, int64_t kind, double gamma, double coef0,
                     int64_t degree, const at::Tensor& ws, const at::Tensor& dA, const at::Tensor& ok,
                     const at::Tensor& y, at::Tensor& G) {
  CHECK_DEV(y);
  CHECK_DTYPE(y, at::kFloat);
  CHECK_DTYPE(G, at::kFloat);
  CHECK_DTYPE(dA, at::kFloat);
  CHECK_DTYPE(ws, at::kLong);
  CHECK_DTYPE(ok, at::kBool);
  const int64_t B = y.size(0), N = y.size(1);
  TORCH_CHECK(G.dim() == 2 && G.size(0) == B && G.size(1) >= N, "G must be [B, >= N]");
  TORCH_CHECK(ws.dim() == 2 && ws.size(0) == B && ws.size(1) <= avk::smo_ws_size() && dA.sizes() == ws.sizes() &&
                  ok.sizes() == ws.sizes(),
              "ws / dA / ok must be [B, Q <= ", avk::smo_ws_size(), "]");
  TORCH_CHECK(ws.numel() == 0 || (ws.min().item<int64_t>() >= 0 && ws.max().item<int64_t>() < N), "ws out of range");
  const avk::SvmKerX k = make_kerx(X, xn, B, N, kind, gamma, coef0, degree);
  DevGuard g(y.device());
  avk::smo_ws_update_x(k, reinterpret_cast<const long long*>(ws.data_ptr<int64_t>()), dA.data_ptr<float>(),
                       ok.data_ptr<bool>(), y.data_ptr<float>(), G.data_ptr<float>(), (int)B, (int)N, (int)G.size(1),
                       (int)ws.size(1), nullptr, -INFINITY, cur_stream(y));
}

// K(A, B) [na, nb] through f32 MFMA for any d (kind 0 linear, 1 poly, 2 rbf, 3 sigmoid)
at::Tensor svm_kernel_matrix(const at::Tensor& A, const at::Tensor& Bm, int64_t kind, double gamma, double coef0,
                             int64_t degree) {
  CHECK_DEV(A);
  CHECK_DEV(Bm);
  CHECK_DTYPE(A, at::kFloat);
  CHECK_DTYPE(Bm, at::kFloat);
  TORCH_CHECK(A.dim() == 2 && Bm.dim() == 2 && A.size(1) == Bm.size(1) && A.size(1) >= 1, "A [na, d], B [nb, d]");
  TORCH_CHECK(A.size(0) < (1LL << 31) / 64 && Bm.size(0) < (1LL << 31) / 64, "too many rows");
  DevGuard g(A.device());
  const auto Ac = A.contiguous(), Bc = Bm.contiguous();
  const auto an = (Ac * Ac).sum(1).contiguous(), bnrm = (Bc * Bc).sum(1).contiguous();
  const avk::SvmKerX k = make_kerx(Ac, an, 1, A.size(0), kind, gamma, coef0, degree);
  auto K = at::empty({A.size(0), Bm.size(0)}, A.options());
  avk::svm_kernel_matrix_mfma(k, Bc.data_ptr<float>(), bnrm.data_ptr<float>(), (int)A.size(0), (int)Bm.size(0),
                              K.data_ptr<float>(), cur_stream(A));
  return K;
}

std::vector<at::Tensor> nb_finalize(const at::Tensor& counts, const at::Tensor& offs, const at::Tensor& bins,
                                    int64_t extent, double laplace, double log_floor) {
  CHECK_DEV(counts);
  CHECK_DTYPE(counts, at::kLong);
  TORCH_CHECK(counts.dim() == 2 && counts.is_contiguous(), "counts must be contiguous [C, TB+1]");
  CHECK_DEV(offs);
  CHECK_DTYPE(offs, at::kInt);
  CHECK_DEV(bins);
  CHECK_DTYPE(bins, at::kInt);
  const int64_t C = counts.size(0), TB = counts.size(1) - 1, F = bins.numel();
  TORCH_CHECK(offs.numel() == F && F >= 1 && TB >= 1, "offs/bins mismatch");
  // extent = offs[F-1] + bins[F-1], computed on the host by the caller (no device sync here, so
  // the call is HIP-graph capturable)
  TORCH_CHECK(extent <= TB, "bins exceed count table");
  DevGuard g(counts.device());
  auto o = counts.options().dtype(at::kFloat);
  auto logp = at::empty({C, TB}, o), logfp = at::empty({TB}, o), logprior = at::empty({C}, o);
  avk::nb_finalize(reinterpret_cast<const long long*>(counts.data_ptr<int64_t>()), (int)C, (int)TB, offs.data_ptr<int>(), bins.data_ptr<int>(), (int)F,
                   (float)laplace, (float)log_floor, logp.data_ptr<float>(), logfp.data_ptr<float>(),
                   logprior.data_ptr<float>(), cur_stream(counts));
  return {logp, logfp, logprior};
}

at::Tensor weighted_gram(const at::Tensor& X, int64_t n, int64_t D, const c10::optional<at::Tensor>& h) {
  CHECK_DEV(X);
  CHECK_DTYPE(X, at::kFloat);
  TORCH_CHECK(X.dim() == 2 && X.is_contiguous() && X.size(0) >= D && D >= 1 && D <= 1024, "X [>=D, ld], D <= 1024");
  TORCH_CHECK(n >= 0 && n <= X.size(1), "n exceeds ld");
  const float* hp = nullptr;
  if (h.has_value() && h->defined()) {
    CHECK_DEV((*h));
    CHECK_DTYPE((*h), at::kFloat);
    TORCH_CHECK(h->is_contiguous() && h->numel() >= n, "h must cover n rows");
    hp = h->data_ptr<float>();
  }
  DevGuard g(X.device());
  if (D <= 32) {
    const int grid = avk::gram_grid(n);
    auto partial = at::empty({(int64_t)grid * 4, 32, 32}, X.options());
    avk::weighted_gram(X.data_ptr<float>(), X.size(1), n, (int)D, hp, partial.data_ptr<float>(), grid, cur_stream(X));
    return partial.to(at::kDouble).sum(0).narrow(0, 0, D).narrow(1, 0, D);
  }
  // block pairs: keep the total work-group count (and the partial buffer) near the D <= 32 launch
  const int64_t nb = (D + 31) / 32, npairs = nb * (nb + 1) / 2;
  const int grid = (int)std::max<int64_t>(8, avk::gram_grid(n) / npairs);
  auto partial = at::empty({(int64_t)grid * 4, npairs, 32, 32}, X.options());
  avk::weighted_gram(X.data_ptr<float>(), X.size(1), n, (int)D, hp, partial.data_ptr<float>(), grid, cur_stream(X));
  auto blocks = partial.to(at::kDouble).sum(0);  // [npairs, 32, 32]
  auto G = at::zeros({nb * 32, nb * 32}, blocks.options());
  int64_t p = 0;
  for (int64_t bi = 0; bi < nb; ++bi)
    for (int64_t bj = bi; bj < nb; ++bj, ++p) {
      G.narrow(0, bi * 32, 32).narrow(1, bj * 32, 32).copy_(blocks[p]);
      if (bj != bi) G.narrow(0, bj * 32, 32).narrow(1, bi * 32, 32).copy_(blocks[p].t());
    }
  return G.narrow(0, 0, D).narrow(1, 0, D).contiguous();
}

// k-means (K16).  Centroids in pair layout C2 [Kp/2, D, 2] (every run padded to an even count),
// norms Cn [Kp] (+inf for padding), run offsets roff [R + 1] (device copy + host copy h_roff).
std::vector<at::Tensor> kmeans_assign(const at::Tensor& X, const at::Tensor& C2, const at::Tensor& Cn,
                                      const at::Tensor& roff, const std::vector<int64_t>& h_roff, bool want_assign) {
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&X, &C2, &Cn}) {
    CHECK_DEV((*t));
    CHECK_DTYPE((*t), at::kFloat);
  }
  CHECK_DEV(roff);
  CHECK_DTYPE(roff, at::kInt);
  TORCH_CHECK(X.dim() == 2, "X must be [n, D]");
  const int64_t n = X.size(0), D = X.size(1), R = (int64_t)h_roff.size() - 1;
  TORCH_CHECK(D == 2 || D == 4 || D == 8 || D == 16 || D == 32 || D == 64, "D must be padded to 2/4/8/16/32/64");
  TORCH_CHECK(R >= 1 && R <= 16, "1..16 runs per launch");
  TORCH_CHECK(roff.numel() == R + 1, "roff must have R + 1 entries");
  TORCH_CHECK(h_roff[0] == 0, "roff[0] must be 0");
  for (int64_t r = 0; r < R; ++r)
    TORCH_CHECK(h_roff[r + 1] >= h_roff[r] + 2 && h_roff[r + 1] % 2 == 0, "every run needs an even count >= 2");
  const int64_t K = h_roff[R];
  TORCH_CHECK(K <= 4096, "at most 4096 centroids per launch");
  TORCH_CHECK(C2.numel() == K * D && Cn.numel() == K, "C2 must hold Kp * D values and Cn Kp norms");
  DevGuard g(X.device());
  const int grid = avk::kmeans_grid(n, (int)D, (int)K, (int)R);
  auto partial = at::empty({grid, K, D + 1}, X.options());
  auto ssep = at::empty({grid, R}, X.options().dtype(at::kDouble));
  at::Tensor assign;
  if (want_assign) assign = at::empty({R, n}, X.options().dtype(at::kInt));
  avk::kmeans_assign(X.data_ptr<float>(), n, (int)D, C2.data_ptr<float>(), Cn.data_ptr<float>(), roff.data_ptr<int>(),
                     (int)R, (int)K, want_assign ? assign.data_ptr<int>() : nullptr, partial.data_ptr<float>(),
                     ssep.data_ptr<double>(), grid, cur_stream(X));
  return {partial, ssep, want_assign ? assign : at::Tensor()};
}

// -> fp64 [K * (D + 1) + R]: per centroid (sums[D], count), then per-run SSE
at::Tensor kmeans_reduce(const at::Tensor& partial, const at::Tensor& ssep) {
  CHECK_DEV(partial);
  CHECK_DTYPE(partial, at::kFloat);
  CHECK_DEV(ssep);
  CHECK_DTYPE(ssep, at::kDouble);
  TORCH_CHECK(partial.dim() == 3 && ssep.dim() == 2 && ssep.size(0) == partial.size(0), "partial [G, K, D+1], ssep [G, R]");
  const int64_t G = partial.size(0), K = partial.size(1), D = partial.size(2) - 1, R = ssep.size(1);
  auto out = at::empty({K * (D + 1) + R}, ssep.options());
  DevGuard g(partial.device());
  avk::kmeans_reduce(partial.data_ptr<float>(), ssep.data_ptr<double>(), (int)G, (int)K, (int)D, (int)R,
                     out.data_ptr<double>(), cur_stream(partial));
  return out;
}

// updates C2 / Cn in place; returns the per-run maximum centroid movement (float [R])
at::Tensor kmeans_update(const at::Tensor& flat, at::Tensor& C2, at::Tensor& Cn, const at::Tensor& run_of,
                         const at::Tensor& frozen, int64_t D) {
  CHECK_DEV(flat);
  CHECK_DTYPE(flat, at::kDouble);
  CHECK_DEV(C2);
  CHECK_DTYPE(C2, at::kFloat);
  CHECK_DEV(Cn);
  CHECK_DTYPE(Cn, at::kFloat);
  CHECK_DEV(run_of);
  CHECK_DTYPE(run_of, at::kInt);
  CHECK_DEV(frozen);
  CHECK_DTYPE(frozen, at::kByte);
  const int64_t K = Cn.numel(), R = frozen.numel();
  TORCH_CHECK(K % 2 == 0 && C2.numel() == K * D && run_of.numel() == K, "layout mismatch");
  TORCH_CHECK(R >= 1 && R <= 16 && flat.numel() == K * (D + 1) + R, "flat must be [K * (D + 1) + R]");
  auto moves = at::empty({2 * R}, C2.options());  // [max shift per run | total squared shift per run]
  DevGuard g(C2.device());
  avk::kmeans_update(flat.data_ptr<double>(), (int)K, (int)D, (int)R, run_of.data_ptr<int>(), frozen.data_ptr<uint8_t>(),
                     C2.data_ptr<float>(), Cn.data_ptr<float>(), moves.data_ptr<float>(), cur_stream(C2));
  return moves;
}

// ---------------------------------------------------------------------------------------------
// sequence mining (K5 / K16 / K19)

// Returns (keys int64 [U], counts int64 [U]); key = (len << 58) | (group * group_mul + packed).
// The table starts at `cap` slots and doubles while the kernel reports that it filled up.
py::tuple ngram_count(const at::Tensor& states, int64_t S, int64_t min_len, int64_t max_len,
                      const c10::optional<at::Tensor>& group, int64_t group_mul, int64_t cap) {
  CHECK_DEV(states);
  CHECK_DTYPE(states, at::kShort);
  TORCH_CHECK(states.dim() == 2, "states must be [N, L]");
  TORCH_CHECK(S >= 1 && S < 32767, "1 <= S < 32767");
  TORCH_CHECK(min_len >= 1 && max_len >= min_len && max_len <= 63, "1 <= min_len <= max_len <= 63");
  const int64_t N = states.size(0), L = states.size(1);
  const int* gp = nullptr;
  if (group.has_value() && group->defined()) {
    CHECK_DEV((*group));
    CHECK_DTYPE((*group), at::kInt);
    TORCH_CHECK(group->numel() == N, "group must be [N]");
    gp = group->data_ptr<int>();
  }
  TORCH_CHECK(cap >= 1024 && (cap & (cap - 1)) == 0, "cap must be a power of two >= 1024");
  DevGuard g(states.device());
  auto dev = states.options();
  for (;;) {
    auto keys = at::full({cap}, -1, dev.dtype(at::kLong));
    auto counts = at::zeros({cap}, dev.dtype(at::kInt));
    auto flag = at::zeros({1}, dev.dtype(at::kInt));
    avk::ngram_count(states.data_ptr<int16_t>(), N, (int)L, (int)S, (int)min_len, (int)max_len, gp,
                     (unsigned long long)group_mul, reinterpret_cast<unsigned long long*>(keys.data_ptr<int64_t>()),
                     reinterpret_cast<unsigned*>(counts.data_ptr<int>()), (unsigned long long)cap,
                     flag.data_ptr<int>(), cur_stream(states));
    if (flag.item<int>() != 0) {
      TORCH_CHECK(cap < (1LL << 30), "ngram_count: more than 2^30 distinct n-grams");
      cap *= 2;
      continue;
    }
    auto ok = at::empty({cap}, dev.dtype(at::kLong));
    auto oc = at::empty({cap}, dev.dtype(at::kLong));
    auto nout = at::zeros({1}, dev.dtype(at::kLong));
    avk::hash_compact(reinterpret_cast<const unsigned long long*>(keys.data_ptr<int64_t>()),
                      reinterpret_cast<const unsigned*>(counts.data_ptr<int>()), (unsigned long long)cap,
                      reinterpret_cast<long long*>(ok.data_ptr<int64_t>()), reinterpret_cast<long long*>(oc.data_ptr<int64_t>()),
                      reinterpret_cast<unsigned long long*>(nout.data_ptr<int64_t>()), cur_stream(states));
    const int64_t U = nout.item<int64_t>();
    return py::make_tuple(ok.narrow(0, 0, U), oc.narrow(0, 0, U));
  }
}

// P fp64 [S, S]; w1, w2 fp64 [B, ldw]; steps int32 [B] (each < ldw) -> out fp64 [B, 2, S, S]
at::Tensor uniformization(const at::Tensor& P, const at::Tensor& w1, const at::Tensor& w2, const at::Tensor& steps,
                          const std::vector<int64_t>& h_steps) {
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&P, &w1, &w2}) {
    CHECK_DEV((*t));
    CHECK_DTYPE((*t), at::kDouble);
  }
  CHECK_DEV(steps);
  CHECK_DTYPE(steps, at::kInt);
  const int64_t S = P.size(0);
  TORCH_CHECK(P.dim() == 2 && P.size(1) == S && S >= 1 && S <= 64, "P must be [S, S], S <= 64");
  TORCH_CHECK(w1.dim() == 2 && w1.sizes() == w2.sizes(), "w1, w2 must be [B, ldw]");
  const int64_t B = w1.size(0), ldw = w1.size(1);
  TORCH_CHECK(steps.numel() == B && (int64_t)h_steps.size() == B, "steps must be [B]");
  for (int64_t s : h_steps) TORCH_CHECK(s >= 0 && s < ldw, "steps[b] must be in [0, ldw)");
  auto out = at::empty({B, 2, S, S}, P.options());
  DevGuard g(P.device());
  avk::uniformization(P.data_ptr<double>(), (int)S, w1.data_ptr<double>(), w2.data_ptr<double>(), steps.data_ptr<int>(),
                      (int)ldw, (int)B, out.data_ptr<double>(), cur_stream(P));
  return out;
}

// A int32 [n, Wa], B int32 [m, Wb] window ids (negative = invalid) -> int32 [n, m] match counts
at::Tensor dot_matrix(const at::Tensor& A, const at::Tensor& B) {
  CHECK_DEV(A);
  CHECK_DTYPE(A, at::kInt);
  CHECK_DEV(B);
  CHECK_DTYPE(B, at::kInt);
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2, "A [n, Wa], B [m, Wb]");
  const int64_t n = A.size(0), m = B.size(0);
  TORCH_CHECK(n < (1LL << 20) && m < (1LL << 31), "too many sequences");
  auto hits = at::empty({n, m}, A.options());
  if (n == 0 || m == 0) return hits;
  DevGuard g(A.device());
  avk::dot_matrix(A.data_ptr<int>(), (int)n, (int)A.size(1), B.data_ptr<int>(), (int)m, (int)B.size(1),
                  hits.data_ptr<int>(), cur_stream(A));
  return hits;
}

// ---- device-resident forest builder (forest.hip) ---------------------------------------------
// codes uint8 [F][ld], lab/wt uint8 [ld] on the device.  Work lists (slot/node int32, start int64,
// len int32, bases int64) are HOST tensors: they are bound-checked here on the CPU and copied to the
// device by the binding, so no chunk outside the row buffer can reach a kernel and no D2H read is
// needed for the check.
static const long long* i64p(const at::Tensor& t) { return reinterpret_cast<const long long*>(t.data_ptr<int64_t>()); }

static void check_host_items(const at::Tensor& node, const at::Tensor& start, const at::Tensor& len, int64_t ld,
                             int64_t n_nodes) {
  TORCH_CHECK(!node.is_cuda() && !start.is_cuda() && !len.is_cuda(), "work lists are host tensors");
  CHECK_DTYPE(node, at::kInt);
  CHECK_DTYPE(start, at::kLong);
  CHECK_DTYPE(len, at::kInt);
  const int64_t n = node.numel();
  TORCH_CHECK(start.numel() == n && len.numel() == n, "work list arrays differ in length");
  const auto node_c = node.contiguous(), start_c = start.contiguous(), len_c = len.contiguous();
  const int* nd = node_c.data_ptr<int>();
  const int64_t* st = start_c.data_ptr<int64_t>();
  const int* ln = len_c.data_ptr<int>();
  for (int64_t i = 0; i < n; ++i) {
    TORCH_CHECK(nd[i] >= 0 && nd[i] < n_nodes, "work item node / slot out of range");
    TORCH_CHECK(st[i] >= 0 && ln[i] >= 0 && st[i] + ln[i] <= ld, "work item outside the row buffer");
  }
}

static at::Tensor to_dev(const at::Tensor& t, const at::Tensor& like) {
  return t.contiguous().to(like.device(), /*non_blocking=*/true);
}

void forest_hist(const at::Tensor& codes, const at::Tensor& lab, const at::Tensor& wt, const at::Tensor& slot,
                 const at::Tensor& start, const at::Tensor& len, const at::Tensor& bins, const at::Tensor& offs,
                 int64_t TB, int64_t C, at::Tensor& hist) {
  CHECK_DEV(codes); CHECK_DTYPE(codes, at::kByte);
  CHECK_DEV(lab); CHECK_DTYPE(lab, at::kByte);
  CHECK_DEV(wt); CHECK_DTYPE(wt, at::kByte);
  CHECK_DEV(hist); CHECK_DTYPE(hist, at::kLong);
  CHECK_DEV(bins); CHECK_DEV(offs);
  const int64_t ld = codes.size(1), F = codes.size(0), n = slot.numel();
  TORCH_CHECK(lab.numel() >= ld && wt.numel() >= ld, "label / weight columns shorter than the code rows");
  TORCH_CHECK(ld % 8 == 0, "row buffers must be padded to a multiple of 8 rows (8-byte lane loads)");
  TORCH_CHECK(bins.numel() == F && offs.numel() == F, "bins / offs per feature");
  TORCH_CHECK(hist.dim() == 3 && hist.size(1) == C && hist.size(2) == TB, "hist [A, C, TB]");
  check_host_items(slot, start, len, ld, hist.size(0));
  if (n == 0) return;
  auto d_slot = to_dev(slot, codes), d_start = to_dev(start, codes), d_len = to_dev(len, codes);
  DevGuard g(codes.device());
  avk::forest_hist(codes.data_ptr<uint8_t>(), ld, lab.data_ptr<uint8_t>(), wt.data_ptr<uint8_t>(),
                   d_slot.data_ptr<int>(), i64p(d_start), d_len.data_ptr<int>(), (int)n, bins.data_ptr<int>(),
                   offs.data_ptr<int>(), (int)F, (int)TB, (int)C,
                   reinterpret_cast<unsigned long long*>(hist.data_ptr<int64_t>()), cur_stream(codes));
}

// X float32 [F, ldx] (rows 0..n), edges float32 concatenated (<= 254 per feature), eoff int32 [F+1]
// (host tensor, checked here) -> uint8 [F, ldo] codes (rows >= n untouched).
void bucketize_u8(const at::Tensor& X, int64_t n, const at::Tensor& edges, const at::Tensor& eoff, at::Tensor& out) {
  CHECK_DEV(X); CHECK_DTYPE(X, at::kFloat);
  CHECK_DEV(edges); CHECK_DTYPE(edges, at::kFloat);
  CHECK_DEV(out); CHECK_DTYPE(out, at::kByte);
  TORCH_CHECK(!eoff.is_cuda(), "eoff is a host tensor");
  CHECK_DTYPE(eoff, at::kInt);
  const int64_t F = X.size(0);
  TORCH_CHECK(eoff.numel() == F + 1 && out.size(0) == F && n <= X.size(1) && n <= out.size(1), "shapes");
  const auto eo = eoff.contiguous();
  const int* e = eo.data_ptr<int>();
  TORCH_CHECK(e[0] == 0 && e[F] == edges.numel(), "edge offsets");
  for (int64_t f = 0; f < F; ++f) TORCH_CHECK(e[f + 1] >= e[f] && e[f + 1] - e[f] <= 254, "at most 254 edges per feature");
  if (n == 0 || F == 0) return;
  auto d_eoff = eo.to(X.device());
  DevGuard g(X.device());
  avk::bucketize_u8(X.data_ptr<float>(), X.size(1), n, (int)F, edges.data_ptr<float>(), d_eoff.data_ptr<int>(),
                    out.data_ptr<uint8_t>(), out.size(1), cur_stream(X));
}

std::vector<at::Tensor> forest_split(const at::Tensor& hist, const at::Tensor& fmask, const at::Tensor& bins,
                                     const at::Tensor& offs, int64_t algo, int64_t topk, const at::Tensor& rnd) {
  CHECK_DEV(hist); CHECK_DTYPE(hist, at::kLong);
  CHECK_DEV(fmask); CHECK_DTYPE(fmask, at::kByte);
  CHECK_DEV(rnd); CHECK_DTYPE(rnd, at::kFloat);
  const int64_t A = hist.size(0), C = hist.size(1), TB = hist.size(2), F = bins.numel();
  TORCH_CHECK(fmask.size(0) == A && fmask.size(1) == F && rnd.numel() >= A, "fmask [A, F], rnd [A]");
  TORCH_CHECK(C <= 16, "forest_split: at most 16 classes");
  auto io = hist.options().dtype(at::kInt), fo = hist.options().dtype(at::kFloat);
  auto feat = at::empty({A}, io), thr = at::empty({A}, io);
  auto score = at::empty({A}, fo), imp = at::empty({A}, fo);
  auto left = at::empty({A, C}, hist.options());
  if (A > 0) {
    DevGuard g(hist.device());
    avk::forest_split(reinterpret_cast<const long long*>(hist.data_ptr<int64_t>()), fmask.data_ptr<uint8_t>(),
                      bins.data_ptr<int>(), offs.data_ptr<int>(), (int)F, (int)TB, (int)C, (int)algo, (int)topk,
                      rnd.data_ptr<float>(), (int)A, feat.data_ptr<int>(), thr.data_ptr<int>(), score.data_ptr<float>(),
                      imp.data_ptr<float>(), reinterpret_cast<long long*>(left.data_ptr<int64_t>()), cur_stream(hist));
  }
  return {feat, thr, score, imp, left};
}

at::Tensor forest_part_count(const at::Tensor& codes, const at::Tensor& node, const at::Tensor& start,
                             const at::Tensor& len, const at::Tensor& feat, const at::Tensor& thr) {
  CHECK_DEV(codes); CHECK_DTYPE(codes, at::kByte);
  CHECK_DEV(feat); CHECK_DTYPE(feat, at::kInt);
  CHECK_DEV(thr); CHECK_DTYPE(thr, at::kInt);
  check_host_items(node, start, len, codes.size(1), feat.numel());
  TORCH_CHECK(codes.size(1) % 8 == 0, "row buffers must be padded to a multiple of 8 rows");
  auto out = at::zeros({node.numel()}, feat.options());
  if (node.numel()) {
    auto d_node = to_dev(node, codes), d_start = to_dev(start, codes), d_len = to_dev(len, codes);
    DevGuard g(codes.device());
    avk::forest_part_count(codes.data_ptr<uint8_t>(), codes.size(1), d_node.data_ptr<int>(), i64p(d_start),
                           d_len.data_ptr<int>(), (int)node.numel(), feat.data_ptr<int>(), thr.data_ptr<int>(),
                           out.data_ptr<int>(), cur_stream(codes));
  }
  return out;
}

void forest_part_scatter(const at::Tensor& codes, const at::Tensor& lab, const at::Tensor& wt, at::Tensor& dcodes,
                         at::Tensor& dlab, at::Tensor& dwt, const at::Tensor& node, const at::Tensor& start,
                         const at::Tensor& len, const at::Tensor& left_base, const at::Tensor& right_base,
                         const at::Tensor& item_left, const at::Tensor& feat, const at::Tensor& thr) {
  CHECK_DEV(codes); CHECK_DTYPE(codes, at::kByte);
  CHECK_DEV(dcodes); CHECK_DTYPE(dcodes, at::kByte);
  CHECK_DEV(lab); CHECK_DEV(wt); CHECK_DEV(dlab); CHECK_DEV(dwt);
  TORCH_CHECK(!item_left.is_cuda(), "item_left (forest_part_count output) is a host tensor");
  CHECK_DTYPE(item_left, at::kInt);
  CHECK_DEV(feat); CHECK_DEV(thr);
  TORCH_CHECK(dcodes.sizes() == codes.sizes() && dlab.numel() == lab.numel() && dwt.numel() == wt.numel(),
              "destination buffers must match the source");
  const int64_t ld = codes.size(1);
  check_host_items(node, start, len, ld, feat.numel());
  TORCH_CHECK(ld % 8 == 0 && lab.numel() >= ld && wt.numel() >= ld, "row buffers padded to a multiple of 8 rows");
  TORCH_CHECK(!left_base.is_cuda() && !right_base.is_cuda(), "bases are host tensors");
  CHECK_DTYPE(left_base, at::kLong);
  CHECK_DTYPE(right_base, at::kLong);
  const int64_t n = node.numel();
  TORCH_CHECK(left_base.numel() == n && right_base.numel() == n && item_left.numel() == n, "one base per work item");
  {  // every chunk's destinations stay inside the buffer: [lb, lb + left) and [rb, rb + len - left)
    const auto lb_c = left_base.contiguous(), rb_c = right_base.contiguous(), len_c = len.contiguous();
    const auto il_c = item_left.contiguous();
    const int64_t* lb = lb_c.data_ptr<int64_t>();
    const int64_t* rb = rb_c.data_ptr<int64_t>();
    const int* ln = len_c.data_ptr<int>();
    const int* il = il_c.data_ptr<int>();
    for (int64_t i = 0; i < n; ++i)
      TORCH_CHECK(il[i] >= 0 && il[i] <= ln[i] && lb[i] >= 0 && rb[i] >= 0 && lb[i] + il[i] <= ld &&
                      rb[i] + (ln[i] - il[i]) <= ld,
                  "forest_part_scatter: destination outside the row buffer");
  }
  if (n == 0) return;
  auto d_node = to_dev(node, codes), d_start = to_dev(start, codes), d_len = to_dev(len, codes);
  auto d_lb = to_dev(left_base, codes), d_rb = to_dev(right_base, codes);
  DevGuard g(codes.device());
  avk::forest_part_scatter(codes.data_ptr<uint8_t>(), lab.data_ptr<uint8_t>(), wt.data_ptr<uint8_t>(),
                           dcodes.data_ptr<uint8_t>(), dlab.data_ptr<uint8_t>(), dwt.data_ptr<uint8_t>(), ld,
                           (int)codes.size(0), d_node.data_ptr<int>(), i64p(d_start), d_len.data_ptr<int>(), (int)n,
                           i64p(d_lb), i64p(d_rb), feat.data_ptr<int>(), thr.data_ptr<int>(), cur_stream(codes));
}

// Bootstrap row buffers of ``keys.numel()`` trees over the first n rows of codes [F, ld] / lab:
// returns (codes [F, ldb], labels [ldb], weights [ldb], rows per tree (host int64)), tree-major.
std::vector<at::Tensor> forest_bootstrap(const at::Tensor& codes, const at::Tensor& lab, int64_t n,
                                         const at::Tensor& keys, int64_t row_off, int64_t mode, int64_t rate32) {
  CHECK_DEV(codes); CHECK_DTYPE(codes, at::kByte);
  CHECK_DEV(lab); CHECK_DTYPE(lab, at::kByte);
  CHECK_DEV(keys); CHECK_DTYPE(keys, at::kLong);
  TORCH_CHECK(codes.dim() == 2 && codes.is_contiguous() && lab.is_contiguous() && keys.is_contiguous(),
              "contiguous codes [F, ld], labels, keys");
  const int64_t ld = codes.size(1), F = codes.size(0), T = keys.numel();
  TORCH_CHECK(ld % 8 == 0 && 0 <= n && n <= ld && lab.numel() >= ld, "row buffers padded to a multiple of 8 rows");
  TORCH_CHECK(0 <= mode && mode <= 2 && 0 <= rate32 && rate32 <= 0xFFFFFFFFLL && row_off >= 0, "bad sampling mode");
  TORCH_CHECK(T > 0 && T < 65536, "1..65535 trees");
  const int64_t tiles = std::max<int64_t>(1, (n + 2047) / 2048);
  auto iopt = codes.options().dtype(at::kInt);
  auto tile_cnt = at::zeros({T, tiles}, iopt);
  DevGuard g(codes.device());
  auto keysu = reinterpret_cast<const unsigned long long*>(keys.data_ptr<int64_t>());
  avk::forest_boot_count(keysu, (int)T, n, row_off, (int)mode, (unsigned)rate32, tile_cnt.data_ptr<int>(),
                         cur_stream(codes));
  auto flat = tile_cnt.view({-1}).to(at::kLong);
  auto incl = flat.cumsum(0);
  auto tile_off = (incl - flat).contiguous();
  auto per_tree = tile_cnt.sum(1, false, at::kLong).cpu();
  const int64_t R = per_tree.sum().item<int64_t>();
  const int64_t ldb = std::max<int64_t>(16, (R + 15) / 16 * 16);
  auto bopt = codes.options();
  auto cb = at::empty({F, ldb}, bopt), lb = at::empty({ldb}, bopt), wb = at::zeros({ldb}, bopt);
  avk::forest_boot_scatter(codes.data_ptr<uint8_t>(), ld, (int)F, lab.data_ptr<uint8_t>(), keysu, (int)T, n, row_off,
                           (int)mode, (unsigned)rate32, i64p(tile_off), cb.data_ptr<uint8_t>(), lb.data_ptr<uint8_t>(),
                           wb.data_ptr<uint8_t>(), ldb, cur_stream(codes));
  return {cb, lb, wb, per_tree};
}

// bf16 term-plane scratch of K27's large-shape split-bf16 path (undefined when not taken)
static at::Tensor k27_planes(const at::Tensor& like, long long M, long long N, long long K, int64_t prec) {
  const long long nb = avk::linear_act_fwd_planes_bytes((int)M, (int)N, (int)K, (int)prec);
  return nb > 0 ? at::empty({nb}, like.options().dtype(at::kByte)) : at::Tensor();
}
static void* ptr_or_null_t(const at::Tensor& t) { return t.defined() ? t.data_ptr() : nullptr; }

// K27: Y = act(X W^T + b) and its backward epilogue (dZ = dY * act'(Y), db = colsum dZ).
// W's bf16 term planes for linear_act_fwd(..., w_planes=) (None when the planes path is off for prec)
py::object sbf16_weight_planes(const at::Tensor& W, int64_t prec) {
  CHECK_DEV(W); CHECK_DTYPE(W, at::kFloat);
  TORCH_CHECK(W.dim() == 2 && W.size(0) < (1LL << 31) && W.size(1) < (1LL << 31), "W [N, K]");
  TORCH_CHECK(prec == -1 || prec == 0 || prec == 3 || prec == 6, "prec: -1 (default), 0, 3 or 6");
  const long long nb = avk::sbf16_weight_planes_bytes((int)W.size(0), (int)W.size(1), (int)prec);
  if (nb == 0) return py::none();
  auto Wc = W.contiguous();
  auto out = at::empty({nb}, W.options().dtype(at::kByte));
  DevGuard g(W.device());
  avk::sbf16_weight_planes(Wc.data_ptr<float>(), (int)W.size(0), (int)W.size(1), (int)prec, out.data_ptr(), cur_stream(W));
  return py::cast(out);
}

at::Tensor linear_act_fwd(const at::Tensor& X, const at::Tensor& W, const c10::optional<at::Tensor>& b, int64_t act,
                          int64_t prec, const c10::optional<at::Tensor>& w_planes) {
  TORCH_CHECK(prec == -1 || prec == 0 || prec == 3 || prec == 6, "prec: -1 (default), 0 (f32), 3 or 6 (split bf16)");
  CHECK_DEV(X); CHECK_DTYPE(X, at::kFloat);
  CHECK_DEV(W); CHECK_DTYPE(W, at::kFloat);
  TORCH_CHECK(X.dim() == 2 && W.dim() == 2 && X.size(1) == W.size(1), "X [M, K], W [N, K]");
  TORCH_CHECK(act >= 0 && act <= 6, "activation code 0..6 (6 = gelu, forward only)");
  TORCH_CHECK(X.size(0) < (1LL << 31) && W.size(0) < (1LL << 31) && X.size(1) < (1LL << 31), "dims < 2^31");
  auto Xc = X.contiguous(), Wc = W.contiguous();
  at::Tensor bc;
  if (b.has_value() && b->defined()) {
    CHECK_DEV((*b)); CHECK_DTYPE((*b), at::kFloat);
    TORCH_CHECK(b->numel() == W.size(0), "bias [N]");
    bc = b->contiguous();
  }
  auto Y = at::empty({X.size(0), W.size(0)}, X.options());
  DevGuard g(X.device());
  const int M = (int)X.size(0), N = (int)W.size(0), K = (int)X.size(1);
  const int S = avk::linear_act_fwd_slices(M, N, K);
  at::Tensor part, planes;
  if (S > 1) part = at::empty({(long long)S * M * N}, X.options());
  else planes = k27_planes(X, M, N, K, prec);
  const void* wp = nullptr;
  if (w_planes.has_value() && w_planes->defined()) {
    CHECK_DEV((*w_planes));
    TORCH_CHECK(w_planes->scalar_type() == at::kByte && w_planes->is_contiguous() &&
                    w_planes->numel() == avk::sbf16_weight_planes_bytes(N, K, (int)prec),
                "w_planes: sbf16_weight_planes(W, prec) of this W and prec");
    wp = w_planes->data_ptr();
  }
  avk::linear_act_fwd(Xc.data_ptr<float>(), Wc.data_ptr<float>(), bc.defined() ? bc.data_ptr<float>() : nullptr,
                      Y.data_ptr<float>(), M, N, K, (int)act, cur_stream(X), S > 1 ? part.data_ptr<float>() : nullptr, S,
                      (int)prec, ptr_or_null_t(planes), wp);
  return Y;
}

std::vector<at::Tensor> linear_act_bwd(const at::Tensor& dY, const at::Tensor& Y, int64_t act) {
  CHECK_DEV(dY); CHECK_DTYPE(dY, at::kFloat);
  CHECK_DEV(Y); CHECK_DTYPE(Y, at::kFloat);
  TORCH_CHECK(dY.sizes() == Y.sizes() && Y.dim() == 2, "dY and Y [M, N]");
  TORCH_CHECK(act >= 0 && act <= 5, "activation code 0..5");
  const int M = (int)Y.size(0), N = (int)Y.size(1);
  auto dYc = dY.contiguous(), Yc = Y.contiguous();
  auto dZ = at::empty_like(Yc);
  auto part = at::empty({std::max(1, avk::linear_act_bwd_blocks(M, N)), N}, Y.options());
  DevGuard g(Y.device());
  if (M == 0) part.zero_();
  avk::linear_act_bwd(dYc.data_ptr<float>(), Yc.data_ptr<float>(), dZ.data_ptr<float>(), part.data_ptr<float>(), M,
                      N, (int)act, cur_stream(Y));
  return {dZ, part.sum(0)};
}

// K27 fused backward of Y = act(X W^T + b): returns (dX | None, dW, db).  dW / db come from the
// fused weight-gradient kernel (dZ formed in-tile), dX = dZ W through the forward MFMA kernel
// (identity activation, W^T as its [K, N] operand).
py::tuple linear_act_backward(const at::Tensor& dY, const at::Tensor& Y, const at::Tensor& X, const at::Tensor& W,
                              int64_t act, bool need_dx) {
  CHECK_DEV(dY); CHECK_DTYPE(dY, at::kFloat);
  CHECK_DEV(Y); CHECK_DTYPE(Y, at::kFloat);
  CHECK_DEV(X); CHECK_DTYPE(X, at::kFloat);
  CHECK_DEV(W); CHECK_DTYPE(W, at::kFloat);
  TORCH_CHECK(Y.dim() == 2 && dY.sizes() == Y.sizes() && X.dim() == 2 && W.dim() == 2, "dY, Y [M, N], X [M, K], W [N, K]");
  TORCH_CHECK(X.size(0) == Y.size(0) && W.size(0) == Y.size(1) && W.size(1) == X.size(1), "shape mismatch");
  TORCH_CHECK(act >= 0 && act <= 5, "activation code 0..5");
  TORCH_CHECK(X.size(0) < (1LL << 31) && W.size(0) < (1LL << 31) && X.size(1) < (1LL << 31), "dims < 2^31");
  const int M = (int)Y.size(0), N = (int)Y.size(1), K = (int)X.size(1);
  auto dYc = dY.contiguous(), Yc = Y.contiguous(), Xc = X.contiguous();
  DevGuard g(Y.device());
  const int S = avk::linear_act_wgrad_slices(M, N, K);
  const int64_t E = (int64_t)N * K + N;
  auto pW = at::empty({S, E}, Y.options());
  auto tmp = at::empty({(S + 63) / 64, E}, Y.options());
  auto outv = at::empty({E}, Y.options());
  auto dW = outv.narrow(0, 0, (int64_t)N * K).view({N, K});
  auto db = outv.narrow(0, (int64_t)N * K, N);
  at::Tensor dZ;
  if (need_dx) dZ = at::empty({M, N}, Y.options());
  if (M == 0) {
    outv.zero_();
    return py::make_tuple(need_dx ? py::cast(at::zeros({0, K}, X.options())) : py::none(), dW, db);
  }
  hipStream_t st = cur_stream(Y);
  avk::linear_act_wgrad(dYc.data_ptr<float>(), Yc.data_ptr<float>(), Xc.data_ptr<float>(),
                        need_dx ? dZ.data_ptr<float>() : nullptr, pW.data_ptr<float>(), tmp.data_ptr<float>(),
                        outv.data_ptr<float>(), M, N, K, (int)act, st);
  if (!need_dx) return py::make_tuple(py::none(), dW, db);
  auto Wt = W.t().contiguous();  // [K, N]
  auto dX = at::empty({M, K}, X.options());
  auto planes = k27_planes(X, M, K, N, -1);
  avk::linear_act_fwd(dZ.data_ptr<float>(), Wt.data_ptr<float>(), nullptr, dX.data_ptr<float>(), M, K, N, 0, st,
                      nullptr, 1, -1, ptr_or_null_t(planes));
  return py::make_tuple(dX, dW, db);
}

// ---------------------------------------------------------------------------------------------
// K1 on the device (csv.hip): upload the file through a ring of pinned staging buffers (host
// copies from the page cache overlap the DMA of the previous slot), index the lines and parse
// every column on the GPU.  specs: the host parser's tuples (ordinal, kind, vocab, bucket_width,
// bucket_offset, max_code, wide); kinds CAT / BUCKET / FLOAT.  Returns (columns, rows, short rows).
#define BIND_HIP_CHECK(expr)                                                         \
  do {                                                                               \
    hipError_t _e = (expr);                                                          \
    TORCH_CHECK(_e == hipSuccess, #expr, " failed: ", hipGetErrorString(_e));        \
  } while (0)

// Pinned staging ring of the device uploads: one per device index (events belong to the device
// that was current when they were created), each behind a mutex so concurrent loads from several
// threads never share a slot; a call waits for every slot's last DMA before reusing it.
constexpr int SLOTS = 4;
constexpr int64_t SLOT = 64LL << 20;
struct StagingRing {
  std::mutex mu;
  void* buf[SLOTS] = {nullptr, nullptr, nullptr, nullptr};
  hipEvent_t done[SLOTS];
  hipStream_t side = nullptr;   // second DMA queue (AVMI_UPLOAD_STREAMS=2, default): odd slots copy on it
  hipEvent_t side_done = nullptr;
};

static int upload_streams() {  // default 2 (measured 30.6 -> 32.7 GB/s at 16 threads)
  const char* e = std::getenv("AVMI_UPLOAD_STREAMS");
  return (e && std::atoi(e) == 1) ? 1 : 2;
}

// DMA of slot k: on ``main`` or (two-queue mode, odd k) on the ring's side stream.
static void ring_dma(StagingRing& R, int slot, int64_t k, uint8_t* dst, int64_t len, hipStream_t main, int ns) {
  hipStream_t s = main;
  if (ns == 2 && (k & 1)) {
    if (!R.side) BIND_HIP_CHECK(hipStreamCreateWithFlags(&R.side, hipStreamNonBlocking));
    s = R.side;
  }
  BIND_HIP_CHECK(hipMemcpyAsync(dst, R.buf[slot], (size_t)len, hipMemcpyHostToDevice, s));
  BIND_HIP_CHECK(hipEventRecord(R.done[slot], s));
}

// the caller's stream waits for every side-stream copy of this upload
static void ring_join(StagingRing& R, hipStream_t main) {
  if (!R.side) return;
  if (!R.side_done) BIND_HIP_CHECK(hipEventCreateWithFlags(&R.side_done, hipEventDisableTiming));
  BIND_HIP_CHECK(hipEventRecord(R.side_done, R.side));
  BIND_HIP_CHECK(hipStreamWaitEvent(main, R.side_done, 0));
}

static StagingRing& staging_ring(int device) {
  static std::mutex reg_mu;
  static std::map<int, std::unique_ptr<StagingRing>> rings;
  std::lock_guard<std::mutex> g(reg_mu);
  auto& r = rings[device];
  if (!r) {
    r = std::make_unique<StagingRing>();
    for (int i = 0; i < SLOTS; ++i) {
      BIND_HIP_CHECK(hipHostMalloc(&r->buf[i], SLOT, hipHostMallocDefault));
      BIND_HIP_CHECK(hipEventCreateWithFlags(&r->done[i], hipEventDisableTiming));
      BIND_HIP_CHECK(hipEventRecord(r->done[i], nullptr));  // completed: the first wait returns at once
    }
  }
  return *r;
}

// Host threads filling one staging slot (AVMI_UPLOAD_THREADS, default 16, 1..32; MI355X box:
// 8 -> 16 threads took the 2.5 GB churn CSV load from 0.10 to 0.08 s, profiles/r3_csv_upload_sweep.jsonl).
static int upload_threads() {
  const char* e = std::getenv("AVMI_UPLOAD_THREADS");
  const int t = e ? std::atoi(e) : 16;
  return std::max(1, std::min(t, 32));
}

// AVMI_UPLOAD_MODE=mmap: copy from a mapping of the file (page faults on every source page);
// default pread: each thread reads its part of the slot straight into the pinned buffer.
static bool upload_pread() {
  const char* e = std::getenv("AVMI_UPLOAD_MODE");
  return !(e && std::string(e) == "mmap");
}

// Persistent host workers for the staging fills (a fill of 64 MB used to spawn and join 16 threads,
// ~15 us each, for every slot).  run(T, fn) calls fn(0..T-1), part 0 on the caller, and returns when
// all parts are done.  The pool is never destroyed (no join at interpreter exit).
class FillPool {
 public:
  static FillPool& get() {  // a forked child has none of the parent's workers: it gets its own pool
    static std::mutex m;
    static FillPool* p = nullptr;
    static pid_t owner = 0;
    std::lock_guard<std::mutex> g(m);
    if (!p || owner != ::getpid()) {
      p = new FillPool();
      owner = ::getpid();
    }
    return *p;
  }
  void run(int T, const std::function<void(int)>& fn) {
    std::unique_lock<std::mutex> call(call_mu_);  // one parallel fill at a time
    while ((int)workers_.size() < T - 1) workers_.emplace_back([this, id = (int)workers_.size() + 1] { loop(id); });
    {
      std::lock_guard<std::mutex> g(mu_);
      fn_ = &fn;
      parts_ = T;
      pending_ = T - 1;
      ++gen_;
    }
    cv_.notify_all();
    fn(0);
    std::unique_lock<std::mutex> g(mu_);
    done_cv_.wait(g, [this] { return pending_ == 0; });
    fn_ = nullptr;
  }

 private:
  void loop(int id) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* f;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return gen_ != seen; });
        seen = gen_;
        if (id >= parts_) continue;
        f = fn_;
      }
      (*f)(id);
      std::lock_guard<std::mutex> g(mu_);
      if (--pending_ == 0) done_cv_.notify_one();
    }
  }
  std::mutex call_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::thread> workers_;
  const std::function<void(int)>* fn_ = nullptr;
  int parts_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
};

// bytes [off, off + len) of fd into dst with T threads; pread may return short counts
static void pread_parallel(int fd, char* dst, int64_t off, int64_t len, int T) {
  std::atomic<bool> bad{false};
  std::function<void(int)> part = [&](int t) {
    int64_t a = len * t / T;
    const int64_t b = len * (t + 1) / T;
    while (a < b) {
      const ssize_t r = ::pread(fd, dst + a, (size_t)(b - a), (off_t)(off + a));
      if (r <= 0) { bad = true; return; }
      a += r;
    }
  };
  FillPool::get().run(T, part);
  TORCH_CHECK(!bad, "pread failed during the device upload");
}

static uint32_t fnv1a_fold(const std::string& v) {
  uint32_t h = 2166136261u;
  for (unsigned char c : v) h = (h ^ c) * 16777619u;
  return h ^ (h >> 15);
}

py::object csv_parse_device(const std::string& path, py::list specs_py, const std::string& delim, bool skip_header,
                           int64_t rank, int64_t world, const at::Tensor& like) {
  CHECK_DEV(like);
  TORCH_CHECK(delim.size() == 1, "device CSV parse: single-character delimiter");
  int fd = ::open(path.c_str(), O_RDONLY);
  TORCH_CHECK(fd >= 0, "cannot open ", path);
  struct stat st;
  TORCH_CHECK(fstat(fd, &st) == 0, "cannot stat ", path);
  const int64_t size = (int64_t)st.st_size;
  const int64_t padded = std::max<int64_t>(16, (size + 15) / 16 * 16);
  auto dopt = like.options().dtype(at::kByte);
  auto dev = at::empty({padded}, dopt);
  DevGuard g(like.device());
  hipStream_t stream = cur_stream(like);
  if (padded > size) BIND_HIP_CHECK(hipMemsetAsync(dev.data_ptr<uint8_t>() + size, 0, padded - size, stream));
  if (size > 0) {
    py::gil_scoped_release rel;
    const bool use_pread = upload_pread();
    const int T = upload_threads();
    const int NS = upload_streams();
    const char* map = nullptr;
    if (!use_pread) {
      map = static_cast<const char*>(mmap(nullptr, (size_t)size, PROT_READ, MAP_PRIVATE, fd, 0));
      TORCH_CHECK(map != MAP_FAILED, "mmap failed for ", path);
      madvise(const_cast<char*>(map), (size_t)size, MADV_SEQUENTIAL);
    }
    StagingRing& R = staging_ring(like.device().index());
    std::lock_guard<std::mutex> hold(R.mu);  // one upload at a time per device ring
    void** ring = R.buf;
    hipEvent_t* done = R.done;
    // a previous call's last DMAs may still read the slots (they ran on that call's stream)
    for (int i = 0; i < SLOTS; ++i) BIND_HIP_CHECK(hipEventSynchronize(done[i]));
    int64_t k = 0;
    // pieces grow 8, 16, 32, 64 MB: the first DMA starts after an 8 MB fill instead of a 64 MB one
    int64_t len = 0;
    for (int64_t off = 0; off < size; off += len, ++k) {
      const int slot = (int)(k % SLOTS);
      len = std::min(std::min(SLOT, (int64_t)(8LL << 20) << std::min<int64_t>(k, 3)), size - off);
      if (k >= SLOTS) BIND_HIP_CHECK(hipEventSynchronize(done[slot]));  // the slot's last DMA is done
      if (use_pread) {  // page cache -> pinned slot, T threads, no source page faults
        pread_parallel(fd, static_cast<char*>(ring[slot]), off, len, T);
      } else {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
          th.emplace_back([&, t] {
            const int64_t a = len * t / T, b = len * (t + 1) / T;
            std::memcpy(static_cast<char*>(ring[slot]) + a, map + off + a, (size_t)(b - a));
          });
        for (auto& x : th) x.join();
      }
      ring_dma(R, slot, k, dev.data_ptr<uint8_t>() + off, len, stream, NS);
    }
    ring_join(R, stream);
    if (map) munmap(const_cast<char*>(map), (size_t)size);
  }
  ::close(fd);
  // ---- line index ----
  const int64_t nch = std::max<int64_t>(1, avk::csv_chunks(size));
  auto counts = at::zeros({nch}, like.options().dtype(at::kInt));
  avk::csv_newline_counts(dev.data_ptr<uint8_t>(), size, reinterpret_cast<unsigned*>(counts.data_ptr<int>()), stream);
  auto c64 = counts.to(at::kLong);
  auto incl = c64.cumsum(0);
  auto offsets = (incl - c64).contiguous();
  const int64_t nl = size > 0 ? incl[-1].item<int64_t>() : 0;
  uint8_t last = '\n';
  if (size > 0) BIND_HIP_CHECK(hipMemcpy(&last, dev.data_ptr<uint8_t>() + size - 1, 1, hipMemcpyDeviceToHost));
  const bool tail = size > 0 && last != '\n';
  auto pos = at::empty({nl + (tail ? 1 : 0)}, like.options().dtype(at::kLong));
  if (nl) avk::csv_newline_positions(dev.data_ptr<uint8_t>(), size, reinterpret_cast<long long*>(offsets.data_ptr<int64_t>()),
                                     reinterpret_cast<long long*>(pos.data_ptr<int64_t>()), stream);
  if (tail) pos.narrow(0, nl, 1).fill_(size);
  // line bounds + blank-line flags in one pass; blank lines (empty after dropping a trailing CR)
  // are skipped, as in the host parser (compaction only when some exist)
  const int64_t nlines = pos.numel();
  auto starts = at::empty({nlines}, pos.options());
  auto ends = at::empty({nlines}, pos.options());
  if (nlines) {
    auto keep = at::empty({nlines}, pos.options().dtype(at::kByte));
    auto blank = at::zeros({1}, pos.options());
    avk::csv_line_bounds(dev.data_ptr<uint8_t>(), reinterpret_cast<const long long*>(pos.data_ptr<int64_t>()), nlines,
                         reinterpret_cast<long long*>(starts.data_ptr<int64_t>()),
                         reinterpret_cast<long long*>(ends.data_ptr<int64_t>()), keep.data_ptr<uint8_t>(),
                         reinterpret_cast<unsigned long long*>(blank.data_ptr<int64_t>()), stream);
    if (blank.item<int64_t>() > 0) {
      auto idx = at::nonzero(keep).view({-1});
      starts = starts.index({idx});
      ends = ends.index({idx});
    }
  }
  if (skip_header && starts.numel()) {
    starts = starts.narrow(0, 1, starts.numel() - 1);
    ends = ends.narrow(0, 1, ends.numel() - 1);
  }
  const int64_t total = starts.numel();
  TORCH_CHECK(world >= 1 && rank >= 0 && rank < world, "bad rank / world");
  // this rank's contiguous balanced row range (data/table.py shard_range)
  const int64_t base = total / world, rem = total % world;
  const int64_t row_begin = rank * base + std::min(rank, rem);
  const int64_t n = base + (rank < rem ? 1 : 0);
  starts = starts.narrow(0, row_begin, n).contiguous();
  ends = ends.narrow(0, row_begin, n).contiguous();
  // ---- specs, vocabulary tables, outputs ----
  const int64_t ld = std::max<int64_t>(16, (n + 15) / 16 * 16);
  struct HostSpec {
    int ordinal, kind, wide, max_code, bucket_offset, tab_off, tab_mask, vbase;
    double bucket_width;
    unsigned long long out;
  };
  TORCH_CHECK(avk::csv_devspec_bytes() == (int)sizeof(HostSpec), "DevSpec layout mismatch");
  std::vector<HostSpec> hs;
  std::vector<int> tabs, voff, vlen;
  std::string vbytes;
  std::vector<at::Tensor> outs;
  std::vector<std::pair<int, int>> order;  // (ordinal, spec index) to sort by ordinal
  int idx = 0;
  for (auto item : specs_py) {
    auto t = item.cast<py::tuple>();
    HostSpec sp{};
    sp.ordinal = t[0].cast<int>();
    sp.kind = t[1].cast<int>();
    auto vocab = t[2].cast<std::vector<std::string>>();
    sp.bucket_width = t[3].cast<double>();
    sp.bucket_offset = t[4].cast<int>();
    sp.max_code = t[5].cast<int>();
    const int width = t.size() > 6 ? t[6].cast<int>() : 0;
    TORCH_CHECK(width <= 1, "device CSV parse: int32 codes take the host parser");
    sp.wide = width >= 1 ? 1 : 0;
    TORCH_CHECK(sp.ordinal >= 0 && sp.kind >= 0 && sp.kind <= 2, "device CSV parse: CAT / BUCKET / FLOAT columns");
    if (sp.kind == 1) TORCH_CHECK(sp.bucket_width > 0, "bucket width must be > 0");
    at::Tensor o;
    if (sp.kind == 2) {
      o = at::empty({std::max<int64_t>(n, 1)}, like.options().dtype(at::kFloat));
    } else {
      o = sp.wide ? at::full({ld}, 65535, like.options().dtype(at::kUInt16)) : at::full({ld}, 255, dopt);
    }
    sp.out = reinterpret_cast<unsigned long long>(o.data_ptr());
    if (sp.kind == 0) {
      TORCH_CHECK(vocab.size() <= (sp.wide ? 65535u : 255u), "categorical cardinality exceeds the code width");
      size_t sz = 16;
      while (sz < 2 * vocab.size()) sz <<= 1;
      sp.tab_off = (int)tabs.size();
      sp.tab_mask = (int)sz - 1;
      sp.vbase = (int)voff.size();
      tabs.resize(tabs.size() + sz, -1);
      for (size_t i = 0; i < vocab.size(); ++i) {
        uint32_t h = fnv1a_fold(vocab[i]) & (uint32_t)(sz - 1);
        bool dup = false;
        while (tabs[sp.tab_off + h] >= 0) {
          if (vocab[(size_t)tabs[sp.tab_off + h]] == vocab[i]) { dup = true; break; }
          h = (h + 1) & (uint32_t)(sz - 1);
        }
        if (!dup) tabs[sp.tab_off + h] = (int)i;
      }
      for (auto& v : vocab) {
        voff.push_back((int)vbytes.size());
        vlen.push_back((int)v.size());
        vbytes += v;
      }
    }
    hs.push_back(sp);
    outs.push_back(o);
    order.push_back({sp.ordinal, idx++});
  }
  std::stable_sort(order.begin(), order.end());
  auto hopt = at::TensorOptions().dtype(at::kByte);
  auto to_i32 = [&](const std::vector<int>& v) {
    auto t = at::empty({(int64_t)std::max<size_t>(1, v.size())}, at::TensorOptions().dtype(at::kInt));
    if (!v.empty()) std::memcpy(t.data_ptr<int>(), v.data(), v.size() * sizeof(int));
    return t.to(like.device());
  };
  auto tabs_d = to_i32(tabs), voff_d = to_i32(voff), vlen_d = to_i32(vlen);
  auto vb_h = at::empty({(int64_t)std::max<size_t>(1, vbytes.size())}, hopt);
  if (!vbytes.empty()) std::memcpy(vb_h.data_ptr<uint8_t>(), vbytes.data(), vbytes.size());
  auto vb_d = vb_h.to(like.device());
  auto bad = at::zeros({1}, like.options().dtype(at::kLong));
  auto bad_scratch = at::zeros({1}, like.options().dtype(at::kLong));
  // wide schemas in passes of up to 64 columns (ordinal order): each pass walks a row only up to
  // its last column; short rows are counted by the pass holding the largest ordinal
  constexpr size_t GROUP = 64;
  const size_t ng = (order.size() + GROUP - 1) / GROUP;
  for (size_t g0 = 0; g0 < order.size(); g0 += GROUP) {
    std::vector<HostSpec> sorted;
    int max_ord = 0;
    for (size_t k = g0; k < std::min(order.size(), g0 + GROUP); ++k) {
      sorted.push_back(hs[(size_t)order[k].second]);
      max_ord = std::max(max_ord, order[k].first);
    }
    auto spec_h = at::empty({(int64_t)(sorted.size() * sizeof(HostSpec))}, hopt);
    std::memcpy(spec_h.data_ptr<uint8_t>(), sorted.data(), sorted.size() * sizeof(HostSpec));
    auto spec_d = spec_h.to(like.device());
    const bool last_group = g0 / GROUP == ng - 1;
    avk::csv_parse_rows(dev.data_ptr<uint8_t>(), dev.numel(), reinterpret_cast<const long long*>(starts.data_ptr<int64_t>()),
                        reinterpret_cast<const long long*>(ends.data_ptr<int64_t>()), n, delim[0], spec_d.data_ptr<uint8_t>(),
                        (int)sorted.size(), max_ord, tabs_d.data_ptr<int>(), voff_d.data_ptr<int>(), vlen_d.data_ptr<int>(),
                        vb_d.data_ptr<uint8_t>(), (int)tabs_d.numel(), (int)vlen_d.numel(), (int)vbytes.size(),
                        reinterpret_cast<unsigned long long*>((last_group ? bad : bad_scratch).data_ptr<int64_t>()),
                        stream);
  }
  // a token of > 19 significant digits the device could not round for certain: the caller
  // re-parses the file on the host (strtod), so both paths keep giving the same bits
  if (avk::csv_slow_tokens_take(stream) != 0) return py::none();
  py::list cols;
  for (auto& o : outs) cols.append(o);
  // the rows' byte spans in the file (raw-line output of the jobs: data/lines.py)
  // plus the uploaded file bytes: the device output formatter (format.hip) copies raw lines from them
  return py::make_tuple(cols, n, bad, total, row_begin, starts, ends, dev);
}

// K18 GSP self-join: X int32 [N, k] lexicographically sorted unique k-sequences; left rows [lo, hi)
// are joined with every row whose (k-1)-prefix equals their (k-1)-suffix -> int32 [M, k+1].
at::Tensor gsp_join(const at::Tensor& X, int64_t lo, int64_t hi) {
  CHECK_DEV(X);
  CHECK_DTYPE(X, at::kInt);
  TORCH_CHECK(X.dim() == 2 && X.size(1) >= 2, "X [N, k], k >= 2");
  const int64_t N = X.size(0), k = X.size(1);
  TORCH_CHECK(N < (1LL << 31) && 0 <= lo && lo <= hi && hi <= N, "bad left range");
  const int64_t n = hi - lo;
  auto opt = X.options();
  if (n == 0) return at::empty({0, k + 1}, opt);
  DevGuard g(X.device());
  auto start = at::empty({n}, opt);
  auto len = at::empty({n}, opt);
  avk::gsp_count(X.data_ptr<int>(), (int)N, (int)k, (int)lo, (int)hi, start.data_ptr<int>(), len.data_ptr<int>(),
                 cur_stream(X));
  auto len64 = len.to(at::kLong);
  auto incl = at::cumsum(len64, 0);
  const int64_t M = incl[n - 1].item<int64_t>();
  auto offs = (incl - len64).contiguous();
  auto out = at::empty({M, k + 1}, opt);
  if (M > 0)
    avk::gsp_emit(X.data_ptr<int>(), (int)k, (int)lo, (int)hi, start.data_ptr<int>(), len.data_ptr<int>(),
                  reinterpret_cast<const long long*>(offs.data_ptr<int64_t>()), out.data_ptr<int>(), cur_stream(X));
  return out;
}

// K26 column moments of a column-major [F, ld] float32 / float64 matrix over its first n rows.
// Returns double [F, 8]: count (non-NaN), sum, min, max, m2, m3, m4 (central power sums / count),
// mean.  Two streaming passes; partials reduced with a fixed-shape sum (reproducible).
at::Tensor col_moments(const at::Tensor& X, int64_t n) {
  CHECK_DEV(X);
  TORCH_CHECK(X.dim() == 2 && n >= 1 && n <= X.size(1), "X [F, ld], 1 <= n <= ld");
  const bool f32 = X.scalar_type() == at::kFloat;
  TORCH_CHECK(f32 || X.scalar_type() == at::kDouble, "X must be float32 or float64");
  const int64_t F = X.size(0), ld = X.size(1);
  TORCH_CHECK(F >= 1 && F < 65536, "1 <= F < 65536 columns");
  if (f32) TORCH_CHECK(ld % 4 == 0 && aligned(X, 16), "float32 X needs ld % 4 == 0 and 16-byte alignment");
  DevGuard g(X.device());
  const int nb = avk::col_moments_blocks(n, (int)F);
  auto opt = X.options().dtype(at::kDouble);
  auto p0 = at::empty({F, nb, 4}, opt);
  auto p1 = at::empty({F, nb, 4}, opt);
  auto st = cur_stream(X);
  if (f32) avk::col_moments_f32(X.data_ptr<float>(), n, ld, (int)F, 0, nullptr, p0.data_ptr<double>(), st);
  else avk::col_moments_f64(X.data_ptr<double>(), n, ld, (int)F, 0, nullptr, p0.data_ptr<double>(), st);
  auto cnt = p0.select(2, 0).sum(1), sm = p0.select(2, 1).sum(1);
  auto lo = std::get<0>(p0.select(2, 2).min(1)), hi = std::get<0>(p0.select(2, 3).max(1));
  auto mean = (sm / cnt.clamp_min(1.0)).contiguous();
  if (f32) avk::col_moments_f32(X.data_ptr<float>(), n, ld, (int)F, 1, mean.data_ptr<double>(), p1.data_ptr<double>(), st);
  else avk::col_moments_f64(X.data_ptr<double>(), n, ld, (int)F, 1, mean.data_ptr<double>(), p1.data_ptr<double>(), st);
  auto c1 = cnt.clamp_min(1.0);
  auto m2 = p1.select(2, 0).sum(1) / c1, m3 = p1.select(2, 1).sum(1) / c1, m4 = p1.select(2, 2).sum(1) / c1;
  return at::stack({cnt, sm, lo, hi, m2, m3, m4, mean}, 1);
}

// K23 leave-one-out statistics: codes [F, ld] uint8 (m = 256) or uint16 (m = 65536), y double [n]
// -> (sum double [F, m], count int32 [F, m]) over the first n rows.
static int64_t loo_slots(const at::Tensor& codes, int64_t slots) {
  if (codes.scalar_type() == at::kInt) {
    TORCH_CHECK(slots >= 2 && slots <= (1LL << 30), "int32 codes: slots (max code + 2) in [2, 2^30]");
    return slots;
  }
  TORCH_CHECK(codes.scalar_type() == at::kUInt16 || codes.scalar_type() == at::kByte,
              "codes must be uint8, uint16 or int32");
  if (codes.scalar_type() == at::kUInt16) {
    // uint16: the table may be cut to the used values (codes >= slots - 1 land in the last slot)
    TORCH_CHECK(slots <= 0 || (slots >= 2 && slots <= 65536), "uint16 codes: slots in [2, 65536]");
    return slots > 0 ? slots : 65536;
  }
  return 256;
}

py::tuple loo_stats(const at::Tensor& codes, int64_t n, const at::Tensor& y, int64_t slots) {
  CHECK_DEV(codes);
  CHECK_DEV(y);
  CHECK_DTYPE(y, at::kDouble);
  TORCH_CHECK(codes.dim() == 2 && n >= 0 && n <= codes.size(1) && y.numel() >= n, "codes [F, ld], y [>= n]");
  const int64_t F = codes.size(0), m = loo_slots(codes, slots);
  const int cb = (int)codes.element_size();
  TORCH_CHECK(F >= 1 && F < 65536, "1 <= F < 65536 columns");
  DevGuard g(codes.device());
  auto sum = at::zeros({F, m}, y.options());
  auto cnt = at::zeros({F, m}, codes.options().dtype(at::kInt));
  if (n > 0)
    avk::loo_stats(codes.data_ptr(), cb, (int)m, codes.size(1), n, (int)F, y.data_ptr<double>(), sum.data_ptr<double>(),
                   reinterpret_cast<unsigned*>(cnt.data_ptr<int>()), cur_stream(codes));
  return py::make_tuple(sum, cnt);
}

// K23 leave-one-out apply -> float32 [n, F] (row-major); noise double [F, n] uniforms or undefined.
at::Tensor loo_apply(const at::Tensor& codes, int64_t n, const at::Tensor& y, const at::Tensor& sum,
                     const at::Tensor& cnt, const at::Tensor& gmean, double reg,
                     const c10::optional<at::Tensor>& noise, double amp, int64_t slots) {
  CHECK_DEV(codes);
  CHECK_DEV(y);
  CHECK_DEV(sum);
  CHECK_DEV(cnt);
  CHECK_DEV(gmean);
  CHECK_DTYPE(y, at::kDouble);
  CHECK_DTYPE(sum, at::kDouble);
  CHECK_DTYPE(cnt, at::kInt);
  CHECK_DTYPE(gmean, at::kDouble);
  const int64_t F = codes.size(0), m = loo_slots(codes, slots);
  const int cb = (int)codes.element_size();
  TORCH_CHECK(codes.dim() == 2 && n >= 0 && n <= codes.size(1) && y.numel() >= n, "codes [F, ld], y [>= n]");
  TORCH_CHECK(sum.numel() == F * m && cnt.numel() == F * m && gmean.numel() >= 1, "stats tables [F, m]");
  TORCH_CHECK((n + 255) / 256 < (1LL << 31), "too many rows");
  const double* nz = nullptr;
  if (noise.has_value() && noise->defined()) {
    CHECK_DEV((*noise));
    CHECK_DTYPE((*noise), at::kDouble);
    TORCH_CHECK(noise->numel() == F * n, "noise [F, n]");
    nz = noise->data_ptr<double>();
  }
  DevGuard g(codes.device());
  auto out = at::empty({n, F}, y.options().dtype(at::kFloat));
  if (n > 0)
    avk::loo_apply(codes.data_ptr(), cb, (int)m, codes.size(1), n, (int)F, y.data_ptr<double>(), sum.data_ptr<double>(),
                   reinterpret_cast<const unsigned*>(cnt.data_ptr<int>()), gmean.data_ptr<double>(), reg, nz, amp,
                   out.data_ptr<float>(), cur_stream(codes));
  return out;
}

// K24 streaming PCA: advances every key's state (W [K, H, D], E / he [K, H], ve / cnt [K], nh int32
// [K]) over its stream X [K, T, D] (first lens[k] records), in place.
void spirit_update(const at::Tensor& X, const at::Tensor& lens, at::Tensor W, at::Tensor E, at::Tensor he,
                   at::Tensor ve, at::Tensor cnt, at::Tensor nh, double lam, double lo, double hi) {
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&X, &W, &E, &he, &ve, &cnt}) {
    CHECK_DEV((*t));
    CHECK_DTYPE((*t), at::kDouble);
  }
  CHECK_DEV(lens);
  CHECK_DEV(nh);
  CHECK_DTYPE(lens, at::kInt);
  CHECK_DTYPE(nh, at::kInt);
  TORCH_CHECK(X.dim() == 3 && W.dim() == 3, "X [K, T, D], W [K, H, D]");
  const int64_t K = X.size(0), T = X.size(1), D = X.size(2), H = W.size(1);
  TORCH_CHECK(D >= 1 && D <= 64 && H >= 1 && H <= D, "spirit kernel: 1 <= H <= D <= 64");
  TORCH_CHECK(W.size(0) == K && W.size(2) == D && E.numel() == K * H && he.numel() == K * H && ve.numel() == K &&
                  cnt.numel() == K && nh.numel() == K && lens.numel() == K, "state shapes");
  if (K == 0) return;
  // host copies bound-check the per-key lengths and unit counts before the launch
  auto lh = lens.cpu(), nhh = nh.cpu();
  TORCH_CHECK(lh.min().item<int>() >= 0 && lh.max().item<int>() <= T, "lens in [0, T]");
  TORCH_CHECK(nhh.min().item<int>() >= 1 && nhh.max().item<int>() <= H, "nh in [1, H]");
  DevGuard g(X.device());
  avk::spirit_update(X.data_ptr<double>(), (int)K, (int)T, (int)D, (int)H, lens.data_ptr<int>(), W.data_ptr<double>(),
                     E.data_ptr<double>(), he.data_ptr<double>(), ve.data_ptr<double>(), cnt.data_ptr<double>(),
                     nh.data_ptr<int>(), lam, lo, hi, cur_stream(X));
}

// ---------------------------------------------------------------------------------------------
// host runtime

// ---------------------------------------------------------------------------------------------
// specs: list of (ordinal, kind, vocab, bucket_width, bucket_offset, max_code).  Returns one
// CPU tensor per spec: uint8 [ld] for CAT/BUCKET (ld = n rounded up to 16, padding = 255),
// float32 [n] for FLOAT, int64 [n] for INT; plus the malformed-row count.
py::tuple csv_parse(avh::CsvFile& f, py::list specs_py, int64_t row_begin, int64_t row_end) {
  std::vector<avh::ColSpec> specs;
  for (auto item : specs_py) {
    auto t = item.cast<py::tuple>();
    avh::ColSpec s;
    s.ordinal = t[0].cast<int>();
    s.kind = t[1].cast<int>();
    s.vocab = t[2].cast<std::vector<std::string>>();
    s.bucket_width = t[3].cast<double>();
    s.bucket_offset = t[4].cast<int>();
    s.max_code = t[5].cast<int>();
    if (t.size() > 6) {  // code width: 0 / False uint8, 1 / True uint16, 2 int32 (CAT only)
      const int w = t[6].cast<int>();
      s.wide = w >= 1;
      s.huge = w >= 2;
      TORCH_CHECK(!s.huge || s.kind == avh::CAT, "int32 codes are for categorical columns");
    }
    TORCH_CHECK(s.ordinal >= 0, "negative ordinal");
    if (s.kind == avh::BUCKET) TORCH_CHECK(s.bucket_width > 0, "bucket width must be > 0");
    specs.push_back(std::move(s));
  }
  row_begin = std::max<int64_t>(0, row_begin);
  if (row_end < 0 || row_end > f.num_rows()) row_end = f.num_rows();
  const int64_t n = std::max<int64_t>(0, row_end - row_begin);
  const int64_t ld = ((n + 15) / 16) * 16;
  std::vector<at::Tensor> outs;
  std::vector<void*> ptrs;
  for (auto& s : specs) {
    at::Tensor t;
    if (s.kind == avh::CAT && s.huge)
      t = at::full({std::max<int64_t>(ld, 16)}, 0x7FFFFFFF, at::TensorOptions().dtype(at::kInt));
    else if ((s.kind == avh::CAT || s.kind == avh::BUCKET) && s.wide)
      t = at::full({std::max<int64_t>(ld, 16)}, 65535, at::TensorOptions().dtype(at::kUInt16));
    else if (s.kind == avh::CAT || s.kind == avh::BUCKET)
      t = at::full({std::max<int64_t>(ld, 16)}, 255, at::TensorOptions().dtype(at::kByte));
    else if (s.kind == avh::FLOAT)
      t = at::empty({n}, at::TensorOptions().dtype(at::kFloat));
    else
      t = at::empty({n}, at::TensorOptions().dtype(at::kLong));
    ptrs.push_back(t.data_ptr());
    outs.push_back(t);
  }
  int64_t bad;
  {
    py::gil_scoped_release rel;
    bad = f.parse(specs, ptrs, row_begin, row_end);
  }
  py::list res;
  for (auto& t : outs) res.append(t);
  return py::make_tuple(res, bad);
}

std::string format_rows(py::object prefix, const at::Tensor& cols, std::vector<int> precision,
                        std::string delim, int nthreads) {
  TORCH_CHECK(!cols.is_cuda() && cols.scalar_type() == at::kDouble && cols.dim() == 2,
              "cols must be CPU float64 [ncol, n]");
  auto c = cols.contiguous();
  std::vector<std::string> pre;
  const std::vector<std::string>* pp = nullptr;
  if (!prefix.is_none()) {
    pre = prefix.cast<std::vector<std::string>>();
    TORCH_CHECK((int64_t)pre.size() == c.size(1), "prefix length != n");
    pp = &pre;
  }
  py::gil_scoped_release rel;
  return avh::format_rows(pp, c.data_ptr<double>(), (int)c.size(0), c.size(1), precision,
                          delim.empty() ? ',' : delim[0], nthreads);
}

// TextShard tokenizer (records.cpp): returns (off int64 [L+1], codes int32 [T], sub int32 [T] or None,
// nums float64 [T] or None, vocab list[str]).
py::tuple text_tokenize(avh::TextShard& sh, const std::string& delims, const std::string& sub_delim,
                        const std::string& modes, const std::string& tail_mode, bool trim, bool want_nums,
                        const std::string& last_mode) {
  TORCH_CHECK(sub_delim.size() <= 1 && tail_mode.size() == 1 && last_mode.size() <= 1,
              "sub_delim / last_mode: 0/1 char, tail_mode: 1 char");
  for (char c : modes + tail_mode + last_mode) TORCH_CHECK(c == 'd' || c == 'n' || c == 'x', "token modes are d / n / x");
  avh::TokenSpec sp;
  sp.delims = delims.empty() ? std::string(",") : delims;
  sp.sub_delim = sub_delim.empty() ? 0 : sub_delim[0];
  sp.modes = modes;
  sp.tail_mode = tail_mode[0];
  sp.trim = trim;
  sp.last_mode = last_mode.empty() ? 0 : last_mode[0];
  const int64_t L = sh.num_lines();
  int64_t T;
  {
    py::gil_scoped_release rel;
    T = sh.count_tokens(sp);
  }
  auto o = at::TensorOptions();
  auto off = at::empty({L + 1}, o.dtype(at::kLong));
  auto codes = at::empty({T}, o.dtype(at::kInt));
  at::Tensor sub, nums;
  if (sp.sub_delim) sub = at::empty({T}, o.dtype(at::kInt));
  if (want_nums) nums = at::empty({T}, o.dtype(at::kDouble));
  {
    py::gil_scoped_release rel;
    sh.tokenize(off.data_ptr<int64_t>(), codes.data_ptr<int32_t>(), sub.defined() ? sub.data_ptr<int32_t>() : nullptr,
                nums.defined() ? nums.data_ptr<double>() : nullptr);
  }
  py::object subo = sub.defined() ? py::cast(sub) : py::none();
  py::object numo = nums.defined() ? py::cast(nums) : py::none();
  return py::make_tuple(off, codes, subo, numo, sh.vocab());
}

std::vector<std::string> text_field_strings(const avh::TextShard& sh, const at::Tensor& line, const at::Tensor& field) {
  TORCH_CHECK(!line.is_cuda() && !field.is_cuda() && line.numel() == field.numel(), "CPU line / field index tensors");
  auto l = line.to(at::kLong).contiguous();
  auto f = field.to(at::kInt).contiguous();
  py::gil_scoped_release rel;
  return sh.field_strings(l.data_ptr<int64_t>(), f.data_ptr<int32_t>(), l.numel());
}

// K1 device tokenizer (records.hip): this rank's byte range is uploaded through the pinned staging
// ring and tokenized on the GPU.  Same result as TextShard.tokenize (codes in first-occurrence
// order, the same vocabulary).  Returns (off, codes, sub | None, nums | None, vocab, stats) with the
// tensors on ``like``'s device, or None when the exactness check found a hash collision (the
// caller then uses the host tokenizer).
py::object text_tokenize_device(std::vector<std::string> paths, int64_t rank, int64_t world,
                                const std::string& delims_in, const std::string& sub_delim, const std::string& modes,
                                const std::string& tail_mode, bool trim, bool want_nums, const at::Tensor& like,
                                int64_t max_initial_slots, const std::string& last_mode) {
  CHECK_DEV(like);
  TORCH_CHECK(max_initial_slots >= 1024, "max_initial_slots >= 1024");
  TORCH_CHECK(sub_delim.size() <= 1 && tail_mode.size() == 1 && last_mode.size() <= 1, "bad tokenizer options");
  // the kernel argument block holds 64 per-field modes: wider mode strings take the host tokenizer
  if (modes.size() > 64) return py::none();
  for (char c : modes + tail_mode + last_mode) TORCH_CHECK(c == 'd' || c == 'n' || c == 'x', "token modes are d / n / x");
  const std::string delims = delims_in.empty() ? std::string(",") : delims_in;
  const char sd = sub_delim.empty() ? 0 : sub_delim[0];
  DevGuard g(like.device());
  hipStream_t stream = cur_stream(like);
  auto t0 = std::chrono::steady_clock::now();
  std::unique_ptr<avh::ByteShard> sh;
  {
    py::gil_scoped_release rel;
    sh = std::make_unique<avh::ByteShard>(paths, rank, world, false);
  }
  // ---- upload: segments streamed through the ring, each newline-terminated ----
  const auto& segs = sh->segments();
  int64_t size = 0;
  for (auto& sg : segs) size += sg.len + ((sg.len > 0 && sg.p[sg.len - 1] != '\n') ? 1 : 0);
  const int64_t padded = std::max<int64_t>(16, (size + 15) / 16 * 16);
  auto dopt = like.options().dtype(at::kByte);
  auto dev = at::empty({padded}, dopt);
  if (padded > size) BIND_HIP_CHECK(hipMemsetAsync(dev.data_ptr<uint8_t>() + size, 0, padded - size, stream));
  {
    py::gil_scoped_release rel;
    struct Piece { const char* p; int64_t len; };
    static const char nl = '\n';
    std::vector<Piece> pieces;
    for (auto& sg : segs) {
      if (sg.len <= 0) continue;
      pieces.push_back({sg.p, sg.len});
      if (sg.p[sg.len - 1] != '\n') pieces.push_back({&nl, 1});
    }
    StagingRing& R = staging_ring(like.device().index());
    std::lock_guard<std::mutex> hold(R.mu);
    for (int i = 0; i < SLOTS; ++i) BIND_HIP_CHECK(hipEventSynchronize(R.done[i]));
    const int NS = upload_streams();
    int64_t out = 0, k = 0;
    size_t pi = 0;
    int64_t pofs = 0;
    while (out < size) {
      const int slot = (int)(k % SLOTS);
      if (k >= SLOTS) BIND_HIP_CHECK(hipEventSynchronize(R.done[slot]));
      // fill the slot from the piece list (parallel memcpy of each run)
      int64_t fill = 0;
      char* dst = static_cast<char*>(R.buf[slot]);
      const int64_t cap = std::min(SLOT, (int64_t)(8LL << 20) << std::min<int64_t>(k, 3));  // 8, 16, 32, 64 MB
      while (fill < cap && pi < pieces.size()) {
        const int64_t n = std::min(cap - fill, pieces[pi].len - pofs);
        const char* src = pieces[pi].p + pofs;
        const int T = n >= (8 << 20) ? upload_threads() : 1;
        std::function<void(int)> part = [&](int t) {
          const int64_t a = n * t / T, b = n * (t + 1) / T;
          std::memcpy(dst + fill + a, src + a, (size_t)(b - a));
        };
        if (T > 1) FillPool::get().run(T, part);
        else part(0);
        fill += n;
        pofs += n;
        if (pofs == pieces[pi].len) { ++pi; pofs = 0; }
      }
      ring_dma(R, slot, k, dev.data_ptr<uint8_t>() + out, fill, stream, NS);
      out += fill;
      ++k;
    }
    ring_join(R, stream);
  }
  // a shard inside ONE file: its lines can be addressed as file offsets (LineSpans.from_file), so
  // the caller needs no host newline scan of the same bytes for raw-line output
  const int seg_file = segs.size() == 1 ? segs[0].file : -1;
  const int64_t seg_off = segs.size() == 1 ? segs[0].file_off : 0;
  sh.reset();
  auto t1 = std::chrono::steady_clock::now();
  const uint8_t* bytes = dev.data_ptr<uint8_t>();
  auto lopt = like.options().dtype(at::kLong);
  auto iopt = like.options().dtype(at::kInt);
  // ---- newline index -> raw lines (every segment ends with '\n') ----
  const int64_t nch = std::max<int64_t>(1, avk::csv_chunks(size));
  auto counts = at::zeros({nch}, iopt);
  avk::csv_newline_counts(bytes, size, reinterpret_cast<unsigned*>(counts.data_ptr<int>()), stream);
  auto c64 = counts.to(at::kLong);
  auto incl = c64.cumsum(0);
  auto coff = (incl - c64).contiguous();
  const int64_t nraw = size > 0 ? incl[-1].item<int64_t>() : 0;
  auto pos = at::empty({std::max<int64_t>(1, nraw)}, lopt);
  if (nraw) avk::csv_newline_positions(bytes, size, reinterpret_cast<long long*>(coff.data_ptr<int64_t>()),
                                       reinterpret_cast<long long*>(pos.data_ptr<int64_t>()), stream);
  auto ls = at::empty({std::max<int64_t>(1, nraw)}, lopt), le = at::empty_like(ls);
  auto nt = at::zeros({std::max<int64_t>(1, nraw)}, iopt);
  avk::rec_lines(bytes, reinterpret_cast<const long long*>(pos.data_ptr<int64_t>()), nraw, delims.data(),
                 (int)delims.size(), reinterpret_cast<long long*>(ls.data_ptr<int64_t>()),
                 reinterpret_cast<long long*>(le.data_ptr<int64_t>()), nt.data_ptr<int>(), stream);
  ls = ls.narrow(0, 0, nraw);
  le = le.narrow(0, 0, nraw);
  nt = nt.narrow(0, 0, nraw);
  if (nraw && !(nt > 0).all().item<bool>()) {  // drop blank lines
    auto idx = at::nonzero(nt > 0).view({-1});
    ls = ls.index({idx});
    le = le.index({idx});
    nt = nt.index({idx});
  }
  ls = ls.contiguous();
  le = le.contiguous();
  const int64_t L = ls.numel();
  auto off = at::zeros({L + 1}, lopt);
  if (L) off.narrow(0, 1, L).copy_(nt.to(at::kLong).cumsum(0));
  const int64_t T = L ? off[L].item<int64_t>() : 0;
  // ---- tokens + dictionary table ----
  auto cap_for = [](int64_t n) {
    int64_t c = 1024;
    while (c < 2 * n) c <<= 1;
    return c;
  };
  const int64_t tdict = T * (sd ? 2 : 1);
  int64_t cap = std::min<int64_t>(cap_for(tdict), max_initial_slots);
  auto tslot = at::empty({std::max<int64_t>(1, T)}, iopt);
  auto th2 = at::empty({std::max<int64_t>(1, T)}, iopt);
  at::Tensor tsub, th2s, nums;
  if (sd) {
    tsub = at::empty({std::max<int64_t>(1, T)}, iopt);
    th2s = at::empty({std::max<int64_t>(1, T)}, iopt);
  }
  if (want_nums) nums = at::empty({std::max<int64_t>(1, T)}, like.options().dtype(at::kDouble));
  at::Tensor keys, h2tab, first;
  auto ctr = at::zeros({2}, iopt);  // inserted, overflow
  while (true) {
    keys = at::zeros({cap}, lopt);
    h2tab = at::empty({cap}, iopt);
    first = at::full({cap}, -1, lopt);  // all ones = EMPTY_FIRST
    ctr.zero_();
    avk::rec_tokens(bytes, reinterpret_cast<const long long*>(ls.data_ptr<int64_t>()),
                    reinterpret_cast<const long long*>(le.data_ptr<int64_t>()),
                    reinterpret_cast<const long long*>(off.data_ptr<int64_t>()), L, delims.data(), (int)delims.size(),
                    modes.data(), (int)modes.size(), tail_mode[0], sd, trim, last_mode.empty() ? 0 : last_mode[0],
                    reinterpret_cast<unsigned long long*>(keys.data_ptr<int64_t>()),
                    reinterpret_cast<unsigned*>(h2tab.data_ptr<int>()),
                    reinterpret_cast<unsigned long long*>(first.data_ptr<int64_t>()), (unsigned long long)(cap - 1),
                    tslot.data_ptr<int>(), reinterpret_cast<unsigned*>(th2.data_ptr<int>()),
                    sd ? tsub.data_ptr<int>() : nullptr, sd ? reinterpret_cast<unsigned*>(th2s.data_ptr<int>()) : nullptr,
                    want_nums ? nums.data_ptr<double>() : nullptr, reinterpret_cast<unsigned*>(ctr.data_ptr<int>()),
                    reinterpret_cast<unsigned*>(ctr.data_ptr<int>()) + 1, stream);
    const bool over = ctr[1].item<int>() != 0;
    if (!over) break;
    TORCH_CHECK(cap < (1LL << 31), "device tokenizer: dictionary table exceeds 2^31 slots");
    cap <<= 2;  // more distinct values than the table holds at load 1/2: retry with a 4x table
  }
  // a number of > 19 significant digits the device could not round for certain: host tokenizer
  if (avk::rec_slow_tokens_take(stream) != 0) return py::none();
  // ---- dense codes in first-occurrence order ----
  auto used = at::nonzero(first != -1).view({-1});
  const int64_t D = used.numel();
  auto focc = first.index({used});
  // first-occurrence keys are unique and non-negative as int64 (< 2^62), so a signed sort orders them
  auto order = std::get<1>(focc.sort());
  auto occ = focc.index({order}).contiguous();
  auto slot_code = at::full({cap}, -1, iopt);
  slot_code.index_put_({used.index({order})}, at::arange(D, iopt));
  auto mism = at::zeros({1}, iopt);
  auto codes = at::empty({std::max<int64_t>(1, T)}, iopt);
  avk::rec_codes(tslot.data_ptr<int>(), reinterpret_cast<const unsigned*>(th2.data_ptr<int>()), T,
                 slot_code.data_ptr<int>(), reinterpret_cast<const unsigned*>(h2tab.data_ptr<int>()),
                 codes.data_ptr<int>(), reinterpret_cast<unsigned*>(mism.data_ptr<int>()), stream);
  at::Tensor subc;
  if (sd) {
    subc = at::empty({std::max<int64_t>(1, T)}, iopt);
    avk::rec_codes(tsub.data_ptr<int>(), reinterpret_cast<const unsigned*>(th2s.data_ptr<int>()), T,
                   slot_code.data_ptr<int>(), reinterpret_cast<const unsigned*>(h2tab.data_ptr<int>()),
                   subc.data_ptr<int>(), reinterpret_cast<unsigned*>(mism.data_ptr<int>()), stream);
  }
  // ---- vocabulary bytes ----
  auto vstart = at::empty({std::max<int64_t>(1, D)}, lopt);
  auto vlen = at::empty({std::max<int64_t>(1, D)}, iopt);
  avk::rec_vocab(bytes, reinterpret_cast<const long long*>(ls.data_ptr<int64_t>()),
                 reinterpret_cast<const long long*>(le.data_ptr<int64_t>()),
                 reinterpret_cast<const long long*>(off.data_ptr<int64_t>()), L,
                 reinterpret_cast<const unsigned long long*>(occ.data_ptr<int64_t>()), D, delims.data(),
                 (int)delims.size(), sd, trim, reinterpret_cast<long long*>(vstart.data_ptr<int64_t>()),
                 vlen.data_ptr<int>(), stream);
  auto vl64 = vlen.narrow(0, 0, D).to(at::kLong);
  auto vincl = vl64.cumsum(0);
  auto vout = (vincl - vl64).contiguous();
  const int64_t VB = D ? vincl[-1].item<int64_t>() : 0;
  auto vbytes = at::empty({std::max<int64_t>(1, VB)}, dopt);
  avk::rec_gather(bytes, reinterpret_cast<const long long*>(vstart.data_ptr<int64_t>()), vlen.data_ptr<int>(),
                  reinterpret_cast<const long long*>(vout.data_ptr<int64_t>()), D, vbytes.data_ptr<uint8_t>(), stream);
  if (mism.item<int>() != 0) return py::none();  // a 64-bit hash collision: let the host path decide
  auto vb_h = vbytes.narrow(0, 0, VB).cpu();
  auto vo_h = vout.cpu();
  auto vl_h = vl64.cpu();
  std::vector<std::string> vocab((size_t)D);
  {
    const char* b = reinterpret_cast<const char*>(vb_h.data_ptr<uint8_t>());
    const int64_t* o = vo_h.data_ptr<int64_t>();
    const int64_t* n = vl_h.data_ptr<int64_t>();
    for (int64_t r = 0; r < D; ++r) vocab[(size_t)r].assign(b + o[r], (size_t)n[r]);
  }
  auto t2 = std::chrono::steady_clock::now();
  py::dict stats;
  stats["bytes"] = size;
  // the uploaded bytes and the lines' spans in them (device output formatter, format.hip)
  stats["line_buf"] = dev;
  stats["line_rel_starts"] = ls;
  stats["line_rel_ends"] = le;
  if (seg_file >= 0) {
    stats["line_file"] = seg_file;
    stats["line_starts"] = ls + seg_off;
    stats["line_ends"] = le + seg_off;
  }
  stats["upload_s"] = std::chrono::duration<double>(t1 - t0).count();
  stats["tokenize_s"] = std::chrono::duration<double>(t2 - t1).count();
  stats["table_slots"] = cap;
  // the dictionary bytes stay on the device too (string-order sorts of keys run there)
  stats["vbytes"] = vbytes.narrow(0, 0, std::max<int64_t>(VB, 0));
  stats["voff"] = vout;
  stats["vlen"] = vl64;
  py::object subo = sd ? py::cast(subc.narrow(0, 0, T)) : py::none();
  py::object numo = want_nums ? py::cast(nums.narrow(0, 0, T)) : py::none();
  return py::make_tuple(off, codes.narrow(0, 0, T), subo, numo, vocab, stats);
}

// format_columns(cols, n, delim, nthreads) -> bytes.  cols: ("s", list[str], idx int32) |
// ("f", float64, prec) | ("i", int64) | ("c", literal) | ("g", literal glued without a delimiter) |
// ("l", list[str], idx int32, off int64 [n+1]).
py::object format_columns_impl(py::list cols_py, int64_t n, const std::string& delim, int nthreads,
                               const std::string* path, bool append) {
  std::vector<avh::FmtCol> cols;
  std::vector<std::unique_ptr<std::vector<std::string>>> tables;
  std::map<PyObject*, const std::vector<std::string>*> table_of;
  std::vector<at::Tensor> keep;
  for (auto item : cols_py) {
    auto t = item.cast<py::tuple>();
    const std::string kind = t[0].cast<std::string>();
    avh::FmtCol c;
    auto cpu_tensor = [&](py::handle h, at::ScalarType st, int64_t len, const char* what) {
      auto x = h.cast<at::Tensor>().to(at::kCPU).to(st).contiguous();
      TORCH_CHECK(x.numel() >= len, "format_columns: ", what, " column shorter than required");
      keep.push_back(x);
      return x;
    };
    if (kind == "s" || kind == "l" || kind == "lp") {
      PyObject* key = t[1].ptr();  // one conversion per distinct table object
      auto hit = table_of.find(key);
      if (hit == table_of.end()) {
        tables.push_back(std::make_unique<std::vector<std::string>>(t[1].cast<std::vector<std::string>>()));
        hit = table_of.emplace(key, tables.back().get()).first;
      }
      c.table = hit->second;
      if (kind == "s") {
        c.kind = avh::FmtCol::STR;
        c.idx = cpu_tensor(t[2], at::kInt, n, "string").data_ptr<int32_t>();
      } else if (kind == "l") {
        c.kind = avh::FmtCol::LIST;
        auto off = cpu_tensor(t[3], at::kLong, n + 1, "list offsets");
        const int64_t m = n ? off.data_ptr<int64_t>()[n] : 0;
        c.idx = cpu_tensor(t[2], at::kInt, m, "list").data_ptr<int32_t>();
        c.off = off.data_ptr<int64_t>();
      } else {  // ("lp", table, idx int32 [m], ints int64 [m], off int64 [n + 1])
        c.kind = avh::FmtCol::PAIRS;
        auto off = cpu_tensor(t[4], at::kLong, n + 1, "list offsets");
        const int64_t m = n ? off.data_ptr<int64_t>()[n] : 0;
        c.idx = cpu_tensor(t[2], at::kInt, m, "list").data_ptr<int32_t>();
        c.iv = cpu_tensor(t[3], at::kLong, m, "pair list ints").data_ptr<int64_t>();
        c.off = off.data_ptr<int64_t>();
      }
    } else if (kind == "f") {
      c.kind = avh::FmtCol::F64;
      c.dv = cpu_tensor(t[1], at::kDouble, n, "float").data_ptr<double>();
      c.prec = t.size() > 2 ? t[2].cast<int>() : 6;
    } else if (kind == "i") {
      c.kind = avh::FmtCol::I64;
      c.iv = cpu_tensor(t[1], at::kLong, n, "int").data_ptr<int64_t>();
    } else if (kind == "c" || kind == "g") {
      c.kind = kind == "c" ? avh::FmtCol::LIT : avh::FmtCol::GLUE;
      c.lit = t[1].cast<std::string>();
    } else if (kind == "r" || kind == "rf" || kind == "rt") {
      // raw input lines: (kind, owner, addr int64 [n], len int64 [n], [field,] from_delims); the
      // owner (a CsvFile / TextShard / mapping) keeps the bytes alive for the call
      TORCH_CHECK(!t[1].is_none(), "format_columns: raw line column without its owner");
      c.kind = kind == "r" ? avh::FmtCol::RAW : (kind == "rf" ? avh::FmtCol::FIELD : avh::FmtCol::TAIL);
      c.raddr = cpu_tensor(t[2], at::kLong, n, "line address").data_ptr<int64_t>();
      c.rlen = cpu_tensor(t[3], at::kLong, n, "line length").data_ptr<int64_t>();
      size_t k = 4;
      if (kind != "r") c.field = t[k++].cast<int>();
      if (t.size() > k) c.from_delims = t[k].cast<std::string>();
    } else {
      TORCH_CHECK(false, "format_columns: unknown column kind ", kind);
    }
    cols.push_back(std::move(c));
  }
  if (path) {
    int64_t w;
    {
      py::gil_scoped_release rel;
      w = avh::format_columns_to_file(cols, n, delim, nthreads, *path, append);
    }
    return py::int_(w);
  }
  std::string out;
  {
    py::gil_scoped_release rel;
    out = avh::format_columns(cols, n, delim, nthreads);
  }
  return py::bytes(out);
}

py::object format_columns_py(py::list cols_py, int64_t n, const std::string& delim, int nthreads) {
  return format_columns_impl(cols_py, n, delim, nthreads, nullptr, false);
}

// format_columns_file(cols, n, delim, nthreads, path, append) -> bytes written (threads pwrite)
py::object format_columns_file_py(py::list cols_py, int64_t n, const std::string& delim, int nthreads,
                                  const std::string& path, bool append) {
  return format_columns_impl(cols_py, n, delim, nthreads, &path, append);
}

// pairs_within(A f32 [nA, D], B f32 [nB, D], nf, scale, thr, tri, a_base, b_base) -> (I, J, dist):
// the pairs with round(|a - b| / nf * scale) <= thr (j > i in global order when ``tri``), sorted by
// (i, j).  Segmented output buffers sized from an estimate, re-run once when a segment overflows.
py::tuple pairs_within(const at::Tensor& A, const at::Tensor& B, double nf, double scale, double thr, bool tri,
                       int64_t a_base, int64_t b_base) {
  CHECK_DEV(A);
  CHECK_DEV(B);
  CHECK_DTYPE(A, at::kFloat);
  CHECK_DTYPE(B, at::kFloat);
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.size(1) == B.size(1) && A.is_contiguous() && B.is_contiguous(),
              "pairs_within: A [nA, D], B [nB, D] contiguous");
  TORCH_CHECK(A.size(1) >= 1 && A.size(1) <= 64, "pairs_within: 1 <= D <= 64");
  TORCH_CHECK(A.size(0) < (1LL << 31) && B.size(0) < (1LL << 31), "pairs_within: too many rows");
  DevGuard g(A.device());
  hipStream_t stream = cur_stream(A);
  const int nA = (int)A.size(0), nB = (int)B.size(0), D = (int)A.size(1);
  const int S = avk::pairs_within_segments();
  auto cnt = at::empty({avk::pairs_within_counter_ints()}, A.options().dtype(at::kInt));
  long long seg_cap = (std::max<long long>(1 << 20, ((long long)nA + nB) * 4) + S - 1) / S;
  std::vector<long long> counts(S);
  for (int attempt = 0; attempt < 2; ++attempt) {
    auto K = at::empty({seg_cap * S}, A.options().dtype(at::kLong));
    auto Dd = at::empty({seg_cap * S}, A.options().dtype(at::kInt));
    const long long mx = avk::pairs_within(A.data_ptr<float>(), nA, B.data_ptr<float>(), nB, D, (float)nf, (float)scale,
                                           (float)thr, tri ? 1 : 0, a_base, b_base, cnt.data_ptr<int>(), seg_cap,
                                           reinterpret_cast<long long*>(K.data_ptr<int64_t>()), Dd.data_ptr<int>(),
                                           counts.data(), stream);
    TORCH_CHECK(mx >= 0 && mx < (1LL << 31) - 1, "pairs_within: pair count overflows int32");
    if (mx <= seg_cap) {
      // the filled prefix of every segment, then one sort by key = i * nB + j
      std::vector<at::Tensor> ks, ds;
      for (int c = 0; c < S; ++c)
        if (counts[c]) {
          ks.push_back(K.narrow(0, c * seg_cap, counts[c]));
          ds.push_back(Dd.narrow(0, c * seg_cap, counts[c]));
        }
      if (ks.empty()) {
        auto e = at::empty({0}, A.options().dtype(at::kLong));
        return py::make_tuple(e, e.clone(), e.clone());
      }
      auto k = at::cat(ks), d = at::cat(ds);
      auto sorted = k.sort();
      auto key = std::get<0>(sorted), order = std::get<1>(sorted);
      const int64_t nb = std::max(nB, 1);
      return py::make_tuple(key.div(nb, "floor"), key.remainder(nb), d.index({order}).to(at::kLong));
    }
    seg_cap = mx;
  }
  TORCH_CHECK(false, "pairs_within: pair buffer overflow after resize");
  return py::make_tuple();
}

// format_device(cols, n, delim, path, append, nthreads, like) -> bytes written, or -1 when a value
// needs the host formatter (a double outside the exact fixed-point fast path, a precision other
// than 0..9): the rows are formatted on ``like``'s device (format.hip: length pass, device scan,
// write pass), copied to pinned host memory once and written by ``nthreads`` pwrite threads.
// Column tuples as format_columns, with device tensors; raw-line kinds read device line bytes:
// ("dr" | "drf" | "drt", bytes uint8, start int64 [n], len int64 [n], [field,] from_delims).
int64_t format_device(py::list cols_py, int64_t n, const std::string& delim, const std::string& path, bool append,
                      int nthreads, const at::Tensor& like) {
  CHECK_DEV(like);
  DevGuard g(like.device());
  hipStream_t stream = cur_stream(like);
  auto dopt = like.options();
  std::vector<avk::DevFmtCol> cols;
  std::vector<at::Tensor> keep;
  std::map<PyObject*, std::pair<at::Tensor, at::Tensor>> tables;
  auto dev_tensor = [&](py::handle h, at::ScalarType st, int64_t len, const char* what) {
    auto x = h.cast<at::Tensor>().to(like.device()).to(st).contiguous();
    TORCH_CHECK(x.numel() >= len, "format_device: ", what, " column shorter than required");
    keep.push_back(x);
    return x;
  };
  auto upload_bytes = [&](const std::string& b) {
    auto h = at::empty({std::max<int64_t>(1, (int64_t)b.size())}, at::kByte);
    if (!b.empty()) std::memcpy(h.data_ptr<uint8_t>(), b.data(), b.size());
    auto d = h.to(like.device());
    keep.push_back(d);
    return d;
  };
  for (auto item : cols_py) {
    auto t = item.cast<py::tuple>();
    const std::string kind = t[0].cast<std::string>();
    avk::DevFmtCol c;
    if (kind == "s" || kind == "l" || kind == "lp") {
      PyObject* key = t[1].ptr();
      auto hit = tables.find(key);
      if (hit == tables.end()) {
        auto strs = t[1].cast<std::vector<std::string>>();
        std::string cat;
        std::vector<int64_t> off(strs.size() + 1, 0);
        for (size_t i = 0; i < strs.size(); ++i) {
          cat += strs[i];
          off[i + 1] = (int64_t)cat.size();
        }
        auto tb = upload_bytes(cat);
        auto to = at::from_blob(off.data(), {(int64_t)off.size()}, at::kLong).to(like.device());
        keep.push_back(to);
        hit = tables.emplace(key, std::make_pair(tb, to)).first;
      }
      c.tbytes = hit->second.first.data_ptr<uint8_t>();
      c.toff = hit->second.second.data_ptr<int64_t>();
      c.tV = hit->second.second.numel() - 1;
      if (kind == "s") {
        c.kind = avk::DevFmtCol::STR;
        c.idx = dev_tensor(t[2], at::kInt, n, "string").data_ptr<int32_t>();
      } else {
        const bool pairs = kind == "lp";
        c.kind = pairs ? avk::DevFmtCol::PAIRS : avk::DevFmtCol::LIST;
        auto off = dev_tensor(t[pairs ? 4 : 3], at::kLong, n + 1, "list offsets");
        const int64_t m = n ? off[n].item<int64_t>() : 0;
        c.idx = dev_tensor(t[2], at::kInt, m, "list").data_ptr<int32_t>();
        if (pairs) c.iv = dev_tensor(t[3], at::kLong, m, "pair list ints").data_ptr<int64_t>();
        c.off = off.data_ptr<int64_t>();
      }
    } else if (kind == "f") {
      c.kind = avk::DevFmtCol::F64;
      c.prec = t.size() > 2 ? t[2].cast<int>() : 6;
      if (c.prec != -2 && (c.prec < 0 || c.prec > 9)) return -1;  // %g / long fractions: host formatter
      c.dv = dev_tensor(t[1], at::kDouble, n, "float").data_ptr<double>();
    } else if (kind == "i") {
      c.kind = avk::DevFmtCol::I64;
      c.iv = dev_tensor(t[1], at::kLong, n, "int").data_ptr<int64_t>();
    } else if (kind == "c" || kind == "g") {
      c.kind = kind == "c" ? avk::DevFmtCol::LIT : avk::DevFmtCol::GLUE;
      const std::string lit = t[1].cast<std::string>();
      c.lit = upload_bytes(lit).data_ptr<uint8_t>();
      c.litlen = (int)lit.size();
    } else if (kind == "dr" || kind == "drf" || kind == "drt") {
      c.kind = kind == "dr" ? avk::DevFmtCol::RAW : (kind == "drf" ? avk::DevFmtCol::FIELD : avk::DevFmtCol::TAIL);
      auto b = t[1].cast<at::Tensor>();
      TORCH_CHECK(b.device() == like.device() && b.scalar_type() == at::kByte && b.is_contiguous(),
                  "format_device: line bytes must be a contiguous uint8 tensor on the device");
      keep.push_back(b);
      c.lbytes = b.data_ptr<uint8_t>();
      auto st = dev_tensor(t[2], at::kLong, n, "line start");
      auto ln = dev_tensor(t[3], at::kLong, n, "line length");
      c.lstart = st.data_ptr<int64_t>();
      c.llen = ln.data_ptr<int64_t>();
      size_t k = 4;
      if (kind != "dr") c.field = t[k++].cast<int>();
      const std::string fd = t.size() > k ? t[k].cast<std::string>() : std::string();
      for (char ch : fd) c.sep[(uint8_t)ch >> 5] |= 1u << ((uint8_t)ch & 31);
      c.same = fd.empty() || fd == delim;
    } else {
      return -1;   // a kind the device formatter does not handle
    }
    cols.push_back(c);
  }
  const int ncols = (int)cols.size();
  auto dcols = at::empty({std::max<int64_t>(1, (int64_t)(ncols * sizeof(avk::DevFmtCol)))}, dopt.dtype(at::kByte));
  if (ncols)
    BIND_HIP_CHECK(hipMemcpyAsync(dcols.data_ptr(), cols.data(), ncols * sizeof(avk::DevFmtCol), hipMemcpyHostToDevice,
                                  stream));
  auto dl = upload_bytes(delim);
  const auto* dc = reinterpret_cast<const avk::DevFmtCol*>(dcols.data_ptr());
  const bool timing = std::getenv("AVMI_FORMAT_TIMING") != nullptr;
  auto tp0 = std::chrono::steady_clock::now();
  auto len = at::empty({std::max<int64_t>(1, n)}, dopt.dtype(at::kLong));
  auto bad = at::zeros({1}, dopt.dtype(at::kInt));
  avk::format_rows_len(dc, ncols, n, dl.data_ptr<uint8_t>(), (int)delim.size(), len.data_ptr<int64_t>(),
                       bad.data_ptr<int>(), stream);
  if (bad.item<int>() != 0) return -1;
  auto lens = len.narrow(0, 0, n);
  auto cs = n ? lens.cumsum(0) : lens;
  const int64_t total = n ? cs[n - 1].item<int64_t>() : 0;
  auto start = (cs - lens).contiguous();
  auto out = at::empty({std::max<int64_t>(1, total)}, dopt.dtype(at::kByte));
  avk::format_rows_write(dc, ncols, n, dl.data_ptr<uint8_t>(), (int)delim.size(), start.data_ptr<int64_t>(),
                         reinterpret_cast<char*>(out.data_ptr<uint8_t>()), stream);
  auto host = at::empty({std::max<int64_t>(1, total)}, at::TensorOptions().dtype(at::kByte).pinned_memory(true));
  if (total)
    BIND_HIP_CHECK(hipMemcpyAsync(host.data_ptr(), out.data_ptr(), (size_t)total, hipMemcpyDeviceToHost, stream));
  BIND_HIP_CHECK(hipStreamSynchronize(stream));
  auto tp1 = std::chrono::steady_clock::now();
  {
    py::gil_scoped_release rel;
    avh::write_file_parallel(path, append, {{reinterpret_cast<const char*>(host.data_ptr()), total}}, nthreads);
  }
  if (timing) {
    auto tp2 = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[format_device] rows %lld bytes %lld format+d2h %.4f s write %.4f s\n", (long long)n,
                 (long long)total, std::chrono::duration<double>(tp1 - tp0).count(),
                 std::chrono::duration<double>(tp2 - tp1).count());
  }
  return total;
}

// pack_spans(addr int64 [n], len int64 [n], nthreads) -> (bytes uint8 [sum len], off int64 [n + 1]):
// the lines behind byte spans (data/lines.py) copied into one contiguous buffer — the payload that
// travels around the ring of the all-pairs similarity jobs.  Rows are split over the threads.
py::tuple pack_spans(const at::Tensor& addr_in, const at::Tensor& len_in, int nthreads) {
  auto addr = addr_in.to(at::kCPU).to(at::kLong).contiguous();
  auto len = len_in.to(at::kCPU).to(at::kLong).contiguous();
  TORCH_CHECK(addr.numel() == len.numel(), "pack_spans: address / length size mismatch");
  const int64_t n = addr.numel();
  auto off = at::empty({n + 1}, at::kLong);
  int64_t* o = off.data_ptr<int64_t>();
  const int64_t* a = addr.data_ptr<int64_t>();
  const int64_t* l = len.data_ptr<int64_t>();
  o[0] = 0;
  for (int64_t i = 0; i < n; ++i) {
    TORCH_CHECK(l[i] >= 0, "pack_spans: negative length");
    o[i + 1] = o[i] + l[i];
  }
  auto bytes = at::empty({std::max<int64_t>(o[n], 1)}, at::kByte);
  uint8_t* dst = bytes.data_ptr<uint8_t>();
  {
    py::gil_scoped_release rel;
    const int T = n < 65536 ? 1 : std::max(1, std::min(nthreads, 64));
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        for (int64_t i = n * t / T; i < n * (t + 1) / T; ++i)
          if (l[i]) std::memcpy(dst + o[i], reinterpret_cast<const void*>(a[i]), (size_t)l[i]);
      });
    for (auto& x : th) x.join();
  }
  return py::make_tuple(bytes.narrow(0, 0, o[n]), off);
}

// smote_lines: the synthetic records of classBasedOverSampler (SMOTE) assembled natively from the
// source lines (byte spans), the K25 kernel's outputs and the field kinds of one record block:
// kind 0 copy the source field (class / non-feature), 1 id (the source id and the picked
// neighbour's id scrambled, truncated to the source id's length), 2 integer feature (the kernel's
// value truncated), 3 double feature (fixed, prec digits), 4 categorical feature (source or
// neighbour field by the kernel's coin).  The scramble is a Fisher-Yates shuffle driven by a
// splitmix64 stream keyed by (seed * 1000003 + global line) * 131 + copy (jobs/core.py mirrors it).
namespace {
inline uint64_t smx_next(uint64_t& x) {
  x += 0x9E3779B97F4A7C15ull;
  uint64_t z = x;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
}  // namespace

py::tuple smote_lines(const at::Tensor& addr_in, const at::Tensor& len_in, int64_t L, const at::Tensor& kinds_in,
                      const at::Tensor& numcol_in, const at::Tensor& newx_in, const at::Tensor& coin_in,
                      const at::Tensor& pick_in, const at::Tensor& gidx_in, int64_t mult, int64_t seed, int64_t prec,
                      const std::string& sep_in, const std::string& delim, int nthreads) {
  auto addr = addr_in.to(at::kCPU).to(at::kLong).contiguous();
  auto len = len_in.to(at::kCPU).to(at::kLong).contiguous();
  auto kinds = kinds_in.to(at::kCPU).to(at::kInt).contiguous();
  auto numcol = numcol_in.to(at::kCPU).to(at::kInt).contiguous();
  auto newx = newx_in.to(at::kCPU).to(at::kFloat).contiguous();
  auto coin = coin_in.to(at::kCPU).to(at::kInt).contiguous();
  auto pick = pick_in.to(at::kCPU).to(at::kLong).contiguous();
  auto gidx = gidx_in.to(at::kCPU).to(at::kLong).contiguous();
  const int64_t n = addr.numel();
  TORCH_CHECK(len.numel() == n && gidx.numel() == n, "smote_lines: one span and global index per line");
  TORCH_CHECK(kinds.numel() == L && numcol.numel() == L && L >= 1, "smote_lines: kinds / numcol are [L]");
  TORCH_CHECK(mult >= 0 && coin.numel() == n * mult && pick.numel() == n * mult, "smote_lines: [n * mult] draws");
  const int64_t C = newx.dim() == 2 ? newx.size(1) : 0;
  TORCH_CHECK(newx.dim() == 2 && newx.size(0) == n * mult, "smote_lines: newx [n * mult, C]");
  TORCH_CHECK(sep_in.size() == 1, "smote_lines: one-character input delimiter");
  const char sep = sep_in[0];
  const int32_t* kd = kinds.data_ptr<int32_t>();
  const int32_t* nc = numcol.data_ptr<int32_t>();
  for (int64_t i = 0; i < L; ++i)
    TORCH_CHECK(kd[i] >= 0 && kd[i] <= 4 && nc[i] < C && ((kd[i] != 2 && kd[i] != 3) || nc[i] >= 0),
                "smote_lines: bad field kind / numeric column");
  const int64_t* a = addr.data_ptr<int64_t>();
  const int64_t* l = len.data_ptr<int64_t>();
  const float* X = newx.data_ptr<float>();
  const int32_t* cn = coin.data_ptr<int32_t>();
  const int64_t* pk = pick.data_ptr<int64_t>();
  const int64_t* gi = gidx.data_ptr<int64_t>();
  const int T = n < 4096 ? 1 : std::max(1, std::min(nthreads, 64));
  std::vector<std::string> parts((size_t)T);
  std::vector<std::vector<int64_t>> lens((size_t)T);
  {
    py::gil_scoped_release rel;
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        std::string& out = parts[(size_t)t];
        std::vector<int64_t>& ol = lens[(size_t)t];
        std::vector<std::pair<const char*, const char*>> fs;
        std::string idb;
        char num[64];
        for (int64_t r = n * t / T; r < n * (t + 1) / T; ++r) {
          // field byte ranges of the source line
          fs.clear();
          const char* p = reinterpret_cast<const char*>(a[r]);
          const char* e = p + l[r];
          while (true) {
            const char* q = static_cast<const char*>(std::memchr(p, sep, (size_t)(e - p)));
            if (!q) q = e;
            fs.emplace_back(p, q);
            if (q >= e) break;
            p = q + 1;
          }
          const int64_t F = (int64_t)fs.size();
          for (int64_t j = 0; j < mult; ++j) {
            const int64_t o = r * mult + j;
            const int64_t pj = std::max<int64_t>(pk[o], 0);
            const size_t start = out.size();
            for (int64_t i = 0; i < L; ++i) {
              if (i) out += delim;
              const auto src = i < F ? fs[(size_t)i] : std::make_pair(e, e);
              const int64_t ni = L + pj * L + i;
              const auto nbr = ni < F ? fs[(size_t)ni] : std::make_pair(e, e);
              switch (kd[i]) {
                case 1: {
                  idb.assign(src.first, src.second);
                  idb.append(nbr.first, nbr.second);
                  uint64_t x = ((uint64_t)seed * 1000003ull + (uint64_t)gi[r]) * 131ull + (uint64_t)j;
                  for (int64_t k = (int64_t)idb.size() - 1; k > 0; --k) {
                    const uint64_t z = smx_next(x) % (uint64_t)(k + 1);
                    std::swap(idb[(size_t)k], idb[(size_t)z]);
                  }
                  out.append(idb.data(), (size_t)(src.second - src.first));
                  break;
                }
                case 2: {
                  const double v = (double)X[o * C + nc[i]];
                  const int k = std::snprintf(num, sizeof num, "%lld", (long long)std::trunc(v));
                  out.append(num, (size_t)k);
                  break;
                }
                case 3: {
                  const double v = (double)X[o * C + nc[i]];
                  const int k = std::snprintf(num, sizeof num, "%.*f", (int)prec, v);
                  out.append(num, (size_t)std::min<int>(k, (int)sizeof num - 1));
                  break;
                }
                case 4: {
                  const auto& f = cn[o] == 0 ? src : nbr;
                  out.append(f.first, f.second);
                  break;
                }
                default:
                  out.append(src.first, src.second);
              }
            }
            ol.push_back((int64_t)(out.size() - start));
          }
        }
      });
    for (auto& x : th) x.join();
  }
  int64_t tot = 0;
  for (auto& s2 : parts) tot += (int64_t)s2.size();
  auto bytes = at::empty({std::max<int64_t>(tot, 1)}, at::kByte);
  auto off = at::empty({n * mult + 1}, at::kLong);
  uint8_t* dst = bytes.data_ptr<uint8_t>();
  int64_t* of = off.data_ptr<int64_t>();
  int64_t at_b = 0, k = 0;
  of[0] = 0;
  for (int t = 0; t < T; ++t) {
    std::memcpy(dst + at_b, parts[(size_t)t].data(), parts[(size_t)t].size());
    at_b += (int64_t)parts[(size_t)t].size();
    int64_t acc = of[k];
    for (int64_t v : lens[(size_t)t]) {
      acc += v;
      of[++k] = acc;
    }
  }
  return py::make_tuple(bytes.narrow(0, 0, tot), off);
}

// ---------------------------------------------------------------------------------------------
// K27 LSTM recurrence.  Fragments are packed by avenir_amd/ops/rnn.py (pack_weights): wfrag holds
// [NW, 4, KS+IS, 64, 8] bf16 (forward, [W_hh | W_ih]), wfragT [NW, 4KS, 64, 8] bf16 (backward,
// W_hhᵀ); NW = 2 KS.
int64_t lstm_ks(int64_t H) {
  TORCH_CHECK(H >= 1 && H <= 128, "fused LSTM supports hidden and input sizes 1..128");
  return H <= 32 ? 1 : (H <= 64 ? 2 : 4);  // padded hidden size HP = 32 KS in {32, 64, 128}
}

void check_opt_f32(const c10::optional<at::Tensor>& t, int64_t numel, const char* name) {
  if (!t.has_value() || !t->defined()) return;
  TORCH_CHECK(t->is_cuda() && t->is_contiguous() && t->scalar_type() == at::kFloat, name,
              " must be a contiguous fp32 GPU tensor");
  TORCH_CHECK(t->numel() == numel, name, " has the wrong size");
}

// x [B, T, I] fp32; wfrag [NW, 4, KS+IS, 64, 8] bf16 ([W_hh | W_ih]); bias [4HP] fp32 kernel order.
// Returns hseq [B,T,H], cseq [B,T,HP] (+ gates [B,T,4HP] bf16, hx [B,T,HP+IP] bf16 when training).
std::vector<at::Tensor> lstm_forward(const at::Tensor& x, const at::Tensor& wfrag, const at::Tensor& bias,
                                     const c10::optional<at::Tensor>& h0, const c10::optional<at::Tensor>& c0,
                                     int64_t H, bool training) {
  const int64_t KS = lstm_ks(H), HP = 32 * KS;
  CHECK_DEV(x);
  CHECK_DTYPE(x, at::kFloat);
  TORCH_CHECK(x.dim() == 3, "x must be [B, T, I]");
  const int64_t B = x.size(0), T = x.size(1), I = x.size(2);
  const int64_t IS = lstm_ks(I), IP = 32 * IS, KT = KS + IS;
  TORCH_CHECK(B >= 1 && T >= 1, "empty LSTM input");
  CHECK_DEV(wfrag);
  CHECK_DTYPE(wfrag, at::kBFloat16);
  TORCH_CHECK(wfrag.numel() == 2 * KS * 4 * KT * 64 * 8, "wfrag must be [NW, 4, KS+IS, 64, 8]");
  TORCH_CHECK(aligned(wfrag, 16), "wfrag must be 16-byte aligned");
  CHECK_DEV(bias);
  CHECK_DTYPE(bias, at::kFloat);
  TORCH_CHECK(bias.numel() == 4 * HP, "bias must be [4HP] (kernel order)");
  check_opt_f32(h0, B * H, "h0");
  check_opt_f32(c0, B * H, "c0");
  DevGuard g(x.device());
  auto f32 = x.options();
  auto bf = x.options().dtype(at::kBFloat16);
  auto hseq = at::empty({B, T, H}, f32), cseq = at::empty({B, T, HP}, f32);
  at::Tensor gates, hx;
  if (training) {
    gates = at::empty({B, T, 4 * HP}, bf);
    hx = at::empty({B, T, HP + IP}, bf);
  }
  const int RT = avk::lstm_row_tiles(B, (int)KS);
  avk::lstm_fwd(x.data_ptr<float>(), (int)I, (int)IS, wfrag.data_ptr(), bias.data_ptr<float>(), ptr_or_null<float>(h0),
                ptr_or_null<float>(c0), (int)B, (int)T, (int)H, (int)KS, RT, hseq.data_ptr<float>(),
                cseq.data_ptr<float>(), training ? reinterpret_cast<unsigned short*>(gates.data_ptr()) : nullptr,
                training ? reinterpret_cast<unsigned short*>(hx.data_ptr()) : nullptr, cur_stream(x));
  if (training) return {hseq, cseq, gates, hx};
  return {hseq, cseq};
}

// K7 split scoring (split.hip): hist int64 [A, C, TBt]; sp int32 [R, 6] (feature, column, bins,
// segments, valid, segment-map offset); seg int8 segment maps; cand uint8 [A, F].  Returns the k best
// splits per node (index, score) and their segment class counts [A, k, G2, C] / impurities [A, k, G2].
std::vector<at::Tensor> ref_split_score(const at::Tensor& hist, const at::Tensor& sp, const at::Tensor& seg,
                                        const at::Tensor& cand, int64_t algo, int64_t k, int64_t G2) {
  CHECK_DEV(hist);
  CHECK_DTYPE(hist, at::kLong);
  CHECK_DEV(sp);
  CHECK_DTYPE(sp, at::kInt);
  CHECK_DEV(seg);
  CHECK_DTYPE(seg, at::kChar);
  CHECK_DEV(cand);
  CHECK_DTYPE(cand, at::kByte);
  TORCH_CHECK(hist.dim() == 3 && hist.is_contiguous(), "hist must be [A, C, TB] contiguous");
  const int64_t A = hist.size(0), C = hist.size(1), TBt = hist.size(2), R = sp.size(0);
  TORCH_CHECK(sp.dim() == 2 && sp.size(1) == 6 && sp.is_contiguous() && R >= 1, "sp must be [R >= 1, 6]");
  TORCH_CHECK(cand.dim() == 2 && cand.size(0) == A && cand.is_contiguous(), "cand must be [A, F]");
  TORCH_CHECK(C >= 1 && C <= 32 && k >= 1 && k <= R && G2 >= 2 && G2 <= 64 && (algo == 0 || algo == 1),
              "1 <= C <= 32, 1 <= k <= R, 2 <= G2 <= 64, algo 0 (entropy) / 1 (gini)");
  // host-side validation of the table against the histogram and the segment maps (no OOB reads)
  auto sph = sp.cpu();
  const int32_t* q = sph.data_ptr<int32_t>();
  const int64_t F = cand.size(1);
  for (int64_t r = 0; r < R; ++r) {
    const int32_t* e = q + 6 * r;
    TORCH_CHECK(e[0] >= 0 && e[0] < F && e[1] >= 0 && e[2] >= 1 && (int64_t)e[1] + e[2] <= TBt && e[3] >= 1 &&
                    e[3] <= G2 && e[5] >= 0 && (int64_t)e[5] + e[2] <= seg.numel(),
                "ref_split_score: split row ", r, " out of range");
  }
  DevGuard g(hist.device());
  auto o = hist.options();
  auto top = at::empty({A, k}, o);
  auto topv = at::empty({A, k}, o.dtype(at::kDouble));
  auto segc = at::empty({A, k, G2, C}, o.dtype(at::kDouble));
  auto cinfo = at::empty({A, k, G2}, o.dtype(at::kDouble));
  at::Tensor scratch;
  if (R > 4096) scratch = at::empty({A, R}, o.dtype(at::kDouble));
  avk::ref_split_score(reinterpret_cast<const long long*>(hist.data_ptr<int64_t>()), (int)A, (int)C, (int)TBt,
                       sp.data_ptr<int32_t>(), seg.data_ptr<int8_t>(), (int)R, cand.data_ptr<uint8_t>(), (int)F,
                       (int)algo, (int)k, (int)G2, reinterpret_cast<long long*>(top.data_ptr<int64_t>()),
                       topv.data_ptr<double>(), segc.data_ptr<double>(), cinfo.data_ptr<double>(),
                       R > 4096 ? scratch.data_ptr<double>() : nullptr, cur_stream(hist));
  return {top, topv, segc, cinfo};
}

// LN(x + res) * gamma + beta over the last dim (transformer.hip); res may be None
at::Tensor add_layernorm(const at::Tensor& x, const c10::optional<at::Tensor>& res, const at::Tensor& gamma,
                         const at::Tensor& beta, double eps) {
  CHECK_DEV(x);
  CHECK_DTYPE(x, at::kFloat);
  TORCH_CHECK(x.is_contiguous() && x.dim() >= 1, "add_layernorm: x contiguous");
  const int64_t H = x.size(-1), rows = x.numel() / std::max<int64_t>(1, H);
  TORCH_CHECK(H >= 4 && H <= 1024 && H % 4 == 0, "add_layernorm: 4 <= H <= 1024, H % 4 == 0");
  check_opt_f32(res, x.numel(), "res");
  check_opt_f32(gamma, H, "gamma");
  check_opt_f32(beta, H, "beta");
  TORCH_CHECK(aligned(x, 16) && aligned(gamma, 16) && aligned(beta, 16) && (!res.has_value() || aligned(*res, 16)),
              "add_layernorm: 16-byte aligned tensors");
  DevGuard g(x.device());
  auto out = at::empty_like(x);
  avk::add_layernorm(x.data_ptr<float>(), ptr_or_null<float>(res), gamma.data_ptr<float>(), beta.data_ptr<float>(),
                     out.data_ptr<float>(), rows, (int)H, (float)eps, cur_stream(x));
  return out;
}

// LN(X W^T + b + res) for X [M, K], W [N, K], res [M, N]: the projection feeding a residual +
// LayerNorm.  With the split-K tile (few output tiles over a long K) the slice sum, bias, residual
// and LayerNorm run in ONE pass over the partials (no [M, N] projection output, no epilogue launch).
at::Tensor linear_add_layernorm(const at::Tensor& X, const at::Tensor& W, const c10::optional<at::Tensor>& b,
                                const at::Tensor& res, const at::Tensor& gamma, const at::Tensor& beta, double eps,
                                int64_t prec, const c10::optional<at::Tensor>& w_planes) {
  TORCH_CHECK(prec == -1 || prec == 0 || prec == 3 || prec == 6, "prec: -1 (default), 0 (f32), 3 or 6 (split bf16)");
  CHECK_DEV(X); CHECK_DTYPE(X, at::kFloat);
  CHECK_DEV(W); CHECK_DTYPE(W, at::kFloat);
  TORCH_CHECK(X.dim() == 2 && W.dim() == 2 && X.size(1) == W.size(1), "X [M, K], W [N, K]");
  const int64_t M = X.size(0), N = W.size(0), K = X.size(1);
  TORCH_CHECK(M < (1LL << 31) && K < (1LL << 31), "dims < 2^31");
  TORCH_CHECK(N >= 4 && N <= 1024 && N % 4 == 0, "linear_add_layernorm: 4 <= N <= 1024, N % 4 == 0");
  CHECK_DEV(res); CHECK_DTYPE(res, at::kFloat);
  TORCH_CHECK(res.is_contiguous() && res.numel() == M * N && aligned(res, 16), "res [M, N] contiguous");
  check_opt_f32(b, N, "bias");
  check_opt_f32(gamma, N, "gamma");
  check_opt_f32(beta, N, "beta");
  TORCH_CHECK(aligned(gamma, 16) && aligned(beta, 16) && (!b.has_value() || !b->defined() || aligned(*b, 16)),
              "linear_add_layernorm: 16-byte aligned parameters");
  auto Xc = X.contiguous(), Wc = W.contiguous();
  DevGuard g(X.device());
  auto out = at::empty({M, N}, X.options());
  const int S = avk::linear_act_fwd_slices((int)M, (int)N, (int)K);
  if (S > 1) {
    auto part = at::empty({(long long)S * M * N}, X.options());
    const int Se = avk::linear_splitk_partial(Xc.data_ptr<float>(), Wc.data_ptr<float>(), part.data_ptr<float>(),
                                              (int)M, (int)N, (int)K, S, cur_stream(X), (int)prec);
    avk::add_layernorm_slices(part.data_ptr<float>(), Se, M * N, ptr_or_null<float>(b), res.data_ptr<float>(),
                              gamma.data_ptr<float>(), beta.data_ptr<float>(), out.data_ptr<float>(), M, (int)N,
                              (float)eps, cur_stream(X));
  } else {
    auto y = at::empty({M, N}, X.options());
    auto planes = k27_planes(X, M, N, K, prec);
    const void* wp = nullptr;
    if (w_planes.has_value() && w_planes->defined()) {
      CHECK_DEV((*w_planes));
      TORCH_CHECK(w_planes->scalar_type() == at::kByte && w_planes->is_contiguous() &&
                      w_planes->numel() == avk::sbf16_weight_planes_bytes((int)N, (int)K, (int)prec),
                  "w_planes: sbf16_weight_planes(W, prec) of this W and prec");
      wp = w_planes->data_ptr();
    }
    avk::linear_act_fwd(Xc.data_ptr<float>(), Wc.data_ptr<float>(), ptr_or_null<float>(b), y.data_ptr<float>(),
                        (int)M, (int)N, (int)K, 0, cur_stream(X), nullptr, 1, (int)prec, ptr_or_null_t(planes), wp);
    avk::add_layernorm(y.data_ptr<float>(), res.data_ptr<float>(), gamma.data_ptr<float>(), beta.data_ptr<float>(),
                       out.data_ptr<float>(), M, (int)N, (float)eps, cur_stream(X));
  }
  return out;
}

// softmax(q k^T * scale + kbias) v per head from the fused projection qkv [B*S, 3H] (Q | K | V,
// heads of 64 columns) -> [B*S, H]; kbias [B, S] additive per key or None
at::Tensor attention_f32(const at::Tensor& qkv, const c10::optional<at::Tensor>& kbias, int64_t B, int64_t S,
                         int64_t nh, double scale) {
  CHECK_DEV(qkv); CHECK_DTYPE(qkv, at::kFloat);
  TORCH_CHECK(B >= 1 && S >= 1 && nh >= 1, "attention_f32: B, S, nh >= 1");
  const int64_t H = nh * 64;
  TORCH_CHECK(qkv.is_contiguous() && qkv.numel() == B * S * 3 * H && aligned(qkv, 16),
              "attention_f32: qkv [B*S, 3 * nh * 64] contiguous, 16-byte aligned");
  TORCH_CHECK(B * S < (1LL << 31) && S < (1LL << 30) && B < 65536 && nh < 65536, "attention_f32: sizes");
  check_opt_f32(kbias, B * S, "kbias");
  DevGuard g(qkv.device());
  auto out = at::empty({B * S, H}, qkv.options());
  avk::attention_f32(qkv.data_ptr<float>(), ptr_or_null<float>(kbias), out.data_ptr<float>(), (int)B, (int)S, (int)nh,
                     (float)scale, cur_stream(qkv));
  return out;
}

// LN(word[ids] + pos[s] + type[tt]) for ids / tt int64 [B, S] (tt may be None: type 0)
at::Tensor embed_layernorm(const at::Tensor& ids, const c10::optional<at::Tensor>& tt, const at::Tensor& word,
                           const at::Tensor& pos, const at::Tensor& type, const at::Tensor& gamma,
                           const at::Tensor& beta, double eps, bool validate) {
  CHECK_DEV(ids);
  CHECK_DTYPE(ids, at::kLong);
  TORCH_CHECK(ids.dim() == 2 && ids.is_contiguous(), "embed_layernorm: ids [B, S]");
  const int64_t B = ids.size(0), S = ids.size(1), H = word.size(1);
  TORCH_CHECK(H >= 4 && H <= 1024 && H % 4 == 0, "embed_layernorm: 4 <= H <= 1024, H % 4 == 0");
  for (const at::Tensor* t : {&word, &pos, &type}) {
    CHECK_DEV((*t));
    CHECK_DTYPE((*t), at::kFloat);
    TORCH_CHECK(t->dim() == 2 && t->size(1) == H && t->is_contiguous() && aligned(*t, 16), "embedding tables [n, H]");
  }
  TORCH_CHECK(S <= pos.size(0), "embed_layernorm: sequence longer than the position table");
  check_opt_f32(gamma, H, "gamma");
  check_opt_f32(beta, H, "beta");
  // host-side index validation (a device -> host copy: callers that checked the ids before their
  // upload pass validate=False; the kernel clamps every gather into the tables regardless)
  if (validate) {
    const auto mm = at::aminmax(ids.cpu());
    TORCH_CHECK(std::get<0>(mm).item<int64_t>() >= 0 && std::get<1>(mm).item<int64_t>() < word.size(0),
                "embed_layernorm: token id out of range");
  }
  if (tt.has_value() && tt->defined()) {
    CHECK_DEV((*tt));
    CHECK_DTYPE((*tt), at::kLong);
    TORCH_CHECK(tt->sizes() == ids.sizes() && tt->is_contiguous(), "token types [B, S]");
    if (validate) {
      const auto tm = at::aminmax(tt->cpu());
      TORCH_CHECK(std::get<0>(tm).item<int64_t>() >= 0 && std::get<1>(tm).item<int64_t>() < type.size(0),
                  "embed_layernorm: token type out of range");
    }
  }
  TORCH_CHECK(word.size(0) >= 1 && type.size(0) >= 1, "embed_layernorm: empty embedding table");
  DevGuard g(ids.device());
  auto out = at::empty({B, S, H}, word.options());
  avk::embed_layernorm(reinterpret_cast<const long long*>(ids.data_ptr<int64_t>()),
                       tt.has_value() && tt->defined() ? reinterpret_cast<const long long*>(tt->data_ptr<int64_t>()) : nullptr,
                       word.data_ptr<float>(), pos.data_ptr<float>(), type.data_ptr<float>(), gamma.data_ptr<float>(),
                       beta.data_ptr<float>(), out.data_ptr<float>(), B * S, (int)S, (int)H, (float)eps, word.size(0),
                       (int)type.size(0), cur_stream(word));
  return out;
}

// C [M, N] = A^T B for A [K, M], B [K, N] fp32 (gemm.hip: split-K f32 MFMA + ordered slice sum)
at::Tensor gemm_tn(const at::Tensor& A, const at::Tensor& B, int64_t prec) {
  CHECK_DEV(A);
  CHECK_DTYPE(A, at::kFloat);
  CHECK_DEV(B);
  CHECK_DTYPE(B, at::kFloat);
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.size(0) == B.size(0) && A.is_contiguous() && B.is_contiguous(),
              "gemm_tn: A [K, M], B [K, N] contiguous");
  TORCH_CHECK(A.size(0) < (1LL << 31) && A.size(1) < (1LL << 31) && B.size(1) < (1LL << 31), "gemm_tn: dims < 2^31");
  const int K = (int)A.size(0), M = (int)A.size(1), N = (int)B.size(1);
  DevGuard g(A.device());
  auto C = at::empty({M, N}, A.options());
  if (K == 0) return C.zero_();
  const int S = avk::gemm_tn_slices(K, M, N);
  auto part = at::empty({(int64_t)S * M * N}, A.options());
  avk::gemm_tn(A.data_ptr<float>(), B.data_ptr<float>(), C.data_ptr<float>(), part.data_ptr<float>(), K, M, N, S,
               cur_stream(A), (int)prec);
  return C;
}

// One launch re-lays an fp32 layer's parameters (rnn_f32.hip lstm_pack_f32_kernel): w_ih [4H, I],
// w_hh [4H, H], b_ih / b_hh [4H] or None -> wfrag [NW,4,HP/4,64], wfragT [NW,HP,64], wihk [4HP, I], biask [4HP],
// wxfrag [NW,4,2,64] (I <= 8; empty otherwise).
std::vector<at::Tensor> lstm_pack_f32(const at::Tensor& w_ih, const at::Tensor& w_hh,
                                      const c10::optional<at::Tensor>& b_ih, const c10::optional<at::Tensor>& b_hh) {
  CHECK_DEV(w_ih);
  CHECK_DTYPE(w_ih, at::kFloat);
  CHECK_DEV(w_hh);
  CHECK_DTYPE(w_hh, at::kFloat);
  TORCH_CHECK(w_hh.dim() == 2 && w_hh.size(0) == 4 * w_hh.size(1) && w_hh.is_contiguous(), "w_hh must be [4H, H]");
  const int64_t H = w_hh.size(1), KS = lstm_ks(H), HP = 32 * KS;
  TORCH_CHECK(w_ih.dim() == 2 && w_ih.size(0) == 4 * H && w_ih.size(1) >= 1 && w_ih.is_contiguous(),
              "w_ih must be [4H, I]");
  const int64_t I = w_ih.size(1);
  check_opt_f32(b_ih, 4 * H, "b_ih");
  check_opt_f32(b_hh, 4 * H, "b_hh");
  DevGuard g(w_hh.device());
  auto f32 = w_hh.options();
  auto wfrag = at::empty({2 * KS, 4, HP / 4, 64}, f32), wfragT = at::empty({2 * KS, HP, 64}, f32);
  auto wihk = at::empty({4 * HP, I}, f32), biask = at::empty({4 * HP}, f32);
  // W_ih fragments of the in-kernel projection (narrow inputs only)
  auto wxfrag = I <= 8 ? at::empty({2 * KS, 4, 2, 64}, f32) : at::empty({0}, f32);
  avk::lstm_pack_f32(w_ih.data_ptr<float>(), w_hh.data_ptr<float>(), ptr_or_null<float>(b_ih), ptr_or_null<float>(b_hh),
                     (int)H, (int)I, (int)KS, wfrag.data_ptr<float>(), wfragT.data_ptr<float>(), wihk.data_ptr<float>(),
                     biask.data_ptr<float>(), I <= 8 ? wxfrag.data_ptr<float>() : nullptr, cur_stream(w_hh));
  return {wfrag, wfragT, wihk, biask, wxfrag};
}

// fp32 recurrence (rnn_f32.hip).  Input: xw [B, T, 4HP] fp32 kernel order (input projection + biases)
// OR, for I <= 8, (x [B, T, I], wxfrag, biask) and the projection runs in the kernel; x is also needed
// when training (the [h_{t-1} | x_t | 1] rows).  wfrag [NW, 4, HP/4, 64] fp32.  Returns hseq [B,T,H],
// cseq [B,T,HP] (+ gates [B,T,4HP] fp32 and hx [B,T,H+I+1] when training).
std::vector<at::Tensor> lstm_forward_f32(const c10::optional<at::Tensor>& xw, const at::Tensor& wfrag,
                                         const c10::optional<at::Tensor>& h0, const c10::optional<at::Tensor>& c0,
                                         int64_t H, bool training, const c10::optional<at::Tensor>& x,
                                         const c10::optional<at::Tensor>& wxfrag,
                                         const c10::optional<at::Tensor>& biask) {
  const int64_t KS = lstm_ks(H), HP = 32 * KS;
  const bool has_xw = xw.has_value() && xw->defined(), has_x = x.has_value() && x->defined();
  TORCH_CHECK(has_xw || has_x, "lstm_forward_f32: xw or x required");
  TORCH_CHECK(!training || has_x, "lstm_forward_f32: training needs x");
  int64_t B, T, I = 0;
  if (has_x) {
    CHECK_DEV((*x));
    CHECK_DTYPE((*x), at::kFloat);
    TORCH_CHECK(x->dim() == 3 && x->is_contiguous(), "x must be [B, T, I] contiguous");
    B = x->size(0), T = x->size(1), I = x->size(2);
  }
  if (has_xw) {
    CHECK_DEV((*xw));
    CHECK_DTYPE((*xw), at::kFloat);
    TORCH_CHECK(xw->dim() == 3 && xw->size(2) == 4 * HP && xw->is_contiguous(), "xw must be [B, T, 4HP] contiguous");
    TORCH_CHECK(aligned(*xw, 16), "xw must be 16-byte aligned");
    TORCH_CHECK(!has_x || (xw->size(0) == B && xw->size(1) == T), "xw / x shapes differ");
    B = xw->size(0), T = xw->size(1);
  } else {
    TORCH_CHECK(I >= 1 && I <= 8, "in-kernel projection needs 1 <= I <= 8");
    TORCH_CHECK(wxfrag.has_value() && wxfrag->defined() && biask.has_value() && biask->defined(),
                "in-kernel projection needs wxfrag and biask");
    check_opt_f32(wxfrag, 2 * KS * 4 * 2 * 64, "wxfrag");
    check_opt_f32(biask, 4 * HP, "biask");
    TORCH_CHECK(aligned(*biask, 16), "biask must be 16-byte aligned");
  }
  TORCH_CHECK(B >= 1 && T >= 1, "empty LSTM input");
  CHECK_DEV(wfrag);
  CHECK_DTYPE(wfrag, at::kFloat);
  TORCH_CHECK(wfrag.numel() == 2 * KS * 4 * (HP / 4) * 64, "wfrag must be [NW, 4, HP/4, 64]");
  check_opt_f32(h0, B * H, "h0");
  check_opt_f32(c0, B * H, "c0");
  DevGuard g(wfrag.device());
  auto f32 = wfrag.options();
  auto hseq = at::empty({B, T, H}, f32), cseq = at::empty({B, T, HP}, f32);
  at::Tensor gates, hx;
  if (training) {
    gates = at::empty({B, T, 4 * HP}, f32);
    hx = at::empty({B, T, H + I + 1}, f32);
  }
  avk::lstm_fwd_f32(has_xw ? xw->data_ptr<float>() : nullptr, has_x ? x->data_ptr<float>() : nullptr,
                    has_xw ? nullptr : wxfrag->data_ptr<float>(), has_xw ? nullptr : biask->data_ptr<float>(),
                    wfrag.data_ptr<float>(), ptr_or_null<float>(h0), ptr_or_null<float>(c0), (int)B, (int)T, (int)H,
                    (int)I, (int)KS, hseq.data_ptr<float>(), cseq.data_ptr<float>(),
                    training ? gates.data_ptr<float>() : nullptr, training ? hx.data_ptr<float>() : nullptr,
                    cur_stream(wfrag));
  if (training) return {hseq, cseq, gates, hx};
  return {hseq, cseq};
}

// fp32 backward recurrence: dz [B,T,4H] fp32 (torch gate order), dh0, dc0 [B,H]; wfragT [NW, HP, 64] fp32
std::vector<at::Tensor> lstm_backward_f32(const at::Tensor& dhseq, const at::Tensor& gates, const at::Tensor& cseq,
                                          const c10::optional<at::Tensor>& c0, const c10::optional<at::Tensor>& dhn,
                                          const c10::optional<at::Tensor>& dcn, const at::Tensor& wfragT, int64_t H) {
  const int64_t KS = lstm_ks(H), HP = 32 * KS;
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&dhseq, &gates, &cseq, &wfragT}) {
    CHECK_DEV((*t));
    CHECK_DTYPE((*t), at::kFloat);
    TORCH_CHECK(t->is_contiguous() && aligned(*t, 16), "LSTM backward inputs must be contiguous and 16-byte aligned");
  }
  TORCH_CHECK(dhseq.dim() == 3 && dhseq.size(2) == H, "dhseq must be [B, T, H]");
  const int64_t B = dhseq.size(0), T = dhseq.size(1);
  TORCH_CHECK(cseq.dim() == 3 && cseq.size(0) == B && cseq.size(1) == T && cseq.size(2) == HP,
              "cseq must be [B, T, HP]");
  TORCH_CHECK(gates.dim() == 3 && gates.size(0) == B && gates.size(1) == T && gates.size(2) == 4 * HP,
              "gates must be [B, T, 4HP]");
  TORCH_CHECK(wfragT.numel() == 2 * KS * HP * 64, "wfragT must be [NW, HP, 64]");
  check_opt_f32(c0, B * H, "c0");
  check_opt_f32(dhn, B * H, "dhn");
  check_opt_f32(dcn, B * H, "dcn");
  DevGuard g(dhseq.device());
  auto dz = at::empty({B, T, 4 * H}, dhseq.options());
  auto dh0 = at::empty({B, H}, dhseq.options()), dc0 = at::empty({B, H}, dhseq.options());
  avk::lstm_bwd_f32(dhseq.data_ptr<float>(), gates.data_ptr<float>(), cseq.data_ptr<float>(), ptr_or_null<float>(c0),
                    ptr_or_null<float>(dhn), ptr_or_null<float>(dcn), wfragT.data_ptr<float>(), (int)B, (int)T, (int)H,
                    (int)KS, dz.data_ptr<float>(), dh0.data_ptr<float>(), dc0.data_ptr<float>(), cur_stream(dhseq));
  return {dz, dh0, dc0};
}

std::vector<at::Tensor> lstm_backward(const at::Tensor& dhseq, const at::Tensor& gates, const at::Tensor& cseq,
                                      const c10::optional<at::Tensor>& c0, const c10::optional<at::Tensor>& dhn,
                                      const c10::optional<at::Tensor>& dcn, const at::Tensor& wfragT, int64_t H) {
  const int64_t KS = lstm_ks(H), HP = 32 * KS;
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&dhseq, &gates, &cseq}) {
    CHECK_DEV((*t));
    CHECK_DTYPE((*t), t == &gates ? at::kBFloat16 : at::kFloat);
    TORCH_CHECK(aligned(*t, 16), "LSTM backward inputs must be 16-byte aligned");
  }
  TORCH_CHECK(dhseq.dim() == 3 && dhseq.size(2) == H, "dhseq must be [B, T, H]");
  const int64_t B = dhseq.size(0), T = dhseq.size(1);
  TORCH_CHECK(cseq.dim() == 3 && cseq.size(0) == B && cseq.size(1) == T && cseq.size(2) == HP,
              "cseq must be [B, T, HP]");
  TORCH_CHECK(gates.dim() == 3 && gates.size(0) == B && gates.size(1) == T && gates.size(2) == 4 * HP,
              "gates must be [B, T, 4HP]");
  CHECK_DEV(wfragT);
  CHECK_DTYPE(wfragT, at::kBFloat16);
  TORCH_CHECK(wfragT.numel() == 2 * KS * 4 * KS * 64 * 8, "wfragT must be [NW, 4KS, 64, 8]");
  TORCH_CHECK(aligned(wfragT, 16), "wfragT must be 16-byte aligned");
  check_opt_f32(c0, B * H, "c0");
  check_opt_f32(dhn, B * H, "dhn");
  check_opt_f32(dcn, B * H, "dcn");
  DevGuard g(dhseq.device());
  auto dz = at::empty({B, T, 4 * HP}, dhseq.options().dtype(at::kBFloat16));
  auto dh0 = at::empty({B, H}, dhseq.options()), dc0 = at::empty({B, H}, dhseq.options());
  const int RT = avk::lstm_row_tiles(B, (int)KS);
  avk::lstm_bwd(dhseq.data_ptr<float>(), reinterpret_cast<const unsigned short*>(gates.data_ptr()),
                cseq.data_ptr<float>(), ptr_or_null<float>(c0), ptr_or_null<float>(dhn), ptr_or_null<float>(dcn),
                wfragT.data_ptr(), (int)B, (int)T, (int)H, (int)KS, RT,
                reinterpret_cast<unsigned short*>(dz.data_ptr()), dh0.data_ptr<float>(), dc0.data_ptr<float>(),
                cur_stream(dhseq));
  return {dz, dh0, dc0};
}

}  // namespace

void register_comm(py::module_& m);  // bind_comm.cpp

PYBIND11_MODULE(_C, m) {
  register_comm(m);
  m.doc() = "avenir_amd native kernels (HIP/CDNA4 gfx950) and host runtime";
  m.def("class_histogram", &class_histogram);
  m.def("pair_histogram", &pair_histogram);
  m.def("class_histogram_rowpacked", &class_histogram_rowpacked);
  m.def("pack_dense", &pack_dense);
  m.def("class_histogram_dense", &class_histogram_dense);
  m.def("bigram_histogram", &bigram_histogram);
  m.def("class_moments", &class_moments);
  m.def("nb_predict", &nb_predict);
  m.def("nb_predict_wide", &nb_predict_wide);
  m.def("node_histogram", &node_histogram, py::arg("codes"), py::arg("n"), py::arg("labels"), py::arg("node"),
        py::arg("weight"), py::arg("bins"), py::arg("offs"), py::arg("total_bins"), py::arg("n_classes"),
        py::arg("n_nodes"), py::arg("hist"), py::arg("node_rows") = py::none());
  m.def("node_grad_histogram", &node_grad_histogram, py::arg("codes"), py::arg("n"), py::arg("node"), py::arg("g"),
        py::arg("h"), py::arg("bins"), py::arg("offs"), py::arg("total_bins"), py::arg("n_nodes"), py::arg("out"),
        py::arg("even_only") = false, py::arg("tot_slot") = -1, py::arg("scale") = 65536.0);
  m.def("gbt_grad", &gbt_grad);
  m.def("gbt_split", &gbt_split);
  m.def("rank_avg", &rank_avg);
  m.def("tfidf_csr", &tfidf_csr);
  m.def("mixed_knn", &mixed_knn);
  m.def("pagerank", &pagerank);
  m.def("pagerank_multi", &pagerank_multi);
  m.def("sgns_hot_replicas", &avk::sgns_hot_replicas);
  m.def("sgns_step", &sgns_step, py::arg("Win"), py::arg("Wout"), py::arg("gIn"), py::arg("gOut"), py::arg("cIn"),
        py::arg("cOut"), py::arg("centre"), py::arg("context"), py::arg("aprob"), py::arg("alias"), py::arg("neg"),
        py::arg("lr"), py::arg("mean_in"), py::arg("seed"), py::arg("step"), py::arg("hot") = py::none(),
        py::arg("gOutHot") = py::none(), py::arg("gInHot") = py::none(), py::arg("cIn_next") = py::none(),
        py::arg("cOut_next") = py::none());
  m.def("kendall_pairs", &kendall_pairs);
  m.def("inversion_count", &inversion_count);
  m.def("resample_uniform", &resample_uniform);
  m.def("smote", &smote);
  m.def("gbt_assign", &gbt_assign);
  m.def("tree_assign", &tree_assign);
  m.def("tree_predict", &tree_predict);
  m.def("knn_topk", &knn_topk, py::arg("Q"), py::arg("R"), py::arg("k"), py::arg("q_base"), py::arg("r_base"),
        py::arg("exclude_self"), py::arg("splits"), py::arg("metric"), py::arg("p"), py::arg("prec") = -1);
  m.def("knn_mode", &avk::knn_mode);
  m.def("knn_vote", &knn_vote);
  m.def("cluster_accumulate", &cluster_accumulate);
  m.def("viterbi", &viterbi);
  m.def("viterbi_chunks", &viterbi_chunks);
  m.def("viterbi_backtrack", &viterbi_backtrack);
  m.def("markov_logodds", &markov_logodds);
  m.def("itemset_support", &itemset_support);
  m.def("build_bitsets", &build_bitsets);
  m.def("bandit_select", &bandit_select);
  m.def("sample", &sample);
  m.def("philox_normal", [](int64_t seed, int64_t offset, int64_t index_base, int64_t n, bool pairs,
                            c10::optional<at::Device> device) {
    TORCH_CHECK(n >= 0 && index_base >= 0, "philox_normal: n, index_base >= 0");
    if (device.has_value() && device->is_cuda()) {
      auto out = pairs ? at::empty({n, 2}, at::TensorOptions().dtype(at::kDouble).device(*device))
                       : at::empty({n}, at::TensorOptions().dtype(at::kDouble).device(*device));
      DevGuard g(*device);
      avk::philox_normal((unsigned long long)seed, (unsigned long long)offset, (unsigned long long)index_base, n,
                         out.data_ptr<double>(), pairs ? 1 : 0, cur_stream(out));
      return out;
    }
    auto out = pairs ? at::empty({n, 2}, at::TensorOptions().dtype(at::kDouble))
                     : at::empty({n}, at::TensorOptions().dtype(at::kDouble));
    {
      py::gil_scoped_release nogil;
      const unsigned hc = std::thread::hardware_concurrency();
      avh::philox_normal((uint64_t)seed, (uint64_t)offset, (uint64_t)index_base, n, out.data_ptr<double>(),
                         (int)std::min(16u, hc ? hc : 4u), pairs ? 1 : 0);
    }
    return out;
  }, "N(0,1) draws of Philox(seed, offset, index_base + i), host, fp64 (pairs: both Box-Muller outputs)",
        py::arg("seed"), py::arg("offset"), py::arg("index_base"), py::arg("n"), py::arg("pairs") = false,
        py::arg("device") = py::none());
  m.def("sa_assign", &sa_assign);
  m.def("ga_assign", &ga_assign);
  m.def("ga_assign_lds", [](int64_t P, int64_t L, int64_t r) { return (int64_t)avk::ga_assign_lds((int)P, (int)L, (int)r); });
  m.def("smote_lines", &smote_lines);
  m.def("format_device", &format_device);
  m.def("pairs_within", &pairs_within);
  m.def("mixed_knn_max_dims", []() { return avk::mixed_knn_max_dims(); });
  m.def("glm_gradient", &glm_gradient);
  m.def("smo_solve", &smo_solve);
  m.def("smo_ws_solve", &smo_ws_solve);
  m.def("smo_ws_select", &smo_ws_select);
  m.def("smo_ws_update", &smo_ws_update);
  m.def("smo_ws_run", &smo_ws_run);
  m.def("smo_ws_run_x", &smo_ws_run_x, py::arg("X"), py::arg("xn"), py::arg("kind"), py::arg("gamma"),
        py::arg("coef0"), py::arg("degree"), py::arg("alpha"), py::arg("G"), py::arg("y"), py::arg("C"), py::arg("eps"),
        py::arg("inner_iter"), py::arg("rel_tol"), py::arg("max_outer"), py::arg("check_every"), py::arg("ws"),
        py::arg("ok"), py::arg("dA"), py::arg("inner_total"), py::arg("gap"), py::arg("cache_slots") = 0,
        py::arg("cache_stats") = py::none());
  m.def("smo_ws_gather_x", &smo_ws_gather_x);
  m.def("smo_ws_update_x", &smo_ws_update_x);
  m.def("svm_kernel_matrix", &svm_kernel_matrix);
  m.def("rbf_matrix", &rbf_matrix);
  m.def("smo_ws_solve_fused", &smo_ws_solve_fused, py::arg("K"), py::arg("ws"), py::arg("ok"), py::arg("alpha"),
        py::arg("G"), py::arg("y"), py::arg("gap"), py::arg("C"), py::arg("eps"), py::arg("max_iter"), py::arg("dA"),
        py::arg("inner_total"), py::arg("rel_tol") = 0.1);
  m.def("smo_ws_size", &avk::smo_ws_size);
  m.def("nb_finalize", &nb_finalize);
  m.def("weighted_gram", &weighted_gram);
  m.def("kmeans_assign", &kmeans_assign);
  m.def("kmeans_reduce", &kmeans_reduce);
  m.def("kmeans_update", &kmeans_update);
  m.def("ngram_count", &ngram_count);
  m.def("uniformization", &uniformization);
  m.def("dot_matrix", &dot_matrix);
  m.def("gsp_join", &gsp_join);
  m.def("spirit_update", &spirit_update);
  m.def("col_moments", &col_moments);
  m.def("loo_stats", &loo_stats, py::arg("codes"), py::arg("n"), py::arg("y"), py::arg("slots") = -1);
  m.def("loo_apply", &loo_apply, py::arg("codes"), py::arg("n"), py::arg("y"), py::arg("sum"), py::arg("cnt"),
        py::arg("gmean"), py::arg("reg"), py::arg("noise") = py::none(), py::arg("amp") = 0.0,
        py::arg("slots") = -1);
  m.def("forest_hist", &forest_hist);
  m.def("bucketize_u8", &bucketize_u8);
  m.def("forest_split", &forest_split);
  m.def("forest_part_count", &forest_part_count);
  m.def("forest_part_scatter", &forest_part_scatter);
  m.def("forest_bootstrap", &forest_bootstrap);
  m.def("csv_parse_device", &csv_parse_device);
  m.def("forest_predict_bin", &forest_predict_bin);
  m.def("linear_act_fwd", &linear_act_fwd, py::arg("X"), py::arg("W"), py::arg("b") = py::none(), py::arg("act") = 0,
        py::arg("prec") = -1, py::arg("w_planes") = py::none());
  m.def("sbf16_weight_planes", &sbf16_weight_planes, py::arg("W"), py::arg("prec") = -1);
  m.def("linear_act_fwd_planes_bytes", [](int64_t M, int64_t N, int64_t K, int64_t prec) {
    return avk::linear_act_fwd_planes_bytes((int)M, (int)N, (int)K, (int)prec); },
        py::arg("M"), py::arg("N"), py::arg("K"), py::arg("prec") = -1);
  m.def("f32_gemm_mode", &avk::f32_gemm_mode);
  m.def("linear_act_bwd", &linear_act_bwd);
  m.def("linear_act_backward", &linear_act_backward);
  m.def("lstm_ks", &lstm_ks);
  m.def("lstm_forward", &lstm_forward);
  m.def("lstm_backward", &lstm_backward);
  m.def("lstm_forward_f32", &lstm_forward_f32, py::arg("xw"), py::arg("wfrag"), py::arg("h0"), py::arg("c0"),
        py::arg("H"), py::arg("training"), py::arg("x") = py::none(), py::arg("wxfrag") = py::none(),
        py::arg("biask") = py::none());
  m.def("lstm_pack_f32", &lstm_pack_f32);
  m.def("gemm_tn", &gemm_tn, py::arg("A"), py::arg("B"), py::arg("prec") = -1);
  m.def("gemm_tn_mode", &avk::gemm_tn_mode);
  m.def("add_layernorm", &add_layernorm);
  m.def("linear_add_layernorm", &linear_add_layernorm, py::arg("X"), py::arg("W"), py::arg("b"), py::arg("res"),
        py::arg("gamma"), py::arg("beta"), py::arg("eps"), py::arg("prec") = -1, py::arg("w_planes") = py::none());
  m.def("attention_f32", &attention_f32);
  m.def("embed_layernorm", &embed_layernorm, py::arg("ids"), py::arg("tt"), py::arg("word"), py::arg("pos"),
        py::arg("type"), py::arg("gamma"), py::arg("beta"), py::arg("eps"), py::arg("validate") = true);
  m.def("ref_split_score", &ref_split_score);
  m.def("lstm_backward_f32", &lstm_backward_f32);

  py::class_<avh::CsvFile>(m, "CsvFile")
      .def(py::init<const std::string&, const std::string&, bool, int>(), py::arg("path"), py::arg("delim") = ",",
           py::arg("skip_header") = false, py::arg("nthreads") = 8)
      .def(py::init([](std::vector<std::string> paths, int64_t rank, int64_t world, std::string delim, bool skip_header,
                       int nthreads) {
             py::gil_scoped_release rel;
             return new avh::CsvFile(paths, rank, world, delim, skip_header, nthreads);
           }),
           py::arg("paths"), py::arg("rank"), py::arg("world"), py::arg("delim") = ",", py::arg("skip_header") = false,
           py::arg("nthreads") = 8)
      .def("num_rows", &avh::CsvFile::num_rows)
      .def("max_fields", &avh::CsvFile::max_fields)
      .def("distinct", &avh::CsvFile::distinct)
      .def("column_strings", &avh::CsvFile::column_strings)
      .def("line", &avh::CsvFile::line)
      .def("lines", &avh::CsvFile::lines)
      .def("line_spans", [](const avh::CsvFile& f, int64_t b, int64_t e) {
        b = std::max<int64_t>(0, b);
        e = std::max(b, std::min<int64_t>(f.num_rows(), e));
        auto addr = at::empty({e - b}, at::kLong), len = at::empty({e - b}, at::kLong);
        f.line_spans(b, e, addr.data_ptr<int64_t>(), len.data_ptr<int64_t>());
        return py::make_tuple(addr, len);
      })
      .def("parse", &csv_parse, py::arg("specs"), py::arg("row_begin") = 0, py::arg("row_end") = -1);
  py::class_<avh::TextShard>(m, "TextShard")
      .def(py::init([](std::vector<std::string> paths, int64_t rank, int64_t world, int nthreads, bool skip_header) {
             py::gil_scoped_release rel;
             return new avh::TextShard(paths, rank, world, nthreads, skip_header);
           }),
           py::arg("paths"), py::arg("rank") = 0, py::arg("world") = 1, py::arg("nthreads") = 8,
           py::arg("skip_header") = false)
      .def("num_lines", &avh::TextShard::num_lines)
      .def("bytes_read", &avh::TextShard::bytes_read)
      .def("total_bytes", &avh::TextShard::total_bytes)
      .def("lines", &avh::TextShard::lines)
      .def("line_spans", [](const avh::TextShard& sh) {
        auto addr = at::empty({sh.num_lines()}, at::kLong), len = at::empty({sh.num_lines()}, at::kLong);
        sh.line_spans(addr.data_ptr<int64_t>(), len.data_ptr<int64_t>());
        return py::make_tuple(addr, len);
      })
      .def("tokenize", &text_tokenize, py::arg("delims") = ",", py::arg("sub_delim") = "", py::arg("modes") = "",
           py::arg("tail_mode") = "d", py::arg("trim") = false, py::arg("want_nums") = false,
           py::arg("last_mode") = "")
      .def("field_strings", &text_field_strings);
  m.def("text_tokenize_device", &text_tokenize_device, py::arg("paths"), py::arg("rank"), py::arg("world"),
        py::arg("delims") = ",", py::arg("sub_delim") = "", py::arg("modes") = "", py::arg("tail_mode") = "d",
        py::arg("trim") = false, py::arg("want_nums") = false, py::arg("like"),
        py::arg("max_initial_slots") = 1LL << 24, py::arg("last_mode") = "");
  m.def("format_columns", &format_columns_py, py::arg("cols"), py::arg("n"), py::arg("delim") = ",",
        py::arg("nthreads") = 8);
  m.def("format_rows", &format_rows);
  m.def("format_columns_file", &format_columns_file_py, py::arg("cols"), py::arg("n"), py::arg("delim"),
        py::arg("nthreads"), py::arg("path"), py::arg("append") = false);
  m.def("pack_spans", &pack_spans, py::arg("addr"), py::arg("len"), py::arg("nthreads") = 16);
  m.def("write_coded_csv", [](const std::string& path, const at::Tensor& codes, int64_t n,
                              std::vector<std::vector<std::string>> vocab, std::string id_prefix, std::string delim,
                              int nthreads) {
    TORCH_CHECK(!codes.is_cuda() && codes.scalar_type() == at::kByte && codes.dim() == 2,
                "codes must be a CPU uint8 [ncol, ld] tensor");
    TORCH_CHECK((int64_t)vocab.size() == codes.size(0) && n <= codes.size(1), "one vocabulary per column");
    auto c = codes.contiguous();
    py::gil_scoped_release rel;
    return avh::write_coded_csv(path, c.data_ptr<uint8_t>(), (int)c.size(0), c.size(1), n, vocab, id_prefix,
                                delim.empty() ? ',' : delim[0], nthreads);
  });
  py::class_<avh::SpscRing>(m, "SpscRing")
      .def(py::init<size_t, int>())
      .def("push", [](avh::SpscRing& r, std::vector<int64_t> rec) {
        TORCH_CHECK((int)rec.size() == r.rec_len(), "record length mismatch");
        return r.push(rec.data());
      })
      .def("pop_batch", [](avh::SpscRing& r, size_t max_n) {
        auto t = at::empty({(int64_t)max_n, r.rec_len()}, at::TensorOptions().dtype(at::kLong));
        size_t k = r.pop_batch(t.data_ptr<int64_t>(), max_n);
        return t.narrow(0, 0, (int64_t)k);
      })
      .def("size", &avh::SpscRing::size);
  m.def("write_container", [](const std::string& path, const std::string& header,
                              std::vector<at::Tensor> blobs) {
    std::vector<const void*> ptrs;
    std::vector<size_t> sizes;
    std::vector<at::Tensor> keep;
    for (auto& b : blobs) {
      auto c = b.cpu().contiguous();
      keep.push_back(c);
      ptrs.push_back(c.data_ptr());
      sizes.push_back((size_t)c.nbytes());
    }
    avh::write_container(path, header, ptrs, sizes);
  });
  m.def("read_container_header", [](const std::string& path) {
    uint64_t off = 0;
    std::string h = avh::read_container_header(path, &off);
    return py::make_tuple(h, off);
  });
  m.def("crc32", [](const at::Tensor& t, uint32_t seed) {
    auto c = t.cpu().contiguous();
    return avh::crc32(c.data_ptr(), (size_t)c.nbytes(), seed);
  }, py::arg("t"), py::arg("seed") = 0);
}
