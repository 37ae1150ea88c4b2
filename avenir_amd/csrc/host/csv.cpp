// K1 host half: memory-mapped multi-threaded CSV -> columnar encoder (see avenir_host.h).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <string_view>
#include <thread>

#include "avenir_host.h"
#include "avenir_numparse.h"

namespace avh {

namespace {

inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\r'; }

inline std::string_view trim(std::string_view s) {
  while (!s.empty() && is_space(s.front())) s.remove_prefix(1);
  while (!s.empty() && is_space(s.back())) s.remove_suffix(1);
  return s;
}

// Decimal parser (avenir_numparse.h, shared with the device K1 kernels): correctly rounded,
// strtod for the rare fields beyond the exact fast path; NaN on garbage / empty.
inline double parse_double(std::string_view s) {
  s = trim(s);
  bool slow = false;
  const double v = avnum::parse_decimal(s.data(), s.data() + s.size(), &slow);
  if (!slow) return v;
  const std::string z(s);
  return std::strtod(z.c_str(), nullptr);
}

inline int64_t parse_int(std::string_view s, bool* ok) {
  s = trim(s);
  *ok = false;
  if (s.empty()) return 0;
  const char* p = s.data();
  const char* e = p + s.size();
  bool neg = false;
  if (*p == '+' || *p == '-') { neg = (*p == '-'); ++p; }
  int64_t v = 0;
  int d = 0;
  while (p < e && *p >= '0' && *p <= '9') { v = v * 10 + (*p - '0'); ++p; ++d; }
  if (p < e && *p == '.') {  // tolerate "12.0" style ints (truncate like the reference's casts)
    ++p;
    while (p < e && *p >= '0' && *p <= '9') ++p;
  }
  if (d == 0 || p != e) return 0;
  *ok = true;
  return neg ? -v : v;
}

// Dictionary encoder: open-addressing table (FNV-1a over the trimmed bytes, linear probing, load
// <= 1/2) — one hash + one verified compare per field whatever the vocabulary size; random values
// no longer mispredict a per-entry comparison chain.
struct CatLookup {
  std::vector<std::string> vocab;
  std::vector<int32_t> slot;  // vocab index or -1
  uint32_t mask = 0;
  static inline uint32_t hash(const char* p, size_t n) {
    uint32_t h = 2166136261u;
    for (size_t i = 0; i < n; ++i) h = (h ^ (uint8_t)p[i]) * 16777619u;
    return h ^ (h >> 15);
  }
  explicit CatLookup(const std::vector<std::string>& v, bool wide, bool huge) : vocab(v) {
    const size_t cap = huge ? 0x7FFFFFFEu : (wide ? 65535 : 255);
    if (vocab.size() > cap)
      throw std::runtime_error("categorical cardinality " + std::to_string(vocab.size()) + " exceeds the " +
                               std::to_string(cap) + "-value code width");
    size_t sz = 16;
    while (sz < 2 * vocab.size()) sz <<= 1;
    slot.assign(sz, -1);
    mask = (uint32_t)(sz - 1);
    for (size_t i = 0; i < vocab.size(); ++i) {
      uint32_t h = hash(vocab[i].data(), vocab[i].size()) & mask;
      bool dup = false;
      while (slot[h] >= 0) {
        const std::string& o = vocab[(size_t)slot[h]];
        if (o == vocab[i]) { dup = true; break; }  // first occurrence keeps its code
        h = (h + 1) & mask;
      }
      if (!dup) slot[h] = (int32_t)i;
    }
  }
  // dictionary code, kUnknown when unknown (store_code clamps it to the column's missing code)
  static constexpr uint32_t kUnknown = 0xFFFFFFFFu;
  inline uint32_t code(std::string_view s) const {
    s = trim(s);
    uint32_t h = hash(s.data(), s.size()) & mask;
    while (true) {
      const int32_t i = slot[h];
      if (i < 0) return kUnknown;
      const std::string& v = vocab[(size_t)i];
      if (v.size() == s.size() && std::memcmp(v.data(), s.data(), s.size()) == 0) return (uint32_t)i;
      h = (h + 1) & mask;
    }
  }
};

inline void store_code(void* out, int64_t r, const ColSpec& sp, uint32_t code) {
  if (sp.huge) static_cast<int32_t*>(out)[r] = (int32_t)(code > 0x7FFFFFFFu ? 0x7FFFFFFFu : code);
  else if (sp.wide) static_cast<uint16_t*>(out)[r] = (uint16_t)(code > 65535 ? 65535 : code);
  else static_cast<uint8_t*>(out)[r] = (uint8_t)(code > 255 ? 255 : code);
}

}  // namespace

CsvFile::CsvFile(const std::string& path, const std::string& delim, bool skip_header, int nthreads)
    : delim_(delim.empty() ? std::string(",") : delim), nthreads_(std::max(1, nthreads)) {
  fd_ = ::open(path.c_str(), O_RDONLY);
  if (fd_ < 0) throw std::runtime_error("cannot open " + path);
  struct stat st;
  if (fstat(fd_, &st) != 0) throw std::runtime_error("cannot stat " + path);
  size_ = (size_t)st.st_size;
  if (size_ > 0) {
    // MAP_POPULATE: the kernel maps the whole (usually page-cached) file up front instead of one
    // fault per 4 KiB page inside the parsing threads
    void* m = mmap(nullptr, size_, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd_, 0);
    if (m == MAP_FAILED) throw std::runtime_error("mmap failed for " + path);
    madvise(m, size_, MADV_SEQUENTIAL);
    data_ = static_cast<const char*>(m);
  }
  index_lines(skip_header);
}

CsvFile::CsvFile(const std::vector<std::string>& paths, int64_t rank, int64_t world, const std::string& delim,
                 bool skip_header, int nthreads)
    : delim_(delim.empty() ? std::string(",") : delim), nthreads_(std::max(1, nthreads)) {
  ByteShard sh(paths, rank, world);
  owned_.resize((size_t)(sh.bytes() + (int64_t)sh.segments().size()) + 16, 0);
  size_ = (size_t)sh.copy_to(owned_.data(), true);
  data_ = owned_.data();
  index_lines(skip_header && rank == 0);
}

CsvFile::~CsvFile() {
  if (data_ && owned_.empty()) munmap(const_cast<char*>(data_), size_);
  if (fd_ >= 0) ::close(fd_);
}

void CsvFile::split(const char* p, const char* e, std::vector<std::string_view>& out, int max_fields) const {
  out.clear();
  const char* s = p;
  if (delim_.size() == 1) {
    const char d = delim_[0];
    for (const char* q = p; q <= e; ++q) {
      if (q == e || *q == d) {
        out.emplace_back(s, (size_t)(q - s));
        s = q + 1;
        if (max_fields >= 0 && (int)out.size() >= max_fields) return;
      }
    }
    return;
  }
  const size_t dl = delim_.size();
  const char* q = p;
  while (true) {
    const char* hit = nullptr;
    for (const char* c = q; c + dl <= e; ++c)
      if (*c == delim_[0] && std::memcmp(c, delim_.data(), dl) == 0) { hit = c; break; }
    if (!hit) { out.emplace_back(s, (size_t)(e - s)); return; }
    out.emplace_back(s, (size_t)(hit - s));
    if (max_fields >= 0 && (int)out.size() >= max_fields) return;
    s = q = hit + dl;
  }
}

void CsvFile::index_lines(bool skip_header) {
  // Two passes over line-aligned chunks, one thread per chunk: count the non-blank lines (and the
  // widest row), then write every line's [start, end) straight into its final slot — no per-thread
  // vectors growing and no concatenation copy (both cost more than the scan itself at 10^8 lines).
  const int T = (size_ < (1u << 20)) ? 1 : nthreads_;
  std::vector<size_t> bounds(T + 1, 0);
  bounds[T] = size_;
  for (int t = 1; t < T; ++t) {
    size_t b = size_ * t / T;
    while (b < size_ && data_[b - 1] != '\n') ++b;
    bounds[t] = b;
  }
  const bool single = delim_.size() == 1;
  const char dch = delim_[0];
  auto for_lines = [&](int t, auto&& fn) {
    size_t p = bounds[t];
    const size_t e = bounds[t + 1];
    while (p < e) {
      const char* nl = static_cast<const char*>(std::memchr(data_ + p, '\n', e - p));
      const size_t q = nl ? (size_t)(nl - data_) : e;
      size_t qe = q;
      if (qe > p && data_[qe - 1] == '\r') --qe;
      if (qe > p) fn(p, qe);  // blank lines are skipped
      p = q + 1;
    }
  };
  std::vector<int64_t> cnt(T, 0);
  std::vector<int> mf(T, 0);
  {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        int64_t c = 0;
        int m = 0;
        std::vector<std::string_view> f;
        for_lines(t, [&](size_t p, size_t qe) {
          ++c;
          int nf = 1;
          if (single) {
            const char* a = data_ + p;
            const size_t len = qe - p;
            for (size_t k = 0; k < len; ++k) nf += (a[k] == dch);
          } else {
            split(data_ + p, data_ + qe, f, -1);
            nf = (int)f.size();
          }
          m = std::max(m, nf);
        });
        cnt[t] = c;
        mf[t] = m;
      });
    for (auto& x : th) x.join();
  }
  std::vector<int64_t> off(T + 1, 0);
  for (int t = 0; t < T; ++t) {
    off[t + 1] = off[t] + cnt[t];
    max_fields_ = std::max(max_fields_, mf[t]);
  }
  line_start_.resize((size_t)off[T]);
  line_end_.resize((size_t)off[T]);
  {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        int64_t* ls = line_start_.data() + off[t];
        int64_t* le = line_end_.data() + off[t];
        int64_t i = 0;
        for_lines(t, [&](size_t p, size_t qe) {
          ls[i] = (int64_t)p;
          le[i] = (int64_t)qe;
          ++i;
        });
      });
    for (auto& x : th) x.join();
  }
  if (skip_header && !line_start_.empty()) {
    line_start_.erase(line_start_.begin());
    line_end_.erase(line_end_.begin());
  }
}

int64_t CsvFile::parse(const std::vector<ColSpec>& specs, const std::vector<void*>& outs,
                       int64_t row_begin, int64_t row_end) {
  if (specs.size() != outs.size()) throw std::runtime_error("specs/outs length mismatch");
  row_begin = std::max<int64_t>(0, row_begin);
  row_end = std::min<int64_t>(num_rows(), row_end < 0 ? num_rows() : row_end);
  const int64_t base = row_begin;
  const int64_t n = std::max<int64_t>(0, row_end - row_begin);
  std::vector<std::unique_ptr<CatLookup>> cats(specs.size());
  int max_ord = 0;
  for (size_t i = 0; i < specs.size(); ++i) {
    if (specs[i].kind == CAT) cats[i] = std::make_unique<CatLookup>(specs[i].vocab, specs[i].wide, specs[i].huge);
    max_ord = std::max(max_ord, specs[i].ordinal);
  }
  // ordinal -> list of spec indices
  std::vector<std::vector<int>> by_ord(max_ord + 1);
  for (size_t i = 0; i < specs.size(); ++i) by_ord[specs[i].ordinal].push_back((int)i);

  const int T = n < 4096 ? 1 : nthreads_;
  std::vector<int64_t> bad(T, 0);
  const bool single = delim_.size() == 1;
  const char dch = delim_[0];
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) {
    th.emplace_back([&, t] {
      const int64_t r0 = n * t / T, r1 = n * (t + 1) / T;
      std::vector<std::string_view> fields;
      fields.reserve(max_ord + 2);
      auto emit = [&](int si, int64_t r, bool have, std::string_view fv) {
        const ColSpec& sp = specs[si];
        switch (sp.kind) {
          case CAT:
            store_code(outs[si], r, sp, have ? cats[si]->code(fv) : CatLookup::kUnknown);
            break;
          case BUCKET: {
            uint32_t c = CatLookup::kUnknown;
            if (have) {
              const double v = parse_double(fv);
              if (!std::isnan(v)) {
                // the reference uses integer division: Integer.parseInt(v) / bucketWidth
                const long long b = (long long)std::floor(v / sp.bucket_width) - sp.bucket_offset;
                if (b >= 0 && b <= sp.max_code) c = (uint32_t)b;
              }
            }
            store_code(outs[si], r, sp, c);
            break;
          }
          case FLOAT:
            static_cast<float*>(outs[si])[r] = have ? (float)parse_double(fv) : NAN;
            break;
          case INT: {
            bool ok = false;
            const int64_t v = have ? parse_int(fv, &ok) : 0;
            static_cast<int64_t*>(outs[si])[r] = ok ? v : INT64_MIN;
            break;
          }
          default:
            break;
        }
      };
      for (int64_t r = r0; r < r1; ++r) {
        const char* p = data_ + line_start_[base + r];
        const char* e = data_ + line_end_[base + r];
        int o = 0;
        if (single) {  // walk the fields in place (no per-row field vector)
          const char* a = p;
          while (o <= max_ord) {
            const char* q = a;
            while (q < e && *q != dch) ++q;
            for (int si : by_ord[o]) emit(si, r, true, std::string_view(a, (size_t)(q - a)));
            ++o;
            if (q >= e) break;
            a = q + 1;
          }
        } else {
          split(p, e, fields, max_ord + 1);
          for (; o <= max_ord && o < (int)fields.size(); ++o)
            for (int si : by_ord[o]) emit(si, r, true, fields[o]);
        }
        bool short_row = false;
        for (; o <= max_ord; ++o)
          for (int si : by_ord[o]) {
            short_row = true;
            emit(si, r, false, std::string_view());
          }
        if (short_row) ++bad[t];
      }
    });
  }
  for (auto& x : th) x.join();
  int64_t b = 0;
  for (auto v : bad) b += v;
  return b;
}

std::vector<std::string> CsvFile::distinct(int ordinal, size_t limit) {
  std::vector<std::string> out;
  std::unordered_map<std::string, int> seen;
  const int64_t n = num_rows();
  std::vector<std::string_view> f;
  for (int64_t r = 0; r < n; ++r) {
    split(data_ + line_start_[r], data_ + line_end_[r], f, ordinal + 1);
    if ((int)f.size() <= ordinal) continue;
    std::string v(trim(f[ordinal]));
    if (seen.emplace(v, 1).second) {
      out.push_back(v);
      if (out.size() >= limit) return out;
    }
  }
  return out;
}

std::vector<std::string> CsvFile::column_strings(int ordinal) {
  const int64_t n = num_rows();
  std::vector<std::string> out(n);
  std::vector<std::string_view> f;
  for (int64_t r = 0; r < n; ++r) {
    split(data_ + line_start_[r], data_ + line_end_[r], f, ordinal + 1);
    if ((int)f.size() > ordinal) out[r] = std::string(trim(f[ordinal]));
  }
  return out;
}

std::string CsvFile::line(int64_t i) const {
  if (i < 0 || i >= num_rows()) throw std::out_of_range("line index");
  return std::string(data_ + line_start_[i], (size_t)(line_end_[i] - line_start_[i]));
}

std::vector<std::string> CsvFile::lines(int64_t b, int64_t e) const {
  b = std::max<int64_t>(0, b);
  e = std::min<int64_t>(num_rows(), e);
  std::vector<std::string> out;
  out.reserve(std::max<int64_t>(0, e - b));
  for (int64_t i = b; i < e; ++i)
    out.emplace_back(data_ + line_start_[i], (size_t)(line_end_[i] - line_start_[i]));
  return out;
}

void CsvFile::line_spans(int64_t b, int64_t e, int64_t* addr, int64_t* len) const {
  b = std::max<int64_t>(0, b);
  e = std::min<int64_t>(num_rows(), e);
  const int64_t base = (int64_t)reinterpret_cast<uintptr_t>(data_);
  for (int64_t i = b; i < e; ++i) {
    addr[i - b] = base + line_start_[(size_t)i];
    len[i - b] = line_end_[(size_t)i] - line_start_[(size_t)i];
  }
}

std::string format_rows(const std::vector<std::string>* prefix, const double* cols, int ncol,
                        int64_t n, const std::vector<int>& precision, char delim, int nthreads) {
  const int T = n < 8192 ? 1 : std::max(1, nthreads);
  std::vector<std::string> parts(T);
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) {
    th.emplace_back([&, t] {
      const int64_t r0 = n * t / T, r1 = n * (t + 1) / T;
      std::string& s = parts[t];
      s.reserve((size_t)(r1 - r0) * (16 + 12 * ncol));
      char buf[64];
      for (int64_t r = r0; r < r1; ++r) {
        bool first = true;
        if (prefix) { s += (*prefix)[r]; first = false; }
        for (int c = 0; c < ncol; ++c) {
          if (!first) s.push_back(delim);
          first = false;
          const double v = cols[(int64_t)c * n + r];
          const int pr = c < (int)precision.size() ? precision[c] : 6;
          int len;
          if (pr < 0) len = snprintf(buf, sizeof buf, "%lld", (long long)std::llround(v));
          else len = snprintf(buf, sizeof buf, "%.*f", pr, v);
          s.append(buf, (size_t)len);
        }
        s.push_back('\n');
      }
    });
  }
  for (auto& x : th) x.join();
  size_t tot = 0;
  for (auto& p : parts) tot += p.size();
  std::string out;
  out.reserve(tot);
  for (auto& p : parts) out += p;
  return out;
}

// Coded records -> delimited text file: row r = id_prefix + r, then vocab[f][codes[f][r]] for every
// column f (uint8 codes, column-major [ncol][ld]).  Threads format contiguous row blocks into
// private buffers which are written to the file in order (the ingest-inclusive benchmark and the
// fixture generators write 10^8-row files at several GB/s instead of through Python strings).
int64_t write_coded_csv(const std::string& path, const uint8_t* codes, int ncol, int64_t ld, int64_t n,
                        const std::vector<std::vector<std::string>>& vocab, const std::string& id_prefix,
                        char delim, int nthreads) {
  FILE* fp = fopen(path.c_str(), "wb");
  if (!fp) throw std::runtime_error("write_coded_csv: cannot open " + path);
  const int64_t block = 1 << 20;
  const int T = std::max(1, nthreads);
  int64_t written = 0;
  std::vector<std::string> bufs(T);
  for (int64_t b0 = 0; b0 < n; b0 += block * T) {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) {
      th.emplace_back([&, t] {
        const int64_t r0 = std::min(n, b0 + block * t), r1 = std::min(n, r0 + block);
        std::string& s = bufs[t];
        s.clear();
        s.reserve((size_t)(r1 - r0) * (size_t)(12 + 8 * ncol));
        char nb[32];
        for (int64_t r = r0; r < r1; ++r) {
          s += id_prefix;
          const int len = snprintf(nb, sizeof nb, "%lld", (long long)r);
          s.append(nb, (size_t)len);
          for (int c = 0; c < ncol; ++c) {
            s.push_back(delim);
            const unsigned v = codes[(int64_t)c * ld + r];
            const auto& vc = vocab[(size_t)c];
            if (v < vc.size()) s += vc[v];
          }
          s.push_back('\n');
        }
      });
    }
    for (auto& x : th) x.join();
    for (int t = 0; t < T; ++t) {
      if (!bufs[t].empty() && fwrite(bufs[t].data(), 1, bufs[t].size(), fp) != bufs[t].size()) {
        fclose(fp);
        throw std::runtime_error("write_coded_csv: short write");
      }
      written += (int64_t)bufs[t].size();
    }
  }
  fclose(fp);
  return written;
}

}  // namespace avh
