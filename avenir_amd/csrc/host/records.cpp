// K1 for the reference's non-schema record layouts: byte-range sharded text input + a
// multi-threaded tokenizer with a shard-wide string dictionary (see avenir_host.h, TextShard).
//
// Every reference mapper splits its line with String.split and then looks the tokens up in a
// HashMap (state sequences J/markov/MarkovStateTransitionModel.java:116-133, transactions
// J/association/FrequentItemsApriori.java:133-196, obs:state tokens
// J/markov/HiddenMarkovModelBuilder.java:136-260, pair-distance rows
// J/explore/TopMatchesByClass.java:133-211 and J/knn/NearestNeighbor.java:130-183, time-stamped
// events S/markov/StateTransitionRate.scala:91-167).  Here one native pass turns a rank's bytes
// into a CSR token table:
//   * the rank reads ONLY its byte range of the concatenated input files (Hadoop's input split:
//     a line belongs to the range holding its first byte), with parallel pread;
//   * blank lines (whitespace only) are dropped, a trailing CR is removed;
//   * every field becomes a token: a dictionary code (first-occurrence order over the shard, one
//     dictionary for all fields), a parsed double, or nothing, by a per-field mode; an optional
//     sub-delimiter splits each token once more (``obs:state``) into a second code;
//   * threads tokenize line blocks with private dictionaries that are merged in block order, so
//     the codes do not depend on the thread count.
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

inline bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\v' || c == '\f'; }

// decimal parser shared with csv.cpp and the device tokenizer (avenir_numparse.h: correctly
// rounded; strtod for the rare fields beyond the exact fast path), NaN on garbage / empty
inline double parse_num(const char* p, const char* e) {
  while (p < e && is_ws(*p)) ++p;
  while (e > p && is_ws(e[-1])) --e;
  bool slow = false;
  const double v = avnum::parse_decimal(p, e, &slow);
  if (!slow) return v;
  const std::string s(p, e);
  return std::strtod(s.c_str(), nullptr);
}

// 64-bit hash of a short byte string in 8-byte words (a partial last word is loaded whole and
// masked when the load cannot cross a page).  The device tokenizer (records.hip) uses the same
// function, so hash partitions agree between the two paths.
inline uint64_t hash_bytes(const char* p, size_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ (n * 0xC2B2AE3D27D4EB4Full);
  while (n >= 8) {
    uint64_t w;
    std::memcpy(&w, p, 8);
    h = (h ^ w) * 0xFF51AFD7ED558CCDull;
    h ^= h >> 32;
    p += 8;
    n -= 8;
  }
  if (n) {
    uint64_t w = 0;
    if (((uintptr_t)p & 4095) <= 4088) {  // the 8-byte load stays inside p's (mapped) page
      std::memcpy(&w, p, 8);
      w &= (~0ull) >> (8 * (8 - n));
    } else {
      std::memcpy(&w, p, n);
    }
    h = (h ^ w) * 0xFF51AFD7ED558CCDull;
    h ^= h >> 32;
  }
  h *= 0xC4CEB9FE1A85EC53ull;
  return h ^ (h >> 29);
}

// Open-addressing string dictionary over views into the shard buffer; ids in insertion order.
struct Dict {
  std::vector<uint64_t> hs;
  std::vector<int32_t> slot;  // id or -1
  std::vector<std::string_view> words;
  std::vector<uint64_t> whash;
  uint64_t mask = 0;
  Dict() { rehash(64); }
  void rehash(size_t sz) {
    slot.assign(sz, -1);
    hs.assign(sz, 0);
    mask = sz - 1;
    for (size_t i = 0; i < words.size(); ++i) {
      uint64_t s = whash[i] & mask;
      while (slot[s] >= 0) s = (s + 1) & mask;
      slot[s] = (int32_t)i;
      hs[s] = whash[i];
    }
  }
  inline int32_t get_or_add(std::string_view w, uint64_t h) {
    uint64_t s = h & mask;
    while (true) {
      const int32_t id = slot[s];
      if (id < 0) break;
      if (hs[s] == h) {
        const std::string_view& o = words[(size_t)id];
        if (o.size() == w.size() && std::memcmp(o.data(), w.data(), w.size()) == 0) return id;
      }
      s = (s + 1) & mask;
    }
    const int32_t id = (int32_t)words.size();
    if (words.size() >= (size_t)INT32_MAX - 1) throw std::runtime_error("TextShard: dictionary exceeds 2^31 entries");
    slot[s] = id;
    hs[s] = h;
    words.push_back(w);
    whash.push_back(h);
    if (2 * words.size() > slot.size()) rehash(slot.size() * 2);
    return id;
  }
};

void pread_all(int fd, char* dst, int64_t off, int64_t len, const std::string& path) {
  while (len > 0) {
    const ssize_t r = ::pread(fd, dst, (size_t)std::min<int64_t>(len, 1LL << 30), off);
    if (r <= 0) throw std::runtime_error("TextShard: read failed for " + path);
    dst += r;
    off += r;
    len -= r;
  }
}

// first position >= from holding '\n' (or size when none)
int64_t find_newline(int fd, int64_t from, int64_t size, const std::string& path) {
  char probe[1 << 16];
  while (from < size) {
    const int64_t n = std::min<int64_t>((int64_t)sizeof probe, size - from);
    pread_all(fd, probe, from, n, path);
    const void* hit = std::memchr(probe, '\n', (size_t)n);
    if (hit) return from + (int64_t)(static_cast<const char*>(hit) - probe);
    from += n;
  }
  return size;
}

}  // namespace

ByteShard::ByteShard(const std::vector<std::string>& paths, int64_t rank, int64_t world, bool populate) {
  if (world < 1 || rank < 0 || rank >= world) throw std::runtime_error("byte shard: bad rank / world");
  std::vector<int64_t> sizes;
  for (const auto& p : paths) {
    struct stat st;
    if (::stat(p.c_str(), &st) != 0) throw std::runtime_error("byte shard: cannot stat " + p);
    sizes.push_back((int64_t)st.st_size);
    total_bytes_ += (int64_t)st.st_size;
  }
  // this rank's global byte range [lo, hi) of the concatenated files
  const int64_t lo = total_bytes_ * rank / world, hi = total_bytes_ * (rank + 1) / world;
  const int64_t page = (int64_t)sysconf(_SC_PAGESIZE);
  int64_t base = 0;
  for (size_t f = 0; f < paths.size(); ++f) {
    const int64_t fs = sizes[f], a0 = std::max(lo, base) - base, b0 = std::min(hi, base + fs) - base;
    base += fs;
    if (a0 >= b0) continue;
    const int fd = ::open(paths[f].c_str(), O_RDONLY);
    if (fd < 0) throw std::runtime_error("byte shard: cannot open " + paths[f]);
    // a line belongs to the range holding its first byte
    const int64_t a = a0 == 0 ? 0 : find_newline(fd, a0 - 1, fs, paths[f]) + 1;
    const int64_t b = std::min(fs, find_newline(fd, b0 - 1, fs, paths[f]) + 1);
    if (a < b0 && a < b) {
      // map only [a, b) (page-aligned): MAP_POPULATE faults in exactly this rank's pages
      const int64_t ma = a / page * page;
      const size_t mlen = (size_t)(b - ma);
      void* m = mmap(nullptr, mlen, PROT_READ, MAP_PRIVATE | (populate ? MAP_POPULATE : 0), fd, (off_t)ma);
      if (m == MAP_FAILED) {
        ::close(fd);
        throw std::runtime_error("byte shard: mmap failed for " + paths[f]);
      }
      madvise(m, mlen, MADV_SEQUENTIAL);
      segs_.push_back({static_cast<const char*>(m) + (a - ma), b - a, m, mlen, (int)f, a});
      bytes_ += b - a;
    }
    ::close(fd);
  }
}

ByteShard::~ByteShard() {
  for (auto& s : segs_) munmap(s.map, s.map_len);
}

int64_t ByteShard::copy_to(char* dst, bool terminate) const {
  int64_t w = 0;
  for (auto& s : segs_) {
    std::memcpy(dst + w, s.p, (size_t)s.len);
    w += s.len;
    if (terminate && s.len > 0 && s.p[s.len - 1] != '\n') dst[w++] = '\n';
  }
  return w;
}

TextShard::TextShard(const std::vector<std::string>& paths, int64_t rank, int64_t world, int nthreads,
                     bool skip_header)
    : bytes_(paths, rank, world), nthreads_(std::max(1, nthreads)) {
  index_lines(skip_header && rank == 0);
}

void TextShard::index_lines(bool skip_header) {
  // chunks: each segment split at newlines into pieces of ~1/T of the shard
  struct Piece {
    const char* a;
    const char* e;
  };
  std::vector<Piece> pieces;
  const int64_t total = std::max<int64_t>(1, bytes_.bytes());
  const int T = total < (1 << 20) ? 1 : nthreads_;
  for (auto& sg : bytes_.segments()) {
    const int k = (int)std::max<int64_t>(1, (int64_t)T * sg.len / total);
    const char* a = sg.p;
    const char* end = sg.p + sg.len;
    for (int i = 1; i <= k; ++i) {
      const char* b = i == k ? end : sg.p + sg.len * i / k;
      while (b < end && b > sg.p && b[-1] != '\n') ++b;
      if (b > a) pieces.push_back({a, b});
      a = std::max(a, b);
    }
  }
  const int P = (int)pieces.size();
  auto for_lines = [&](int t, auto&& fn) {
    const char* p = pieces[t].a;
    const char* e = pieces[t].e;
    while (p < e) {
      const char* nl = static_cast<const char*>(std::memchr(p, '\n', (size_t)(e - p)));
      const char* q = nl ? nl : e;
      const char* qe = q;
      if (qe > p && qe[-1] == '\r') --qe;
      const char* k = p;
      while (k < qe && is_ws(*k)) ++k;
      if (k < qe) fn(p, qe);
      p = q + 1;
    }
  };
  std::vector<int64_t> cnt(P, 0);
  auto run = [&](auto&& body) {
    std::vector<std::thread> th;
    for (int t = 0; t < P; ++t) th.emplace_back([&, t] { body(t); });
    for (auto& x : th) x.join();
  };
  run([&](int t) {
    int64_t c = 0;
    for_lines(t, [&](const char*, const char*) { ++c; });
    cnt[t] = c;
  });
  std::vector<int64_t> off(P + 1, 0);
  for (int t = 0; t < P; ++t) off[t + 1] = off[t] + cnt[t];
  ls_.resize((size_t)off[P]);
  le_.resize((size_t)off[P]);
  run([&](int t) {
    int64_t i = off[t];
    for_lines(t, [&](const char* p, const char* qe) {
      ls_[(size_t)i] = p;
      le_[(size_t)i] = qe;
      ++i;
    });
  });
  if (skip_header && !ls_.empty()) {
    ls_.erase(ls_.begin());
    le_.erase(le_.begin());
  }
}

std::vector<std::string> TextShard::lines(int64_t b, int64_t e) const {
  b = std::max<int64_t>(0, b);
  e = std::min<int64_t>(num_lines(), e);
  std::vector<std::string> out;
  out.reserve((size_t)std::max<int64_t>(0, e - b));
  for (int64_t i = b; i < e; ++i) out.emplace_back(ls_[(size_t)i], (size_t)(le_[(size_t)i] - ls_[(size_t)i]));
  return out;
}

void TextShard::line_spans(int64_t* addr, int64_t* len) const {
  for (size_t i = 0; i < ls_.size(); ++i) {
    addr[i] = (int64_t)reinterpret_cast<uintptr_t>(ls_[i]);
    len[i] = (int64_t)(le_[i] - ls_[i]);
  }
}

int64_t TextShard::count_tokens(const TokenSpec& spec) {
  spec_ = spec;
  if (spec_.delims.empty()) spec_.delims = ",";
  for (int c = 0; c < 256; ++c) sep_[c] = 0;
  for (char c : spec_.delims) sep_[(uint8_t)c] = 1;
  const int64_t L = num_lines();
  const int T = L < 4096 ? 1 : nthreads_;
  tok_lines_.assign(T + 1, 0);
  for (int t = 0; t <= T; ++t) tok_lines_[t] = L * t / T;
  tok_cnt_.assign(T + 1, 0);
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      int64_t c = 0;
      for (int64_t l = tok_lines_[t]; l < tok_lines_[t + 1]; ++l) {
        int64_t n = 1;
        for (const char* k = ls_[(size_t)l]; k < le_[(size_t)l]; ++k) n += sep_[(uint8_t)*k];
        c += n;
      }
      tok_cnt_[t + 1] = c;
    });
  for (auto& x : th) x.join();
  for (int t = 0; t < T; ++t) tok_cnt_[t + 1] += tok_cnt_[t];
  return tok_cnt_[T];
}

void TextShard::tokenize(int64_t* off, int32_t* codes, int32_t* sub, double* nums) {
  const int T = (int)tok_lines_.size() - 1;
  if (T < 1) throw std::runtime_error("TextShard: count_tokens() first");
  const TokenSpec& sp = spec_;
  const int nm = (int)sp.modes.size();
  std::vector<Dict> dicts(T);
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      Dict& D = dicts[t];
      int64_t k = tok_cnt_[t];
      for (int64_t l = tok_lines_[t]; l < tok_lines_[t + 1]; ++l) {
        off[l] = k;
        const char* p = ls_[(size_t)l];
        const char* e = le_[(size_t)l];
        int f = 0;
        while (true) {
          const char* q = p;
          while (q < e && !sep_[(uint8_t)*q]) ++q;
          const char m = (q >= e && sp.last_mode) ? sp.last_mode : (f < nm ? sp.modes[(size_t)f] : sp.tail_mode);
          const char* a = p;
          const char* b = q;
          if (sp.trim) {
            while (a < b && is_ws(*a)) ++a;
            while (b > a && is_ws(b[-1])) --b;
          }
          int32_t c = -1, s2 = -1;
          double v = std::nan("");
          if (m == 'd') {
            const char* mid = b;
            if (sp.sub_delim) {
              const void* h = std::memchr(a, sp.sub_delim, (size_t)(b - a));
              if (h) mid = static_cast<const char*>(h);
            }
            c = D.get_or_add(std::string_view(a, (size_t)(mid - a)), hash_bytes(a, (size_t)(mid - a)));
            if (mid < b) s2 = D.get_or_add(std::string_view(mid + 1, (size_t)(b - mid - 1)), hash_bytes(mid + 1, (size_t)(b - mid - 1)));
          } else if (m == 'n') {
            v = parse_num(a, b);
          }
          codes[k] = c;
          if (sub) sub[k] = s2;
          if (nums) nums[k] = v;
          ++k;
          ++f;
          if (q >= e) break;
          p = q + 1;
        }
      }
    });
  for (auto& x : th) x.join();
  off[num_lines()] = tok_cnt_[T];
  // merge the block dictionaries in block order (= first occurrence over the shard)
  Dict G;
  std::vector<std::vector<int32_t>> remap(T);
  for (int t = 0; t < T; ++t) {
    const Dict& D = dicts[t];
    remap[t].resize(D.words.size());
    for (size_t i = 0; i < D.words.size(); ++i) remap[t][i] = G.get_or_add(D.words[i], D.whash[i]);
  }
  vocab_.clear();
  vocab_.reserve(G.words.size());
  for (auto& w : G.words) vocab_.emplace_back(w);
  th.clear();
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      const int32_t* r = remap[t].data();
      bool ident = true;
      for (size_t i = 0; i < remap[t].size(); ++i) ident &= (r[i] == (int32_t)i);
      if (ident) return;  // block 0 (and any block adding nothing new) keeps its codes
      for (int64_t k = tok_cnt_[t]; k < tok_cnt_[t + 1]; ++k) {
        if (codes[k] >= 0) codes[k] = r[codes[k]];
        if (sub && sub[k] >= 0) sub[k] = r[sub[k]];
      }
    });
  for (auto& x : th) x.join();
}

std::vector<std::string> TextShard::field_strings(const int64_t* line, const int32_t* field, int64_t n) const {
  std::vector<std::string> out((size_t)n);
  const bool have_spec = !spec_.delims.empty();
  for (int64_t i = 0; i < n; ++i) {
    const int64_t l = line[i];
    if (l < 0 || l >= num_lines()) throw std::out_of_range("TextShard::field_strings: line index");
    const char* p = ls_[(size_t)l];
    const char* e = le_[(size_t)l];
    int f = 0;
    while (true) {
      const char* q = p;
      while (q < e && !(have_spec ? sep_[(uint8_t)*q] : *q == ',')) ++q;
      if (f == field[i]) {
        out[(size_t)i].assign(p, (size_t)(q - p));
        break;
      }
      if (q >= e) break;
      p = q + 1;
      ++f;
    }
  }
  return out;
}

}  // namespace avh
