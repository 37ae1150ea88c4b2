// Native output formatting for the CLI jobs: rows assembled from string-table lookups, numbers,
// literals and variable-length string lists (CSR), by several threads into one buffer.  The
// reference's reducers write one Text line per record through Hadoop's TextOutputFormat; jobs here
// produce millions of output lines per rank (neighbour lists, per-entity predictions), which Python
// string joins would spend seconds on.
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <array>
#include <atomic>
#include <fcntl.h>
#include <sys/mman.h>
#include <algorithm>
#include <unistd.h>
#include <thread>

#include "avenir_host.h"

namespace avh {

namespace {

// Output cursor over a growable buffer: every row first reserves an upper bound of its bytes
// (``ensure``), then the writers copy with plain pointer arithmetic — no per-append capacity check.
struct Out {
  std::string buf;
  size_t pos = 0;
  char* w = nullptr;
  void ensure(size_t k) {
    if (buf.size() - pos < k) {
      buf.resize(std::max(buf.size() * 2, pos + k + (1u << 16)));
    }
    w = buf.data() + pos;
  }
  void commit() { pos = (size_t)(w - buf.data()); }
  void put(const char* p, size_t n) {
    std::memcpy(w, p, n);
    w += n;
  }
  void put(char c) { *w++ = c; }
};

// Python's repr(float): the shortest digit string that round-trips (std::to_chars), written in
// fixed notation for decimal exponents -4 <= e < 16 and as d.ddde[+-]XX otherwise.  <= 32 bytes.
inline void put_pyrepr(Out& o, double v) {
  if (std::isnan(v)) {
    o.put("nan", 3);
    return;
  }
  if (std::isinf(v)) {
    if (v < 0) o.put("-inf", 4);
    else o.put("inf", 3);
    return;
  }
  char buf[40];
  auto res = std::to_chars(buf, buf + sizeof buf, v, std::chars_format::scientific);
  const char* p = buf;
  const char* end = res.ptr;
  if (*p == '-') {
    o.put('-');
    ++p;
  }
  char dig[24];
  int nd = 0;
  const char* q = p;
  for (; q < end && *q != 'e'; ++q)
    if (*q != '.') dig[nd++] = *q;
  int ex = 0;  // to_chars does not terminate the buffer: parse the exponent up to ``end``
  bool eneg = false;
  for (const char* c = q + 1; c < end; ++c) {
    if (*c == '-') eneg = true;
    else if (*c >= '0' && *c <= '9') ex = ex * 10 + (*c - '0');
  }
  if (eneg) ex = -ex;
  if (ex >= -4 && ex < 16) {
    if (ex >= 0) {
      for (int i = 0; i <= ex; ++i) o.put(i < nd ? dig[i] : '0');
      o.put('.');
      if (nd > ex + 1) o.put(dig + ex + 1, (size_t)(nd - ex - 1));
      else o.put('0');
    } else {
      o.put("0.", 2);
      for (int i = 0; i < -ex - 1; ++i) o.put('0');
      o.put(dig, (size_t)nd);
    }
    return;
  }
  o.put(dig[0]);
  if (nd > 1) {
    o.put('.');
    o.put(dig + 1, (size_t)(nd - 1));
  }
  char eb[8];
  const int el = snprintf(eb, sizeof eb, "e%c%02d", ex < 0 ? '-' : '+', ex < 0 ? -ex : ex);
  o.put(eb, (size_t)el);
}

constexpr size_t F64_BOUND = 352;  // fixed notation of the largest double at precision <= 15 + repr

inline void put_double(Out& o, double v, int prec) {
  if (prec == -2) {
    put_pyrepr(o, v);
    return;
  }
  if (std::isnan(v)) {
    o.put("NaN", 3);
    return;
  }
  // std::to_chars with a precision formats exactly as printf's %.*f / %g (and several times faster)
  auto res = prec >= 0 ? std::to_chars(o.w, o.w + F64_BOUND, v, std::chars_format::fixed, prec)
                       : std::to_chars(o.w, o.w + F64_BOUND, v, std::chars_format::general, 6);  // "{:g}"
  if (res.ec != std::errc()) {  // beyond the bound (very large values at a high precision)
    // one format with a precision argument in both cases ("%.*g" at 6 == "%g"), so the varargs
    // always match the format (int precision, double value)
    const char* fmt = prec >= 0 ? "%.*f" : "%.*g";
    const int p = prec >= 0 ? prec : 6;
    const int len = snprintf(nullptr, 0, fmt, p, v);
    std::string tmp((size_t)len + 1, '\0');
    snprintf(tmp.data(), tmp.size(), fmt, p, v);
    o.commit();
    o.ensure((size_t)len + (1u << 20));  // the rest of the row: its bound was reserved before
    o.put(tmp.data(), (size_t)len);
    return;
  }
  o.w = res.ptr;
}

inline void put_int(Out& o, int64_t v) { o.w = std::to_chars(o.w, o.w + 24, v).ptr; }

// [a, e) of field ``f`` of the line [p, p + n) split at any character with sep[c] set (f < 0:
// counted from the end); false when the line has fewer fields
inline bool field_span(const char* p, int64_t n, int f, const uint8_t* sep, const char** a, const char** e) {
  const char* end = p + n;
  if (f >= 0) {
    const char* s = p;
    for (int k = 0; k < f; ++k) {
      while (s < end && !sep[(uint8_t)*s]) ++s;
      if (s >= end) return false;
      ++s;
    }
    const char* t = s;
    while (t < end && !sep[(uint8_t)*t]) ++t;
    *a = s;
    *e = t;
    return true;
  }
  const char* t = end;
  for (int k = -1; k > f; --k) {
    while (t > p && !sep[(uint8_t)t[-1]]) --t;
    if (t <= p) return false;
    --t;
  }
  const char* s = t;
  while (s > p && !sep[(uint8_t)s[-1]]) --s;
  *a = s;
  *e = t;
  return true;
}

// append [p, p + n) with every separator character replaced by ``delim`` (copied as is when the
// only separator is the delimiter itself)
inline void put_rejoined(Out& o, const char* p, int64_t n, const uint8_t* sep, bool same, const std::string& delim) {
  if (same) {
    o.put(p, (size_t)n);
    return;
  }
  const char* end = p + n;
  const char* a = p;
  for (const char* c = p; c < end; ++c)
    if (sep[(uint8_t)*c]) {
      o.put(a, (size_t)(c - a));
      o.put(delim.data(), delim.size());
      a = c + 1;
    }
  o.put(a, (size_t)(end - a));
}

struct Tab {
  std::vector<const char*> p;
  std::vector<uint32_t> n;
  size_t maxlen = 0;
};

}  // namespace

// the rows split over ``nthreads`` threads, each formatting its block into its own buffer
static std::vector<std::string> format_parts(const std::vector<FmtCol>& cols, int64_t n, const std::string& delim,
                                             int nthreads) {
  // (no rows: empty columns hold no buffers — an empty selection of lines has null span pointers)
  for (const auto& c : (n > 0 ? cols : std::vector<FmtCol>{})) {
    if ((c.kind == FmtCol::STR || c.kind == FmtCol::LIST || c.kind == FmtCol::PAIRS) && (!c.table || !c.idx))
      throw std::runtime_error("format_columns: string column without table / index");
    if ((c.kind == FmtCol::LIST || c.kind == FmtCol::PAIRS) && !c.off)
      throw std::runtime_error("format_columns: list column without offsets");
    if (c.kind == FmtCol::PAIRS && !c.iv) throw std::runtime_error("format_columns: pair list without integers");
    if ((c.kind == FmtCol::RAW || c.kind == FmtCol::FIELD || c.kind == FmtCol::TAIL) && (!c.raddr || !c.rlen))
      throw std::runtime_error("format_columns: line column without spans");
  }
  // per column: separator table of the raw-line kinds, whether re-joining changes nothing, and the
  // string table as (pointer, length) pairs
  std::vector<std::array<uint8_t, 256>> seps(cols.size());
  std::vector<char> same(cols.size(), 0);
  std::vector<Tab> tabs(cols.size());
  const size_t dl = delim.size();
  for (size_t k = 0; k < cols.size(); ++k) {
    seps[k].fill(0);
    for (char ch : cols[k].from_delims) seps[k][(uint8_t)ch] = 1;
    same[k] = cols[k].from_delims.empty() || cols[k].from_delims == delim;
    if (cols[k].table) {
      Tab& t = tabs[k];
      for (const auto& str : *cols[k].table) {
        t.p.push_back(str.data());
        t.n.push_back((uint32_t)str.size());
        t.maxlen = std::max(t.maxlen, str.size());
      }
    }
  }
  const int T = n < 16384 ? 1 : std::max(1, nthreads);
  std::vector<std::string> parts(T);
  std::vector<std::string> err(T);
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) {
    th.emplace_back([&, t] {
      try {
        const int64_t r0 = n * t / T, r1 = n * (t + 1) / T;
        Out o;
        o.buf.resize((size_t)(r1 - r0) * (8 * cols.size() + 8) + 4096);
        for (int64_t r = r0; r < r1; ++r) {
          // upper bound of this row's bytes
          size_t bound = 1;
          for (size_t ci = 0; ci < cols.size(); ++ci) {
            const auto& c = cols[ci];
            switch (c.kind) {
              case FmtCol::STR: bound += tabs[ci].maxlen + dl; break;
              case FmtCol::LIST:
              case FmtCol::PAIRS:
                bound += (size_t)(c.off[r + 1] - c.off[r]) *
                         (tabs[ci].maxlen + dl + (c.kind == FmtCol::PAIRS ? 24 + dl : 0));
                break;
              case FmtCol::F64: bound += F64_BOUND + dl; break;
              case FmtCol::I64: bound += 24 + dl; break;
              case FmtCol::LIT:
              case FmtCol::GLUE: bound += c.lit.size() + dl; break;
              default: bound += (size_t)c.rlen[r] * std::max<size_t>(dl, 1) + dl;
            }
          }
          o.ensure(bound);
          bool first = true;
          for (size_t ci = 0; ci < cols.size(); ++ci) {
            const auto& c = cols[ci];
            if (c.kind == FmtCol::GLUE) {
              o.put(c.lit.data(), c.lit.size());
              continue;
            }
            if (c.kind == FmtCol::LIST || c.kind == FmtCol::PAIRS) {
              const Tab& tb = tabs[ci];
              const int64_t a = c.off[r], b = c.off[r + 1];
              for (int64_t j = a; j < b; ++j) {
                if (!first) o.put(delim.data(), dl);
                first = false;
                const int32_t k = c.idx[j];
                if (k >= 0 && (size_t)k < tb.p.size()) o.put(tb.p[(size_t)k], tb.n[(size_t)k]);
                if (c.kind == FmtCol::PAIRS) {
                  o.put(delim.data(), dl);
                  put_int(o, c.iv[j]);
                }
              }
              continue;
            }
            if (!first) o.put(delim.data(), dl);
            first = false;
            switch (c.kind) {
              case FmtCol::STR: {
                const Tab& tb = tabs[ci];
                const int32_t k = c.idx[r];
                if (k >= 0 && (size_t)k < tb.p.size()) o.put(tb.p[(size_t)k], tb.n[(size_t)k]);
                break;
              }
              case FmtCol::F64:
                put_double(o, c.dv[r], c.prec);
                break;
              case FmtCol::I64:
                put_int(o, c.iv[r]);
                break;
              case FmtCol::LIT:
                o.put(c.lit.data(), c.lit.size());
                break;
              case FmtCol::RAW:
                put_rejoined(o, reinterpret_cast<const char*>(c.raddr[r]), c.rlen[r], seps[ci].data(), same[ci],
                             delim);
                break;
              case FmtCol::FIELD: {
                const char *a, *e;
                if (field_span(reinterpret_cast<const char*>(c.raddr[r]), c.rlen[r], c.field, seps[ci].data(), &a, &e))
                  o.put(a, (size_t)(e - a));
                break;
              }
              case FmtCol::TAIL: {
                const char* p = reinterpret_cast<const char*>(c.raddr[r]);
                const char *a, *e;
                if (field_span(p, c.rlen[r], c.field, seps[ci].data(), &a, &e))
                  put_rejoined(o, a, (int64_t)(p + c.rlen[r] - a), seps[ci].data(), false, delim);
                break;
              }
              default:
                break;
            }
          }
          o.put('\n');
          o.commit();
        }
        o.buf.resize(o.pos);
        parts[t] = std::move(o.buf);
      } catch (const std::exception& e) {
        err[t] = e.what();
      }
    });
  }
  for (auto& x : th) x.join();
  for (auto& e : err)
    if (!e.empty()) throw std::runtime_error(e);
  return parts;
}

std::string format_columns(const std::vector<FmtCol>& cols, int64_t n, const std::string& delim, int nthreads) {
  std::vector<std::string> parts = format_parts(cols, n, delim, nthreads);
  size_t tot = 0;
  for (auto& p : parts) tot += p.size();
  std::string out;
  out.reserve(tot);
  for (auto& p : parts) out += p;
  return out;
}

}  // namespace avh

namespace avh {

// format_columns straight into a file (created / truncated, or appended to): every thread formats
// its block of rows, then writes it with pwrite at its offset — no concatenated copy, no Python
// bytes object.  Returns the bytes written.
int64_t write_file_parallel(const std::string& path, bool append,
                            const std::vector<std::pair<const char*, int64_t>>& parts, int nthreads) {
  int64_t total = 0;
  for (auto& p : parts) total += p.second;
  const int fd = ::open(path.c_str(), O_RDWR | O_CREAT | (append ? 0 : O_TRUNC), 0644);
  if (fd < 0) throw std::runtime_error("cannot open " + path + " for writing");
  const off_t base = append ? ::lseek(fd, 0, SEEK_END) : 0;
  bool done = false;
  if (total >= (16 << 20) && nthreads > 1) {
    // large outputs: byte ranges written by several threads (pwrite at their offsets)
    std::vector<int64_t> off(parts.size() + 1, 0);
    for (size_t k = 0; k < parts.size(); ++k) off[k + 1] = off[k] + parts[k].second;
    const int T = std::max(1, std::min(nthreads, 16));
    std::vector<std::thread> th;
    std::atomic<bool> bad{false};
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        const int64_t a = total * t / T, b = total * (t + 1) / T;
        size_t k = (size_t)(std::upper_bound(off.begin(), off.end(), a) - off.begin()) - 1;
        for (int64_t x = a; x < b && k < parts.size(); ++k) {
          const int64_t e = std::min(b, off[k + 1]);
          while (x < e) {
            const ssize_t w = ::pwrite(fd, parts[k].first + (x - off[k]), (size_t)(e - x), (off_t)(base + x));
            if (w <= 0) {
              bad = true;
              return;
            }
            x += w;
          }
        }
      });
    for (auto& x : th) x.join();
    if (bad) {
      ::close(fd);
      throw std::runtime_error("write failed: " + path);
    }
    done = true;
  }
  if (!done) {
    int64_t at = base;
    for (auto& p : parts) {
      const char* q = p.first;
      int64_t left = p.second;
      while (left > 0) {
        const ssize_t w = ::pwrite(fd, q, (size_t)left, (off_t)at);
        if (w <= 0) {
          ::close(fd);
          throw std::runtime_error("write failed: " + path);
        }
        q += w;
        left -= w;
        at += w;
      }
    }
  }
  ::close(fd);
  return total;
}

int64_t format_columns_to_file(const std::vector<FmtCol>& cols, int64_t n, const std::string& delim, int nthreads,
                               const std::string& path, bool append) {
  std::vector<std::string> parts = format_parts(cols, n, delim, nthreads);
  std::vector<std::pair<const char*, int64_t>> pv;
  for (auto& p : parts) pv.emplace_back(p.data(), (int64_t)p.size());
  return write_file_parallel(path, append, pv, nthreads);
}

}  // namespace avh
