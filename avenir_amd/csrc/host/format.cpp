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
#include <unistd.h>
#include <thread>

#include "avenir_host.h"

namespace avh {

namespace {

// Python's repr(float): the shortest digit string that round-trips (std::to_chars), written in
// fixed notation for decimal exponents -4 <= e < 16 and as d.ddde[+-]XX otherwise.
inline void put_pyrepr(std::string& s, double v) {
  if (std::isnan(v)) {
    s += "nan";
    return;
  }
  if (std::isinf(v)) {
    s += v < 0 ? "-inf" : "inf";
    return;
  }
  char buf[40];
  auto res = std::to_chars(buf, buf + sizeof buf, v, std::chars_format::scientific);
  const char* p = buf;
  const char* end = res.ptr;
  if (*p == '-') {
    s.push_back('-');
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
      for (int i = 0; i <= ex; ++i) s.push_back(i < nd ? dig[i] : '0');
      s.push_back('.');
      if (nd > ex + 1) s.append(dig + ex + 1, (size_t)(nd - ex - 1));
      else s.push_back('0');
    } else {
      s += "0.";
      s.append((size_t)(-ex - 1), '0');
      s.append(dig, (size_t)nd);
    }
    return;
  }
  s.push_back(dig[0]);
  if (nd > 1) {
    s.push_back('.');
    s.append(dig + 1, (size_t)(nd - 1));
  }
  char eb[8];
  const int el = snprintf(eb, sizeof eb, "e%c%02d", ex < 0 ? '-' : '+', ex < 0 ? -ex : ex);
  s.append(eb, (size_t)el);
}

inline void put_double(std::string& s, double v, int prec) {
  char buf[352];
  int len;
  if (prec == -2) {
    put_pyrepr(s, v);
    return;
  }
  if (std::isnan(v)) {
    s += "NaN";
    return;
  }
  // std::to_chars with a precision formats exactly as printf's %.*f / %g (and several times faster)
  auto res = prec >= 0 ? std::to_chars(buf, buf + sizeof buf, v, std::chars_format::fixed, prec)
                       : std::to_chars(buf, buf + sizeof buf, v, std::chars_format::general, 6);  // "{:g}"
  if (res.ec != std::errc()) {  // very large values at a high precision: printf into a heap buffer
    len = snprintf(nullptr, 0, prec >= 0 ? "%.*f" : "%g", prec >= 0 ? prec : 6, v);
    std::string tmp((size_t)len + 1, '\0');
    snprintf(tmp.data(), tmp.size(), prec >= 0 ? "%.*f" : "%g", prec >= 0 ? prec : 6, v);
    s.append(tmp.data(), (size_t)len);
    return;
  }
  s.append(buf, (size_t)(res.ptr - buf));
}

inline void put_int(std::string& s, int64_t v) {
  char buf[24];
  auto res = std::to_chars(buf, buf + sizeof buf, v);
  s.append(buf, (size_t)(res.ptr - buf));
}

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
inline void put_rejoined(std::string& s, const char* p, int64_t n, const uint8_t* sep, bool same,
                         const std::string& delim) {
  if (same) {
    s.append(p, (size_t)n);
    return;
  }
  const char* end = p + n;
  const char* a = p;
  for (const char* c = p; c < end; ++c)
    if (sep[(uint8_t)*c]) {
      s.append(a, (size_t)(c - a));
      s += delim;
      a = c + 1;
    }
  s.append(a, (size_t)(end - a));
}

}  // namespace

// the rows split over ``nthreads`` threads, each formatting its block into its own buffer
static std::vector<std::string> format_parts(const std::vector<FmtCol>& cols, int64_t n, const std::string& delim,
                                             int nthreads) {
  for (const auto& c : cols) {
    if ((c.kind == FmtCol::STR || c.kind == FmtCol::LIST || c.kind == FmtCol::PAIRS) && (!c.table || !c.idx))
      throw std::runtime_error("format_columns: string column without table / index");
    if ((c.kind == FmtCol::LIST || c.kind == FmtCol::PAIRS) && !c.off)
      throw std::runtime_error("format_columns: list column without offsets");
    if (c.kind == FmtCol::PAIRS && !c.iv) throw std::runtime_error("format_columns: pair list without integers");
    if ((c.kind == FmtCol::RAW || c.kind == FmtCol::FIELD || c.kind == FmtCol::TAIL) && (!c.raddr || !c.rlen))
      throw std::runtime_error("format_columns: line column without spans");
  }
  // per column: separator table of the raw-line kinds, and whether re-joining changes nothing
  std::vector<std::array<uint8_t, 256>> seps(cols.size());
  std::vector<char> same(cols.size(), 0);
  for (size_t k = 0; k < cols.size(); ++k) {
    seps[k].fill(0);
    for (char ch : cols[k].from_delims) seps[k][(uint8_t)ch] = 1;
    same[k] = cols[k].from_delims.empty() || cols[k].from_delims == delim;
  }
  const int T = n < 16384 ? 1 : std::max(1, nthreads);
  std::vector<std::string> parts(T);
  std::vector<std::string> err(T);
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) {
    th.emplace_back([&, t] {
      try {
        const int64_t r0 = n * t / T, r1 = n * (t + 1) / T;
        std::string& s = parts[t];
        s.reserve((size_t)(r1 - r0) * (8 * cols.size() + 8));
        for (int64_t r = r0; r < r1; ++r) {
          bool first = true;
          for (size_t ci = 0; ci < cols.size(); ++ci) {
            const auto& c = cols[ci];
            if (c.kind == FmtCol::GLUE) {
              s += c.lit;
              continue;
            }
            if (c.kind == FmtCol::LIST || c.kind == FmtCol::PAIRS) {
              const int64_t a = c.off[r], b = c.off[r + 1];
              for (int64_t j = a; j < b; ++j) {
                if (!first) s += delim;
                first = false;
                const int32_t k = c.idx[j];
                if (k >= 0 && (size_t)k < c.table->size()) s += (*c.table)[(size_t)k];
                if (c.kind == FmtCol::PAIRS) {
                  s += delim;
                  put_int(s, c.iv[j]);
                }
              }
              continue;
            }
            if (!first) s += delim;
            first = false;
            switch (c.kind) {
              case FmtCol::STR: {
                const int32_t k = c.idx[r];
                if (k >= 0 && (size_t)k < c.table->size()) s += (*c.table)[(size_t)k];
                break;
              }
              case FmtCol::F64:
                put_double(s, c.dv[r], c.prec);
                break;
              case FmtCol::I64:
                put_int(s, c.iv[r]);
                break;
              case FmtCol::LIT:
                s += c.lit;
                break;
              case FmtCol::RAW:
                put_rejoined(s, reinterpret_cast<const char*>(c.raddr[r]), c.rlen[r], seps[ci].data(), same[ci],
                             delim);
                break;
              case FmtCol::FIELD: {
                const char *a, *e;
                if (field_span(reinterpret_cast<const char*>(c.raddr[r]), c.rlen[r], c.field, seps[ci].data(), &a, &e))
                  s.append(a, (size_t)(e - a));
                break;
              }
              case FmtCol::TAIL: {
                const char* p = reinterpret_cast<const char*>(c.raddr[r]);
                const char *a, *e;
                if (field_span(p, c.rlen[r], c.field, seps[ci].data(), &a, &e))
                  put_rejoined(s, a, (int64_t)(p + c.rlen[r] - a), seps[ci].data(), false, delim);
                break;
              }
              default:
                break;
            }
          }
          s.push_back('\n');
        }
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
int64_t format_columns_to_file(const std::vector<FmtCol>& cols, int64_t n, const std::string& delim, int nthreads,
                               const std::string& path, bool append) {
  std::vector<std::string> parts = format_parts(cols, n, delim, nthreads);
  const int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | (append ? 0 : O_TRUNC), 0644);
  if (fd < 0) throw std::runtime_error("cannot open " + path + " for writing");
  off_t base = 0;
  if (append) base = ::lseek(fd, 0, SEEK_END);
  std::vector<int64_t> off(parts.size() + 1, 0);
  for (size_t t = 0; t < parts.size(); ++t) off[t + 1] = off[t] + (int64_t)parts[t].size();
  std::vector<std::thread> th;
  std::atomic<bool> bad{false};
  for (size_t t = 0; t < parts.size(); ++t)
    th.emplace_back([&, t] {
      const char* p = parts[t].data();
      int64_t left = (int64_t)parts[t].size(), at = base + off[t];
      while (left > 0) {
        const ssize_t w = ::pwrite(fd, p, (size_t)left, (off_t)at);
        if (w <= 0) {
          bad = true;
          return;
        }
        p += w;
        left -= w;
        at += w;
      }
    });
  for (auto& x : th) x.join();
  ::close(fd);
  if (bad) throw std::runtime_error("write failed: " + path);
  return off.back();
}

}  // namespace avh
