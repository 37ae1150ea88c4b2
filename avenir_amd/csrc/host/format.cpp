// Native output formatting for the CLI jobs: rows assembled from string-table lookups, numbers,
// literals and variable-length string lists (CSR), by several threads into one buffer.  The
// reference's reducers write one Text line per record through Hadoop's TextOutputFormat; jobs here
// produce millions of output lines per rank (neighbour lists, per-entity predictions), which Python
// string joins would spend seconds on.
#include <cmath>
#include <cstdio>
#include <stdexcept>
#include <thread>

#include "avenir_host.h"

namespace avh {

namespace {

inline void put_double(std::string& s, double v, int prec) {
  char buf[64];
  int len;
  if (std::isnan(v)) {
    s += "NaN";
    return;
  }
  if (prec >= 0) len = snprintf(buf, sizeof buf, "%.*f", prec, v);
  else len = snprintf(buf, sizeof buf, "%g", v);  // Python's "{:g}"
  s.append(buf, (size_t)len);
}

inline void put_int(std::string& s, int64_t v) {
  char buf[24];
  const int len = snprintf(buf, sizeof buf, "%lld", (long long)v);
  s.append(buf, (size_t)len);
}

}  // namespace

std::string format_columns(const std::vector<FmtCol>& cols, int64_t n, const std::string& delim, int nthreads) {
  for (const auto& c : cols) {
    if ((c.kind == FmtCol::STR || c.kind == FmtCol::LIST) && (!c.table || !c.idx))
      throw std::runtime_error("format_columns: string column without table / index");
    if (c.kind == FmtCol::LIST && !c.off) throw std::runtime_error("format_columns: list column without offsets");
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
          for (const auto& c : cols) {
            if (c.kind == FmtCol::GLUE) {
              s += c.lit;
              continue;
            }
            if (c.kind == FmtCol::LIST) {
              const int64_t a = c.off[r], b = c.off[r + 1];
              for (int64_t j = a; j < b; ++j) {
                if (!first) s += delim;
                first = false;
                const int32_t k = c.idx[j];
                if (k >= 0 && (size_t)k < c.table->size()) s += (*c.table)[(size_t)k];
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
  size_t tot = 0;
  for (auto& p : parts) tot += p.size();
  std::string out;
  out.reserve(tot);
  for (auto& p : parts) out += p;
  return out;
}

}  // namespace avh
