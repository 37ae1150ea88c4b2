// Host check of csrc/include/avenir_numparse.h against strtod: random full-precision doubles
// (%.17g / %.15g / %.Ne), subnormals, extremes, midpoints and 20-25 digit mantissas must give the
// same bits (tokens flagged slow are skipped: the parsers hand those to strtod).  Built and run by
// tests/test_numparse.py.
#include "avenir_numparse.h"
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
int main() {
  std::mt19937_64 rng(42);
  long bad = 0, slow = 0, total = 0;
  char buf[64];
  auto check = [&](const char* s) {
    bool sl;
    double v = avnum::parse_decimal(s, s + strlen(s), &sl);
    double r = strtod(s, nullptr);
    ++total;
    if (sl) { ++slow; return; }
    uint64_t a, b; memcpy(&a, &v, 8); memcpy(&b, &r, 8);
    if (a != b) { if (bad < 10) printf("MISMATCH %s: %.17g vs %.17g\n", s, v, r); ++bad; }
  };
  for (int i = 0; i < 400000; ++i) {
    uint64_t u = rng();
    double d; memcpy(&d, &u, 8);
    if (d != d || __builtin_isinf(d)) continue;
    snprintf(buf, sizeof buf, "%.17g", d); check(buf);
    snprintf(buf, sizeof buf, "%.15g", d); check(buf);
    snprintf(buf, sizeof buf, "%.*e", (int)(rng() % 19), d); check(buf);
  }
  // subnormals, extremes, halfway cases, long digit strings
  const char* fixed[] = {"4.9e-324", "2.4703282292062327e-324", "2.4703282292062328e-324", "1e-400", "1e309",
    "1.7976931348623157e308", "1.7976931348623158e308", "2.2250738585072011e-308", "2.2250738585072014e-308",
    "9007199254740993", "9007199254740992.5", "0.1", "0.3", "123456789012345678901234567890", "1.00000000000000011102230246251565404236316680908203125",
    "1.00000000000000011102230246251565404236316680908203124", "7.2057594037927933e16", "0.000001", "1e23", "8.98846567431158e307"};
  for (auto s : fixed) check(s);
  for (int i = 0; i < 50000; ++i) {  // random 20-25 digit mantissas
    std::string s;
    int nd = 20 + rng() % 6;
    for (int k = 0; k < nd; ++k) s += char('0' + rng() % 10);
    s.insert(1 + rng() % (nd - 1), ".");
    s += "e" + std::to_string((int)(rng() % 600) - 300);
    check(s.c_str());
  }
  for (int i = 0; i < 50000; ++i) {  // subnormal range
    snprintf(buf, sizeof buf, "%.*fe-%d", (int)(rng() % 17), 1.0 + (double)(rng() % 9000000) / 1000000.0, 300 + (int)(rng() % 30));
    check(buf);
  }
  printf("total %ld bad %ld slow %ld\n", total, bad, slow);
  return bad != 0;
}
