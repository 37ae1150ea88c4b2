// Host runtime self-test, built by tests/test_host_sanitizers.py under AddressSanitizer +
// UndefinedBehaviorSanitizer and, separately, ThreadSanitizer (race detection and
// sanitizers; GPU-side ASan is unavailable on the target pool, so the sanitised surface is the
// native host runtime: the multi-threaded CSV encoder, the SPSC ring shared by the bandit
// service's producer / consumer threads, the multi-threaded row formatter and the checkpoint
// container).  Prints "OK" and exits 0 when every check passes; any sanitizer report aborts.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include "avenir_host.h"

#define CHECK(cond)                                                        \
  do {                                                                     \
    if (!(cond)) {                                                         \
      std::fprintf(stderr, "FAILED %s at %s:%d\n", #cond, __FILE__, __LINE__); \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

static void test_csv(const std::string& dir) {
  const std::string path = dir + "/selftest.csv";
  const int n = 50000;
  {
    std::ofstream f(path);
    f << "id,color,size,score\n";
    const char* colors[] = {"red", "green", "blue"};
    for (int i = 0; i < n; ++i) {
      // every 97th row is short (malformed), every 101st has an unknown colour
      if (i % 97 == 0) { f << i << "," << colors[i % 3] << "\n"; continue; }
      f << i << "," << (i % 101 == 0 ? "mauve" : colors[i % 3]) << "," << (i % 50) << "," << (i * 0.5) << "\n";
    }
  }
  avh::CsvFile csv(path, ",", true, 8);
  CHECK(csv.num_rows() == n);
  std::vector<avh::ColSpec> specs(3);
  specs[0].ordinal = 1; specs[0].kind = avh::CAT; specs[0].vocab = {"red", "green", "blue"};
  specs[1].ordinal = 2; specs[1].kind = avh::BUCKET; specs[1].bucket_width = 10.0; specs[1].max_code = 254;
  specs[2].ordinal = 3; specs[2].kind = avh::FLOAT;
  const int64_t ld = ((n + 15) / 16) * 16;
  std::vector<uint8_t> color(ld, 255), size(ld, 255);
  std::vector<float> score(n, 0.f);
  std::vector<void*> outs = {color.data(), size.data(), score.data()};
  const int64_t bad = csv.parse(specs, outs, 0, -1);
  if (bad != (n + 96) / 97) std::fprintf(stderr, "malformed rows: %lld\n", (long long)bad);
  CHECK(bad == (n + 96) / 97);
  for (int i = 1; i < n; ++i) {
    if (i % 97 == 0) continue;
    CHECK(color[i] == (i % 101 == 0 ? 255 : i % 3));
    CHECK(size[i] == (i % 50) / 10);
    CHECK(score[i] == (float)(i * 0.5));
  }
  // a row range parsed on its own agrees with the full parse
  std::vector<uint8_t> c2(ld, 255), s2(ld, 255);
  std::vector<float> f2(n, 0.f);
  std::vector<void*> outs2 = {c2.data(), s2.data(), f2.data()};
  csv.parse(specs, outs2, 1000, 2000);
  for (int i = 1000; i < 2000; ++i)
    if (i % 97) CHECK(c2[i - 1000] == color[i] && s2[i - 1000] == size[i]);
  CHECK(csv.distinct(1, 10).size() == 4);
  std::remove(path.c_str());
}

static void test_ring() {
  // one producer thread, one consumer thread, many wrap-arounds of a small ring
  avh::SpscRing ring(64, 3);
  const int64_t N = 200000;
  std::thread prod([&] {
    int64_t rec[3];
    for (int64_t i = 0; i < N; ++i) {
      rec[0] = i; rec[1] = 2 * i; rec[2] = -i;
      while (!ring.push(rec)) std::this_thread::yield();
    }
  });
  int64_t expect = 0;
  std::vector<int64_t> buf(3 * 16);
  while (expect < N) {
    const size_t k = ring.pop_batch(buf.data(), 16);
    for (size_t j = 0; j < k; ++j, ++expect) {
      CHECK(buf[3 * j] == expect && buf[3 * j + 1] == 2 * expect && buf[3 * j + 2] == -expect);
    }
    if (!k) std::this_thread::yield();
  }
  prod.join();
  CHECK(ring.size() == 0);
}

static void test_format_and_container(const std::string& dir) {
  const int64_t n = 20000;
  std::vector<double> cols(2 * n);
  for (int64_t i = 0; i < n; ++i) { cols[i] = (double)i; cols[n + i] = i * 0.25; }
  const std::string out = avh::format_rows(nullptr, cols.data(), 2, n, {0, 2}, ',', 8);
  CHECK(out.compare(0, 11, "0,0.00\n1,0.") == 0);
  size_t lines = 0;
  for (char c : out) lines += c == '\n';
  CHECK(lines == (size_t)n);
  const std::string path = dir + "/selftest.ckpt";
  std::vector<float> a(1000);
  for (int i = 0; i < 1000; ++i) a[i] = i * 1.5f;
  const std::string hdr = "{\"a\":{\"dtype\":\"F32\",\"shape\":[1000],\"data_offsets\":[0,4000]}}";
  avh::write_container(path, hdr, {a.data()}, {a.size() * sizeof(float)});
  uint64_t off = 0;
  const std::string got = avh::read_container_header(path, &off);
  CHECK(got.compare(0, hdr.size(), hdr) == 0 && off % 8 == 0);
  std::ifstream f(path, std::ios::binary);
  f.seekg((std::streamoff)off);
  std::vector<float> b(1000);
  f.read(reinterpret_cast<char*>(b.data()), 4000);
  CHECK(std::memcmp(a.data(), b.data(), 4000) == 0);
  CHECK(avh::crc32("123456789", 9) == 0xCBF43926u);
  std::remove(path.c_str());
}

// byte-range shards over two files: every line lands on exactly one rank whatever the world size,
// the tokens of the union equal the world-1 tokens, and the dictionaries agree in merged order
static void test_text_shards(const std::string& dir) {
  const std::string p1 = dir + "/shard_a.txt", p2 = dir + "/shard_b.txt";
  const char* st[] = {"L", "M", "H", "LL", "MMM"};
  int nlines = 0;
  {
    std::ofstream a(p1), b(p2);
    for (int i = 0; i < 20000; ++i) {
      std::ofstream& f = i < 12000 ? a : b;
      if (i % 501 == 0) { f << "   \n"; continue; }  // blank lines are dropped
      f << "id" << i;
      for (int k = 0; k < 1 + i % 7; ++k) f << "," << st[(i + k) % 5] << ":" << (k % 2 ? "x" : "y");
      if (i != 19999) f << (i % 3 ? "\n" : "\r\n");  // the last line has no newline
      ++nlines;
    }
  }
  avh::TokenSpec spec;
  spec.sub_delim = ':';
  spec.modes = "x";
  avh::TextShard whole({p1, p2}, 0, 1, 8, false);
  CHECK(whole.num_lines() == nlines);
  const int64_t T1 = whole.count_tokens(spec);
  std::vector<int64_t> off1(whole.num_lines() + 1);
  std::vector<int32_t> c1(T1), s1(T1);
  whole.tokenize(off1.data(), c1.data(), s1.data(), nullptr);
  for (int world : {2, 3, 8}) {
    int64_t lines = 0, toks = 0;
    for (int r = 0; r < world; ++r) {
      avh::TextShard sh({p1, p2}, r, world, 3, false);
      const int64_t T = sh.count_tokens(spec);
      std::vector<int64_t> off(sh.num_lines() + 1);
      std::vector<int32_t> c(T), s(T);
      sh.tokenize(off.data(), c.data(), s.data(), nullptr);
      for (int64_t k = 0; k < T; ++k) {
        if (c[k] < 0) { CHECK(c1[toks + k] < 0); continue; }
        CHECK(sh.vocab()[(size_t)c[k]] == whole.vocab()[(size_t)c1[toks + k]]);
        CHECK(sh.vocab()[(size_t)s[k]] == whole.vocab()[(size_t)s1[toks + k]]);
      }
      lines += sh.num_lines();
      toks += T;
    }
    CHECK(lines == nlines && toks == T1);
  }
  std::remove(p1.c_str());
  std::remove(p2.c_str());
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  test_csv(dir);
  test_ring();
  test_format_and_container(dir);
  test_text_shards(dir);
  std::printf("OK\n");
  return 0;
}
