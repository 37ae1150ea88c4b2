// SPSC ring buffer (bandit serving) and checkpoint container I/O (see avenir_host.h).
#include <cstdio>
#include <cstring>
#include <fstream>
#include <stdexcept>

#include "avenir_host.h"

namespace avh {

SpscRing::SpscRing(size_t capacity_pow2, int rec_len) : rec_len_(rec_len) {
  size_t cap = 1;
  while (cap < capacity_pow2) cap <<= 1;
  buf_.assign(cap * (size_t)rec_len, 0);
  mask_ = cap - 1;
}

bool SpscRing::push(const int64_t* rec) {
  const size_t h = head_.load(std::memory_order_relaxed);
  const size_t t = tail_.load(std::memory_order_acquire);
  if (h - t > mask_) return false;  // full
  std::memcpy(&buf_[(h & mask_) * rec_len_], rec, sizeof(int64_t) * rec_len_);
  head_.store(h + 1, std::memory_order_release);
  return true;
}

bool SpscRing::pop(int64_t* rec) {
  const size_t t = tail_.load(std::memory_order_relaxed);
  const size_t h = head_.load(std::memory_order_acquire);
  if (t == h) return false;
  std::memcpy(rec, &buf_[(t & mask_) * rec_len_], sizeof(int64_t) * rec_len_);
  tail_.store(t + 1, std::memory_order_release);
  return true;
}

size_t SpscRing::pop_batch(int64_t* recs, size_t max_n) {
  const size_t t = tail_.load(std::memory_order_relaxed);
  const size_t h = head_.load(std::memory_order_acquire);
  const size_t k = std::min(max_n, h - t);
  for (size_t i = 0; i < k; ++i)
    std::memcpy(recs + i * rec_len_, &buf_[((t + i) & mask_) * rec_len_], sizeof(int64_t) * rec_len_);
  tail_.store(t + k, std::memory_order_release);
  return k;
}

size_t SpscRing::size() const {
  return head_.load(std::memory_order_acquire) - tail_.load(std::memory_order_acquire);
}

static uint32_t crc_table[256];
static bool crc_init = [] {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    crc_table[i] = c;
  }
  return true;
}();

uint32_t crc32(const void* data, size_t n, uint32_t seed) {
  (void)crc_init;
  const uint8_t* p = static_cast<const uint8_t*>(data);
  uint32_t c = seed ^ 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) c = crc_table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

void write_container(const std::string& path, const std::string& header_json,
                     const std::vector<const void*>& blobs, const std::vector<size_t>& sizes) {
  if (blobs.size() != sizes.size()) throw std::runtime_error("blobs/sizes mismatch");
  const std::string tmp = path + ".tmp";
  {
    std::ofstream f(tmp, std::ios::binary | std::ios::trunc);
    if (!f) throw std::runtime_error("cannot write " + tmp);
    // pad header to 8 bytes so tensor data is aligned (safetensors convention)
    std::string hdr = header_json;
    while ((hdr.size() % 8) != 0) hdr.push_back(' ');
    uint64_t hl = hdr.size();
    f.write(reinterpret_cast<const char*>(&hl), 8);
    f.write(hdr.data(), (std::streamsize)hdr.size());
    for (size_t i = 0; i < blobs.size(); ++i)
      f.write(static_cast<const char*>(blobs[i]), (std::streamsize)sizes[i]);
    f.flush();
    if (!f) throw std::runtime_error("short write " + tmp);
  }
  if (std::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("rename failed " + path);
}

std::string read_container_header(const std::string& path, uint64_t* data_offset) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  uint64_t hl = 0;
  f.read(reinterpret_cast<char*>(&hl), 8);
  if (!f || hl > (1ull << 30)) throw std::runtime_error("corrupt checkpoint header in " + path);
  std::string hdr(hl, '\0');
  f.read(&hdr[0], (std::streamsize)hl);
  if (!f) throw std::runtime_error("truncated checkpoint header in " + path);
  *data_offset = 8 + hl;
  return hdr;
}

}  // namespace avh
