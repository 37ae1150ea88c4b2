// Host-side (CPU) C++ runtime of avenir_amd: declarations.
//
//  * CsvFile   — K1: memory-mapped, multi-threaded CSV -> columnar encoder driven by the JSON
//                FeatureSchema (categoricals dictionary-coded to uint8 with 255 = unknown/missing,
//                ints bucketized by bucketWidth, doubles parsed to f32).  Replaces every mapper's
//                `value.toString().split(fieldDelimRegex)` + schema lookup in the reference
//                (e.g. J/bayesian/BayesianDistribution.java:137-178).
//  * SpscRing  — lock-free single-producer/single-consumer ring buffer used by the online bandit
//                service (replaces the Storm spout/bolt + Redis queues, J/storm/*).
//  * checkpoint container read/write (safetensors-compatible layout, JSON header).
#pragma once
#include <atomic>
#include <cstdint>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

namespace avh {

enum ColKind : int { CAT = 0, BUCKET = 1, FLOAT = 2, INT = 3 };

struct ColSpec {
  int ordinal = 0;
  int kind = CAT;
  std::vector<std::string> vocab;  // CAT: known values, code = index (255 = unknown)
  double bucket_width = 1.0;       // BUCKET: code = (int)(v / width) - offset
  int bucket_offset = 0;
  int max_code = 254;              // BUCKET: codes > max_code -> missing
  bool wide = false;               // CAT/BUCKET: uint16 codes (missing = 65535) for > 255 values
  bool huge = false;               // CAT: int32 codes (missing = INT32_MAX) for > 65534 values
};

// Rank ``rank``'s byte range of the concatenated ``paths`` as memory-mapped segments of whole lines
// (a line belongs to the range holding its first byte; one segment per file touched).  Only the
// rank's own pages are mapped and faulted in (MAP_POPULATE over the segment).
class ByteShard {
 public:
  struct Segment {
    const char* p;
    int64_t len;
    void* map;
    size_t map_len;
    int file = 0;          // index into the constructor's paths
    int64_t file_off = 0;  // byte offset of p inside that file
  };
  // populate: fault the pages in at map time (host tokenizer); the device upload faults them in
  // from its parallel copy threads instead
  ByteShard(const std::vector<std::string>& paths, int64_t rank, int64_t world, bool populate = true);
  ~ByteShard();
  ByteShard(const ByteShard&) = delete;
  ByteShard& operator=(const ByteShard&) = delete;
  const std::vector<Segment>& segments() const { return segs_; }
  int64_t bytes() const { return bytes_; }
  int64_t total_bytes() const { return total_bytes_; }
  // concatenate the segments into dst (a '\n' after a segment lacking one when ``terminate``);
  // dst needs bytes() + segments().size() bytes; returns the bytes written
  int64_t copy_to(char* dst, bool terminate) const;

 private:
  std::vector<Segment> segs_;
  int64_t bytes_ = 0, total_bytes_ = 0;
};

class CsvFile {
 public:
  // byte-range shard of several files (records.cpp read_byte_shard): no bytes of other ranks are read
  CsvFile(const std::vector<std::string>& paths, int64_t rank, int64_t world, const std::string& delim,
          bool skip_header, int nthreads);
  // ``delim``: one character (fast path) or a multi-character literal separator (e.g. ",," of
  // the reference's REST record lists).
  CsvFile(const std::string& path, const std::string& delim, bool skip_header, int nthreads);
  ~CsvFile();
  int64_t num_rows() const { return (int64_t)line_start_.size(); }
  int max_fields() const { return max_fields_; }
  // Parse the given specs into caller-owned buffers.  out_u8[i] is [ld] for CAT/BUCKET specs,
  // out_f32 for FLOAT, out_i64 for INT (nullptr for kinds not matching).  Returns number of
  // malformed (short) rows encountered.
  int64_t parse(const std::vector<ColSpec>& specs, const std::vector<void*>& outs,
                int64_t row_begin = 0, int64_t row_end = -1);
  // Discover distinct values of a column (in first-seen order) — used when the schema omits
  // cardinality.
  std::vector<std::string> distinct(int ordinal, size_t limit);
  std::vector<std::string> column_strings(int ordinal);
  std::string line(int64_t i) const;
  std::vector<std::string> lines(int64_t begin, int64_t end) const;
  // absolute address and byte length of lines [begin, end) (valid while the CsvFile lives)
  void line_spans(int64_t begin, int64_t end, int64_t* addr, int64_t* len) const;

 private:
  void index_lines(bool skip_header);
  // split [p, e) at the delimiter into at most max_fields fields (all when max_fields < 0)
  void split(const char* p, const char* e, std::vector<std::string_view>& out, int max_fields) const;
  const char* data_ = nullptr;
  size_t size_ = 0;
  int fd_ = -1;
  std::vector<char> owned_;  // the byte-shard buffer (empty for a mapped file)
  std::string delim_;
  int nthreads_;
  int max_fields_ = 0;
  std::vector<int64_t> line_start_;
  std::vector<int64_t> line_end_;
};

// Tokenizer options of TextShard: ``delims`` — every listed character separates fields; per field
// index a mode ('d' dictionary code, 'n' parsed double, 'x' nothing) from ``modes``, ``tail_mode``
// beyond it; ``sub_delim`` (0 = none) splits a 'd' token once more into (code, sub code);
// ``trim`` strips spaces / tabs around fields (the reference's String.split does not).
struct TokenSpec {
  std::string delims = ",";
  char sub_delim = 0;
  std::string modes;
  char tail_mode = 'd';
  bool trim = false;
  char last_mode = 0;  // the mode of every line's LAST field (0: by position like the others)
};

// K1 for non-schema layouts (records.cpp): this rank's byte range of the concatenated input files
// (a line belongs to the rank whose range holds its first byte), its non-blank lines, and a CSR
// token table with a shard-wide first-occurrence dictionary.
class TextShard {
 public:
  TextShard(const std::vector<std::string>& paths, int64_t rank, int64_t world, int nthreads, bool skip_header);
  int64_t num_lines() const { return (int64_t)ls_.size(); }
  int64_t bytes_read() const { return bytes_.bytes(); }
  int64_t total_bytes() const { return bytes_.total_bytes(); }
  const ByteShard& byte_shard() const { return bytes_; }
  std::vector<std::string> lines(int64_t begin, int64_t end) const;
  // absolute address and byte length of every line (valid while the TextShard lives)
  void line_spans(int64_t* addr, int64_t* len) const;
  // pass 1: number of tokens under ``spec``; pass 2 fills off [L + 1], codes [T] (-1 for non-'d'
  // fields) and, when non-null, sub [T] (-1 without a sub-delimiter) and nums [T] (NaN for non-'n').
  int64_t count_tokens(const TokenSpec& spec);
  void tokenize(int64_t* off, int32_t* codes, int32_t* sub, double* nums);
  const std::vector<std::string>& vocab() const { return vocab_; }
  // raw text of field ``field[i]`` of line ``line[i]`` (empty when the line is shorter)
  std::vector<std::string> field_strings(const int64_t* line, const int32_t* field, int64_t n) const;

 private:
  void index_lines(bool skip_header);
  ByteShard bytes_;
  int nthreads_;
  std::vector<const char*> ls_, le_;
  TokenSpec spec_;
  uint8_t sep_[256] = {0};
  std::vector<int64_t> tok_lines_, tok_cnt_;
  std::vector<std::string> vocab_;
};

// Format rows of numeric columns to CSV text quickly (multi-threaded).  prefix: optional per-row
// leading text (e.g. the original record); cols are f64 column-major [ncol][n].
std::string format_rows(const std::vector<std::string>* prefix, const double* cols, int ncol,
                        int64_t n, const std::vector<int>& precision, char delim, int nthreads);

// One output column of format_columns: STR = table[idx[r]], F64 = dv[r] ("%.*f"; prec -1: "%g",
// prec -2: Python's repr, the shortest round-trip digits), I64 = iv[r], LIT = a constant, LIST =
// table[idx[j]] for j in [off[r], off[r+1]) (delimited, nothing when empty), GLUE = a constant
// appended with no delimiter (brackets), RAW = the input line at raddr[r] (rlen[r] bytes) with every
// character of ``from_delims`` replaced by the output delimiter (no replacement when empty), FIELD =
// field ``field`` of that line split at any character of ``from_delims`` (negative: from the end;
// empty when the line is shorter), TAIL = the fields ``field``.. of the line re-joined with the
// output delimiter, PAIRS = LIST with an integer iv[j] after every string (``w,count,w,count``).
// An index outside the table writes an empty field.
struct FmtCol {
  enum Kind : int { STR = 0, F64 = 1, I64 = 2, LIT = 3, LIST = 4, GLUE = 5, RAW = 6, FIELD = 7, TAIL = 8,
                    PAIRS = 9 };
  int kind = STR;
  const std::vector<std::string>* table = nullptr;
  const int32_t* idx = nullptr;
  const double* dv = nullptr;
  int prec = 6;
  const int64_t* iv = nullptr;
  const int64_t* off = nullptr;
  std::string lit;
  const int64_t* raddr = nullptr;
  const int64_t* rlen = nullptr;
  int field = 0;
  std::string from_delims;
};
std::string format_columns(const std::vector<FmtCol>& cols, int64_t n, const std::string& delim, int nthreads);
int64_t format_columns_to_file(const std::vector<FmtCol>& cols, int64_t n, const std::string& delim, int nthreads,
                               const std::string& path, bool append);
// write (or append) the concatenation of ``parts`` to ``path``: large outputs as byte ranges
// pwritten by several threads, small ones by one; returns the bytes written
int64_t write_file_parallel(const std::string& path, bool append,
                            const std::vector<std::pair<const char*, int64_t>>& parts, int nthreads);

// Lock-free SPSC ring of fixed-size int64 records.
class SpscRing {
 public:
  SpscRing(size_t capacity_pow2, int rec_len);
  bool push(const int64_t* rec);
  bool pop(int64_t* rec);
  size_t pop_batch(int64_t* recs, size_t max_n);
  size_t size() const;
  int rec_len() const { return rec_len_; }

 private:
  std::vector<int64_t> buf_;
  size_t mask_;
  int rec_len_;
  alignas(64) std::atomic<size_t> head_{0};
  alignas(64) std::atomic<size_t> tail_{0};
};

// Checkpoint container: 8-byte little-endian header length, JSON header, raw tensor bytes
// (exactly the safetensors layout, so files open with the safetensors library too).
void write_container(const std::string& path, const std::string& header_json,
                     const std::vector<const void*>& blobs, const std::vector<size_t>& sizes);
std::string read_container_header(const std::string& path, uint64_t* data_offset);
uint32_t crc32(const void* data, size_t n, uint32_t seed = 0);

int64_t write_coded_csv(const std::string& path, const uint8_t* codes, int ncol, int64_t ld, int64_t n,
                        const std::vector<std::vector<std::string>>& vocab, const std::string& id_prefix,
                        char delim, int nthreads);

// Gaussian draws out[i] = N(0, 1) of Philox(seed, offset, index_base + i), fp64, threaded (host/random.cpp);
// with `pairs`, both Box-Muller outputs per index: out [n][2]
void philox_normal(uint64_t seed, uint64_t offset, uint64_t index_base, int64_t n, double* out, int nthreads,
                   int pairs = 0);

}  // namespace avh
