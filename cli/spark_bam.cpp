// spark-bam CLI on MI355X: the reference's commands (cli/.../Main.scala:19-28) over the
// C-ABI in include/sparkbam.h.  Host side in C++ (the reference's Scala/JVM toolchain
// is not part of this build); all byte work runs in libsparkbam_hip.so on the GPU.
//
//   spark-bam compute-splits [-s] [-m SIZE] [-l N] BAM      (ComputeSplits.scala:18-156)
//   spark-bam count-reads   [-s] [-m SIZE] BAM              (compare/CountReads.scala:21-213)
//   spark-bam check-bam -s  [-m SIZE] [-i RANGES] [-r RECORDS] BAM  (check/eager/CheckBam.scala)
//   spark-bam full-check    [-m SIZE] [-i RANGES] [-l N] BAM       (check/full/FullCheck.scala)
//   spark-bam index-blocks  BAM [OUT]                        (bgzf/index/IndexBlocks.scala)
//   spark-bam index-records BAM [OUT]                        (check/index/IndexRecords.scala)
//   spark-bam check-blocks -s [-r RECORDS] [-l N] BAM        (cli/.../check/blocks/CheckBlocks.scala)
//   spark-bam htsjdk-rewrite [-r READS] [-b] [-i] BAM OUT     (cli/.../rewrite/HTSJDKRewrite.scala)
//
// The hadoop-bam ("seqdoop", -u) comparisons are out of scope: hadoop-bam's
// BAMSplitGuesser is a competitor's algorithm, not part of spark-bam's path.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "../include/sparkbam.h"

namespace {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

sbh_ctx *g_ctx = nullptr;

void chk(int rc, const char *what) {
  if (rc != SBH_OK) throw Error(rc, std::string(what) + ": " + sbh_last_error(g_ctx));
}

// hammerlab Bytes parser: integers or shorthands (k = 1024, "230k" = 235520)
uint64_t parse_bytes(const std::string &s) {
  size_t i = 0;
  while (i < s.size() && (isdigit((unsigned char)s[i]) || s[i] == '.')) ++i;
  double v = std::stod(s.substr(0, i));
  std::string u = s.substr(i);
  for (auto &c : u) c = (char)tolower(c);
  if (!u.empty() && u.back() == 'b') u.pop_back();
  double m = 1;
  if (u == "k") m = 1024.0;
  else if (u == "m") m = 1024.0 * 1024;
  else if (u == "g") m = 1024.0 * 1024 * 1024;
  else if (u == "t") m = 1024.0 * 1024 * 1024 * 1024;
  else if (!u.empty()) throw Error(SBH_E_ARG, "bad byte size: " + s);
  return (uint64_t)(v * m);
}

// ByteRanges (check/.../args/ByteRanges.scala, Range.scala): a-b | a+len | pos
std::vector<std::pair<uint64_t, uint64_t>> parse_ranges(const std::string &s) {
  std::vector<std::pair<uint64_t, uint64_t>> out;
  size_t p = 0;
  while (p <= s.size()) {
    size_t q = s.find(',', p);
    std::string t = s.substr(p, q == std::string::npos ? std::string::npos : q - p);
    size_t d = t.find('-'), pl = t.find('+');
    if (d != std::string::npos) out.push_back({parse_bytes(t.substr(0, d)), parse_bytes(t.substr(d + 1))});
    else if (pl != std::string::npos) {
      uint64_t a = parse_bytes(t.substr(0, pl));
      out.push_back({a, a + parse_bytes(t.substr(pl + 1))});
    } else {
      uint64_t a = parse_bytes(t);
      out.push_back({a, a + 1});
    }
    if (q == std::string::npos) break;
    p = q + 1;
  }
  return out;
}

std::vector<uint8_t> read_file(const std::string &path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw Error(SBH_E_ARG, "cannot open " + path);
  return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

struct Pos {
  uint64_t block = 0;
  uint32_t off = 0;
  std::string str() const { return std::to_string(block) + ":" + std::to_string(off); }
  double minus(const Pos &o, double ratio = 3.0) const {  // Pos.- (Pos.scala:17-22)
    int64_t v = (int64_t)block - (int64_t)o.block + (int64_t)(((int64_t)off - (int64_t)o.off) / ratio);
    return (double)std::max<int64_t>(0, v);
  }
};

struct BamHeader {
  std::vector<std::string> names;
  std::vector<int32_t> lens;
  uint64_t end = 0;
};

int32_t rd32(const uint8_t *p) { return (int32_t)((uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24); }

// header.Header.apply (check/.../header/Header.scala:26-60)
BamHeader parse_header(sbh_shard *sh, uint64_t flat_size) {
  uint64_t n = std::min<uint64_t>(flat_size, 1 << 16);
  for (;;) {
    std::vector<uint8_t> b(n);
    chk(sbh_read_flat(sh, 0, n, b.data()), "read header");
    BamHeader h;
    bool ok = n >= 12 && std::memcmp(b.data(), "BAM\1", 4) == 0;
    if (!ok) throw Error(SBH_E_ARG, "not a BAM file");
    uint64_t c = 8 + (uint64_t)rd32(&b[4]);
    bool done = false;
    if (c + 4 <= n) {
      int32_t nref = rd32(&b[c]);
      c += 4;
      done = true;
      for (int32_t i = 0; i < nref; ++i) {
        if (c + 4 > n) { done = false; break; }
        int32_t l = rd32(&b[c]);
        if (c + 8 + (uint64_t)l > n) { done = false; break; }
        h.names.emplace_back((const char *)&b[c + 4], strnlen((const char *)&b[c + 4], l));
        h.lens.push_back(rd32(&b[c + 4 + l]));
        c += 8 + l;
      }
    }
    if (done) { h.end = c; return h; }
    if (n >= flat_size) throw Error(SBH_E_TRUNCATED, "truncated BAM header");
    n = std::min<uint64_t>(flat_size, n * 4);
  }
}

struct Loaded {
  std::vector<uint8_t> data;
  sbh_shard *sh = nullptr;
  uint64_t nblocks = 0, flat = 0;
  BamHeader hdr;
  std::vector<sbh_block> blocks;
  explicit Loaded(const std::string &path) : data(read_file(path)) {
    chk(sbh_shard_create(g_ctx, data.data(), data.size(), 0, data.size(), 0, &sh), "shard");
    chk(sbh_index(sh, 0, &nblocks, &flat), "index");
    chk(sbh_inflate(sh, nullptr), "inflate");
    hdr = parse_header(sh, flat);
    chk(sbh_set_contigs(sh, hdr.lens.data(), (int32_t)hdr.lens.size()), "contigs");
    blocks.resize(nblocks);
    if (nblocks) chk(sbh_get_blocks(sh, 0, nblocks, blocks.data()), "blocks");
  }
  ~Loaded() { sbh_shard_destroy(sh); }
  Pos pos(uint64_t flat_pos) const {
    Pos p;
    chk(sbh_pos_of(sh, flat_pos, &p.block, &p.off), "pos");
    return p;
  }
};

std::vector<std::pair<uint64_t, uint64_t>> file_splits(uint64_t size, uint64_t split) {
  std::vector<std::pair<uint64_t, uint64_t>> out;
  uint64_t rem = size;
  while ((double)rem / (double)split > 1.1) {
    out.push_back({size - rem, size - rem + split});
    rem -= split;
  }
  if (rem) out.push_back({size - rem, size});
  return out;
}

// hammerlab stats number rendering (as in the reference's golden outputs)
std::string num(double v) {
  char b[64];
  if (std::fabs(v) >= 1e5) {
    snprintf(b, sizeof b, "%.1e", v);
    std::string s(b);
    size_t e = s.find('e');
    std::string mant = s.substr(0, e), ex = s.substr(e + 1);
    int x = std::stoi(ex);
    return mant + "e" + std::to_string(x);
  }
  if (std::fabs(v - std::round(v)) < 1e-9 || std::fabs(v) >= 100) {
    snprintf(b, sizeof b, "%.0f", v);
    return b;
  }
  snprintf(b, sizeof b, "%.1f", v);
  return b;
}

std::string stats_lines(const std::vector<double> &xs) {
  std::string out;
  size_t n = xs.size();
  if (!n) return "(empty)\n";
  double mean = 0;
  for (double x : xs) mean += x;
  mean /= n;
  double var = 0;
  for (double x : xs) var += (x - mean) * (x - mean);
  double sd = std::sqrt(var / n);
  auto median = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    size_t m = v.size();
    return m % 2 ? v[m / 2] : (v[m / 2 - 1] + v[m / 2]) / 2;
  };
  double med = median(xs);
  std::vector<double> dev;
  for (double x : xs) dev.push_back(std::fabs(x - med));
  double mad = median(dev);
  out += "N: " + std::to_string(n) + ", μ/σ: " + num(mean) + "/" + num(sd) + ", med/mad: " + num(med) + "/" + num(mad) + "\n";
  std::string el = " elems:", so = "sorted:";
  std::vector<double> s = xs;
  std::sort(s.begin(), s.end());
  for (double x : xs) el += " " + std::to_string((long long)x);
  for (double x : s) so += " " + std::to_string((long long)x);
  out += el + "\n" + so + "\n";
  return out;
}

// hammerlab Bytes.format: 583K, 25.6K, 1.2M ...
std::string bytes_fmt(uint64_t b) {
  const char *u[] = {"B", "K", "M", "G", "T"};
  double v = (double)b;
  int i = 0;
  while (v >= 1024 && i < 4) { v /= 1024; ++i; }
  char buf[64];
  if (i == 0) snprintf(buf, sizeof buf, "%lluB", (unsigned long long)b);
  else if (v >= 100) snprintf(buf, sizeof buf, "%.0f%s", std::floor(v + 0.5 - 1e-9), u[i]);
  else snprintf(buf, sizeof buf, "%.1f%s", v, u[i]);
  return buf;
}

struct Args {
  std::string cmd, path, out, records, blocks_path;
  uint64_t split = 0;
  bool has_split = false, s = false, u = false;
  long limit = 1000000;
  std::vector<std::pair<uint64_t, uint64_t>> ranges;
  bool has_ranges = false;
  int reads_to_check = 10, max_read_size = 100000000, blocks_to_check = 5;
  // htsjdk-rewrite: -r record-index ranges (IntRanges), -b / -i write OUT.blocks / OUT.records
  std::vector<std::pair<uint64_t, uint64_t>> read_ranges;
  bool has_read_ranges = false, idx_blocks = false, idx_records = false;
};

Args parse(int argc, char **argv) {
  Args a;
  if (argc < 2) throw Error(SBH_E_ARG, "usage: spark-bam <command> [options] <bam>");
  a.cmd = argv[1];
  const bool rewrite = a.cmd == "htsjdk-rewrite";
  std::vector<std::string> pos;
  for (int i = 2; i < argc; ++i) {
    std::string t = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) throw Error(SBH_E_ARG, "missing value for " + t);
      return argv[++i];
    };
    if (rewrite && (t == "-r" || t == "--read-ranges")) { a.read_ranges = parse_ranges(next()); a.has_read_ranges = true; }
    else if (rewrite && (t == "-b" || t == "--index-blocks")) a.idx_blocks = true;
    else if (rewrite && (t == "-i" || t == "--index-records")) a.idx_records = true;
    else if (t == "-m" || t == "--max-split-size") { a.split = parse_bytes(next()); a.has_split = true; }
    else if (t == "-s" || t == "--spark-bam") a.s = true;
    else if (t == "-u" || t == "--upstream" || t == "--hadoop-bam") a.u = true;
    else if (t == "-l" || t == "--print-limit") a.limit = std::stol(next());
    else if (t == "-i" || t == "--intervals") { a.ranges = parse_ranges(next()); a.has_ranges = true; }
    else if (t == "-r" || t == "--records-path") a.records = next();
    else if (t == "-b" || t == "--blocks-path") a.blocks_path = next();
    else if (t == "--reads-to-check") a.reads_to_check = std::stoi(next());
    else if (t == "--max-read-size") a.max_read_size = std::stoi(next());
    else if (t == "-z" || t == "--bgzf-blocks-to-check") a.blocks_to_check = std::stoi(next());
    else if (t == "-w" || t == "--warn") {}
    else pos.push_back(t);
  }
  if (pos.empty()) throw Error(SBH_E_ARG, "missing BAM path");
  a.path = pos[0];
  if (pos.size() > 1) a.out = pos[1];
  return a;
}

void no_hadoop_bam() {
  throw Error(SBH_E_ARG, "hadoop-bam (seqdoop) comparison is not part of the MI355X build; use -s");
}

struct SplitsResult {
  std::vector<std::pair<Pos, Pos>> splits;
  std::vector<uint64_t> counts;
};

SplitsResult splits_from(const std::vector<std::pair<uint64_t, uint64_t>> &sp, const std::vector<uint64_t> &v,
                         const std::vector<uint64_t> &cnt, const std::vector<int32_t> &status, uint64_t file_size) {
  SplitsResult r;
  std::vector<Pos> firsts;
  for (uint64_t i = 0; i < sp.size(); ++i) {
    if (status[i]) throw Error(status[i], "split " + std::to_string(sp[i].first) + "-" + std::to_string(sp[i].second));
    r.counts.push_back(cnt[i]);
    if (cnt[i]) firsts.push_back(Pos{v[i] >> 16, (uint32_t)(v[i] & 0xffff)});
  }
  for (size_t i = 0; i < firsts.size(); ++i)
    r.splits.push_back({firsts[i], i + 1 < firsts.size() ? firsts[i + 1] : Pos{file_size, 0}});
  return r;
}

// CanLoadBam.loadSplitsAndReads (load/.../CanLoadBam.scala:268-302)
SplitsResult spark_bam_splits(Loaded &L, const Args &a, uint64_t split_size) {
  // every split in one batch: FindBlockStart + FindRecordStart + counts on the device
  const auto sp = file_splits(L.data.size(), split_size);
  const uint64_t n = sp.size();
  std::vector<uint64_t> st(n), en(n), v(n), cnt(n);
  std::vector<int32_t> status(n);
  for (uint64_t i = 0; i < n; ++i) st[i] = sp[i].first, en[i] = sp[i].second;
  chk(sbh_split_starts(L.sh, st.data(), en.data(), n, a.blocks_to_check, a.reads_to_check, a.max_read_size,
                       v.data(), cnt.data(), status.data(), nullptr),
      "splits");
  return splits_from(sp, v, cnt, status, L.data.size());
}

uint64_t default_split(const Args &a) { return a.has_split ? a.split : 32ull << 20; }

// A file larger than this many compressed bytes (SBH_RESIDENT_MAX, default 24 GiB) is not held
// resident: it is memory-mapped and streamed through HBM in windows cut at split starts
// (sbh_run_stream2), each split decided in its window -- the same per-split answer in bounded
// HBM, as the reference bounds its memory per split (SplitRDD.scala:33-52, Stream.scala:80-122).
uint64_t resident_max() {
  const char *e = std::getenv("SBH_RESIDENT_MAX");
  return e && *e ? std::strtoull(e, nullptr, 10) : 24ull << 30;
}

struct Mapped {  // read-only mapping of a whole file
  const uint8_t *p = nullptr;
  uint64_t n = 0;
  explicit Mapped(const std::string &path) {
    const int fd = open(path.c_str(), O_RDONLY);
    if (fd < 0) throw Error(SBH_E_ARG, "cannot open " + path);
    struct stat st;
    if (fstat(fd, &st) != 0) {
      close(fd);
      throw Error(SBH_E_ARG, "cannot stat " + path);
    }
    n = (uint64_t)st.st_size;
    void *m = n ? mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0) : nullptr;
    close(fd);
    if (n && m == MAP_FAILED) throw Error(SBH_E_ARG, "cannot map " + path);
    p = static_cast<const uint8_t *>(m);
  }
  ~Mapped() {
    if (p) munmap(const_cast<uint8_t *>(p), n);
  }
};

// Header(path) from the file's leading bytes (grown x4 until the header fits)
BamHeader header_of(const uint8_t *data, uint64_t size) {
  for (uint64_t m = std::min<uint64_t>(size, 1 << 20);; m = std::min<uint64_t>(size, m * 4)) {
    sbh_shard *sh = nullptr;
    chk(sbh_shard_create(g_ctx, data, m, 0, size, 0, &sh), "shard");
    uint64_t nb = 0, flat = 0;
    int rc = sbh_index(sh, 0, &nb, &flat);
    if (!rc) rc = sbh_inflate(sh, nullptr);
    try {
      if (rc) throw Error(rc, "header blocks");
      BamHeader h = parse_header(sh, flat);
      sbh_shard_destroy(sh);
      return h;
    } catch (const Error &) {
      sbh_shard_destroy(sh);
      if (m >= size) throw;
    }
  }
}

// loadSplitsAndReads over a file streamed through HBM (sbh_run_stream2 with every split)
SplitsResult spark_bam_splits_streamed(const std::string &path, const Args &a, uint64_t split_size) {
  Mapped f(path);
  const BamHeader h = header_of(f.p, f.n);
  const auto sp = file_splits(f.n, split_size);
  const uint64_t n = sp.size();
  std::vector<uint64_t> st(n), en(n), v(n), cnt(n);
  std::vector<int32_t> status(n);
  for (uint64_t i = 0; i < n; ++i) st[i] = sp[i].first, en[i] = sp[i].second;
  sbh_stream_opts o{};
  o.window = 1ull << 30;
  o.halo = 4ull << 20;
  o.reads_to_check = a.reads_to_check;
  o.max_read_size = a.max_read_size;
  o.bgzf_blocks_to_check = a.blocks_to_check;
  o.split_start = st.data(), o.split_end = en.data(), o.n_splits = n;
  o.split_first_vpos = v.data(), o.split_count = cnt.data(), o.split_status = status.data();
  sbh_stream_result res;
  chk(sbh_run_stream2(g_ctx, f.p, f.n, 0, f.n, UINT64_MAX, f.n, h.lens.data(), (int32_t)h.lens.size(), &o, &res),
      "stream");
  return splits_from(sp, v, cnt, status, f.n);
}

// the resident path for files that fit, the streamed one otherwise
SplitsResult spark_bam_splits_any(const Args &a, uint64_t split_size) {
  struct stat st;
  if (stat(a.path.c_str(), &st) == 0 && (uint64_t)st.st_size > resident_max())
    return spark_bam_splits_streamed(a.path, a, split_size);
  Loaded L(a.path);
  return spark_bam_splits(L, a, split_size);
}

int compute_splits(const Args &a) {
  if (a.u && !a.s) no_hadoop_bam();
  auto t0 = std::chrono::steady_clock::now();
  SplitsResult r = spark_bam_splits_any(a, default_split(a));
  long ms = (long)std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
  printf("Get spark-bam splits: %ldms\n\n", ms);
  std::vector<double> lens;
  for (auto &s : r.splits) lens.push_back((double)(int64_t)s.second.minus(s.first));
  printf("Split-size distribution:\n%s\n", stats_lines(lens).c_str());
  size_t n = r.splits.size();
  if ((long)n <= a.limit) printf("%zu splits:\n", n);
  else printf("First %ld of %zu splits:\n", a.limit, n);
  for (size_t i = 0; i < n && (long)i < a.limit; ++i)
    printf("\t%s-%s\n", r.splits[i].first.str().c_str(), r.splits[i].second.str().c_str());
  if ((long)n > a.limit) printf("\t…\n");
  printf("\n");
  return 0;
}

int count_reads(const Args &a) {
  auto t0 = std::chrono::steady_clock::now();
  SplitsResult r = spark_bam_splits_any(a, default_split(a));
  uint64_t total = 0;
  for (uint64_t c : r.counts) total += c;
  long ms = (long)std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
  printf("spark-bam read-count time: %ld\n\n", ms);
  printf("spark-bam found %llu reads, hadoop-bam threw exception:\n", (unsigned long long)total);
  printf("\thadoop-bam is not part of the MI355X build\n");
  return 0;
}

std::vector<Pos> read_records_file(const std::string &p) {
  std::ifstream f(p);
  if (!f) throw Error(SBH_E_ARG, "no records file " + p + " (run index-records first)");
  std::vector<Pos> out;
  std::string line;
  while (std::getline(f, line)) {
    size_t c = line.find(',');
    if (c == std::string::npos) continue;
    out.push_back(Pos{std::stoull(line.substr(0, c)), (uint32_t)std::stoul(line.substr(c + 1))});
  }
  return out;
}

// Set bits of an LSB-first bitmap as positions base + i (64 positions per step).
std::vector<uint64_t> bits_to_positions(const std::vector<uint8_t> &bits, uint64_t base, uint64_t n) {
  std::vector<uint64_t> out;
  for (uint64_t i = 0; i < n; i += 64) {
    uint64_t w = 0;
    std::memcpy(&w, bits.data() + i / 8, std::min<uint64_t>(8, bits.size() - i / 8));
    if (n - i < 64) w &= (1ull << (n - i)) - 1;
    for (; w; w &= w - 1) out.push_back(base + i + (uint64_t)__builtin_ctzll(w));
  }
  return out;
}

// Blocks.apply (check/src/main/scala/org/hammerlab/bam/check/Blocks.scala:47-208): the blocks the
// all-positions modes examine, per partition.  With a `.blocks` file (-b, default BAM.blocks): its
// blocks whose start is in -i, partitioned by cumulative compressed size / split size (:86-139);
// without one: the file cut every split size, the splits meeting -i, each one's blocks found on
// the device (FindBlockStart, then MetadataStream while start < split end: sbh_find_blocks,
// :141-206).  The split size is -m, default 2 MB (:74-78).
struct BlockMeta {
  uint64_t start;
  uint32_t csize, usize;
};
struct BlocksPartitions {
  std::vector<std::vector<BlockMeta>> parts;
  std::vector<std::pair<uint64_t, uint64_t>> bounds;
  std::vector<uint64_t> starts() const {
    std::vector<uint64_t> v;
    for (auto &p : parts)
      for (auto &m : p) v.push_back(m.start);
    return v;
  }
};

bool in_ranges(const Args &a, uint64_t x) {
  if (!a.has_ranges) return true;
  for (auto &r : a.ranges)
    if (r.first <= x && x < r.second) return true;
  return false;
}

BlocksPartitions blocks_apply(const Args &a, const uint8_t *data, uint64_t size) {
  const uint64_t split = a.has_split ? a.split : 2ull << 20;
  const std::string bp = a.blocks_path.empty() ? a.path + ".blocks" : a.blocks_path;
  BlocksPartitions R;
  std::ifstream f(bp);
  if (f) {
    std::vector<BlockMeta> metas;
    std::string line;
    while (std::getline(f, line)) {
      if (line.empty()) continue;
      const size_t c1 = line.find(','), c2 = c1 == std::string::npos ? c1 : line.find(',', c1 + 1);
      if (c2 == std::string::npos) throw Error(SBH_E_ARG, "Bad blocks-index line: " + line);
      BlockMeta m{std::stoull(line.substr(0, c1)), (uint32_t)std::stoul(line.substr(c1 + 1, c2 - c1 - 1)),
                  (uint32_t)std::stoul(line.substr(c2 + 1))};
      if (in_ranges(a, m.start)) metas.push_back(m);
    }
    // partition = (compressed bytes of the blocks before it) / split; the partition count is the last
    // block's partition + 1 (as BlocksTest's "block boundaries" case pins it)
    uint64_t off = 0;
    for (auto &m : metas) {
      const uint64_t k = off / split;
      if (R.parts.size() <= k) R.parts.resize(k + 1);
      R.parts[k].push_back(m);
      off += m.csize;
    }
    for (uint64_t i = 0; i < R.parts.size(); ++i) R.bounds.push_back({i * split, (i + 1) * split});
    return R;
  }
  std::vector<uint64_t> idx, st, en;
  for (uint64_t i = 0; i * split < size; ++i) {
    bool meets = !a.has_ranges;
    for (auto &r : a.ranges) meets |= r.first < r.second && r.first < (i + 1) * split && r.second > i * split;
    if (!meets) continue;
    idx.push_back(i);
    st.push_back(i * split);
    en.push_back(std::min(size, (i + 1) * split));
    R.bounds.push_back({i * split, (i + 1) * split});
  }
  R.parts.resize(idx.size());
  std::vector<sbh_block> out(size / 16384 + 4096);  // BAM blocks average 15-25 KB; regrown if short
  uint64_t n = 0;
  for (;;) {
    chk(sbh_find_blocks(g_ctx, data, size, st.data(), en.data(), st.size(), a.blocks_to_check, 1ull << 30, out.data(),
                        out.size(), &n),
        "find blocks");
    if (n <= out.size()) break;
    out.resize(n);
  }
  for (uint64_t i = 0; i < n; ++i)
    if (in_ranges(a, out[i].start)) R.parts[out[i].ustart].push_back(BlockMeta{out[i].start, out[i].csize, out[i].usize});
  return R;
}

uint64_t stream_window() {
  const char *e = std::getenv("SBH_STREAM_WINDOW");
  return e && *e ? std::strtoull(e, nullptr, 10) : 1ull << 30;
}

// The file's record at/after a vpos, for PosMetadata (a few KB of the file around it inflated on
// the device; grown x4 while the search needs more bytes).
struct NextRecord {
  bool found = false;
  int32_t delta = 0, ref = 0, pos = 0, lseq = 0;
  uint32_t flag = 0;
  std::string name;
};
NextRecord next_record(const uint8_t *data, uint64_t size, const BamHeader &h, const Args &a, uint64_t vpos) {
  NextRecord r;
  const uint64_t blk = vpos >> 16;
  for (uint64_t span = 4ull << 20;; span *= 4) {
    const uint64_t n = std::min(size - blk, span);
    sbh_shard *sh = nullptr;
    chk(sbh_shard_create(g_ctx, data + blk, n, blk, size, 0, &sh), "shard");
    uint64_t nb = 0, flat = 0, nxt = 0;
    int rc = sbh_index(sh, blk, &nb, &flat);
    if (!rc) rc = sbh_inflate(sh, nullptr);
    if (!rc) rc = sbh_set_contigs(sh, h.lens.data(), (int32_t)h.lens.size());
    if (!rc) rc = sbh_find_record_start(sh, vpos & 0xffff, a.reads_to_check, a.max_read_size, &nxt, &r.delta);
    if (rc == SBH_E_NEED_HALO && blk + n < size) {
      sbh_shard_destroy(sh);
      continue;
    }
    if (!rc && nxt + 36 <= flat) {
      uint8_t f[36];
      chk(sbh_read_flat(sh, nxt, 36, f), "read record");
      r.ref = rd32(f + 4), r.pos = rd32(f + 8), r.lseq = rd32(f + 20);
      const uint32_t rnl = (uint32_t)rd32(f + 12) & 0xff;
      r.flag = (uint32_t)rd32(f + 16) >> 16;
      std::vector<uint8_t> name(rnl ? rnl : 1, 0);
      if (rnl && nxt + 36 + rnl <= flat) chk(sbh_read_flat(sh, nxt + 36, rnl, name.data()), "read name");
      r.name.assign((const char *)name.data(), strnlen((const char *)name.data(), rnl));
      r.found = true;
    }
    sbh_shard_destroy(sh);
    return r;
  }
}

// check-bam -s and full-check's pass over Blocks.apply's blocks: sbh_check_stream moves the file
// through HBM in windows, so any file size runs in bounded HBM.
struct AllPositions {
  sbh_check_result res{};
  std::vector<uint64_t> fp, fn, close_v, counts, rbe;
  std::vector<uint32_t> close_w;
};
AllPositions all_positions(const Args &a, const Mapped &f, const BamHeader &h, const std::vector<uint64_t> *truth,
                           bool full, uint64_t cap) {
  const BlocksPartitions B = blocks_apply(a, f.p, f.n);
  const std::vector<uint64_t> starts = B.starts();
  AllPositions R;
  sbh_check_opts o{};
  o.window = stream_window();
  o.halo = 4ull << 20;
  o.reads_to_check = a.reads_to_check;
  o.blocks = starts.data();
  o.n_blocks = starts.size();
  if (truth) {
    R.fp.resize(cap + 1);
    R.fn.resize(cap + 1);
    o.truth_vpos = truth->data();
    o.n_truth = truth->size();
    o.fp_vpos = R.fp.data(), o.fn_vpos = R.fn.data();
    o.fp_cap = o.fn_cap = cap;
  }
  if (full) {
    const uint64_t ccap = 1 << 22;
    R.counts.resize(21 * 19);
    R.rbe.resize(21 * 64);
    R.close_v.resize(ccap);
    R.close_w.resize(ccap);
    o.full = 1;
    o.counts = R.counts.data(), o.rbe_hist = R.rbe.data();
    o.close_vpos = R.close_v.data(), o.close_word = R.close_w.data(), o.close_cap = ccap;
  }
  chk(sbh_check_stream(g_ctx, f.p, f.n, h.lens.data(), (int32_t)h.lens.size(), &o, &R.res), "check");
  R.fp.resize(std::min<uint64_t>(R.res.fp, cap));
  R.fn.resize(std::min<uint64_t>(R.res.fn, cap));
  if (full) {
    R.close_v.resize(std::min<uint64_t>(R.res.n_close, R.close_v.size()));
    R.close_w.resize(R.close_v.size());
  }
  return R;
}

Pos pos_of_vpos(uint64_t v) { return Pos{v >> 16, (uint32_t)(v & 0xffff)}; }

// CheckerApp's summary (CheckerApp.scala:150-227) of the eager calls vs the `.records` truth
void print_check_summary(const Args &a, const AllPositions &R) {
  const uint64_t tp = R.res.tp, fp = R.res.fp, fn = R.res.fn, positions = R.res.positions, comp = R.res.comp_bytes;
  if (R.res.unknown)
    throw Error(SBH_E_NOT_FOUND, std::to_string(R.res.unknown) + " records-file positions are not block starts");
  printf("%llu uncompressed positions\n%s compressed\nCompression ratio: %.2f\n%llu reads\n",
         (unsigned long long)positions, bytes_fmt(comp).c_str(), (double)positions / (double)comp,
         (unsigned long long)(tp + fn));
  if (!fp && !fn) {
    printf("All calls matched!\n");
    return;
  }
  printf("%llu false positives, %llu false negatives\n\n", (unsigned long long)fp, (unsigned long long)fn);
  if (fp) {
    printf("False positives:\n");
    for (uint64_t v : R.fp) printf("\t%s\n", pos_of_vpos(v).str().c_str());
  }
  if (fn) {
    printf("%llu false negatives:\n", (unsigned long long)fn);
    for (uint64_t v : R.fn) printf("\t%s\n", pos_of_vpos(v).str().c_str());
  }
}

std::vector<uint64_t> truth_of(const Args &a) {
  std::vector<Pos> recs = read_records_file(a.records.empty() ? a.path + ".records" : a.records);
  std::vector<uint64_t> truth(recs.size());
  for (size_t i = 0; i < recs.size(); ++i) truth[i] = recs[i].block << 16 | recs[i].off;
  std::sort(truth.begin(), truth.end());
  return truth;
}

int check_bam(const Args &a) {
  if (!a.s) no_hadoop_bam();
  Mapped f(a.path);
  const BamHeader h = header_of(f.p, f.n);
  const std::vector<uint64_t> truth = truth_of(a);
  const AllPositions R = all_positions(a, f, h, &truth, false, (uint64_t)std::max(a.limit, 0L));
  print_check_summary(a, R);
  return 0;
}

const char *FLAG_NAMES[19] = {
    "tooFewFixedBlockBytes", "negativeReadIdx", "tooLargeReadIdx", "negativeReadPos", "tooLargeReadPos",
    "negativeNextReadIdx", "tooLargeNextReadIdx", "negativeNextReadPos", "tooLargeNextReadPos",
    "tooFewBytesForReadName", "nonNullTerminatedReadName", "nonASCIIReadName", "noReadName", "emptyReadName",
    "tooFewBytesForCigarOps", "invalidCigarOp", "emptyMappedCigar", "emptyMappedSeq",
    "tooFewRemainingBytesImplied"};

std::string flags_str(uint32_t w) {
  std::string s;
  for (int i = 0; i < 19; ++i)
    if (w & (1u << i)) s += (s.empty() ? "" : ",") + std::string(FLAG_NAMES[i]);
  return s;
}

// PosMetadata show (check/.../PosMetadata.scala:20-53) with htsjdk SAMRecord.toString
std::string pos_metadata(const Mapped &f, const BamHeader &h, const Args &a, uint64_t vpos, uint32_t word) {
  std::string rec = "no next record";
  const NextRecord r = next_record(f.p, f.n, h, a, vpos);
  if (r.found) {
    std::string s = std::to_string(r.delta) + " before " + r.name;
    if (r.flag & 1) s += (r.flag & 0x40) ? " 1/2" : " 2/2";
    s += " " + std::to_string(r.lseq) + "b";
    const bool unmapped = r.flag & 4;
    s += unmapped ? " unmapped read" : " aligned read";
    auto where = [&]() { return h.names[r.ref] + ":" + std::to_string(r.pos + 1); };
    if (unmapped && r.pos + 1 >= 0 && r.ref >= 0 && r.ref < (int32_t)h.names.size()) s += " (placed at " + where() + ")";
    else if (!unmapped && r.ref >= 0 && r.ref < (int32_t)h.names.size()) s += " @ " + where();
    rec = s;
  }
  return pos_of_vpos(vpos).str() + ":\t" + rec + ". Failing checks: " + flags_str(word & SBH_FULL_FLAGS_MASK);
}

std::vector<std::string> counts_lines(const std::vector<uint64_t> &c, const std::map<uint32_t, uint64_t> &rbe,
                                      bool include_zeros, bool hide_first) {
  std::vector<std::pair<std::string, uint64_t>> kv;
  for (int i = 0; i < 19; ++i) kv.push_back({FLAG_NAMES[i], c[i]});
  std::stable_sort(kv.begin(), kv.end(), [](auto &x, auto &y) { return x.second > y.second; });
  std::vector<std::pair<std::string, std::string>> pairs;
  for (auto &p : kv) {
    if ((p.second > 0 || include_zeros) && (p.first != "tooFewFixedBlockBytes" || !hide_first))
      pairs.push_back({p.first, std::to_string(p.second)});
  }
  if (!rbe.empty()) {
    std::string v;
    for (auto &r : rbe) v += (v.empty() ? "" : " ") + std::to_string(r.first) + "ⅹ" + std::to_string(r.second);
    pairs.push_back({"readsBeforeError", v});
  }
  size_t mk = 0, mv = 0;
  for (auto &p : pairs) { mk = std::max(mk, p.first.size()); mv = std::max(mv, p.second.size()); }
  std::vector<std::string> out;
  for (auto &p : pairs)
    out.push_back(std::string(mk - p.first.size(), ' ') + p.first + ":\t" + std::string(mv - p.second.size(), ' ') + p.second);
  return out;
}

int full_check(const Args &a) {
  Mapped f(a.path);
  const BamHeader h = header_of(f.p, f.n);
  // records file, if present: the indexed comparison summary first (FullCheck.scala:94-106), from
  // the same pass over the blocks
  const std::string rp = a.records.empty() ? a.path + ".records" : a.records;
  const bool have_records = (bool)std::ifstream(rp);
  std::vector<uint64_t> truth;
  if (have_records) {
    Args e = a;
    e.records = rp;
    truth = truth_of(e);
  }
  const AllPositions R = all_positions(a, f, h, have_records ? &truth : nullptr, true, (uint64_t)std::max(a.limit, 0L));
  if (have_records) {
    print_check_summary(a, R);
    printf("\n");
  }
  const std::vector<uint64_t> &counts = R.counts, &rbe = R.rbe;
  std::vector<std::pair<uint64_t, uint32_t>> close;
  for (size_t i = 0; i < R.close_v.size(); ++i) close.push_back({R.close_v[i], R.close_w[i]});
  auto nnz_of = [](uint32_t w) { return __builtin_popcount(w & SBH_FULL_FLAGS_MASK) + (((w >> SBH_FULL_N_SHIFT) & 0x3FF) > 0); };
  auto per = [&](int k) {
    std::vector<uint64_t> c(19);
    for (int i = 0; i < 19; ++i) c[i] = counts[k * 19 + i];
    std::map<uint32_t, uint64_t> r;
    for (int j = 1; j < 64; ++j)
      if (rbe[k * 64 + j]) r[j] = rbe[k * 64 + j];
    return std::make_pair(c, r);
  };
  std::vector<std::pair<uint64_t, uint32_t>> ones, twos;
  for (auto &c : close) (nnz_of(c.second) == 1 ? ones : twos).push_back(c);
  if (ones.empty()) {
    printf("No positions where only one check failed\n");
  } else {
    auto pc = per(1);
    printf("Critical error counts (true negatives where only one check failed):\n");
    for (auto &l : counts_lines(pc.first, pc.second, false, false)) printf("\t%s\n", l.c_str());
    printf("\n");
    if ((long)ones.size() <= a.limit) printf("%zu critical positions:\n", ones.size());
    else printf("%ld of %zu critical positions:\n", a.limit, ones.size());
    for (size_t i = 0; i < ones.size() && (long)i < a.limit; ++i)
      printf("\t%s\n", pos_metadata(f, h, a, ones[i].first, ones[i].second).c_str());
    if ((long)ones.size() > a.limit) printf("\t…\n");
  }
  printf("\n");
  if (twos.empty()) {
    printf("No positions where exactly two checks failed\n\n");
  } else {
    if ((long)twos.size() <= a.limit) printf("%zu positions where exactly two checks failed:\n", twos.size());
    else printf("%ld of %zu positions where exactly two checks failed:\n", a.limit, twos.size());
    for (size_t i = 0; i < twos.size() && (long)i < a.limit; ++i)
      printf("\t%s\n", pos_metadata(f, h, a, twos[i].first, twos[i].second).c_str());
    if ((long)twos.size() > a.limit) printf("\t…\n");
    printf("\n");
    std::map<uint32_t, uint64_t> hist;
    for (auto &t : twos) hist[t.second & SBH_FULL_FLAGS_MASK]++;
    std::vector<std::pair<uint64_t, uint32_t>> h;
    for (auto &x : hist) h.push_back({x.second, x.first});
    std::stable_sort(h.begin(), h.end(), [](auto &x, auto &y) { return x.first > y.first; });
    if (h.front().first > 1) {
      printf("\tHistogram:\n");
      for (size_t i = 0; i < h.size() && (long)i < a.limit; ++i)
        printf("\t\t%llu:\t%s\n", (unsigned long long)h[i].first, flags_str(h[i].second).c_str());
      printf("\n");
    }
    auto pc = per(2);
    printf("\tPer-flag totals:\n");
    for (auto &l : counts_lines(pc.first, pc.second, false, false)) printf("\t\t%s\n", l.c_str());
    printf("\n");
  }
  std::vector<uint64_t> tot(19, 0);
  std::map<uint32_t, uint64_t> trbe;
  for (int k = 0; k < 21; ++k) {
    for (int i = 0; i < 19; ++i) tot[i] += counts[k * 19 + i];
    for (int j = 1; j < 64; ++j)
      if (rbe[k * 64 + j]) trbe[j] += rbe[k * 64 + j];
  }
  printf("Total error counts:\n");
  for (auto &l : counts_lines(tot, trbe, true, true)) printf("\t%s\n", l.c_str());
  printf("\n");
  return 0;
}

int index_blocks(const Args &a) {
  Loaded L(a.path);
  std::string out = a.out.empty() ? a.path + ".blocks" : a.out;
  FILE *f = fopen(out.c_str(), "w");
  if (!f) throw Error(SBH_E_ARG, "cannot write " + out);
  for (const sbh_block &b : L.blocks) {
    if (b.flags & SBH_BLOCK_EMPTY) break;  // MetadataStream ends at the first empty block
    fprintf(f, "%llu,%u,%u\n", (unsigned long long)b.start, b.csize, b.usize);
  }
  fclose(f);
  return 0;
}

int index_records(const Args &a) {
  Loaded L(a.path);
  uint64_t seg_end = L.flat;
  for (const sbh_block &b : L.blocks)
    if (b.flags & SBH_BLOCK_EMPTY) { seg_end = b.ustart; break; }
  std::vector<uint8_t> bits((seg_end - L.hdr.end + 7) / 8);
  uint64_t n = 0, chain = 0;
  chk(sbh_check_eager(L.sh, L.hdr.end, seg_end, a.reads_to_check, bits.data(), &n), "eager");
  chk(sbh_count_records(L.sh, L.hdr.end, seg_end, &chain), "records");
  if (chain != n) throw Error(SBH_E_STATE, "record chain and eager calls disagree; refusing to write .records");
  std::string out = a.out.empty() ? a.path + ".records" : a.out;
  FILE *f = fopen(out.c_str(), "w");
  if (!f) throw Error(SBH_E_ARG, "cannot write " + out);
  for (uint64_t p : bits_to_positions(bits, L.hdr.end, seg_end - L.hdr.end)) {
    Pos q = L.pos(p);
    fprintf(f, "%llu,%u\n", (unsigned long long)q.block, q.off);
  }
  fclose(f);
  return 0;
}

// HTSJDKRewrite (cli/.../rewrite/HTSJDKRewrite.scala:40-92): the BAM's uncompressed stream --
// header, then every record, or only the records whose index is in -r (:48-58) -- re-cut into
// 65498-byte BGZF members on the GPU (sbh_bgzf_compress) plus the EOF member; -b / -i then
// index the output like IndexBlocks / IndexRecords (:72-90).  Records pass through byte for
// byte (htsjdk's decode/re-encode is the identity on a BAM it wrote), and each member is
// deflated exactly as htsjdk's Deflater(5) does (zlib 1.2.11 deflate_slow, include/sparkbam.h),
// so the output and its .blocks / .records equal htsjdk's (HTSJDKRewriteTest's dirMatch).
int htsjdk_rewrite(const Args &a) {
  if (a.out.empty()) throw Error(SBH_E_ARG, "htsjdk-rewrite: missing output path");
  std::vector<uint8_t> payload;
  {
    Loaded L(a.path);
    uint64_t seg_end = L.flat;
    for (const sbh_block &b : L.blocks)
      if (b.flags & SBH_BLOCK_EMPTY) { seg_end = b.ustart; break; }
    std::vector<uint8_t> flat(seg_end);
    if (seg_end) chk(sbh_read_flat(L.sh, 0, seg_end, flat.data()), "read stream");
    if (!a.has_read_ranges) {
      payload.swap(flat);
    } else {
      // record starts: the eager calls over the records, proven equal to the record chain
      std::vector<uint8_t> bits((seg_end - L.hdr.end + 7) / 8);
      uint64_t n = 0, chain = 0;
      chk(sbh_check_eager(L.sh, L.hdr.end, seg_end, a.reads_to_check, bits.data(), &n), "eager");
      chk(sbh_count_records(L.sh, L.hdr.end, seg_end, &chain), "records");
      if (chain != n) throw Error(SBH_E_STATE, "record chain and eager calls disagree");
      const std::vector<uint64_t> st = bits_to_positions(bits, L.hdr.end, seg_end - L.hdr.end);
      payload.assign(flat.begin(), flat.begin() + (ptrdiff_t)L.hdr.end);
      for (uint64_t i = 0; i < st.size(); ++i) {
        bool in = false;
        for (auto &r : a.read_ranges) in |= r.first <= i && i < r.second;
        if (!in) continue;
        const uint64_t e = i + 1 < st.size() ? st[i + 1] : seg_end;
        payload.insert(payload.end(), flat.begin() + (ptrdiff_t)st[i], flat.begin() + (ptrdiff_t)e);
      }
    }
  }
  std::vector<uint8_t> out(sbh_bgzf_compress_bound(payload.size()));
  uint64_t size = 0, nb = 0;
  chk(sbh_bgzf_compress(g_ctx, payload.data(), payload.size(), 0, out.data(), out.size(), &size, &nb, nullptr),
      "bgzf compress");
  FILE *f = fopen(a.out.c_str(), "wb");
  if (!f) throw Error(SBH_E_ARG, "cannot write " + a.out);
  const bool ok = fwrite(out.data(), 1, size, f) == size;
  fclose(f);
  if (!ok) throw Error(SBH_E_ARG, "short write to " + a.out);
  Args ix = a;
  ix.path = a.out;
  ix.out.clear();
  if (a.idx_blocks) index_blocks(ix);
  if (a.idx_records) index_records(ix);
  return 0;
}

// hammerlab Stats.fromHist rendered with the truncating Show[Double] CheckBlocks installs
// (CheckBlocks.scala:123-131): N, mean / population sigma, median / MAD, the histogram's
// first and last 10 runs ("v" or "v×n", "…" between), and the percentiles whose
// interpolation index (N + 1) p - 1 lies inside [0, N - 1].
std::string stats_hist(const std::map<long long, uint64_t> &hist) {
  std::vector<double> v;
  for (auto &kv : hist) v.insert(v.end(), kv.second, (double)kv.first);
  const size_t n = v.size();
  if (!n) return "(empty)\n";
  auto rnd = [](double x) { return std::to_string((long long)std::floor(x + 0.5)); };
  auto pct = [&](const std::vector<double> &s, double p) {  // s sorted
    const double idx = (double)(s.size() + 1) * p - 1;
    const size_t lo = (size_t)std::floor(idx);
    const double f = idx - (double)lo;
    return lo + 1 < s.size() ? s[lo] + f * (s[lo + 1] - s[lo]) : s[lo];
  };
  double mean = 0, var = 0;
  for (double x : v) mean += x;
  mean /= (double)n;
  for (double x : v) var += (x - mean) * (x - mean);
  const double sd = std::sqrt(var / (double)n), med = pct(v, 0.5);
  std::vector<double> dev;
  for (double x : v) dev.push_back(std::fabs(x - med));
  std::sort(dev.begin(), dev.end());
  std::string out = "N: " + std::to_string(n) + ", μ/σ: " + rnd(mean) + "/" + rnd(sd) + ", med/mad: " + rnd(med) +
                    "/" + rnd(pct(dev, 0.5)) + "\n";
  std::vector<std::string> runs;
  for (auto &kv : hist)
    runs.push_back(std::to_string(kv.first) + (kv.second > 1 ? "×" + std::to_string(kv.second) : ""));
  out += " elems:";
  for (size_t i = 0; i < runs.size(); ++i) {
    if (runs.size() > 20 && i == 10) {
      out += " …";
      i = runs.size() - 10;
    }
    out += " " + runs[i];
  }
  out += "\n";
  const double ps[] = {0.01, 0.05, 0.10, 0.25, 0.50, 0.75, 0.90, 0.95, 0.99};
  for (double p : ps) {
    const double idx = (double)(n + 1) * p - 1;
    if (idx < 0 || idx > (double)(n - 1)) continue;
    char lab[16];
    snprintf(lab, sizeof lab, "%.2f", p);
    out += std::string("  ") + (lab + 1) + ":\t" + rnd(pct(v, p)) + "\n";
  }
  return out;
}

// java.lang.Double.toString for 1e-3 <= |x| < 1e7: the shortest digits that read back
std::string jdouble(double x) {
  char b[64];
  for (int p = 1; p <= 17; ++p) {
    snprintf(b, sizeof b, "%.*g", p, x);
    if (std::strtod(b, nullptr) == x) break;
  }
  std::string s(b);
  if (s.find('.') == std::string::npos && s.find('e') == std::string::npos) s += ".0";
  return s;
}

// CheckBlocks (cli/.../check/blocks/CheckBlocks.scala:30-195), -s mode: for every BGZF
// block, the next read start from Pos(start, 0) by the indexed checker (the .records
// ground truth) and by the eager checker; blocks where they differ are reported with the
// compressed positions whose splits they would break.
int check_blocks(const Args &a) {
  if (!a.s || a.u) no_hadoop_bam();
  Loaded L(a.path);
  std::vector<uint64_t> truth;
  for (auto &r : read_records_file(a.records.empty() ? a.path + ".records" : a.records)) {
    uint64_t f = 0;
    chk(sbh_flat_of(L.sh, r.block, r.off, &f), "records file position");
    truth.push_back(f);
  }
  std::sort(truth.begin(), truth.end());
  uint64_t seg_end = L.flat;
  std::vector<const sbh_block *> blocks;
  for (const sbh_block &b : L.blocks) {
    if (b.flags & SBH_BLOCK_EMPTY) { seg_end = b.ustart; break; }  // the stream (and the block list) ends
    blocks.push_back(&b);
  }
  std::vector<uint8_t> bits((seg_end + 7) / 8);
  uint64_t ncalled = 0;
  if (seg_end) chk(sbh_check_eager(L.sh, 0, seg_end, a.reads_to_check, bits.data(), &ncalled), "eager");
  auto next_set = [&](uint64_t f) -> int64_t {  // eager nextReadStart: first call in [f, f + maxReadSize)
    const uint64_t lim = std::min<uint64_t>(seg_end, f + (uint64_t)a.max_read_size);
    for (uint64_t i = f; i < lim; ++i)
      if (bits[i >> 3] & (1u << (i & 7))) return (int64_t)i;
    return -1;
  };
  auto show = [&](int64_t f) { return f < 0 ? std::string("-") : L.pos((uint64_t)f).str(); };
  std::map<long long, uint64_t> offsets;  // first read's offset in its block -> blocks
  uint64_t no_read = 0, wrong_pos = 0;
  std::vector<std::string> bad;
  for (size_t i = 0; i < blocks.size(); ++i) {
    const sbh_block &b = *blocks[i];
    auto it = std::lower_bound(truth.begin(), truth.end(), b.ustart);
    const int64_t p1 = it == truth.end() ? -1 : (int64_t)*it;
    const int64_t p2 = next_set(b.ustart);
    if (p1 >= 0 && L.pos((uint64_t)p1).block == b.start) ++offsets[(long long)L.pos((uint64_t)p1).off];
    else ++no_read;
    if (p1 != p2) {
      const uint64_t prev = i ? blocks[i - 1]->csize : 1;
      wrong_pos += prev;
      bad.push_back(std::to_string(b.start) + " (prev block size: " + std::to_string(prev) + "):\t" + show(p1) +
                    "\t" + show(p2));
    }
  }
  const uint64_t total = L.data.size();
  auto offsets_info = [&]() {
    if (no_read && offsets.size() == 1 && offsets.count(0))
      printf("\n%llu blocks start with a read, %llu blocks didn't contain a read\n",
             (unsigned long long)offsets[0], (unsigned long long)no_read);
    else if (!no_read && offsets.size() == 1 && offsets.count(0))
      printf("\nAll blocks start with reads\n");
    else
      printf("\nOffsets of blocks' first reads (%llu blocks didn't contain a read start):\n%s",
             (unsigned long long)no_read, stats_hist(offsets).c_str());
  };
  if (bad.empty()) {
    printf("First read-position matched in %zu BGZF blocks totaling %sB (compressed)\n", blocks.size(),
           bytes_fmt(total).c_str());
    offsets_info();
  } else {
    printf("First read-position mismatched in %zu of %zu BGZF blocks\n\n", bad.size(), blocks.size());
    printf("%llu of %llu (%s) compressed positions would lead to bad splits\n", (unsigned long long)wrong_pos,
           (unsigned long long)total, jdouble((double)wrong_pos / (double)total).c_str());
    offsets_info();
    printf("\n");
    if ((long)bad.size() <= a.limit) printf("%zu mismatched blocks:\n", bad.size());
    else printf("%ld of %zu mismatched blocks:\n", a.limit, bad.size());
    for (size_t i = 0; i < bad.size() && (long)i < a.limit; ++i) printf("\t%s\n", bad[i].c_str());
  }
  return 0;
}

}  // namespace

int main(int argc, char **argv) {
  try {
    Args a = parse(argc, argv);
    chk(sbh_ctx_create(0, &g_ctx), "context");
    int rc;
    if (a.cmd == "compute-splits") rc = compute_splits(a);
    else if (a.cmd == "count-reads") rc = count_reads(a);
    else if (a.cmd == "check-bam") rc = check_bam(a);
    else if (a.cmd == "full-check") rc = full_check(a);
    else if (a.cmd == "index-blocks") rc = index_blocks(a);
    else if (a.cmd == "index-records") rc = index_records(a);
    else if (a.cmd == "check-blocks") rc = check_blocks(a);
    else if (a.cmd == "htsjdk-rewrite") rc = htsjdk_rewrite(a);
    else throw Error(SBH_E_ARG, "unknown command " + a.cmd);
    sbh_ctx_destroy(g_ctx);
    return rc;
  } catch (const Error &e) {
    fprintf(stderr, "spark-bam: %s\n", e.what());
    if (g_ctx) sbh_ctx_destroy(g_ctx);
    return 1;
  } catch (const std::exception &e) {
    fprintf(stderr, "spark-bam: %s\n", e.what());
    return 1;
  }
}
