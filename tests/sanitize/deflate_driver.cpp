// ASan/UBSan driver for the BGZF writer's host build (tools/deflate_host.cpp = deflate_core.h,
// the coder k_deflate runs): compresses patterned, random and file inputs of awkward sizes
// and inflates every member back with zlib.  Test infrastructure only.
#include <zlib.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <random>
#include <vector>

extern "C" uint64_t sbh_host_bgzf_compress(const uint8_t *src, uint64_t n, uint8_t *out);

static int roundtrip(const std::vector<uint8_t> &in) {
  const uint64_t nb = (in.size() + 65497) / 65498;
  std::vector<uint8_t> out(nb * 65536 + 28 + 64);
  const uint64_t m = sbh_host_bgzf_compress(in.data(), in.size(), out.data());
  std::vector<uint8_t> back;
  uint64_t o = 0;
  while (o + 18 <= m) {
    const uint32_t bsize = (uint32_t)out[o + 16] | (uint32_t)out[o + 17] << 8;
    const uint32_t cs = bsize + 1;
    uint32_t isize = 0;
    std::memcpy(&isize, &out[o + cs - 4], 4);
    std::vector<uint8_t> buf(isize + 1);
    z_stream z{};
    if (inflateInit2(&z, -15) != Z_OK) return 1;
    z.next_in = &out[o + 18];
    z.avail_in = cs - 26;
    z.next_out = buf.data();
    z.avail_out = (uInt)buf.size();
    const int rc = inflate(&z, Z_FINISH);
    inflateEnd(&z);
    if (rc != Z_STREAM_END || z.total_out != isize) return 1;
    back.insert(back.end(), buf.begin(), buf.begin() + isize);
    o += cs;
  }
  return o == m && back == in ? 0 : 1;
}

int main(int argc, char **argv) {
  std::mt19937_64 rng(7);
  int bad = 0, n = 0;
  for (uint64_t size : {0ull, 1ull, 3ull, 65497ull, 65498ull, 65499ull, 200000ull}) {
    std::vector<uint8_t> a(size), b(size), c(size);
    for (uint64_t i = 0; i < size; ++i) {
      a[i] = (uint8_t)rng();
      b[i] = (uint8_t)(i % 7 == 0 ? rng() % 4 : 'A' + i % 3);
      c[i] = 0;
    }
    bad += roundtrip(a) + roundtrip(b) + roundtrip(c);
    n += 3;
  }
  for (int k = 1; k < argc; ++k) {
    std::ifstream f(argv[k], std::ios::binary);
    std::vector<uint8_t> d((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    bad += roundtrip(d);
    ++n;
  }
  std::printf("%d inputs, %d failed round trips\n", n, bad);
  return bad ? 1 : 0;
}
