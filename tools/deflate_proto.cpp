// Host prototype for the writer's next coder: per-segment LZ77 (lanes of a member) with a
// window reaching back into earlier segments, hash chains, lazy matching, and ONE dynamic
// Huffman block per member.  Prints the compression ratio over a flat stream for parameter
// variants, with a zlib round trip of every member.  Not product code (a design probe).
// usage: deflate_proto <flat-file>
#include <zlib.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <vector>

static const uint16_t LBASE[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                   31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const uint8_t LEXT[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint16_t DBASE[30] = {1,    2,    3,    4,    5,    7,    9,    13,    17,    25,
                                   33,   49,   65,   97,   129,  193,  257,  385,   513,   769,
                                   1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
static const uint8_t DEXT[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
static const uint8_t CLORD[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

struct Tok {
  uint16_t lit_or_len;  // < 256 literal; else 256 + len
  uint16_t dist;
};

struct Params {
  uint32_t seg, win, depth;
  bool lazy;
  uint32_t hbits;
};

static uint32_t lcode(uint32_t len) {
  uint32_t c = 0;
  while (c + 1 < 29 && LBASE[c + 1] <= len) ++c;
  return c;
}
static uint32_t dcode(uint32_t d) {
  uint32_t c = 0;
  while (c + 1 < 30 && DBASE[c + 1] <= d) ++c;
  return c;
}

// LZ77 of [lo, hi) of the member with matches back to max(0, lo - win) (chain depth `depth`)
static void lz(const uint8_t *m, uint32_t lo, uint32_t hi, const Params &P, std::vector<Tok> &out) {
  const uint32_t H = 1u << P.hbits;
  std::vector<int32_t> head(H, -1), prev(hi, -1);
  auto h3 = [&](uint32_t p) {
    const uint32_t v = m[p] | m[p + 1] << 8 | m[p + 2] << 16;
    return (v * 2654435761u) >> (32 - P.hbits);
  };
  auto ins = [&](uint32_t p) {
    if (p + 3 > hi) return;
    const uint32_t h = h3(p);
    prev[p] = head[h];
    head[h] = (int32_t)p;
  };
  const uint32_t w0 = lo > P.win ? lo - P.win : 0;
  for (uint32_t p = w0; p < lo; ++p) ins(p);
  auto best = [&](uint32_t p, uint32_t &bl, uint32_t &bd) {
    bl = 0;
    bd = 0;
    if (p + 3 > hi) return;
    int32_t q = head[h3(p)];
    const uint32_t lim = std::min<uint32_t>(258, hi - p);
    for (uint32_t k = 0; k < P.depth && q >= 0 && p - (uint32_t)q <= 32768; ++k, q = prev[q]) {
      uint32_t l = 0;
      while (l < lim && m[q + l] == m[p + l]) ++l;
      if (l > bl) {
        bl = l;
        bd = p - (uint32_t)q;
        if (l == lim) break;
      }
    }
  };
  uint32_t p = lo;
  while (p < hi) {
    uint32_t l1, d1;
    best(p, l1, d1);
    if (l1 >= 3 && P.lazy && p + 1 < hi) {
      ins(p);
      uint32_t l2, d2;
      best(p + 1, l2, d2);
      if (l2 > l1) {
        out.push_back({m[p], 0});
        p += 1;
        continue;  // p+1 will be re-searched (already inserted p)
      }
      out.push_back({(uint16_t)(256 + l1), (uint16_t)d1});
      for (uint32_t q = p + 1; q < p + l1; ++q) ins(q);
      p += l1;
      continue;
    }
    ins(p);
    if (l1 >= 3) {
      out.push_back({(uint16_t)(256 + l1), (uint16_t)d1});
      for (uint32_t q = p + 1; q < p + l1; ++q) ins(q);
      p += l1;
    } else {
      out.push_back({m[p], 0});
      ++p;
    }
  }
}

// length-limited Huffman code lengths (heuristic: build, then zlib-style overflow fix)
static void huff_lengths(const uint32_t *freq, uint32_t n, uint32_t maxbits, uint8_t *len) {
  std::vector<std::pair<uint32_t, uint32_t>> s;
  for (uint32_t i = 0; i < n; ++i) {
    len[i] = 0;
    if (freq[i]) s.push_back({freq[i], i});
  }
  if (s.empty()) return;
  if (s.size() == 1) {
    len[s[0].second] = 1;
    return;
  }
  std::sort(s.begin(), s.end());
  // two-queue Huffman on sorted leaves
  const uint32_t m = (uint32_t)s.size();
  std::vector<uint64_t> w(2 * m);
  std::vector<int32_t> parent(2 * m, -1);
  for (uint32_t i = 0; i < m; ++i) w[i] = s[i].first;
  uint32_t a = 0, b = m, nxt = m;
  auto take = [&]() {
    if (a < m && (b >= nxt || w[a] <= w[b])) return a++;
    return b++;
  };
  while (nxt < 2 * m - 1) {
    const uint32_t x = take(), y = take();
    w[nxt] = w[x] + w[y];
    parent[x] = parent[y] = (int32_t)nxt;
    ++nxt;
  }
  std::vector<uint32_t> depth(2 * m, 0);
  for (int32_t i = (int32_t)nxt - 2; i >= 0; --i) depth[i] = depth[parent[i]] + 1;
  // overflow fix: count per length, push down
  std::vector<uint32_t> bl(64, 0);
  for (uint32_t i = 0; i < m; ++i) bl[std::min<uint32_t>(depth[i], 63)]++;
  uint32_t overflow = 0;
  for (uint32_t l = maxbits + 1; l < 64; ++l) {
    overflow += bl[l];
    bl[maxbits] += bl[l];
    bl[l] = 0;
  }
  // Kraft repair (zlib gen_bitlen style)
  while (true) {
    uint64_t kraft = 0;
    for (uint32_t l = 1; l <= maxbits; ++l) kraft += (uint64_t)bl[l] << (maxbits - l);
    if (kraft <= (1ull << maxbits)) break;
    uint32_t l = maxbits - 1;
    while (bl[l] == 0) --l;
    bl[l]--;
    bl[l + 1] += 2;
    bl[maxbits]--;
  }
  (void)overflow;
  // assign lengths: longest codes to the least frequent (s sorted ascending)
  uint32_t idx = 0;
  for (uint32_t l = maxbits; l >= 1 && idx < m; --l)
    for (uint32_t k = 0; k < bl[l] && idx < m; ++k) len[s[idx++].second] = (uint8_t)l;
}

struct BW {
  std::vector<uint8_t> o;
  uint64_t acc = 0;
  uint32_t nb = 0;
  void put(uint32_t v, uint32_t n) {
    acc |= (uint64_t)v << nb;
    nb += n;
    while (nb >= 8) {
      o.push_back((uint8_t)acc);
      acc >>= 8;
      nb -= 8;
    }
  }
  void flush() {
    if (nb) o.push_back((uint8_t)acc);
    acc = 0;
    nb = 0;
  }
};
static uint32_t rev(uint32_t c, uint32_t n) {
  uint32_t r = 0;
  for (uint32_t i = 0; i < n; ++i) r |= ((c >> i) & 1u) << (n - 1 - i);
  return r;
}
static void canon(const uint8_t *len, uint32_t n, uint32_t *code) {
  uint32_t cnt[16] = {0}, next[16] = {0};
  for (uint32_t i = 0; i < n; ++i) cnt[len[i]]++;
  cnt[0] = 0;
  uint32_t c = 0;
  for (uint32_t l = 1; l < 16; ++l) {
    c = (c + cnt[l - 1]) << 1;
    next[l] = c;
  }
  for (uint32_t i = 0; i < n; ++i)
    if (len[i]) code[i] = rev(next[len[i]]++, len[i]);
}

static std::vector<uint8_t> encode_dynamic(const std::vector<Tok> &toks) {
  uint32_t fl[286] = {0}, fd[30] = {0};
  for (auto &t : toks) {
    if (t.lit_or_len < 256) fl[t.lit_or_len]++;
    else {
      fl[257 + lcode(t.lit_or_len - 256)]++;
      fd[dcode(t.dist)]++;
    }
  }
  fl[256] = 1;
  uint8_t ll[286], dl[30];
  huff_lengths(fl, 286, 15, ll);
  huff_lengths(fd, 30, 15, dl);
  bool anyd = false;
  for (int i = 0; i < 30; ++i) anyd |= dl[i] != 0;
  if (!anyd) dl[0] = 1;
  uint32_t nlit = 286, ndist = 30;
  while (nlit > 257 && !ll[nlit - 1]) --nlit;
  while (ndist > 1 && !dl[ndist - 1]) --ndist;
  // RLE of lengths
  std::vector<uint8_t> all(ll, ll + nlit);
  all.insert(all.end(), dl, dl + ndist);
  std::vector<std::pair<uint8_t, uint8_t>> rle;  // (sym, extra)
  for (size_t i = 0; i < all.size();) {
    size_t j = i;
    while (j < all.size() && all[j] == all[i]) ++j;
    size_t run = j - i;
    if (all[i] == 0) {
      while (run >= 11) { const size_t r = std::min<size_t>(run, 138); rle.push_back({18, (uint8_t)(r - 11)}); run -= r; }
      if (run >= 3) { rle.push_back({17, (uint8_t)(run - 3)}); run = 0; }
      while (run--) rle.push_back({0, 0});
    } else {
      rle.push_back({all[i], 0});
      --run;
      while (run >= 3) { const size_t r = std::min<size_t>(run, 6); rle.push_back({16, (uint8_t)(r - 3)}); run -= r; }
      while (run--) rle.push_back({all[i], 0});
    }
    i = j;
  }
  uint32_t fc[19] = {0};
  for (auto &r : rle) fc[r.first]++;
  uint8_t cl[19];
  huff_lengths(fc, 19, 7, cl);
  uint32_t ncl = 19;
  while (ncl > 4 && !cl[CLORD[ncl - 1]]) --ncl;
  uint32_t cc[19] = {0}, lc[286] = {0}, dc[30] = {0};
  canon(cl, 19, cc);
  canon(ll, 286, lc);
  canon(dl, 30, dc);
  BW b;
  b.put(1, 1);
  b.put(2, 2);
  b.put(nlit - 257, 5);
  b.put(ndist - 1, 5);
  b.put(ncl - 4, 4);
  for (uint32_t i = 0; i < ncl; ++i) b.put(cl[CLORD[i]], 3);
  for (auto &r : rle) {
    b.put(cc[r.first], cl[r.first]);
    if (r.first == 16) b.put(r.second, 2);
    if (r.first == 17) b.put(r.second, 3);
    if (r.first == 18) b.put(r.second, 7);
  }
  for (auto &t : toks) {
    if (t.lit_or_len < 256) {
      b.put(lc[t.lit_or_len], ll[t.lit_or_len]);
    } else {
      const uint32_t len = t.lit_or_len - 256, c = lcode(len), d = dcode(t.dist);
      b.put(lc[257 + c], ll[257 + c]);
      b.put(len - LBASE[c], LEXT[c]);
      b.put(dc[d], dl[d]);
      b.put(t.dist - DBASE[d], DEXT[d]);
    }
  }
  b.put(lc[256], ll[256]);
  b.flush();
  return b.o;
}

int main(int argc, char **argv) {
  std::ifstream f(argv[1], std::ios::binary);
  std::vector<uint8_t> U((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  const uint32_t PAY = 65498;
  const Params vars[] = {
      {4096, 32768, 4, true, 15}, {1024, 32768, 4, true, 15}, {512, 32768, 4, true, 15},
      {256, 32768, 4, true, 15},  {256, 32768, 8, true, 15},  {256, 32768, 4, false, 15},
      {256, 32768, 4, true, 13},  {512, 32768, 8, true, 14},  {1024, 32768, 8, true, 14},
  };
  for (const Params &P : vars) {
    uint64_t total = 0;
    bool ok = true;
    for (size_t s = 0; s < U.size(); s += PAY) {
      const uint32_t n = (uint32_t)std::min<size_t>(PAY, U.size() - s);
      const uint8_t *m = U.data() + s;
      std::vector<Tok> toks;
      for (uint32_t lo = 0; lo < n; lo += P.seg) lz(m, lo, std::min(n, lo + P.seg), P, toks);
      auto o = encode_dynamic(toks);
      total += o.size() + 26;
      std::vector<uint8_t> back(n + 16);
      z_stream z{};
      inflateInit2(&z, -15);
      z.next_in = o.data();
      z.avail_in = (uInt)o.size();
      z.next_out = back.data();
      z.avail_out = (uInt)back.size();
      const int rc = inflate(&z, Z_FINISH);
      ok &= rc == Z_STREAM_END && z.total_out == n && !memcmp(back.data(), m, n);
      inflateEnd(&z);
    }
    std::printf("seg %5u win %5u depth %2u lazy %d hbits %u: ratio %.3f %s\n", P.seg, P.win, P.depth, P.lazy,
                P.hbits, (double)U.size() / (double)total, ok ? "ok" : "ROUNDTRIP FAILED");
  }
  return 0;
}
