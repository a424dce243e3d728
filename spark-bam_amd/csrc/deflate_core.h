// deflate_core.h -- one BGZF member of the writer: LZ77 over hash chains with lazy matching,
// ONE dynamic-Huffman deflate block per member, the BGZF framing (RFC 1952 + the BC extra
// subfield) and its CRC32 / ISIZE footer.
//
// Replaces, for HTSJDKRewrite (cli/src/main/scala/org/hammerlab/bam/rewrite/HTSJDKRewrite.scala:62-67),
// the block compressor htsjdk's BAM writer drives (BlockCompressedOutputStream -> java.util.zip
// Deflater level 5; third-party: htsjdk, not in /root/reference): the uncompressed stream is cut
// every 65498 bytes (the payload size visible in every full block of test_bams/.../2.bam.blocks)
// and each piece becomes one member; a piece whose deflate output would not fit the 64 KiB
// member is stored instead.  The deflate bytes are this coder's own, not zlib's: member
// boundaries and the uncompressed layout match htsjdk's, the compressed bytes do not.
//
// The coder, defined so that a GPU can run it with one workgroup per member and one lane per
// 256-byte segment and give exactly the bytes of the serial definition below:
//  1. prev[p] = the latest q < p whose 3-byte hash (HB bits) equals p's (chains, as zlib's);
//  2. each segment [256 t, 256 t + 256) is parsed on its own (matches end inside it, but reach
//     back up to 32 KiB into the member): at p the best of DEPTH chain candidates (longest,
//     nearest first on ties; a NICE-long match ends the walk), lazily -- a match shorter than
//     LAZY is deferred by one literal when p + 1 has a longer one (zlib level 5's nice 32 /
//     lazy 16);
//  3. the member's token histogram gives length-limited Huffman codes (a two-queue Huffman
//     tree on the (frequency, symbol)-sorted symbols, then zlib's overflow repair), the block
//     header codes them with the RFC 1951 code-length alphabet;
//  4. the bit stream is the header, every segment's tokens in order, the end-of-block code.
// Measured on the reference's 2.bam / 5k.bam streams (tools/deflate_host.cpp): ratio 2.875 /
// 2.932, against 1.85 for round 1's fixed-Huffman 4 KiB segments and 3.02 / 3.11 for the
// reference files themselves (htsjdk, zlib level 5).
//
// Written once for both sides: the device kernel (deflate.hip) and tests/ build the same
// header for the host (tools/deflate_host.cpp) to round-trip it through zlib without a GPU.
// SBH_HD is __host__ __device__ under hipcc, empty otherwise.
#pragma once
#include <stdint.h>

#ifndef SBH_HD
#define SBH_HD
#endif

namespace sbh_deflate {

constexpr uint32_t PAYLOAD = 65498;  // htsjdk DEFAULT_UNCOMPRESSED_BLOCK_SIZE (2.bam.blocks)
constexpr uint32_t SLOT = 65536;     // max BGZF member size (BSIZE is u16)
constexpr uint32_t BUDGET = SLOT - 26;  // deflate bytes that fit a member with header + footer
constexpr uint32_t MAXD = 32768;
constexpr uint32_t LSEG = 256;                       // bytes parsed per lane
constexpr uint32_t NLANE = (PAYLOAD + LSEG - 1) / LSEG;  // 256 segments per member
constexpr uint32_t HB = 12, HN = 1u << HB;           // hash bits defining prev[]
constexpr uint32_t DEPTH = 4;                        // chain candidates per position
#ifndef SBH_DEFLATE_NICE
#define SBH_DEFLATE_NICE 32
#endif
#ifndef SBH_DEFLATE_LAZY
#define SBH_DEFLATE_LAZY 16
#endif
constexpr uint32_t NICE = SBH_DEFLATE_NICE;  // a match this long ends the chain walk
constexpr uint32_t LAZY = SBH_DEFLATE_LAZY;  // a match this long is taken without a look at p + 1
constexpr uint16_t NONE16 = 0xffff;
constexpr uint32_t TOK_M = 0x80000000u;  // token: literal = byte; match = TOK_M | (len - 3) << 16 | (dist - 1)
constexpr uint32_t HDR_CAP = 512;        // bytes of a dynamic block header, at most
static_assert(NLANE * LSEG >= PAYLOAD && NLANE <= 256, "one lane per segment");

struct Bits {
  uint8_t *p;
  uint64_t acc;
  uint32_t nb;
  SBH_HD void put(uint32_t v, uint32_t n) {  // n <= 32, LSB first (RFC 1951 3.1.1)
    acc |= (uint64_t)v << nb;
    nb += n;
    while (nb >= 8) {
      *p++ = (uint8_t)acc;
      acc >>= 8;
      nb -= 8;
    }
  }
  SBH_HD void flush() {
    if (nb) *p++ = (uint8_t)acc;
    acc = 0;
    nb = 0;
  }
};

SBH_HD inline uint32_t rev(uint32_t c, uint32_t n) {
  uint32_t r = 0;
  for (uint32_t i = 0; i < n; ++i) r |= ((c >> i) & 1u) << (n - 1 - i);
  return r;
}

SBH_HD inline uint32_t lg2(uint32_t x) { return 31u - (uint32_t)__builtin_clz(x); }

SBH_HD inline uint32_t hash3(const uint8_t *s) {
  const uint32_t v = (uint32_t)s[0] | (uint32_t)s[1] << 8 | (uint32_t)s[2] << 16;
  return (v * 2654435761u) >> (32 - HB);
}

// Length 3..258 -> symbol 257..285 and its extra bits (RFC 1951 3.2.5).
SBH_HD inline uint32_t len_sym(uint32_t len, uint32_t *xb, uint32_t *xv) {
  if (len == 258) {
    *xb = 0, *xv = 0;
    return 285;
  }
  const uint32_t m = len - 3;
  if (m < 8) {
    *xb = 0, *xv = 0;
    return 257 + m;
  }
  const uint32_t l = lg2(m), x = l - 2;
  *xb = x, *xv = m & ((1u << x) - 1);
  return 257 + 4 * (l - 1) + ((m >> x) & 3u);
}
// Distance 1..32768 -> symbol 0..29 and its extra bits.
SBH_HD inline uint32_t dist_sym(uint32_t dist, uint32_t *xb, uint32_t *xv) {
  const uint32_t d = dist - 1;
  if (d < 4) {
    *xb = 0, *xv = 0;
    return d;
  }
  const uint32_t l = lg2(d), x = l - 1;
  *xb = x, *xv = d & ((1u << x) - 1);
  return 2 * l + ((d >> x) & 1u);
}

// Bytes equal from q and p (q < p), at most lim; `ld` reads 8 bytes at any offset (up to 7
// past the last byte compared, which the callers pad).
template <typename Load>
SBH_HD inline uint32_t match_len(const Load &ld, uint32_t q, uint32_t p, uint32_t lim) {
  uint32_t l = 0;
  while (l + 8 <= lim) {
    const uint64_t x = ld(q + l) ^ ld(p + l);
    if (x) return l + ((uint32_t)__builtin_ctzll(x) >> 3);
    l += 8;
  }
  if (l < lim) {
    const uint64_t x = ld(q + l) ^ ld(p + l);
    const uint32_t e = x ? (uint32_t)__builtin_ctzll(x) >> 3 : 8u;
    l += e < lim - l ? e : lim - l;
  }
  return l;
}

// The best of DEPTH chain candidates at p (matches ending by hi): longest, nearest first.
template <typename Load, typename Prev>
SBH_HD inline void best_match(const Load &ld, const Prev &prev, uint32_t p, uint32_t hi, uint32_t *bl,
                              uint32_t *bd) {
  *bl = 0, *bd = 0;
  if (p + 3 > hi) return;
  const uint32_t lim = hi - p < 258u ? hi - p : 258u;
  uint32_t q = prev(p);
  for (uint32_t k = 0; k < DEPTH && q != NONE16 && p - q <= MAXD; ++k) {
    const uint32_t l = match_len(ld, q, p, lim);
    if (l > *bl) {
      *bl = l, *bd = p - q;
      if (l >= lim || l >= NICE) break;
    }
    q = prev(q);
  }
}

// The segment [lo, hi) of the member as tokens (lazy matching); emit(token) per token.
template <typename Load, typename Prev, typename Emit>
SBH_HD inline void parse_seg(const Load &ld, const Prev &prev, uint32_t lo, uint32_t hi, Emit &&emit) {
  uint32_t p = lo, l1 = 0, d1 = 0;
  bool have = false;  // l1 / d1 already hold best_match(p)
  while (p < hi) {
    if (!have) best_match(ld, prev, p, hi, &l1, &d1);
    have = false;
    if (l1 >= 3 && l1 < LAZY && p + 1 < hi) {
      uint32_t l2, d2;
      best_match(ld, prev, p + 1, hi, &l2, &d2);
      if (l2 > l1) {  // defer: a literal, then the longer match is reconsidered at p + 1
        emit((uint32_t)(uint8_t)ld(p));
        ++p;
        l1 = l2, d1 = d2, have = true;
        continue;
      }
    }
    if (l1 >= 3) {
      emit(TOK_M | (l1 - 3) << 16 | (d1 - 1));
      p += l1;
    } else {
      emit((uint32_t)(uint8_t)ld(p));
      ++p;
    }
  }
}

SBH_HD inline uint32_t tok_len(uint32_t t) { return ((t >> 16) & 0xff) + 3; }
SBH_HD inline uint32_t tok_dist(uint32_t t) { return (t & 0xffff) + 1; }

// Length-limited Huffman code lengths, in stages so that the device can run them from LDS
// (no per-thread arrays) and split the sort over threads:
//  huff_rank: position of symbol i among the nonzero symbols in (frequency, symbol) order;
//  huff_tree: from that order, a two-queue Huffman tree, then zlib's repair of lengths past
//  maxbits (gen_bitlen); longest codes go to the least frequent symbols.  One nonzero symbol
//  gets length 1.
struct HuffWork {          // n <= 286 symbols
  uint16_t sym[286];       // nonzero symbols, (frequency, symbol) order
  uint16_t par[2 * 286];
  uint32_t w[2 * 286];
  uint32_t bl[33];
};
SBH_HD inline uint32_t huff_rank(const uint32_t *freq, uint32_t n, uint32_t i) {
  const uint32_t f = freq[i];
  uint32_t r = 0;
  for (uint32_t j = 0; j < n; ++j) {
    const uint32_t g = freq[j];
    r += (g != 0 && (g < f || (g == f && j < i))) ? 1u : 0u;
  }
  return r;
}
SBH_HD inline void huff_sort(const uint32_t *freq, uint32_t n, HuffWork &W) {  // serial huff_rank
  for (uint32_t i = 0; i < n; ++i)
    if (freq[i]) W.sym[huff_rank(freq, n, i)] = (uint16_t)i;
}
SBH_HD inline void huff_tree(const uint32_t *freq, uint32_t n, uint32_t maxbits, uint8_t *len, HuffWork &W) {
  uint32_t m = 0;
  for (uint32_t i = 0; i < n; ++i) {
    len[i] = 0;
    m += freq[i] != 0;
  }
  if (m == 0) return;
  if (m == 1) {
    len[W.sym[0]] = 1;
    return;
  }
  uint32_t *w = W.w;
  uint16_t *par = W.par;
  for (uint32_t i = 0; i < m; ++i) w[i] = freq[W.sym[i]];
  uint32_t a = 0, b = m, nxt = m;
  while (nxt < 2 * m - 1) {
    uint32_t x, y;
    x = (a < m && (b >= nxt || w[a] <= w[b])) ? a++ : b++;
    y = (a < m && (b >= nxt || w[a] <= w[b])) ? a++ : b++;
    w[nxt] = w[x] + w[y];
    par[x] = (uint16_t)nxt;
    par[y] = (uint16_t)nxt;
    ++nxt;
  }
  // depths, root first (parents have larger indices); reuse w[] for them
  uint32_t *bl = W.bl;
  for (uint32_t l = 0; l < 33; ++l) bl[l] = 0;
  w[nxt - 1] = 0;
  for (int32_t i = (int32_t)nxt - 2; i >= 0; --i) {
    const uint32_t d = w[par[i]] + 1;
    w[i] = d;
    if ((uint32_t)i < m) bl[d < 32 ? d : 32]++;
  }
  for (uint32_t l = maxbits + 1; l < 33; ++l) {
    bl[maxbits] += bl[l];
    bl[l] = 0;
  }
  for (;;) {  // Kraft repair: move a leaf down from the longest level below maxbits
    uint64_t kraft = 0;
    for (uint32_t l = 1; l <= maxbits; ++l) kraft += (uint64_t)bl[l] << (maxbits - l);
    if (kraft <= (1ull << maxbits)) break;
    uint32_t l = maxbits - 1;
    while (bl[l] == 0) --l;
    bl[l]--;
    bl[l + 1] += 2;
    bl[maxbits]--;
  }
  uint32_t idx = 0;
  for (uint32_t l = maxbits; l >= 1 && idx < m; --l)
    for (uint32_t k = 0; k < bl[l] && idx < m; ++k) len[W.sym[idx++]] = (uint8_t)l;
}

// Canonical codes (bit-reversed for the LSB-first writer) packed as code | len << 16.
// cnt, next: 16 u32 of scratch each.
SBH_HD inline void canon(const uint8_t *len, uint32_t n, uint32_t *code, uint32_t *cnt, uint32_t *next) {
  for (uint32_t l = 0; l < 16; ++l) cnt[l] = 0;
  for (uint32_t i = 0; i < n; ++i) cnt[len[i]]++;
  cnt[0] = 0;
  uint32_t c = 0;
  next[0] = 0;
  for (uint32_t l = 1; l < 16; ++l) {
    c = (c + cnt[l - 1]) << 1;
    next[l] = c;
  }
  for (uint32_t i = 0; i < n; ++i) code[i] = len[i] ? rev(next[len[i]]++, len[i]) | (uint32_t)len[i] << 16 : 0u;
}

constexpr uint8_t CLORD[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// A member's codes: lit/len and distance (code | len << 16).
struct Codes {
  uint32_t lit[286], dist[30];
};
// Header stage scratch: the lit/len and distance code lengths (inputs) and the
// run-length-coded lengths with their code-length code.
struct HdrWork {
  uint8_t ll[286], dl[30], cl[19];
  uint16_t rle[286 + 30];
  uint32_t fc[19], cc[19], cnt[16], next[16];
};

// From ll / dl (the member's code lengths): codes into cd and the dynamic block header
// bits (BFINAL set) into hdr (HDR_CAP bytes, zeroed), returning the header's bit count.
// hw: scratch for the code-length code's tree.
SBH_HD inline uint32_t build_header(HdrWork &H, HuffWork &hw, Codes &cd, uint8_t *hdr) {
  uint8_t *ll = H.ll, *dl = H.dl, *cl = H.cl;
  bool anyd = false;
  for (uint32_t i = 0; i < 30; ++i) anyd = anyd || dl[i] != 0;
  if (!anyd) dl[0] = 1;  // no matches: one unused distance code (RFC 1951 3.2.7)
  uint32_t nlit = 286, ndist = 30;
  while (nlit > 257 && !ll[nlit - 1]) --nlit;
  while (ndist > 1 && !dl[ndist - 1]) --ndist;
  // run-length coded lengths (symbol | extra << 8) of ll[0, nlit) ++ dl[0, ndist)
  uint16_t *rle = H.rle;
  uint32_t nr = 0;
  const uint32_t tot = nlit + ndist;
  for (uint32_t i = 0; i < tot;) {
    const uint32_t v = i < nlit ? ll[i] : dl[i - nlit];
    uint32_t j = i + 1;
    while (j < tot && (j < nlit ? ll[j] : dl[j - nlit]) == v) ++j;
    uint32_t run = j - i;
    if (v == 0) {
      while (run >= 11) {
        const uint32_t r = run < 138 ? run : 138;
        rle[nr++] = (uint16_t)(18 | (r - 11) << 8);
        run -= r;
      }
      if (run >= 3) {
        rle[nr++] = (uint16_t)(17 | (run - 3) << 8);
        run = 0;
      }
      while (run) rle[nr++] = 0, --run;
    } else {
      rle[nr++] = (uint16_t)v;
      --run;
      while (run >= 3) {
        const uint32_t r = run < 6 ? run : 6;
        rle[nr++] = (uint16_t)(16 | (r - 3) << 8);
        run -= r;
      }
      while (run) rle[nr++] = (uint16_t)v, --run;
    }
    i = j;
  }
  uint32_t *fc = H.fc;
  for (uint32_t i = 0; i < 19; ++i) fc[i] = 0;
  for (uint32_t i = 0; i < nr; ++i) fc[rle[i] & 0xff]++;
  huff_sort(fc, 19, hw);
  huff_tree(fc, 19, 7, cl, hw);
  uint32_t ncl = 19;
  while (ncl > 4 && !cl[CLORD[ncl - 1]]) --ncl;
  canon(cl, 19, H.cc, H.cnt, H.next);
  canon(ll, 286, cd.lit, H.cnt, H.next);
  canon(dl, 30, cd.dist, H.cnt, H.next);
  Bits b{hdr, 0, 0};
  b.put(1, 1);  // BFINAL
  b.put(2, 2);  // BTYPE = 10, dynamic
  b.put(nlit - 257, 5);
  b.put(ndist - 1, 5);
  b.put(ncl - 4, 4);
  for (uint32_t i = 0; i < ncl; ++i) b.put(cl[CLORD[i]], 3);
  const uint32_t *cc = H.cc;
  for (uint32_t i = 0; i < nr; ++i) {
    const uint32_t s = rle[i] & 0xff, x = rle[i] >> 8;
    b.put(cc[s] & 0xffff, cc[s] >> 16);
    if (s == 16) b.put(x, 2);
    if (s == 17) b.put(x, 3);
    if (s == 18) b.put(x, 7);
  }
  const uint32_t nbits = (uint32_t)(b.p - hdr) * 8 + b.nb;
  b.flush();
  return nbits;
}

// The whole code build, serially (host): fl[256] must count the end-of-block code.
SBH_HD inline uint32_t build_codes(const uint32_t *fl, const uint32_t *fd, Codes &cd, uint8_t *hdr, HuffWork &wl,
                                   HuffWork &wd, HdrWork &H) {
  huff_sort(fl, 286, wl);
  huff_tree(fl, 286, 15, H.ll, wl);
  huff_sort(fd, 30, wd);
  huff_tree(fd, 30, 15, H.dl, wd);
  return build_header(H, wl, cd, hdr);
}

// Histogram entries of a token.
SBH_HD inline void tok_syms(uint32_t t, uint32_t *ls, int32_t *ds) {
  if (!(t & TOK_M)) {
    *ls = t, *ds = -1;
    return;
  }
  uint32_t xb, xv;
  *ls = len_sym(tok_len(t), &xb, &xv);
  *ds = (int32_t)dist_sym(tok_dist(t), &xb, &xv);
}

// A token's bits: up to 48 (15 + 5 + 15 + 13) as (value, count).
SBH_HD inline uint32_t tok_bits(uint32_t t, const Codes &cd, uint64_t *v) {
  if (!(t & TOK_M)) {
    *v = cd.lit[t] & 0xffff;
    return cd.lit[t] >> 16;
  }
  uint32_t lx, lv, dx, dv;
  const uint32_t ls = len_sym(tok_len(t), &lx, &lv), ds = dist_sym(tok_dist(t), &dx, &dv);
  const uint32_t lc = cd.lit[ls], dc = cd.dist[ds];
  uint32_t n = lc >> 16;
  uint64_t x = lc & 0xffff;
  x |= (uint64_t)lv << n;
  n += lx;
  x |= (uint64_t)(dc & 0xffff) << n;
  n += dc >> 16;
  x |= (uint64_t)dv << n;
  n += dx;
  *v = x;
  return n;
}

SBH_HD inline void put_le32(uint8_t *o, uint32_t v) {
  o[0] = (uint8_t)v;
  o[1] = (uint8_t)(v >> 8);
  o[2] = (uint8_t)(v >> 16);
  o[3] = (uint8_t)(v >> 24);
}

SBH_HD inline void put_header(uint8_t *out, uint32_t total) {
  const uint8_t hdr[16] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0};
  for (int i = 0; i < 16; ++i) out[i] = hdr[i];
  out[16] = (uint8_t)(total - 1);
  out[17] = (uint8_t)((total - 1) >> 8);
}

SBH_HD inline uint32_t stored_dsize(uint32_t n) { return 5 + n; }
SBH_HD inline void put_stored_head(uint8_t *d0, uint32_t n) {  // BFINAL=1 BTYPE=00, LEN, NLEN
  d0[0] = 1;
  d0[1] = (uint8_t)n;
  d0[2] = (uint8_t)(n >> 8);
  d0[3] = (uint8_t)~n;
  d0[4] = (uint8_t)(~n >> 8);
}

SBH_HD inline uint32_t crc32_bytes(const uint8_t *s, uint32_t n, const uint32_t *crctab) {
  uint32_t crc = 0xffffffffu;
  for (uint32_t i = 0; i < n; ++i) crc = crctab[(crc ^ s[i]) & 0xff] ^ (crc >> 8);
  return crc ^ 0xffffffffu;
}

// The empty member htsjdk appends at close (BlockCompressedStreamConstants.EMPTY_GZIP_BLOCK).
constexpr uint32_t EOF_SIZE = 28;
SBH_HD inline void put_eof(uint8_t *o) {
  const uint8_t e[28] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0, 27, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 28; ++i) o[i] = e[i];
}

}  // namespace sbh_deflate
