// zdeflate_core.h -- one BGZF member exactly as htsjdk writes it: java.util.zip.Deflater at
// level 5, nowrap (raw deflate, windowBits -15, memLevel 8, default strategy), i.e. zlib 1.2.11's
// deflate_slow + trees.c, bit for bit (levels 4..9 share that path; 6 is samtools' default).
//
// Reference call site: HTSJDKRewrite (cli/src/main/scala/org/hammerlab/bam/rewrite/
// HTSJDKRewrite.scala:62-67) -> SAMFileWriterFactory.makeBAMWriter -> htsjdk
// BlockCompressedOutputStream.deflateBlock: deflater.reset(); setInput(65498 bytes); finish();
// deflate(compressedBuffer, 0, 65518) -- if that does not finish (the output reached 65518
// bytes) the block is re-deflated at level 0 (one final stored block).  htsjdk and zlib are
// third-party (not in /root/reference); what follows restates zlib 1.2.11's published
// algorithm (deflate.c: deflate_slow, longest_match, fill_window; trees.c: _tr_tally,
// _tr_flush_block, build_tree, gen_bitlen, gen_codes, build_bl_tree, scan_tree, send_tree,
// compress_block, _tr_stored_block), pinned by tests/test_zdeflate_cpu.py against the
// container's zlib 1.2.11 (zlib.compressobj(5, DEFLATED, -15, 8)) and against every member of
// the reference's own BAMs (2.bam, 1.bam, 5k.bam, slice/2.100-1000.bam).
//
// Restated so that a GPU can run it in parallel stages and still give zlib's bytes:
//  (1) hash chains.  Every position p with 3 bytes left is inserted in order, so prev[p] is
//      simply the latest q < p with the same 15-bit hash ((b0 << 10) ^ (b1 << 5) ^ b2), 0 = NIL
//      (position 0 is never a match candidate, as in zlib).  A 65498-byte member fits the
//      2 x 32 KiB window at once; the one window slide (when strstart reaches 65274) only NILs
//      entries <= 32768, which longest_match's `limit` already excludes -- except the head at
//      exactly 32768 seen from 65274, handled in z_info.
//  (2) match info.  longest_match(p) depends on the parse only through prev_length (its
//      starting best_len, and chain 32 vs 8 when prev_length >= good 8).  Its result is
//      max(prev_length, M) where M is the longest of the first `chain` candidates up to the
//      first one reaching nice (first such candidate on ties), so z_info computes (M, start)
//      for both chain lengths at every position independently (one GPU lane per position).
//  (3) the lazy parse (deflate_slow) is a short serial state machine over those records;
//      blocks close when 16383 symbols are tallied (lit_bufsize - 1).
//  (4) per block the exact zlib tree construction (heap order, depth tie-break, overflow
//      repair), the stored / static / dynamic choice, and the bits.
// SBH_HD is __host__ __device__ under hipcc, empty otherwise.
//
// This file is an altered restatement of zlib 1.2.11's deflate.c / trees.c (marked as such
// above and below: the parse and tree construction are re-structured into parallel stages), so
// zlib's licence notice travels with it:
//
//   zlib 1.2.11, Copyright (C) 1995-2017 Jean-loup Gailly and Mark Adler
//
//   This software is provided 'as-is', without any express or implied warranty.  In no event
//   will the authors be held liable for any damages arising from the use of this software.
//
//   Permission is granted to anyone to use this software for any purpose, including commercial
//   applications, and to alter it and redistribute it freely, subject to the following
//   restrictions:
//   1. The origin of this software must not be misrepresented; you must not claim that you
//      wrote the original software. If you use this software in a product, an acknowledgment in
//      the product documentation would be appreciated but is not required.
//   2. Altered source versions must be plainly marked as such, and must not be misrepresented
//      as being the original software.
//   3. This notice may not be removed or altered from any source distribution.
//
//   Jean-loup Gailly jloup@gzip.org, Mark Adler madler@alumni.caltech.edu
#pragma once
#include <stdint.h>

#ifndef SBH_HD
#define SBH_HD
#endif

namespace sbh_zlib {

constexpr uint32_t WSIZE = 32768;
constexpr uint32_t MIN_MATCH = 3, MAX_MATCH = 258;
constexpr uint32_t MIN_LOOKAHEAD = MAX_MATCH + MIN_MATCH + 1;  // 262
constexpr uint32_t MAX_DIST = WSIZE - MIN_LOOKAHEAD;            // 32506
constexpr uint32_t HASH_MASK = (1u << 15) - 1;                  // hash_bits = memLevel + 7
constexpr uint32_t SLIDE_AT = WSIZE + MAX_DIST;                 // fill_window slides here
// deflate.c configuration_table for the deflate_slow levels 4..9: good_length, max_lazy,
// nice_length, max_chain (level 5 is htsjdk's; level 6 is zlib's / samtools' default)
struct ZCfg {
  uint32_t good, lazy, nice, chain;
};
SBH_HD inline ZCfg z_config(int level) {
  switch (level) {
    case 4: return ZCfg{4, 4, 16, 16};
    case 5: return ZCfg{8, 16, 32, 32};
    case 6: return ZCfg{8, 16, 128, 128};
    case 7: return ZCfg{8, 32, 128, 256};
    case 8: return ZCfg{32, 128, 258, 1024};
    default: return ZCfg{32, 258, 258, 4096};
  }
}
constexpr uint32_t TOO_FAR = 4096;
constexpr uint32_t LIT_BUFSIZE = 1u << (8 + 6);  // memLevel 8
constexpr uint32_t MAX_SYMS = LIT_BUFSIZE - 1;   // a block closes at this many symbols
constexpr uint32_t OUT_CAP = 65536 - 18;         // htsjdk's compressedBuffer
constexpr uint32_t MAX_MEMBER = 65536;           // inputs this definition supports
constexpr uint32_t MAX_BLOCKS = 8;               // ceil(65536 / 16383) + the final one, rounded up
constexpr uint32_t L_CODES = 286, D_CODES = 30, BL_CODES = 19, HEAP_SIZE = 2 * L_CODES + 1;
constexpr uint32_t TOK_M = 0x80000000u;  // token: literal = byte; match = TOK_M | (len - 3) << 16 | dist

SBH_HD inline uint32_t zhash(uint32_t b0, uint32_t b1, uint32_t b2) {
  return ((b0 << 10) ^ (b1 << 5) ^ b2) & HASH_MASK;
}

// ---- (2) match records --------------------------------------------------------------------
// One u64 per position p: M | S << 9 | M' << 25 | S' << 34 | byte(p) << 50, where (M, S) is
// longest_match's (length, match_start) over the full chain and (M', S') over the chain >> 2
// it walks once prev_length >= good (M = 0: no candidate improves on MIN_MATCH - 1, or
// longest_match is not called at all).  Lengths are capped at the lookahead N - p, which
// changes none of zlib's decisions (a candidate reaching the lookahead also reaches nice, and
// nice <= lookahead).  `prv(i)` returns prev[i]; `cmp(a, b, lim)` how many bytes from a and b
// are equal, at most lim.  z_info leaves the byte field 0 (z_rec_with_byte adds it).
SBH_HD inline uint32_t z_rec_len(uint64_t r, bool quarter) { return (uint32_t)(r >> (quarter ? 25 : 0)) & 0x1ffu; }
SBH_HD inline uint32_t z_rec_start(uint64_t r, bool quarter) { return (uint32_t)(r >> (quarter ? 34 : 9)) & 0xffffu; }
SBH_HD inline uint32_t z_rec_byte(uint64_t r) { return (uint32_t)(r >> 50) & 0xffu; }
SBH_HD inline uint64_t z_rec_with_byte(uint64_t r, uint32_t byte) { return r | (uint64_t)(byte & 0xffu) << 50; }
template <typename Prv, typename Cmp>
SBH_HD inline uint64_t z_info(const Prv &prv, const Cmp &cmp, uint32_t p, uint32_t N, const ZCfg &cf) {
  if (p + MIN_MATCH > N) return 0;  // lookahead < MIN_MATCH: no INSERT_STRING, hash_head = NIL
  uint32_t cur = prv(p);            // hash_head
  if (cur == 0 || p - cur > MAX_DIST) return 0;
  if (p == SLIDE_AT && cur == WSIZE && N < MAX_MEMBER) return 0;  // NIL after the slide
  const uint32_t limit = p > MAX_DIST ? p - MAX_DIST : 0;
  const uint32_t look = N - p;
  const uint32_t nice = look < cf.nice ? look : cf.nice;
  const uint32_t cap = look < MAX_MATCH ? look : MAX_MATCH;
  const uint32_t c2 = cf.chain >> 2;
  uint32_t best = MIN_MATCH - 1, start = 0, best2 = 0, start2 = 0;
  for (uint32_t i = 0; i < cf.chain; ++i) {
    const uint32_t len = cmp(cur, p, cap);
    if (len > best) {
      best = len, start = cur;
      if (len >= nice) {
        if (i < c2) best2 = best, start2 = start;
        break;
      }
    }
    if (i + 1 == c2) best2 = best, start2 = start;
    const uint32_t nx = prv(cur);
    if (nx <= limit) {
      if (i + 1 < c2) best2 = best, start2 = start;
      break;
    }
    cur = nx;
  }
  if (best < MIN_MATCH) best = 0;
  if (best2 < MIN_MATCH) best2 = 0;
  return (uint64_t)best | (uint64_t)start << 9 | (uint64_t)best2 << 25 | (uint64_t)start2 << 34;
}

// ---- (3) the lazy parse (deflate_slow) -----------------------------------------------------
struct ZBlock {
  uint32_t tok0, tok1;    // tokens [tok0, tok1)
  uint32_t byte0, byte1;  // uncompressed bytes [block_start, strstart) at the flush
  uint32_t nobuf;         // block_start < 0 after the window slide: a stored block is impossible
};

// Runs deflate_slow over the member (all N bytes present, flush = Z_FINISH) at level cf.  info(p)
// gives position p's record (z_info with its byte), read once per loop iteration in increasing
// p; tok(k, t) receives token k.  Fills blocks[] (the last one is the final block) and returns
// the number of blocks; *ntok = tokens.
template <typename Info, typename Tok>
SBH_HD inline uint32_t z_parse(uint32_t N, const ZCfg &cf, const Info &info, const Tok &tok, ZBlock *blocks,
                               uint32_t *ntok) {
  uint32_t strstart = 0, match_length = MIN_MATCH - 1, match_start = 0, prev_length, prev_match;
  bool match_available = false, slid = false, nobuf = false;
  uint32_t block_start = 0, last_lit = 0, nt = 0, nb = 0, tb = 0, prev_byte = 0;
  auto flush = [&](uint32_t end) {
    blocks[nb++] = ZBlock{tb, nt, block_start, end, nobuf ? 1u : 0u};
    tb = nt;
    block_start = end;
    last_lit = 0;
    nobuf = false;
  };
  for (;;) {
    const uint32_t look = N - strstart;
    if (look < MIN_LOOKAHEAD) {  // fill_window: the one slide of the 64 KiB window
      if (!slid && strstart >= SLIDE_AT) {
        slid = true;
        if (block_start < WSIZE) nobuf = true;
      }
      if (look == 0) break;
    }
    const uint64_t r = info(strstart);  // (its byte is window[strstart])
    prev_length = match_length, prev_match = match_start;
    match_length = MIN_MATCH - 1;
    if (prev_length < cf.lazy) {
      // longest_match (the chain, or a quarter of it once prev_length >= good) starts at best_len =
      // prev_length: only a longer candidate changes match_start.  When none is longer,
      // zlib's match_length is min(prev_length, lookahead) <= prev_length; keeping
      // MIN_MATCH - 1 instead takes the same branch below (the previous match is emitted,
      // or with prev_length = 2 a literal), so it is not spelled out.
      const uint32_t M = z_rec_len(r, prev_length >= cf.good), S = z_rec_start(r, prev_length >= cf.good);
      if (M > prev_length) {
        match_length = M;
        match_start = S;
        if (match_length == MIN_MATCH && strstart - match_start > TOO_FAR) match_length = MIN_MATCH - 1;
      }
    }
    if (prev_length >= MIN_MATCH && match_length <= prev_length) {
      tok(nt++, TOK_M | (prev_length - MIN_MATCH) << 16 | (strstart - 1 - prev_match));
      const bool bflush = ++last_lit == MAX_SYMS;
      strstart += prev_length - 1;
      match_available = false;
      match_length = MIN_MATCH - 1;
      if (bflush) flush(strstart);
    } else if (match_available) {
      tok(nt++, prev_byte);  // window[strstart - 1]: the previous iteration's position
      if (++last_lit == MAX_SYMS) flush(strstart);
      ++strstart;
    } else {
      match_available = true;
      ++strstart;
    }
    prev_byte = z_rec_byte(r);
  }
  if (match_available) {
    tok(nt++, prev_byte);
    ++last_lit;
  }
  flush(strstart);
  *ntok = nt;
  return nb;
}

// ---- (4) trees (trees.c) -------------------------------------------------------------------
struct ct_data {
  uint16_t fc;  // freq / code
  uint16_t dl;  // dad / len
};

constexpr int32_t EXTRA_LBITS[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
constexpr int32_t EXTRA_DBITS[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
constexpr int32_t EXTRA_BLBITS[19] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 3, 7};
constexpr uint8_t BL_ORDER[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
constexpr uint16_t BASE_LENGTH[29] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 14, 16, 20, 24, 28, 32, 40, 48, 56, 64, 80, 96, 112, 128, 160, 192, 224, 0};
constexpr uint16_t BASE_DIST[30] = {0, 1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64, 96, 128, 192, 256, 384, 512, 768, 1024, 1536, 2048, 3072, 4096, 6144, 8192, 12288, 16384, 24576};

// _length_code[lc] for lc = match length - 3 in [0, 255]
SBH_HD inline uint32_t length_code(uint32_t lc) {
  if (lc == 255) return 28;
  uint32_t c = 0;
  while (c < 27 && BASE_LENGTH[c + 1] <= lc) ++c;
  return c;
}
// d_code(dist - 1)
SBH_HD inline uint32_t dist_code(uint32_t d) {
  uint32_t c = 0;
  while (c < 29 && BASE_DIST[c + 1] <= d) ++c;
  return c;
}
SBH_HD inline uint32_t bi_reverse(uint32_t code, uint32_t len) {
  uint32_t res = 0;
  do {
    res |= code & 1;
    code >>= 1, res <<= 1;
  } while (--len > 0);
  return res >> 1;
}
SBH_HD inline uint32_t static_llen(uint32_t n) { return n < 144 ? 8 : n < 256 ? 9 : n < 280 ? 7 : 8; }
// static_ltree[n].Code (bit-reversed, as trees.c's tr_static_init builds it)
SBH_HD inline uint32_t static_lcode(uint32_t n) {
  if (n < 144) return bi_reverse(0x30 + n, 8);
  if (n < 256) return bi_reverse(0x190 + (n - 144), 9);
  if (n < 280) return bi_reverse(n - 256, 7);
  return bi_reverse(0xc0 + (n - 280), 8);
}

struct ZTreeState {
  ct_data dyn_ltree[HEAP_SIZE];
  ct_data dyn_dtree[2 * D_CODES + 1];
  ct_data bl_tree[2 * BL_CODES + 1];
  int32_t heap[HEAP_SIZE];
  int32_t heap_len, heap_max;
  uint8_t depth[HEAP_SIZE];
  uint16_t bl_count[16];
  int64_t opt_len, static_len;
  int32_t l_max_code, d_max_code, bl_max_code;
};

SBH_HD inline bool z_smaller(const ct_data *tree, int32_t n, int32_t m, const uint8_t *depth) {
  return tree[n].fc < tree[m].fc || (tree[n].fc == tree[m].fc && depth[n] <= depth[m]);
}
SBH_HD inline void z_pqdownheap(ZTreeState &s, const ct_data *tree, int32_t k) {
  const int32_t v = s.heap[k];
  int32_t j = k << 1;
  while (j <= s.heap_len) {
    if (j < s.heap_len && z_smaller(tree, s.heap[j + 1], s.heap[j], s.depth)) j++;
    if (z_smaller(tree, v, s.heap[j], s.depth)) break;
    s.heap[k] = s.heap[j];
    k = j;
    j <<= 1;
  }
  s.heap[k] = v;
}

// kind: 0 literal/length, 1 distance, 2 bit lengths
SBH_HD inline void z_gen_bitlen(ZTreeState &s, ct_data *tree, int32_t max_code, int32_t kind) {
  const int32_t max_length = kind == 2 ? 7 : 15;
  const int32_t base = kind == 0 ? 257 : 0;
  int32_t overflow = 0;
  for (int32_t bits = 0; bits <= 15; bits++) s.bl_count[bits] = 0;
  tree[s.heap[s.heap_max]].dl = 0;  // root
  int32_t h;
  for (h = s.heap_max + 1; h < (int32_t)HEAP_SIZE; h++) {
    const int32_t n = s.heap[h];
    int32_t bits = tree[tree[n].dl].dl + 1;
    if (bits > max_length) bits = max_length, overflow++;
    tree[n].dl = (uint16_t)bits;
    if (n > max_code) continue;  // not a leaf
    s.bl_count[bits]++;
    int32_t xbits = 0;
    if (n >= base) xbits = kind == 0 ? EXTRA_LBITS[n - base] : kind == 1 ? EXTRA_DBITS[n - base] : EXTRA_BLBITS[n - base];
    const uint32_t f = tree[n].fc;
    s.opt_len += (int64_t)f * (bits + xbits);
    if (kind == 0) s.static_len += (int64_t)f * ((int32_t)static_llen((uint32_t)n) + xbits);
    else if (kind == 1) s.static_len += (int64_t)f * (5 + xbits);
  }
  if (overflow == 0) return;
  do {
    int32_t bits = max_length - 1;
    while (s.bl_count[bits] == 0) bits--;
    s.bl_count[bits]--;
    s.bl_count[bits + 1] += 2;
    s.bl_count[max_length]--;
    overflow -= 2;
  } while (overflow > 0);
  for (int32_t bits = max_length; bits != 0; bits--) {
    int32_t n = s.bl_count[bits];
    while (n != 0) {
      const int32_t m = s.heap[--h];
      if (m > max_code) continue;
      if ((int32_t)tree[m].dl != bits) {
        s.opt_len += ((int64_t)bits - tree[m].dl) * tree[m].fc;
        tree[m].dl = (uint16_t)bits;
      }
      n--;
    }
  }
}

SBH_HD inline void z_gen_codes(ct_data *tree, int32_t max_code, const uint16_t *bl_count) {
  uint16_t next_code[16];
  uint32_t code = 0;
  for (int32_t bits = 1; bits <= 15; bits++) {
    code = (code + bl_count[bits - 1]) << 1;
    next_code[bits] = (uint16_t)code;
  }
  for (int32_t n = 0; n <= max_code; n++) {
    const int32_t len = tree[n].dl;
    if (len == 0) continue;
    tree[n].fc = (uint16_t)bi_reverse(next_code[len]++, (uint32_t)len);
  }
}

SBH_HD inline int32_t z_build_tree(ZTreeState &s, ct_data *tree, int32_t elems, int32_t kind) {
  int32_t max_code = -1, node;
  s.heap_len = 0, s.heap_max = HEAP_SIZE;
  for (int32_t n = 0; n < elems; n++) {
    if (tree[n].fc != 0) {
      s.heap[++(s.heap_len)] = max_code = n;
      s.depth[n] = 0;
    } else {
      tree[n].dl = 0;
    }
  }
  while (s.heap_len < 2) {
    node = s.heap[++(s.heap_len)] = (max_code < 2 ? ++max_code : 0);
    tree[node].fc = 1;
    s.depth[node] = 0;
    s.opt_len--;
    if (kind == 0) s.static_len -= static_llen((uint32_t)node);
    else if (kind == 1) s.static_len -= 5;
  }
  for (int32_t n = s.heap_len / 2; n >= 1; n--) z_pqdownheap(s, tree, n);
  node = elems;
  do {
    const int32_t n = s.heap[1];  // pqremove
    s.heap[1] = s.heap[s.heap_len--];
    z_pqdownheap(s, tree, 1);
    const int32_t m = s.heap[1];
    s.heap[--(s.heap_max)] = n;
    s.heap[--(s.heap_max)] = m;
    tree[node].fc = (uint16_t)(tree[n].fc + tree[m].fc);
    s.depth[node] = (uint8_t)((s.depth[n] >= s.depth[m] ? s.depth[n] : s.depth[m]) + 1);
    tree[n].dl = tree[m].dl = (uint16_t)node;
    s.heap[1] = node++;
    z_pqdownheap(s, tree, 1);
  } while (s.heap_len >= 2);
  s.heap[--(s.heap_max)] = s.heap[1];
  z_gen_bitlen(s, tree, max_code, kind);
  z_gen_codes(tree, max_code, s.bl_count);
  return max_code;
}

SBH_HD inline void z_scan_tree(ZTreeState &s, ct_data *tree, int32_t max_code) {
  int32_t prevlen = -1, curlen, nextlen = tree[0].dl, count = 0, max_count = 7, min_count = 4;
  if (nextlen == 0) max_count = 138, min_count = 3;
  tree[max_code + 1].dl = (uint16_t)0xffff;  // guard
  for (int32_t n = 0; n <= max_code; n++) {
    curlen = nextlen;
    nextlen = tree[n + 1].dl;
    if (++count < max_count && curlen == nextlen) {
      continue;
    } else if (count < min_count) {
      s.bl_tree[curlen].fc = (uint16_t)(s.bl_tree[curlen].fc + count);
    } else if (curlen != 0) {
      if (curlen != prevlen) s.bl_tree[curlen].fc++;
      s.bl_tree[16].fc++;
    } else if (count <= 10) {
      s.bl_tree[17].fc++;
    } else {
      s.bl_tree[18].fc++;
    }
    count = 0;
    prevlen = curlen;
    if (nextlen == 0) max_count = 138, min_count = 3;
    else if (curlen == nextlen) max_count = 6, min_count = 3;
    else max_count = 7, min_count = 4;
  }
}

// Block decision of _tr_flush_block.
enum : uint32_t { ZB_STORED = 0, ZB_STATIC = 1, ZB_DYN = 2 };

// The trees of one block (_tr_flush_block's build_tree x 2, build_bl_tree) and its
// stored / static / dynamic choice, from the block's symbol counts already in
// dyn_ltree[].fc / dyn_dtree[].fc (END_BLOCK counted).  Returns ZB_*; max_blindex in *mbl.
SBH_HD inline uint32_t z_block_decide(ZTreeState &s, const ZBlock &b, int32_t *mbl) {
  for (uint32_t n = 0; n < BL_CODES; n++) s.bl_tree[n].fc = 0;
  s.opt_len = s.static_len = 0;
  s.l_max_code = z_build_tree(s, s.dyn_ltree, L_CODES, 0);
  s.d_max_code = z_build_tree(s, s.dyn_dtree, D_CODES, 1);
  z_scan_tree(s, s.dyn_ltree, s.l_max_code);  // build_bl_tree
  z_scan_tree(s, s.dyn_dtree, s.d_max_code);
  s.bl_max_code = z_build_tree(s, s.bl_tree, BL_CODES, 2);
  int32_t max_blindex;
  for (max_blindex = BL_CODES - 1; max_blindex >= 3; max_blindex--)
    if (s.bl_tree[BL_ORDER[max_blindex]].dl != 0) break;
  s.opt_len += 3 * ((int64_t)max_blindex + 1) + 5 + 5 + 4;
  *mbl = max_blindex;
  int64_t opt_lenb = (s.opt_len + 3 + 7) >> 3;
  const int64_t static_lenb = (s.static_len + 3 + 7) >> 3;
  if (static_lenb <= opt_lenb) opt_lenb = static_lenb;
  const int64_t stored_len = (int64_t)b.byte1 - b.byte0;
  if (stored_len + 4 <= opt_lenb && !b.nobuf) return ZB_STORED;
  if (static_lenb == opt_lenb) return ZB_STATIC;
  return ZB_DYN;
}

// A token's lit/len and distance symbols (the tally's counts).
SBH_HD inline void z_tok_syms(uint32_t t, uint32_t *ls, int32_t *ds) {
  if (!(t & TOK_M)) {
    *ls = t & 0xff, *ds = -1;
    return;
  }
  *ls = length_code((t >> 16) & 0xff) + 257;
  *ds = (int32_t)dist_code((t & 0xffff) - 1);
}

// Serially: the block's histogram (init_block + _tr_tally) then z_block_decide.
template <typename TokAt>
SBH_HD inline uint32_t z_block_trees(ZTreeState &s, const TokAt &tokat, const ZBlock &b, int32_t *mbl) {
  for (uint32_t n = 0; n < L_CODES; n++) s.dyn_ltree[n].fc = 0;  // init_block
  for (uint32_t n = 0; n < D_CODES; n++) s.dyn_dtree[n].fc = 0;
  s.dyn_ltree[256].fc = 1;
  for (uint32_t k = b.tok0; k < b.tok1; ++k) {
    uint32_t ls;
    int32_t ds;
    z_tok_syms(tokat(k), &ls, &ds);
    s.dyn_ltree[ls].fc++;
    if (ds >= 0) s.dyn_dtree[ds].fc++;
  }
  return z_block_decide(s, b, mbl);
}

// The block's codes as code | len << 16 tables (static or the dynamic trees).
SBH_HD inline void z_code_tables(const ZTreeState &s, uint32_t type, uint32_t *lit, uint32_t *dist) {
  for (uint32_t n = 0; n < L_CODES; ++n)
    lit[n] = type == ZB_STATIC ? static_lcode(n) | static_llen(n) << 16
                               : (uint32_t)s.dyn_ltree[n].fc | (uint32_t)s.dyn_ltree[n].dl << 16;
  for (uint32_t n = 0; n < D_CODES; ++n)
    dist[n] = type == ZB_STATIC ? bi_reverse(n, 5) | 5u << 16
                                : (uint32_t)s.dyn_dtree[n].fc | (uint32_t)s.dyn_dtree[n].dl << 16;
}

// A token's bits from code | len << 16 tables: up to 15 + 5 + 15 + 13 = 48 bits.
SBH_HD inline uint32_t z_tok_bits_tab(uint32_t t, const uint32_t *lit, const uint32_t *dist, uint64_t *v) {
  if (!(t & TOK_M)) {
    const uint32_t c = lit[t & 0xff];
    *v = c & 0xffff;
    return c >> 16;
  }
  const uint32_t lc = (t >> 16) & 0xff, d = (t & 0xffff) - 1;
  const uint32_t code = length_code(lc), dc = dist_code(d);
  const uint32_t l = lit[code + 257], dd = dist[dc];
  uint64_t x = l & 0xffff;
  uint32_t n = l >> 16;
  const uint32_t el = (uint32_t)EXTRA_LBITS[code];
  if (el) {  // (length 258 is code 28 with base 0 and no extra bits)
    x |= (uint64_t)(lc - BASE_LENGTH[code]) << n;
    n += el;
  }
  x |= (uint64_t)(dd & 0xffff) << n;
  n += dd >> 16;
  x |= (uint64_t)(d - BASE_DIST[dc]) << n;
  n += (uint32_t)EXTRA_DBITS[dc];
  *v = x;
  return n;
}

// LSB-first bit sink (send_bits / bi_windup).
struct ZBits {
  uint8_t *p;
  uint32_t cap, n;  // bytes available, bytes written
  uint64_t acc;
  uint32_t nb;
  SBH_HD void put(uint32_t v, uint32_t k) {  // k <= 32
    acc |= (uint64_t)v << nb;
    nb += k;
    while (nb >= 8) {
      if (n < cap) p[n] = (uint8_t)acc;
      ++n;
      acc >>= 8;
      nb -= 8;
    }
  }
  SBH_HD void windup() {
    if (nb) {
      if (n < cap) p[n] = (uint8_t)acc;
      ++n;
    }
    acc = 0;
    nb = 0;
  }
};

// send_tree
template <typename Put>
SBH_HD inline void z_send_tree(const ZTreeState &s, const ct_data *tree, int32_t max_code, const Put &put) {
  int32_t prevlen = -1, curlen, nextlen = tree[0].dl, count = 0, max_count = 7, min_count = 4;
  if (nextlen == 0) max_count = 138, min_count = 3;
  auto code = [&](int32_t c) { put(s.bl_tree[c].fc, s.bl_tree[c].dl); };
  for (int32_t n = 0; n <= max_code; n++) {
    curlen = nextlen;
    nextlen = tree[n + 1].dl;
    if (++count < max_count && curlen == nextlen) {
      continue;
    } else if (count < min_count) {
      do {
        code(curlen);
      } while (--count != 0);
    } else if (curlen != 0) {
      if (curlen != prevlen) {
        code(curlen);
        count--;
      }
      code(16);
      put((uint32_t)(count - 3), 2);
    } else if (count <= 10) {
      code(17);
      put((uint32_t)(count - 3), 3);
    } else {
      code(18);
      put((uint32_t)(count - 11), 7);
    }
    count = 0;
    prevlen = curlen;
    if (nextlen == 0) max_count = 138, min_count = 3;
    else if (curlen == nextlen) max_count = 6, min_count = 3;
    else max_count = 7, min_count = 4;
  }
}

// The dynamic block header after the 3 block-type bits (send_all_trees).
template <typename Put>
SBH_HD inline void z_send_all_trees(const ZTreeState &s, int32_t max_blindex, const Put &put) {
  const int32_t lcodes = s.l_max_code + 1, dcodes = s.d_max_code + 1, blcodes = max_blindex + 1;
  put((uint32_t)(lcodes - 257), 5);
  put((uint32_t)(dcodes - 1), 5);
  put((uint32_t)(blcodes - 4), 4);
  for (int32_t rank = 0; rank < blcodes; rank++) put(s.bl_tree[BL_ORDER[rank]].dl, 3);
  z_send_tree(s, s.dyn_ltree, lcodes - 1, put);
  z_send_tree(s, s.dyn_dtree, dcodes - 1, put);
}

// The whole member serially (host reference of the GPU stages): raw deflate bytes of
// src[0, N) into out (cap bytes); returns the deflate size, or 0 when it does not fit
// OUT_CAP - 1 bytes (htsjdk then stores the block at level 0).  tok / prev / info: scratch
// of N entries each; st: tree scratch.
SBH_HD inline void z_prev_serial(const uint8_t *src, uint32_t N, uint16_t *prev, uint16_t *head) {
  for (uint32_t h = 0; h <= HASH_MASK; ++h) head[h] = 0;
  for (uint32_t p = 0; p + MIN_MATCH <= N; ++p) {
    const uint32_t h = zhash(src[p], src[p + 1], src[p + 2]);
    prev[p] = head[h];
    head[h] = (uint16_t)p;
  }
}

// One block's bits (_tr_flush_block after the decision): stored (byte-aligned, LEN, NLEN, the
// bytes), static or dynamic (header, tokens, end of block); the last block ends with bi_windup.
template <typename TokAt, typename ByteAt>
SBH_HD inline void z_emit_block(ZBits &o, const ZTreeState &s, uint32_t type, int32_t mbl, const ZBlock &b, bool last,
                                const TokAt &tokat, const ByteAt &byteat) {
  const uint32_t lb = last ? 1u : 0u;
  auto put = [&](uint32_t v, uint32_t k) { o.put(v, k); };
  if (type == ZB_STORED) {
    const uint32_t len = b.byte1 - b.byte0;
    o.put(lb, 3);
    o.windup();
    o.put(len & 0xffff, 16);
    o.put(~len & 0xffff, 16);
    for (uint32_t i = b.byte0; i < b.byte1; ++i) o.put(byteat(i), 8);
  } else {
    uint32_t lit[L_CODES], dist[D_CODES];  // (the tables the GPU's k_zemit codes with)
    z_code_tables(s, type, lit, dist);
    o.put((type == ZB_STATIC ? 2u : 4u) + lb, 3);
    if (type == ZB_DYN) z_send_all_trees(s, mbl, put);
    for (uint32_t k = b.tok0; k < b.tok1; ++k) {
      uint64_t v;
      const uint32_t n = z_tok_bits_tab(tokat(k), lit, dist, &v);
      if (n > 32) {
        o.put((uint32_t)v & 0xffffu, 16);
        o.put((uint32_t)(v >> 16), n - 16);
      } else {
        o.put((uint32_t)v, n);
      }
    }
    o.put(lit[256] & 0xffff, lit[256] >> 16);
  }
  if (last) o.windup();
}

// The whole member serially (the host definition the GPU stages reproduce): raw deflate of
// src[0, N) into out (cap bytes, writes past cap are dropped but counted); returns the size.
// prev / head / tok / info: N, 32768, N and N entries of scratch; st: tree scratch.
SBH_HD inline uint32_t z_deflate_serial(const uint8_t *src, uint32_t N, int level, uint8_t *out, uint32_t cap,
                                        uint16_t *prev, uint16_t *head, uint32_t *tok, uint64_t *info,
                                        ZTreeState &st) {
  const ZCfg cf = z_config(level);
  z_prev_serial(src, N, prev, head);
  auto prv = [&](uint32_t i) -> uint32_t { return prev[i]; };
  auto cmp = [&](uint32_t a, uint32_t b, uint32_t lim) -> uint32_t {
    uint32_t l = 0;
    while (l < lim && src[a + l] == src[b + l]) ++l;
    return l;
  };
  for (uint32_t p = 0; p < N; ++p) info[p] = z_rec_with_byte(z_info(prv, cmp, p, N, cf), src[p]);
  ZBlock blocks[MAX_BLOCKS];
  uint32_t ntok = 0;
  const uint32_t nb = z_parse(
      N, cf, [&](uint32_t p) { return info[p]; }, [&](uint32_t k, uint32_t t) { tok[k] = t; }, blocks, &ntok);
  ZBits o{out, cap, 0, 0, 0};
  for (uint32_t i = 0; i < nb; ++i) {
    int32_t mbl = 0;
    auto tokat = [&](uint32_t k) { return tok[k]; };
    const uint32_t type = z_block_trees(st, tokat, blocks[i], &mbl);
    z_emit_block(o, st, type, mbl, blocks[i], i + 1 == nb, tokat, [&](uint32_t p) -> uint32_t { return src[p]; });
  }
  return o.n;
}

}  // namespace sbh_zlib
