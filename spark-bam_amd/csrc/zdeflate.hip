// zdeflate.hip -- the byte-exact BGZF writer on CDNA4: every 65498-byte member deflated exactly
// as htsjdk's java.util.zip.Deflater (zlib 1.2.11 deflate_slow; level 5 by default, 4..9 on
// request), in the parallel stages of zdeflate_core.h (whose serial definition the CPU tests
// pin to zlib).  Members run in batches; per member:
//  k_zprev   one wave: prev[] (the previous position with the same 15-bit hash) in steps of 64
//            positions -- the step's (hash, lane) keys bitonic-sorted across the wave, so a
//            position's predecessor inside the step is its sorted neighbour and the first of a
//            hash takes the 32768-entry LDS head table's entry;
//  k_zinfo   one 1024-thread workgroup, one thread per position: longest_match's result for both
//            chain lengths (z_info), the member processed in 16 Ki-position slabs with the slab's
//            prev[] and bytes, and the 32 KiB of history before it, staged in LDS (145 KiB);
//  k_zparse  one wave: deflate_slow's lazy parse (z_parse) over those records, 64 of them held
//            in VGPRs and read with v_readlane, tokens gathered one per lane and stored 64 at a
//            time; blocks close at 16383 symbols;
//  k_ztrees  four waves, one block each: the block's histogram (LDS atomics), then on one lane
//            zlib's build_tree / gen_bitlen / gen_codes / build_bl_tree and the stored / static
//            / dynamic choice; the block's code tables, dynamic header bits and token bit count;
//  k_zemit   256 threads: the blocks' bit offsets (stored blocks byte-aligned), the tokens'
//            offsets by a workgroup scan, the bits written as dwords (atomicOr where a run
//            shares a dword); a deflate stream of 65518 bytes or more becomes htsjdk's level-0
//            fallback (one final stored block);
//  then the CRC32 / ISIZE footer and the gather (deflate.hip's k_footer / k_gather).
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
#define SBH_HD __host__ __device__
#include "sbh_internal.h"
#include "zdeflate_core.h"

namespace sbh {
namespace {

using namespace sbh_zlib;

constexpr uint32_t ZPAY = 65498;  // htsjdk's uncompressed payload per member (2.bam.blocks)

struct ZRec {  // per-member record between the kernels
  uint32_t nblocks, ntok;
  ZBlock blocks[MAX_BLOCKS];
  uint32_t type[MAX_BLOCKS], hbits[MAX_BLOCKS];
  uint32_t tbits[MAX_BLOCKS];
  uint32_t lit[MAX_BLOCKS][L_CODES];
  uint32_t dist[MAX_BLOCKS][D_CODES];
  uint8_t hdr[MAX_BLOCKS][ZDEFLATE_HDR_BYTES];
};
static_assert(sizeof(ZRec) <= ZDEFLATE_REC_BYTES, "member record fits its scratch");

__device__ __forceinline__ uint32_t member_len(uint64_t n, uint64_t b) {
  const uint64_t s0 = b * ZPAY;
  return (uint32_t)((n - s0) < ZPAY ? (n - s0) : ZPAY);
}

// ---- k_zprev ------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_zprev(const uint8_t *__restrict__ src, uint64_t n, uint64_t b0,
                                              uint64_t nblocks, uint16_t *__restrict__ prevg) {
  __shared__ uint32_t head32[(HASH_MASK + 1) / 2];
  uint16_t *head = reinterpret_cast<uint16_t *>(head32);
  const uint32_t lane = threadIdx.x;
  const uint64_t b = b0 + blockIdx.x;
  if (b >= nblocks) return;
  const uint32_t len = member_len(n, b);
  const uint8_t *m = src + b * ZPAY;
  uint16_t *pv = prevg + (uint64_t)blockIdx.x * ZDEFLATE_PREV_ENTRIES;
  for (uint32_t i = lane; i < (HASH_MASK + 1) / 2; i += WAVE) head32[i] = 0;
  __syncthreads();
  const uint32_t hp = len >= MIN_MATCH ? len - (MIN_MATCH - 1) : 0;  // positions with 3 bytes
  uint32_t c0 = 0, c1 = 0, c2 = 0;
  if (lane < hp) c0 = m[lane], c1 = m[lane + 1], c2 = m[lane + 2];
  for (uint32_t base = 0; base < hp; base += WAVE) {
    const uint32_t p = base + lane;
    const bool live = p < hp;
    // dead lanes get keys past every hash, so they sort last
    const uint32_t h = live ? zhash(c0, c1, c2) : (HASH_MASK + 1) + lane;
    const uint32_t np = p + WAVE;
    if (np < hp) c0 = m[np], c1 = m[np + 1], c2 = m[np + 2];
    const uint32_t k = bitonic64(h << 6 | lane, lane);
    const uint32_t kp = (uint32_t)__shfl_up((int)k, 1), kn = (uint32_t)__shfl_down((int)k, 1);
    const uint32_t hs = k >> 6, ps = base + (k & 63);
    if (hs <= HASH_MASK) {
      const uint32_t pr = (lane > 0 && (kp >> 6) == hs) ? base + (kp & 63) : head[hs];
      pv[ps] = (uint16_t)pr;
      if (lane == WAVE - 1 || (kn >> 6) != hs) head[hs] = (uint16_t)ps;
    }
  }
}

// ---- k_zinfo ------------------------------------------------------------------------------
constexpr uint32_t ZSLAB = 16384, ZBACK = 32768, ZWIN = ZSLAB + ZBACK;
constexpr uint32_t ZBYTES = ZWIN + MAX_MATCH + 16;  // window bytes staged (+ the look-ahead of the slab's last match)
constexpr uint32_t ZINFO_T = 1024;

__global__ __launch_bounds__(ZINFO_T) void k_zinfo(const uint8_t *__restrict__ src, uint64_t n, uint64_t b0,
                                                   uint64_t nblocks, const uint16_t *__restrict__ prevg,
                                                   uint64_t *__restrict__ infog, ZCfg cf) {
  __shared__ uint32_t pw32[ZWIN / 2];                 // prev[base, base + ZWIN)
  __shared__ uint32_t bw32[(ZBYTES + 3) / 4 + 4];     // bytes [base, base + ZBYTES), zero padded
  const uint32_t t = threadIdx.x;
  const uint64_t b = b0 + blockIdx.x;
  if (b >= nblocks) return;
  const uint32_t len = member_len(n, b);
  const uint8_t *m = src + b * ZPAY;
  const uint32_t *pv32 = reinterpret_cast<const uint32_t *>(prevg + (uint64_t)blockIdx.x * ZDEFLATE_PREV_ENTRIES);
  uint64_t *info = infog + (uint64_t)blockIdx.x * ZDEFLATE_INFO_ENTRIES;
  const uint16_t *pw = reinterpret_cast<const uint16_t *>(pw32);
  const uintptr_t lim = (uintptr_t)(src + n);  // first address past the source buffer
  for (uint32_t s0 = 0; s0 < len; s0 += ZSLAB) {
    const uint32_t s1 = s0 + ZSLAB < len ? s0 + ZSLAB : len;
    const uint32_t base = s0 > ZBACK ? s0 - ZBACK : 0;  // even: prev dwords line up
    const uint32_t np = s1 - base;
    for (uint32_t i = t; i < (np + 1) / 2; i += ZINFO_T) pw32[i] = pv32[base / 2 + i];
    // bytes [base, bend) from aligned source dwords realigned with alignbyte, zero past bend
    {
      const uint32_t bend = s1 + MAX_MATCH + 8 < len ? s1 + MAX_MATCH + 8 : len;
      const uint8_t *q = m + base;
      const uintptr_t a0 = (uintptr_t)q & ~(uintptr_t)3;
      const uint32_t sh = (uint32_t)((uintptr_t)q & 3);
      const uint32_t nb = bend - base;
      for (uint32_t j = t; j < (ZBYTES + 3) / 4 + 4; j += ZINFO_T) {
        uint32_t v = 0;
        if (4 * j < nb) {
          const uintptr_t a = a0 + 4 * (uintptr_t)j;
          const uint32_t lo = *reinterpret_cast<const uint32_t *>(a);
          const uint32_t hi = a + 4 < lim ? *reinterpret_cast<const uint32_t *>(a + 4) : 0u;
          v = __builtin_amdgcn_alignbyte(hi, lo, sh);
          if (4 * j + 4 > nb) v &= (uint32_t)((1ull << (8 * (nb - 4 * j))) - 1);
        }
        bw32[j] = v;
      }
    }
    __syncthreads();
    const auto ld8 = [&](uint32_t i) -> uint64_t {  // window bytes [i, i + 8)
      const uint32_t a = i >> 2, r = i & 3;
      const uint32_t x0 = bw32[a], x1 = bw32[a + 1], x2 = bw32[a + 2];
      return (uint64_t)__builtin_amdgcn_alignbyte(x2, x1, r) << 32 | __builtin_amdgcn_alignbyte(x1, x0, r);
    };
    const auto prv = [&](uint32_t i) -> uint32_t { return pw[i - base]; };
    const auto cmp = [&](uint32_t a, uint32_t c, uint32_t lim8) -> uint32_t {
      uint32_t l = 0;
      const uint32_t ra = a - base, rc = c - base;
      while (l < lim8) {
        const uint64_t x = ld8(ra + l) ^ ld8(rc + l);
        if (x) {
          const uint32_t e = l + ((uint32_t)__builtin_ctzll(x) >> 3);
          return e < lim8 ? e : lim8;
        }
        l += 8;
      }
      return lim8;
    };
    for (uint32_t p = s0 + t; p < s1; p += ZINFO_T) {
      const uint32_t byte = (bw32[(p - base) >> 2] >> (8 * ((p - base) & 3))) & 0xffu;
      info[p] = z_rec_with_byte(z_info(prv, cmp, p, len, cf), byte);
    }
    __syncthreads();
  }
}

// ---- k_zparse -----------------------------------------------------------------------------
__device__ __forceinline__ uint64_t rdlane64(uint64_t v, uint32_t l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)l);
  return (uint64_t)hi << 32 | lo;
}

__global__ __launch_bounds__(64) void k_zparse(uint64_t n, uint64_t b0, uint64_t nblocks,
                                               const uint64_t *__restrict__ infog, uint32_t *__restrict__ tokg,
                                               uint8_t *__restrict__ recs, ZCfg cf) {
  const uint32_t lane = threadIdx.x;
  const uint64_t b = b0 + blockIdx.x;
  if (b >= nblocks) return;
  const uint32_t len = member_len(n, b);
  const uint64_t *inf = infog + (uint64_t)blockIdx.x * ZDEFLATE_INFO_ENTRIES;
  uint32_t *tk = tokg + (uint64_t)blockIdx.x * ZDEFLATE_TOK_ENTRIES;
  ZRec &R = *reinterpret_cast<ZRec *>(recs + (uint64_t)blockIdx.x * ZDEFLATE_REC_BYTES);
  // records [w0, w0 + 64) in vc, [w0 + 64, w0 + 128) in vn (one per lane)
  uint32_t w0 = 0;
  uint64_t vc = lane < len ? inf[lane] : 0, vn = WAVE + lane < len ? inf[WAVE + lane] : 0;
  const auto info = [&](uint32_t p) -> uint64_t {
    if (p >= w0 + WAVE) {
      if (p < w0 + 2 * WAVE) {
        vc = vn;
        w0 += WAVE;
      } else {
        w0 = p & ~(WAVE - 1);
        vc = w0 + lane < len ? inf[w0 + lane] : 0;
      }
      vn = w0 + WAVE + lane < len ? inf[w0 + WAVE + lane] : 0;
    }
    return rdlane64(vc, p - w0);
  };
  uint32_t tv = 0;  // lane (k & 63) holds token k until its group of 64 is stored
  const auto tok = [&](uint32_t k, uint32_t v) {
    if (lane == (k & (WAVE - 1))) tv = v;
    if ((k & (WAVE - 1)) == WAVE - 1) tk[k - (WAVE - 1) + lane] = tv;
  };
  ZBlock blocks[MAX_BLOCKS];
  uint32_t ntok = 0;
  const uint32_t nb = z_parse(len, cf, info, tok, blocks, &ntok);
  if (lane < (ntok & (WAVE - 1))) tk[(ntok & ~(WAVE - 1)) + lane] = tv;
  if (lane == 0) {
    R.nblocks = nb;
    R.ntok = ntok;
    for (uint32_t i = 0; i < nb; ++i) R.blocks[i] = blocks[i];
  }
}

// ---- k_ztrees -----------------------------------------------------------------------------
struct TreesLds {
  ZTreeState st;
  uint32_t cnt[L_CODES + D_CODES];  // histogram, then the code tables
};

__global__ __launch_bounds__(256) void k_ztrees(uint64_t n, uint64_t b0, uint64_t nblocks,
                                                const uint32_t *__restrict__ tokg, uint8_t *__restrict__ recs) {
  __shared__ TreesLds S[4];
  const uint32_t t = threadIdx.x, w = t / WAVE, lane = t % WAVE;
  const uint64_t b = b0 + blockIdx.x;
  if (b >= nblocks) return;
  const uint32_t *tk = tokg + (uint64_t)blockIdx.x * ZDEFLATE_TOK_ENTRIES;
  ZRec &R = *reinterpret_cast<ZRec *>(recs + (uint64_t)blockIdx.x * ZDEFLATE_REC_BYTES);
  TreesLds &L = S[w];
  const uint32_t nbk = R.nblocks;
  const auto wsync = []() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
  };
  for (uint32_t bi = w; bi < nbk; bi += 4) {
    const ZBlock blk = R.blocks[bi];
    for (uint32_t i = lane; i < L_CODES + D_CODES; i += WAVE) L.cnt[i] = 0;
    wsync();
    for (uint32_t k = blk.tok0 + lane; k < blk.tok1; k += WAVE) {
      uint32_t ls;
      int32_t ds;
      z_tok_syms(tk[k], &ls, &ds);
      atomicAdd(&L.cnt[ls], 1u);
      if (ds >= 0) atomicAdd(&L.cnt[L_CODES + ds], 1u);
    }
    wsync();
    for (uint32_t i = lane; i < L_CODES; i += WAVE) L.st.dyn_ltree[i].fc = (uint16_t)(L.cnt[i] + (i == 256 ? 1u : 0u));
    for (uint32_t i = lane; i < D_CODES; i += WAVE) L.st.dyn_dtree[i].fc = (uint16_t)L.cnt[L_CODES + i];
    wsync();
    uint32_t type = 0;
    if (lane == 0) {
      int32_t mbl = 0;
      type = z_block_decide(L.st, blk, &mbl);
      uint32_t hb = 0;
      if (type == ZB_DYN) {
        ZBits o{R.hdr[bi], ZDEFLATE_HDR_BYTES, 0, 0, 0};
        z_send_all_trees(L.st, mbl, [&](uint32_t v, uint32_t k) { o.put(v, k); });
        hb = o.n * 8 + o.nb;
        o.windup();
      }
      R.type[bi] = type;
      R.hbits[bi] = hb;
    }
    type = (uint32_t)__builtin_amdgcn_readfirstlane((int)type);
    wsync();
    // the code tables (static or the dynamic trees), to the record and to LDS for the bit count
    for (uint32_t i = lane; i < L_CODES; i += WAVE) {
      const uint32_t c = type == ZB_STATIC ? static_lcode(i) | static_llen(i) << 16
                                           : (uint32_t)L.st.dyn_ltree[i].fc | (uint32_t)L.st.dyn_ltree[i].dl << 16;
      L.cnt[i] = c;
      R.lit[bi][i] = c;
    }
    for (uint32_t i = lane; i < D_CODES; i += WAVE) {
      const uint32_t c = type == ZB_STATIC ? bi_reverse(i, 5) | 5u << 16
                                           : (uint32_t)L.st.dyn_dtree[i].fc | (uint32_t)L.st.dyn_dtree[i].dl << 16;
      L.cnt[L_CODES + i] = c;
      R.dist[bi][i] = c;
    }
    wsync();
    uint32_t bits = 0;
    if (type != ZB_STORED)
      for (uint32_t k = blk.tok0 + lane; k < blk.tok1; k += WAVE) {
        uint64_t v;
        bits += z_tok_bits_tab(tk[k], L.cnt, L.cnt + L_CODES, &v);
      }
    for (uint32_t d = WAVE / 2; d > 0; d >>= 1) bits += (uint32_t)__shfl_down((int)bits, d, WAVE);
    if (lane == 0) R.tbits[bi] = bits;
    wsync();
  }
}

// ---- k_zemit ------------------------------------------------------------------------------
// A run of bits into the zeroed slot from bit `bit0` on: interior dwords stored, the first and
// last (which other runs may share) through atomicOr.
struct RunBits {
  uint32_t *base;
  uint32_t wi, nb;
  uint64_t acc;
  bool first;
  __device__ void start(uint32_t *b, uint32_t bit0) {
    base = b, wi = bit0 / 32, nb = bit0 % 32, acc = 0, first = true;
  }
  __device__ void put(uint32_t v, uint32_t k) {  // k <= 32
    acc |= (uint64_t)v << nb;
    nb += k;
    if (nb >= 32) {
      if (first) {
        atomicOr(base + wi, (uint32_t)acc);
        first = false;
      } else {
        base[wi] = (uint32_t)acc;
      }
      ++wi;
      acc >>= 32;
      nb -= 32;
    }
  }
  __device__ void put48(uint64_t v, uint32_t k) {
    if (k > 32) {
      put((uint32_t)v & 0xffffu, 16);
      put((uint32_t)(v >> 16), k - 16);
    } else {
      put((uint32_t)v, k);
    }
  }
  __device__ void finish() {
    if (nb) atomicOr(base + wi, (uint32_t)acc);
  }
};

constexpr uint32_t ZE_T = 256;

__global__ __launch_bounds__(ZE_T) void k_zemit(const uint8_t *__restrict__ src, uint64_t n, uint64_t b0,
                                                uint64_t nblocks, const uint32_t *__restrict__ tokg,
                                                const uint8_t *__restrict__ recs, uint8_t *__restrict__ slots,
                                                uint32_t *__restrict__ sizes, int level0) {
  __shared__ uint32_t lit[MAX_BLOCKS][L_CODES], dist[MAX_BLOCKS][D_CODES];
  __shared__ uint32_t bstart[MAX_BLOCKS], tbs[MAX_BLOCKS], btype[MAX_BLOCKS], bhb[MAX_BLOCKS];
  __shared__ ZBlock blk[MAX_BLOCKS];
  __shared__ uint32_t wsum[ZE_T / WAVE], total_bytes;
  const uint32_t t = threadIdx.x, w = t / WAVE, lane = t % WAVE;
  const uint64_t b = b0 + blockIdx.x;
  if (b >= nblocks) return;
  const uint32_t len = member_len(n, b);
  const uint8_t *m = src + b * ZPAY;
  const uint32_t *tk = tokg + (uint64_t)blockIdx.x * ZDEFLATE_TOK_ENTRIES;
  const ZRec &R = *reinterpret_cast<const ZRec *>(recs + (uint64_t)blockIdx.x * ZDEFLATE_REC_BYTES);
  uint8_t *slot = slots + (uint64_t)blockIdx.x * ZDEFLATE_SLOT;
  uint32_t *words = reinterpret_cast<uint32_t *>(slot);
  const uint32_t nbk = level0 ? 0u : R.nblocks, ntok = level0 ? 0u : R.ntok;
  for (uint32_t i = t; i < nbk * L_CODES; i += ZE_T) lit[i / L_CODES][i % L_CODES] = R.lit[i / L_CODES][i % L_CODES];
  for (uint32_t i = t; i < nbk * D_CODES; i += ZE_T) dist[i / D_CODES][i % D_CODES] = R.dist[i / D_CODES][i % D_CODES];
  if (t < nbk) {
    blk[t] = R.blocks[t];
    btype[t] = R.type[t];
    bhb[t] = R.hbits[t];
  }
  if (t == 0) {  // the blocks' bit offsets
    uint32_t pos = 0, tb = 0;
    for (uint32_t i = 0; i < nbk; ++i) {
      const ZBlock &k = R.blocks[i];
      bstart[i] = pos;
      tbs[i] = tb;
      if (R.type[i] == ZB_STORED) {
        pos = (pos + 3 + 7) & ~7u;
        pos += 32 + 8 * (k.byte1 - k.byte0);
      } else {
        pos += 3 + R.hbits[i] + R.tbits[i] + (R.lit[i][256] >> 16);
        tb += R.tbits[i];
      }
    }
    total_bytes = level0 ? OUT_CAP : (pos + 7) / 8;  // the last block ends with bi_windup
  }
  __syncthreads();
  uint32_t dsize = total_bytes;
  if (dsize >= OUT_CAP) {
    // htsjdk: the level-5 stream did not finish in 65518 bytes -> NO_COMPRESSION deflater: one
    // final stored block (zlib 1.2.11 deflate_stored with 65518 bytes of output space); the
    // same bytes at level 0
    dsize = 5 + len;
    uint8_t *d0 = slot + 18;
    if (t == 0) {
      d0[0] = 1;
      d0[1] = (uint8_t)len;
      d0[2] = (uint8_t)(len >> 8);
      d0[3] = (uint8_t)~len;
      d0[4] = (uint8_t)(~len >> 8);
    }
    for (uint32_t i = t; i < len; i += ZE_T) d0[5 + i] = m[i];
  } else {
    const uint32_t bit0 = 8 * 18;  // the deflate stream follows the 18-byte BGZF header
    const uint32_t wend = (18 + dsize + 3) / 4;
    for (uint32_t i = 4 + t; i < wend; i += ZE_T) words[i] = 0;  // (dword 4 = BSIZE + 2 stream bytes)
    __syncthreads();
    // the tokens: a contiguous range per thread
    const uint32_t K = (ntok + ZE_T - 1) / ZE_T;
    const uint32_t k0 = t * K < ntok ? t * K : ntok, k1 = k0 + K < ntok ? k0 + K : ntok;
    uint32_t bi = 0;
    while (bi + 1 < nbk && blk[bi].tok1 <= k0) ++bi;
    uint32_t mine = 0;
    {
      uint32_t bj = bi;
      for (uint32_t k = k0; k < k1; ++k) {
        while (blk[bj].tok1 <= k) ++bj;
        if (btype[bj] == ZB_STORED) continue;
        uint64_t v;
        mine += z_tok_bits_tab(tk[k], lit[bj], dist[bj], &v);
      }
    }
    const uint32_t incl = wave_incl_scan(mine);
    if (lane == WAVE - 1) wsum[w] = incl;
    __syncthreads();
    uint32_t tb = incl - mine;
    for (uint32_t q = 0; q < w; ++q) tb += wsum[q];
    RunBits o;
    bool open = false;
    for (uint32_t k = k0; k < k1; ++k) {
      if (blk[bi].tok1 <= k) {
        while (blk[bi].tok1 <= k) ++bi;
        if (open) o.finish();
        open = false;
      }
      if (btype[bi] == ZB_STORED) continue;
      if (!open) {
        o.start(words, bit0 + bstart[bi] + 3 + bhb[bi] + (tb - tbs[bi]));
        open = true;
      }
      uint64_t v;
      const uint32_t nbits = z_tok_bits_tab(tk[k], lit[bi], dist[bi], &v);
      o.put48(v, nbits);
      tb += nbits;
    }
    if (open) o.finish();
    // block headers, end-of-block codes and stored blocks (one wave per block)
    for (uint32_t i = w; i < nbk; i += ZE_T / WAVE) {
      const uint32_t last = i + 1 == nbk ? 1u : 0u;
      const uint32_t s = bit0 + bstart[i];
      if (btype[i] == ZB_STORED) {
        const ZBlock &k = blk[i];
        const uint32_t sl = k.byte1 - k.byte0;
        if (lane == 0) {
          RunBits h;
          h.start(words, s);
          h.put(last, 3);  // STORED_BLOCK << 1 | last
          h.finish();
        }
        // LEN, NLEN and the bytes from the next byte boundary on, as a byte string
        const uint32_t by0 = (s + 3 + 7) / 8, nby = 4 + sl;
        const auto sb = [&](uint32_t j) -> uint32_t {
          if (j == 0) return sl & 0xff;
          if (j == 1) return (sl >> 8) & 0xff;
          if (j == 2) return ~sl & 0xff;
          if (j == 3) return (~sl >> 8) & 0xff;
          return m[k.byte0 + j - 4];
        };
        const uint32_t dw0 = by0 / 4, dw1 = (by0 + nby + 3) / 4;
        for (uint32_t d = dw0 + lane; d < dw1; d += WAVE) {
          uint32_t v = 0;
          bool partial = false;
          for (uint32_t c = 0; c < 4; ++c) {
            const uint32_t by = 4 * d + c;
            if (by < by0 || by >= by0 + nby) {
              partial = true;
              continue;
            }
            v |= sb(by - by0) << (8 * c);
          }
          if (partial) atomicOr(words + d, v);
          else words[d] = v;
        }
      } else if (lane == 0) {
        RunBits h;
        h.start(words, s);
        h.put((btype[i] == ZB_STATIC ? 2u : 4u) + last, 3);
        const uint8_t *hd = R.hdr[i];
        for (uint32_t q = 0; q < bhb[i]; q += 8) h.put(hd[q / 8], bhb[i] - q < 8 ? bhb[i] - q : 8);
        h.finish();
        // end of block after the header and the tokens
        const uint32_t eb = s + 3 + bhb[i] + R.tbits[i];
        RunBits e;
        e.start(words, eb);
        e.put(lit[i][256] & 0xffff, lit[i][256] >> 16);
        e.finish();
      }
    }
  }
  __syncthreads();
  if (t == 0) {
    const uint32_t total = 18 + dsize + 8;
    const uint8_t hdr[16] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0};
    for (int i = 0; i < 4; ++i)
      words[i] = (uint32_t)hdr[4 * i] | (uint32_t)hdr[4 * i + 1] << 8 | (uint32_t)hdr[4 * i + 2] << 16 |
                 (uint32_t)hdr[4 * i + 3] << 24;
    // BSIZE: htsjdk writes totalBlockSize - 1 as a u16 (bytes 16..17; the rest of that dword
    // is the stream's, complete after the barrier)
    slot[16] = (uint8_t)(total - 1);
    slot[17] = (uint8_t)((total - 1) >> 8);
    sizes[blockIdx.x] = total;
  }
}

}  // namespace

hipError_t launch_zdeflate(const uint8_t *src, uint64_t n, uint64_t b0, uint32_t nbatch, int level, uint16_t *prev,
                           uint64_t *info, uint32_t *toks, uint8_t *recs, uint8_t *slots, uint32_t *sizes,
                           hipStream_t st) {
  const uint64_t nb = (n + ZPAY - 1) / ZPAY;
  if (!nbatch || b0 >= nb) return hipSuccess;
  if (nbatch > ZDEFLATE_BATCH || b0 + nbatch > nb || level < 0 || (level > 0 && level < 4) || level > 9)
    return hipErrorInvalidValue;
  if (level > 0) {
    const ZCfg cf = z_config(level);
    hipLaunchKernelGGL(k_zprev, dim3(nbatch), dim3(64), 0, st, src, n, b0, nb, prev);
    hipLaunchKernelGGL(k_zinfo, dim3(nbatch), dim3(ZINFO_T), 0, st, src, n, b0, nb, prev, info, cf);
    hipLaunchKernelGGL(k_zparse, dim3(nbatch), dim3(64), 0, st, n, b0, nb, info, toks, recs, cf);
    hipLaunchKernelGGL(k_ztrees, dim3(nbatch), dim3(256), 0, st, n, b0, nb, toks, recs);
  }
  hipLaunchKernelGGL(k_zemit, dim3(nbatch), dim3(ZE_T), 0, st, src, n, b0, nb, toks, recs, slots, sizes,
                     level == 0 ? 1 : 0);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_member_footer(src, n, b0, nb, nbatch, slots, ZDEFLATE_SLOT, sizes, st);
}

}  // namespace sbh
