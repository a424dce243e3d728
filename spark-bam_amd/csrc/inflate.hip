// inflate.hip -- BGZF block inflate on CDNA4: one 64-lane wave per BGZF block.
//
// Replaces StreamI._advance's `new Inflater(true).inflate(decBuf, 0, ISIZE)`
// (bgzf/src/main/scala/org/hammerlab/bgzf/block/Stream.scala:31-71) for every block
// of a shard at once.  Semantics follow java.util.zip.Inflater over raw DEFLATE
// (the JDK's zlib): output is exactly the first ISIZE bytes of the stream; fewer is
// an "Expected N decompressed bytes" error, a malformed stream a DataFormatException,
// and -- like zlib -- decoding continues past a full output buffer until a byte would
// have to be written, so a malformed header/code right after the last byte is still
// reported.  No CRC is checked (the reference does not check it either).
//
// Design (MI355X-first):
//  * The Huffman decode of a DEFLATE stream is serial, so each wave runs ONE
//    wave-uniform decoder: the bit buffer, counters and symbol state live in SGPRs
//    (SALU work); lanes are used for the parallel parts: table construction, LZ77
//    copies (64 bytes per instruction), stored-block copies and coalesced write-out.
//  * Compressed input is streamed through two VGPR windows (64 lanes x 4 B each,
//    prefetched 256 B ahead) and pulled into the bit buffer with v_readlane -- no LDS
//    round trip on the bit path.
//  * Decode tables (10-bit literal/length, 8-bit distance primary tables; canonical
//    slow path beyond) live in LDS, one set per wave.
//  * Output goes through a 32 KiB LDS ring (the whole DEFLATE window) indexed by the
//    *flat* destination address, so 16-byte granules are aligned both in LDS and in
//    HBM; 1 KiB groups are flushed with one 16 B store per lane.  Every LZ77 copy is
//    served from the ring: measured on synthetic and real BAM data, ~39% of matches
//    reach back more than 4 KiB (distances are spread over the whole window), so a
//    smaller ring with HBM read-back was latency-bound.
//  * ~39 KiB LDS per wave -> one 4-wave workgroup (one wave per SIMD) per CU.
#include "sbh_internal.h"

namespace sbh {
namespace {

constexpr int LIT_FAST = 10;
constexpr int DIST_FAST = 8;
constexpr int CL_FAST = 7;
#ifndef SBH_RING
#define SBH_RING 32768
#endif
#ifndef SBH_WAVES
#define SBH_WAVES 4
#endif
constexpr uint32_t RING = SBH_RING;  // 32768 = the whole DEFLATE window
constexpr uint32_t RMASK = RING - 1;
constexpr uint32_t GROUP = 1024;  // flush group: 64 lanes x 16 B
constexpr int WAVES = SBH_WAVES;
// With RING = 32768 a round of 64 lanes reads its sources before writing and a slot is
// rewritten only by a position 32768 later, so dist <= 32768 never reads a clobbered
// slot.  A smaller ring serves dist > NEAR_MAX from HBM (bytes flushed >= 2 groups
// earlier, drained by s_waitcnt vmcnt(0) before the read).
constexpr uint32_t NEAR_MAX = RING >= 32768 ? 32768 : RING - 258;
static_assert(RING >= 2 * GROUP + 2 * 258 + 16, "ring too small");

// Table entry: [4:0] code length, [7:5] kind, [15:8] byte/extra/sym, [31:16] base.
constexpr uint32_t K_LIT = 0, K_LEN = 1, K_EOB = 2, K_BAD = 3, K_DIST = 4, K_CL = 5, K_SLOW = 7;

__constant__ uint16_t LBASE[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                   31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t LEXT[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t DBASE[30] = {1,    2,    3,    4,    5,    7,    9,    13,    17,    25,
                                   33,   49,   65,   97,   129,  193,  257,  385,   513,   769,
                                   1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t DEXT[30] = {0, 0, 0, 0, 1, 1, 2, 2,  3,  3,  4,  4,  5,  5,  6,
                                 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t CL_ORDER[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

struct __attribute__((aligned(16))) WaveSmem {
  uint8_t ring[RING];
  uint32_t lit[1 << LIT_FAST];  // also the code-length-code table while reading headers
  uint32_t dist[1 << DIST_FAST];
  uint16_t sorted[320];  // canonical order: [0,288) lit/len (or CL), [288,320) dist
  uint8_t lens[320];     // [0,288) lit/len lengths, [288,320) dist lengths
  uint8_t cl_lens[20];
  uint32_t cnt[2][16];  // per-length counts (slow path)
};

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t l) {
  return __builtin_amdgcn_readlane(v, l);
}

__device__ __forceinline__ uint32_t lit_entry(uint32_t sym, uint32_t L) {
  if (sym < 256) return L | (K_LIT << 5) | (sym << 8);
  if (sym == 256) return L | (K_EOB << 5);
  if (sym < 286)
    return L | (K_LEN << 5) | ((uint32_t)LEXT[sym - 257] << 8) | ((uint32_t)LBASE[sym - 257] << 16);
  return L | (K_BAD << 5);
}
__device__ __forceinline__ uint32_t dist_entry(uint32_t sym, uint32_t L) {
  if (sym < 30) return L | (K_DIST << 5) | ((uint32_t)DEXT[sym] << 8) | ((uint32_t)DBASE[sym] << 16);
  return L | (K_BAD << 5);
}
__device__ __forceinline__ uint32_t make_entry(uint32_t kind, uint32_t sym, uint32_t L) {
  if (kind == 0) return lit_entry(sym, L);
  if (kind == 1) return dist_entry(sym, L);
  return L | (K_CL << 5) | (sym << 8);
}

// Canonical Huffman table (zlib inflate_table validity: over-subscribed -> error;
// incomplete -> error unless type != CODES and max == 1; max == 0 -> all invalid).
// kind: 0 lit/len, 1 dist, 2 code-length code.  Returns 0 ok, 1 error, 2 empty.
__device__ __forceinline__ uint32_t build_table(WaveSmem &sm, const uint8_t *lens, uint32_t nsym, uint32_t kind,
                                uint32_t *tab, int fast, uint32_t lane) {
  const uint32_t w = kind == 1 ? 1 : 0;
  uint16_t *sorted = sm.sorted + (kind == 1 ? 288 : 0);
  // counts per length: lane v (1..15) accumulates count[v]
  uint32_t my_cnt = 0;
  for (uint32_t base = 0; base < nsym; base += WAVE) {
    uint32_t s = base + lane;
    uint32_t l = s < nsym ? lens[s] : 0;
#pragma unroll
    for (uint32_t v = 1; v <= 15; ++v) {
      uint32_t c = (uint32_t)__popcll(__ballot(l == v));
      my_cnt += lane == v ? c : 0;
    }
  }
  // scalar prefix: offsets, first codes, validity
  int32_t left = 1;
  uint32_t max = 0, acc = 0, code = 0, prev = 0;
  uint32_t my_offs = 0, my_first = 0;
  for (uint32_t v = 1; v <= 15; ++v) {
    uint32_t c = uni(rdlane(my_cnt, v));
    left = 2 * left - (int32_t)c;
    if (c) max = v;
    code = (code + prev) << 1;
    prev = c;
    my_offs = lane == v ? acc : my_offs;
    my_first = lane == v ? code : my_first;
    acc += c;
  }
  if (lane < 16) sm.cnt[w][lane] = lane == 0 ? 0 : my_cnt;
  if (max == 0) {  // no symbols: every entry invalid
    for (uint32_t i = lane; i < (1u << fast); i += WAVE) tab[i] = 1u | (K_BAD << 5);
    return 2;
  }
  if (left < 0) return 1;
  if (left > 0 && (kind == 2 || max != 1)) return 1;
  // sorted symbols (stable by symbol within a length)
  uint32_t my_run = 0;
  for (uint32_t base = 0; base < nsym; base += WAVE) {
    uint32_t s = base + lane;
    uint32_t l = s < nsym ? lens[s] : 0;
    uint32_t rank = 0;
    for (uint32_t v = 1; v <= max; ++v) {
      uint64_t m = __ballot(l == v);
      if (m == 0) continue;
      uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
      uint32_t ov = uni(rdlane(my_offs, v)), rv = uni(rdlane(my_run, v));
      if (l == v) rank = ov + rv + below;
      my_run += lane == v ? (uint32_t)__popcll(m) : 0;
    }
    if (l) sorted[rank] = (uint16_t)s;
  }
  __builtin_amdgcn_wave_barrier();
  // fill the primary table: entry idx holds the code whose bit-reversed value is a
  // prefix of idx (DEFLATE codes are sent MSB first into an LSB-first bit buffer)
  const uint32_t n_ent = 1u << fast;
  const uint32_t per_lane = n_ent / WAVE;
  uint32_t found = 0;  // bit k: entry lane + 64k resolved
  for (uint32_t l = 1; l <= (uint32_t)fast && l <= max; ++l) {
    uint32_t fl = uni(rdlane(my_first, l));
    uint32_t cl = uni(rdlane(my_cnt, l));
    uint32_t ol = uni(rdlane(my_offs, l));
    if (cl == 0) continue;
    for (uint32_t k = 0; k < per_lane; ++k) {
      uint32_t idx = lane + WAVE * k;
      uint32_t c = __builtin_bitreverse32(idx) >> (32 - l);
      uint32_t v = c - fl;
      if (!(found & (1u << k)) && v < cl) {
        tab[idx] = make_entry(kind, sorted[ol + v], l);
        found |= 1u << k;
      }
    }
  }
  for (uint32_t k = 0; k < per_lane; ++k)
    if (!(found & (1u << k))) tab[lane + WAVE * k] = max > (uint32_t)fast ? (K_SLOW << 5) : (1u | (K_BAD << 5));
  __builtin_amdgcn_wave_barrier();
  return 0;
}

// Canonical slow-path decode (codes longer than the primary table): returns the
// table entry for the symbol, or a K_BAD entry.
__device__ __forceinline__ uint32_t slow_decode(const WaveSmem &sm, uint64_t buf, uint32_t kind) {
  const uint32_t w = kind == 1 ? 1 : 0;
  const uint16_t *sorted = sm.sorted + (kind == 1 ? 288 : 0);
  uint32_t code = 0, first = 0, index = 0;
  for (uint32_t len = 1; len <= 15; ++len) {
    code |= (uint32_t)(buf >> (len - 1)) & 1u;
    uint32_t count = uni(sm.cnt[w][len]);
    if (code - first < count) {
      uint32_t sym = uni(sorted[index + code - first]);
      return make_entry(kind, sym, len);
    }
    index += count;
    first += count;
    first <<= 1;
    code <<= 1;
  }
  return 1u | (K_BAD << 5);
}

// Wave-uniform bit reader over the VGPR windows.
struct Bits {
  const uint32_t *base32;  // dword-aligned view of the compressed shard
  uint32_t win, nwin;      // VGPR windows: lane l holds base32[wbase + l] / [wbase + 64 + l]
  uint32_t wbase;          // dword index of `win`
  uint32_t widx;           // next dword to pull into buf
  uint64_t buf;
  uint32_t cnt;
  uint32_t pos;    // bits consumed, relative to dword index a0
  uint32_t a0;     // dword index of the start of the block's deflate data (aligned down)
  uint32_t limit;  // bits available (relative to a0): Inflater input ends here
  uint32_t lane;

  __device__ __forceinline__ void seek(uint32_t bitpos) {
    pos = bitpos;
    widx = a0 + (bitpos >> 5);
    wbase = widx;
    win = base32[wbase + lane];
    nwin = base32[wbase + WAVE + lane];
    buf = 0;
    cnt = 0;
    refill();
    uint32_t d = bitpos & 31;
    buf >>= d;
    cnt -= d;
  }
  __device__ __forceinline__ void refill() {
    while (cnt <= 32) {
      uint32_t rel = widx - wbase;
      uint32_t w = rel < WAVE ? rdlane(win, rel) : rdlane(nwin, rel - WAVE);
      buf |= (uint64_t)w << cnt;
      cnt += 32;
      ++widx;
      if (widx - wbase == WAVE + 1) {  // moved into nwin: slide and prefetch
        win = nwin;
        wbase += WAVE;
        nwin = base32[wbase + WAVE + lane];
      }
    }
  }
  __device__ __forceinline__ void drop(uint32_t n) {
    buf >>= n;
    cnt -= n;
    pos += n;
  }
  __device__ __forceinline__ uint32_t peek(uint32_t n) const {
    return (uint32_t)buf & ((1u << n) - 1u);
  }
  __device__ __forceinline__ uint32_t take(uint32_t n) {
    uint32_t v = peek(n);
    drop(n);
    return v;
  }
  __device__ __forceinline__ bool avail(uint32_t n) const { return pos + n <= limit; }
};

// Flush granules [from_g, to_g) of the ring to U (flat addresses; from_g 16-aligned);
// bytes outside [G, to_g) are left alone (they belong to neighbouring blocks).
__device__ __forceinline__ void flush(const WaveSmem &sm, uint8_t *U, uint64_t from_g, uint64_t to_g,
                                      uint64_t G, uint32_t lane) {
  for (uint64_t g0 = from_g; g0 < to_g; g0 += GROUP) {
    uint64_t ga = g0 + 16ull * lane;
    if (ga < to_g) {
      if (ga >= G && ga + 16 <= to_g) {
        uint4 v = *reinterpret_cast<const uint4 *>(&sm.ring[(uint32_t)ga & RMASK]);
        *reinterpret_cast<uint4 *>(U + ga) = v;
      } else {
        for (uint32_t k = 0; k < 16; ++k) {
          uint64_t a = ga + k;
          if (a >= G && a < to_g) U[a] = sm.ring[(uint32_t)a & RMASK];
        }
      }
    }
  }
}

__global__ __launch_bounds__(WAVES *WAVE) void k_inflate(const uint8_t *__restrict__ comp, DevBlocks bl,
                                                          uint64_t nblocks, uint8_t *__restrict__ U) {
  __shared__ WaveSmem smem[WAVES];
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  const uint32_t wid = uni(threadIdx.x / WAVE);
  const uint64_t b = (uint64_t)blockIdx.x * WAVES + wid;
  if (b >= nblocks) return;
  WaveSmem &sm = smem[wid];

  const uint64_t cstart = bl.cstart[b];
  const uint32_t csize = bl.csize[b], hsize = bl.hsize[b], usize = bl.usize[b];
  const uint64_t G = bl.ustart[b];
  const uint32_t bflags = bl.flags[b];
  if (bflags & BLK_TRUNCATED) {
    if (lane == 0) bl.status[b] = INF_SIZE;
    return;
  }
  if (usize > 65536u) {
    if (lane == 0) bl.status[b] = INF_BAD_ISIZE;
    return;
  }
  if ((int32_t)csize - (int32_t)hsize - 8 < 0) {
    if (lane == 0) bl.status[b] = INF_DATA;
    return;
  }
  const uint32_t data_len = csize - hsize - 8;

  Bits br;
  br.base32 = reinterpret_cast<const uint32_t *>(comp);
  br.lane = lane;
  const uint64_t dbyte = cstart + hsize;
  br.a0 = (uint32_t)(dbyte >> 2);
  const uint32_t skip = (uint32_t)(dbyte & 3) * 8;
  br.limit = skip + data_len * 8;
  br.seek(skip);

  uint32_t out = 0;                 // bytes produced
  uint64_t flushed = G & ~15ull;     // flat address up to which stores were issued
  uint32_t status = INF_OK;
  bool fixed_built = false;
  bool last = false;
  bool done = false;

  // ---- block loop (deflate blocks inside the BGZF block) ----
  while (!done) {
    br.refill();
    if (!br.avail(3)) break;  // needs input: stop
    last = br.take(1);
    const uint32_t type = br.take(2);
    if (type == 0) {
      // stored block: byte-align, LEN, NLEN
      br.drop((8 - (br.pos & 7)) & 7);
      br.refill();
      if (!br.avail(32)) break;
      const uint32_t len = br.take(16), nlen = br.take(16);
      if (len != (~nlen & 0xffffu)) { status = INF_DATA; break; }
      uint32_t src_byte = br.pos >> 3;  // relative to a0*4
      uint32_t avail_bytes = (br.limit - br.pos) >> 3;
      uint32_t n = len;
      if (n > avail_bytes) n = avail_bytes;
      if (n > usize - out) n = usize - out;
      const uint8_t *src = comp + (uint64_t)br.a0 * 4 + src_byte;
      for (uint32_t c0 = 0; c0 < n; c0 += 512) {
        uint32_t piece = n - c0 < 512 ? n - c0 : 512;
        for (uint32_t k = 0; k < 8; ++k) {
          uint32_t i = lane * 8 + k;
          if (i < piece) sm.ring[(uint32_t)(G + out + i) & RMASK] = src[c0 + i];
        }
        out += piece;
        while (G + out >= flushed + GROUP) {
          flush(sm, U, flushed, flushed + GROUP, G, lane);
          flushed += GROUP;
        }
      }
      if (n < len) {  // output full or input exhausted
        done = true;
        break;
      }
      br.seek(br.pos + len * 8);
    } else if (type == 1 || type == 2) {
      if (type == 1) {
        if (!fixed_built) {
          for (uint32_t s = lane; s < 288; s += WAVE)
            sm.lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
          if (lane < 32) sm.lens[288 + lane] = 5;
          __builtin_amdgcn_wave_barrier();
          build_table(sm, sm.lens, 288, 0, sm.lit, LIT_FAST, lane);
          build_table(sm, sm.lens + 288, 32, 1, sm.dist, DIST_FAST, lane);
          fixed_built = true;
        }
      } else {
        fixed_built = false;
        br.refill();
        if (!br.avail(14)) break;
        const uint32_t nlen = br.take(5) + 257, ndist = br.take(5) + 1, ncode = br.take(4) + 4;
        if (nlen > 286 || ndist > 30) { status = INF_DATA; break; }
        if (!br.avail(ncode * 3)) break;
        if (lane < 20) sm.cl_lens[lane] = 0;
        __builtin_amdgcn_wave_barrier();
        // 3 bits each, in CL_ORDER; read serially (<= 57 bits)
        for (uint32_t i = 0; i < ncode; ++i) {
          br.refill();
          uint32_t v = br.take(3);
          if (lane == 0) sm.cl_lens[CL_ORDER[i]] = (uint8_t)v;
        }
        __builtin_amdgcn_wave_barrier();
        uint32_t rc = uni(build_table(sm, sm.cl_lens, 19, 2, sm.lit, CL_FAST, lane));
        if (rc == 1) { status = INF_DATA; break; }
        const uint32_t total = nlen + ndist;
        if (rc == 2) {  // no code-length codes: zlib decodes each as 0 (1 bit) then fails
          if (!br.avail(total)) break;
          status = INF_DATA;
          break;
        }
        uint32_t i = 0, prevlen = 0;
        bool hdr_ok = true, starved = false;
        while (i < total) {
          br.refill();
          uint32_t e = uni(sm.lit[br.peek(CL_FAST)]);
          uint32_t L = e & 31;
          if (!br.avail(L)) { starved = true; break; }
          br.drop(L);
          uint32_t sym = (e >> 8) & 0xff;
          if (sym < 16) {
            if (lane == 0) sm.lens[i] = (uint8_t)sym;
            prevlen = sym;
            ++i;
            continue;
          }
          uint32_t rep, val;
          if (sym == 16) {
            if (i == 0) { hdr_ok = false; break; }
            if (!br.avail(2)) { starved = true; break; }
            rep = 3 + br.take(2);
            val = prevlen;
          } else if (sym == 17) {
            if (!br.avail(3)) { starved = true; break; }
            rep = 3 + br.take(3);
            val = 0;
          } else {
            if (!br.avail(7)) { starved = true; break; }
            rep = 11 + br.take(7);
            val = 0;
          }
          if (i + rep > total) { hdr_ok = false; break; }
          for (uint32_t k = lane; k < rep; k += WAVE) sm.lens[i + k] = (uint8_t)val;
          prevlen = val;
          i += rep;
        }
        if (starved) break;
        if (!hdr_ok) { status = INF_DATA; break; }
        __builtin_amdgcn_wave_barrier();
        // split: lit lens [0,nlen) (+zeros to 288); dist lens -> [288, 288+ndist)
        uint32_t dv = lane < ndist ? sm.lens[nlen + lane] : 0;
        __builtin_amdgcn_wave_barrier();
        for (uint32_t s = nlen + lane; s < 288; s += WAVE) sm.lens[s] = 0;
        __builtin_amdgcn_wave_barrier();
        if (lane < 32) sm.lens[288 + lane] = (uint8_t)dv;
        __builtin_amdgcn_wave_barrier();
        if (uni(sm.lens[256]) == 0) { status = INF_DATA; break; }  // missing end-of-block
        if (uni(build_table(sm, sm.lens, nlen, 0, sm.lit, LIT_FAST, lane)) == 1) { status = INF_DATA; break; }
        if (uni(build_table(sm, sm.lens + 288, ndist, 1, sm.dist, DIST_FAST, lane)) == 1) { status = INF_DATA; break; }
      }
      // ---- symbol loop ----
      bool eob = false;
      for (;;) {
        br.refill();
        uint32_t e = uni(sm.lit[br.peek(LIT_FAST)]);
        uint32_t kind = (e >> 5) & 7;
        if (kind == K_SLOW) {
          e = uni(slow_decode(sm, br.buf, 0));
          kind = (e >> 5) & 7;
        }
        uint32_t L = e & 31;
        if (kind == K_BAD) {
          if (br.avail(1)) status = INF_DATA;
          done = true;
          break;
        }
        if (!br.avail(L)) { done = true; break; }
        br.drop(L);
        if (kind == K_LIT) {
          if (out == usize) { done = true; break; }
          if (lane == 0) sm.ring[(uint32_t)(G + out) & RMASK] = (uint8_t)(e >> 8);
          ++out;
        } else if (kind == K_EOB) {
          eob = true;
          break;
        } else {  // length
          const uint32_t lx = (e >> 8) & 0xff;
          if (!br.avail(lx)) { done = true; break; }
          const uint32_t mlen = (e >> 16) + br.take(lx);
          br.refill();
          uint32_t d = uni(sm.dist[br.peek(DIST_FAST)]);
          uint32_t dk = (d >> 5) & 7;
          if (dk == K_SLOW) {
            d = uni(slow_decode(sm, br.buf, 1));
            dk = (d >> 5) & 7;
          }
          if (dk == K_BAD) {
            if (br.avail(1)) status = INF_DATA;
            done = true;
            break;
          }
          const uint32_t DL = d & 31;
          if (!br.avail(DL)) { done = true; break; }
          br.drop(DL);
          const uint32_t dx = (d >> 8) & 0xff;
          if (!br.avail(dx)) { done = true; break; }
          const uint32_t dist = (d >> 16) + br.take(dx);
          if (out == usize) { done = true; break; }  // zlib stops at MATCH when full
          if (dist > out) { status = INF_DATA; done = true; break; }  // too far back
          const uint32_t n = mlen < usize - out ? mlen : usize - out;
          const uint64_t dst_g = G + out;
          if (dist > NEAR_MAX) {  // far (only with a ring smaller than the window)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            for (uint32_t i0 = 0; i0 < n; i0 += WAVE) {
              uint32_t i = i0 + lane;
              if (i < n) sm.ring[(uint32_t)(dst_g + i) & RMASK] = U[dst_g - dist + i];
            }
          } else if (dist >= WAVE || dist >= n) {
            for (uint32_t i0 = 0; i0 < n; i0 += WAVE) {
              uint32_t i = i0 + lane;
              if (i < n) sm.ring[(uint32_t)(dst_g + i) & RMASK] = sm.ring[(uint32_t)(dst_g - dist + i) & RMASK];
            }
          } else {  // overlapping short period: out[i] = out[i mod dist - dist]
            const uint32_t inv = dist == 1 ? 0 : (uint32_t)((0x100000000ull + dist - 1) / dist);
            for (uint32_t i0 = 0; i0 < n; i0 += WAVE) {
              uint32_t i = i0 + lane;
              uint32_t q = dist == 1 ? i : __umulhi(i, inv);
              uint32_t si = i - q * dist;
              if (i < n) sm.ring[(uint32_t)(dst_g + i) & RMASK] = sm.ring[(uint32_t)(dst_g - dist + si) & RMASK];
            }
          }
          out += n;
          if (n < mlen) { done = true; break; }  // output full mid-match
        }
        while (G + out >= flushed + GROUP) {
          flush(sm, U, flushed, flushed + GROUP, G, lane);
          flushed += GROUP;
        }
      }
      if (done) break;
      (void)eob;
    } else {
      status = INF_DATA;  // invalid block type
      break;
    }
    if (last) break;
  }
  // final flush of [flushed, G + out)
  if (G + out > flushed) flush(sm, U, flushed, G + out, G, lane);
  if (status == INF_OK && out != usize) status = INF_SIZE;
  if (lane == 0) bl.status[b] = status;
}

}  // namespace

hipError_t launch_inflate(const uint8_t *comp, DevBlocks blocks, uint64_t nblocks, uint8_t *U,
                          hipStream_t stream) {
  if (nblocks == 0) return hipSuccess;
  const uint64_t grid = (nblocks + WAVES - 1) / WAVES;
  hipLaunchKernelGGL(k_inflate, dim3((uint32_t)grid), dim3(WAVES * WAVE), 0, stream, comp, blocks,
                     nblocks, U);
  return hipGetLastError();
}

}  // namespace sbh
