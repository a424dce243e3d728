// inflate.hip -- BGZF block inflate on CDNA4, in two kernels.
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
//  * k_hdr -- the first deflate block of a BGZF block starts at its first data bit, so
//    its dynamic header is decoded and tabled before k_huff, one 64-lane wave per block,
//    into the end of the block's token region; k_huff copies the tables into LDS.
//  * k_huff -- Huffman decode to LZ77 tokens.  One 256-lane workgroup per BGZF block
//    stages the deflate bytes in LDS and decodes lane-parallel: each lane takes a slice
//    of the bits, decodes speculatively (Huffman/DEFLATE self-synchronises), repairs
//    from its left neighbour's exit until no exit changes, and after two prefix sums
//    emits its tokens (see "Lane-parallel Huffman decode" below).  Anything it cannot
//    prove well-formed goes to k_huff_serial, the exact one-wave zlib-semantics decoder
//    (stored blocks, errors, short/long streams), so block status always equals zlib's.
//  * k_lz -- LZ77 resolution.  One 512-thread workgroup per block builds the block's
//    64 KiB image in LDS, 1024 tokens per chunk: token starts are marked (one slot
//    value + one start bit each), a divergence-free slot pass gives every byte the
//    position it copies from, and barrier-free pointer chasing settles them; the image
//    goes to HBM with 16-byte stores aligned to the flat address.
//  * Token buffer: tokens of block b live at tok[ustart_b ...]; a block has at most
//    usize tokens (every token yields >= 1 byte), so the buffer is 4 B per flat byte.
#include "sbh_internal.h"

namespace sbh {
namespace {

#ifndef SBH_LIT_FAST
#define SBH_LIT_FAST 10
#endif
#ifndef SBH_HUFF_WAVES
#define SBH_HUFF_WAVES 4
#endif
constexpr int LIT_FAST = SBH_LIT_FAST;
#ifndef SBH_HUFF_PAIRS
#define SBH_HUFF_PAIRS 1  // literal-pair table entries and two-byte literal tokens (see PE_PAIR)
#endif
constexpr int DIST_FAST = 8;
constexpr int CL_FAST = 7;
constexpr int PDIST_FAST = 10;  // PAR-format distance table: one dword per entry, as wide as the literal one
constexpr int WAVES = SBH_HUFF_WAVES;  // waves (blocks) per k_huff workgroup
#ifndef SBH_LZ_THREADS
#define SBH_LZ_THREADS 512
#endif
constexpr uint32_t LZ_THREADS = SBH_LZ_THREADS;
#ifndef SBH_LZ_SHORT
#define SBH_LZ_SHORT 32
#endif
constexpr uint32_t LZ_SHORT = SBH_LZ_SHORT;  // longer matches get their pointers from the whole wave
static_assert(LZ_SHORT <= 33, "k_lz finds a short match's start within 32 slots back");
constexpr uint32_t NTOK_STORED = 0xffffffffu;  // ntok of a block whose payload is one stored deflate block
constexpr uint32_t TOK_PAIR = 1u << 24;  // a literal token of two bytes (byte2 at [23:16])
constexpr uint32_t TOK_MATCH = 0x80000000u;  // token: literal = byte << 8 (bit 31 clear); match = bit31 | len << 16 | dist

// Table entries (32-bit; laid out so the asm hot loop decodes with few scalar ops):
//   literal   [4:0] code length L, [7:5] K_LIT, [15:8] byte          (the entry is the token)
//   length    [4:0] L, [7:5] K_LEN, [15:8] L + extra bits, [22:16] extra bits, [31:23] base
//             (s_bfe_u32 with the entry as operand extracts the extra bits: offset L, width lx)
//   distance  [4:0] L, [7:5] K_DIST, [15:8] L + extra, [22:16] extra, [27:23] symbol, bit 31 set;
//             the distance table holds (entry, base) dword pairs
//   code-length code  [4:0] L, [7:5] K_CL, [15:8] symbol;  EOB / BAD / SLOW: [4:0] L, [7:5] kind
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

static_assert((1 << PDIST_FAST) >= (2 << DIST_FAST), "the serial distance table fits the PAR one");

// PAR-format entry flags (see pentry)
constexpr uint32_t PE_LEN = 1u << 12;      // a length code: a distance code follows (= the distance
                                           // table's byte offset in WaveSmem::tab)
constexpr uint32_t PE_EOB = 1u << 13;      // (with PE_SPECIAL) end of block
constexpr uint32_t PE_SLOW = 1u << 14;     // (with PE_SPECIAL) code longer than the table: slow_lane
constexpr uint32_t PE_SPECIAL = 1u << 31;  // not a token: end of block, invalid, or long code
// (SBH_HUFF_PAIRS) a literal entry that decodes two literal codes at once (their lengths summed in
// [4:0]; the first byte at [23:16], the second's low 7 bits at [30:24] and its bit 7 at PE_L2B7):
// one token of two bytes, (byte1 << 8) | (byte2 << 16) | TOK_PAIR
constexpr uint32_t PE_L2B7 = 1u << 9;
constexpr uint32_t PE_PAIR = 1u << 10;

struct __attribute__((aligned(16))) WaveSmem {
  union {
    struct {
      uint32_t lit[1 << LIT_FAST];    // also the code-length-code table while reading headers
      uint32_t dist[1 << PDIST_FAST];  // serial format: (entry, base) pairs in the first 2 << DIST_FAST
    };
    uint32_t tab[(1 << LIT_FAST) + (1 << PDIST_FAST)];
  };
  uint16_t sorted[320];  // canonical order: [0,288) lit/len (or CL), [288,320) dist
  uint8_t lens[320];     // [0,288) lit/len lengths, [288,320) dist lengths
  uint8_t cl_lens[20];
  uint32_t cnt[2][16];  // per-length counts (slow path)
  uint32_t pk[2][16];   // PAR format, per length: left-justified (15-bit) code limit << 16 |
                        // sorted index of the length's code 0 (offs - first, mod 2^16)
  uint32_t sent[320];   // PAR format: entry of each sorted symbol ([0,288) lit/len, [288,320) dist)
};

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t l) {
  return __builtin_amdgcn_readlane(v, l);
}


__device__ __forceinline__ uint32_t lit_entry(uint32_t sym, uint32_t L) {
  if (sym < 256) return L | (K_LIT << 5) | (sym << 8);
  if (sym == 256) return L | (K_EOB << 5);
  if (sym < 286) {
    const uint32_t lx = LEXT[sym - 257];
    return L | (K_LEN << 5) | ((L + lx) << 8) | (lx << 16) | ((uint32_t)LBASE[sym - 257] << 23);
  }
  return L | (K_BAD << 5);
}
__device__ __forceinline__ uint32_t dist_entry(uint32_t sym, uint32_t L) {
  if (sym < 30) {
    const uint32_t dx = DEXT[sym];
    return L | (K_DIST << 5) | ((L + dx) << 8) | (dx << 16) | (sym << 23) | 0x80000000u;
  }
  return L | (K_BAD << 5);
}
__device__ __forceinline__ uint32_t len_extra(uint32_t e) { return (e >> 16) & 0x7f; }
__device__ __forceinline__ uint32_t len_base(uint32_t e) { return e >> 23; }
__device__ __forceinline__ uint32_t dist_base(uint32_t e) { return DBASE[(e >> 23) & 31]; }
__device__ __forceinline__ uint32_t make_entry(uint32_t kind, uint32_t sym, uint32_t L) {
  if (kind == 0) return lit_entry(sym, L);
  if (kind == 1) return dist_entry(sym, L);
  return L | (K_CL << 5) | (sym << 8);
}

// Distance tables hold (entry, base) pairs; the others one entry per index.
__device__ __forceinline__ void put_entry(uint32_t *tab, uint32_t kind, uint32_t idx, uint32_t e) {
  if (kind == 1) {
    tab[2 * idx] = e;
    tab[2 * idx + 1] = (e & 0x80000000u) ? (uint32_t)DBASE[(e >> 23) & 31] : 0u;
  } else {
    tab[idx] = e;
  }
}

// Canonical Huffman table (zlib inflate_table validity: over-subscribed -> error;
// incomplete -> error unless type != CODES and max == 1; max == 0 -> all invalid).
// kind: 0 lit/len, 1 dist, 2 code-length code.  Returns 0 ok, 1 error, 2 empty.
template <class SM>
__device__ __forceinline__ uint32_t build_table(SM &sm, const uint8_t *lens, uint32_t nsym, uint32_t kind,
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
    for (uint32_t i = lane; i < (1u << fast); i += WAVE) put_entry(tab, kind, i, 1u | (K_BAD << 5));
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
        put_entry(tab, kind, idx, make_entry(kind, sorted[ol + v], l));
        found |= 1u << k;
      }
    }
  }
  for (uint32_t k = 0; k < per_lane; ++k)
    if (!(found & (1u << k)))
      put_entry(tab, kind, lane + WAVE * k, max > (uint32_t)fast ? (K_SLOW << 5) : (1u | (K_BAD << 5)));
  __builtin_amdgcn_wave_barrier();
  return 0;
}

// PAR-format entries (the lane-parallel decoder): [4:0] code length L, [8:5] extra bits,
// [12] PE_LEN, [13] PE_EOB, [14] PE_SLOW, [30:16] base (a literal's byte; a length's base
// MINUS ONE; a distance base), [31] PE_SPECIAL, so any code decodes as base + bits(L, extra),
// a special entry is a negative one, and PE_LEN doubles as the distance table's offset.
__device__ __forceinline__ uint32_t pentry(uint32_t kind, uint32_t sym, uint32_t L) {
  // base / extra bits of length symbols 257 + i and distance symbols i, computed
  // (RFC 1951 3.2.5) rather than looked up: no constant-memory loads in the table build
  if (kind == 0) {
    if (sym < 256) return L | (sym << 16);
    if (sym == 256) return L | PE_SPECIAL | PE_EOB;
    if (sym < 286) {
      const uint32_t i = sym - 257;
      const uint32_t x = (i < 8 || i == 28) ? 0u : (i - 4) >> 2;
      const uint32_t base = i < 8 ? 3 + i : i == 28 ? 258u : ((4 + (i & 3)) << x) + 3;
      return L | PE_LEN | (x << 5) | ((base - 1) << 16);
    }
    return L | PE_SPECIAL;
  }
  if (sym < 30) {
    const uint32_t x = sym < 4 ? 0u : (sym - 2) >> 1;
    const uint32_t base = sym < 4 ? sym + 1 : ((2 + (sym & 1)) << x) + 1;
    return L | (x << 5) | (base << 16);
  }
  return L | PE_SPECIAL;
}

// Canonical table in the PAR format (kind 0 lit/len, 1 dist), same validity rules as
// build_table.  Codes are located by their left-justified limits: the codes of length
// v occupy [lj[v-1], lj[v]) of the 15-bit left-justified code space, so a reversed
// index's length is 1 + #{v : lj[v] <= code}.  Entries whose code is longer than
// `fast` bits are K_SLOW (slow_lane finishes them); prefixes of no code are K_BAD.
template <class SM>
__device__ __forceinline__ uint32_t ptable_meta(SM &sm, const uint8_t *lens, uint32_t nsym, uint32_t kind,
                                                uint32_t lane) {
  uint16_t *sorted = sm.sorted + (kind ? 288 : 0);
  uint32_t my_cnt = 0;  // lane v (1..15): count of length v
  for (uint32_t base = 0; base < nsym; base += WAVE) {
    const uint32_t s = base + lane;
    const uint32_t l = s < nsym ? lens[s] : 0;
#pragma unroll
    for (uint32_t v = 1; v <= 15; ++v) {
      const uint32_t c = (uint32_t)__popcll(__ballot(l == v));
      my_cnt += lane == v ? c : 0;
    }
  }
  int32_t left = 1;
  uint32_t max = 0, acc = 0, code = 0, prev = 0, my_offs = 0;
  uint32_t ljv[16];
#pragma unroll
  for (uint32_t v = 1; v <= 15; ++v) {
    const uint32_t c = uni(rdlane(my_cnt, v));
    left = 2 * left - (int32_t)c;
    if (c) max = v;
    code = (code + prev) << 1;
    prev = c;
    ljv[v] = (code + c) << (15 - v);
    if (lane == v) {
      sm.pk[kind][v] = (ljv[v] << 16) | ((acc - code) & 0xffffu);
      my_offs = acc;
    }
    acc += c;
  }
  if (max == 0) {  // no symbols: all-zero limits make every entry invalid (ptable_entry)
    if (lane < 16) sm.pk[kind][lane] = 0;
    return 2;
  }
  if (left < 0) return 1;
  if (left > 0 && max != 1) return 1;
  uint32_t my_run = 0;
  for (uint32_t base = 0; base < nsym; base += WAVE) {
    const uint32_t s = base + lane;
    const uint32_t l = s < nsym ? lens[s] : 0;
    uint32_t rank = 0;
    for (uint32_t v = 1; v <= max; ++v) {
      const uint64_t m = __ballot(l == v);
      if (m == 0) continue;
      const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
      const uint32_t ov = uni(rdlane(my_offs, v)), rv = uni(rdlane(my_run, v));
      if (l == v) rank = ov + rv + below;
      my_run += lane == v ? (uint32_t)__popcll(m) : 0;
    }
    if (l) {
      sorted[rank] = (uint16_t)s;
      sm.sent[(kind ? 288 : 0) + rank] = pentry(kind, s, l);
    }
  }
  return 0;
}

// Entry i of the PAR table of `kind` from its limits lj[v] (= pk[kind][v] >> 16) and
// ptable_meta's canonical order: the code's length is 1 + #{v : lj[v] <= code}.
template <class SM>
__device__ __forceinline__ uint32_t ptable_entry(const SM &sm, const uint32_t *lj, uint32_t kind, uint32_t fast,
                                                 uint32_t i) {
  const uint32_t c15 = (__builtin_bitreverse32(i) >> (32 - fast)) << (15 - fast);
  uint32_t len = 1;
#pragma unroll
  for (uint32_t v = 1; v <= 15; ++v) len += lj[v] <= c15 ? 1u : 0u;
  if (len > 15) return 1u | PE_SPECIAL;
  if (len > fast) return PE_SPECIAL | PE_SLOW;
  return sm.sent[(kind ? 288 : 0) + (((sm.pk[kind][len] & 0xffffu) + (c15 >> (15 - len))) & 0xffffu)];
}

// Entry i of the literal/length table (PAR format), paired (SBH_HUFF_PAIRS): a literal code of
// L1 < LIT_FAST bits whose next LIT_FAST - L1 bits hold a whole literal code gives both at once.
// (The entry of i >> L1 is that second code's whatever the bits past the window: codes are
// prefix-free, and a code of at most LIT_FAST - L1 bits lies inside it.)
template <class SM>
__device__ __forceinline__ uint32_t ptable_lit_entry(const SM &sm, const uint32_t *lj, uint32_t i) {
  const uint32_t e1 = ptable_entry(sm, lj, 0, LIT_FAST, i);
  if (!SBH_HUFF_PAIRS || (int32_t)e1 < 0 || (e1 & PE_LEN) || (e1 & 31) >= (uint32_t)LIT_FAST) return e1;
  const uint32_t L1 = e1 & 31;
  const uint32_t e2 = ptable_entry(sm, lj, 0, LIT_FAST, i >> L1);
  if ((int32_t)e2 < 0 || (e2 & PE_LEN) || L1 + (e2 & 31) > (uint32_t)LIT_FAST) return e1;
  const uint32_t b2 = (e2 >> 16) & 0xffu;
  return (L1 + (e2 & 31)) | (e1 & 0x00ff0000u) | ((b2 & 0x7fu) << 24) | ((b2 >> 7) ? PE_L2B7 : 0u) | PE_PAIR;
}

// Canonical table in the PAR format (kind 0 lit/len, 1 dist), same validity rules as
// build_table, built by one wave.  Returns 0 ok, 1 error, 2 empty.
__device__ __forceinline__ uint32_t build_ptable(WaveSmem &sm, const uint8_t *lens, uint32_t nsym, uint32_t kind,
                                                 uint32_t *tab, uint32_t fast, uint32_t lane) {
  const uint32_t rc = ptable_meta(sm, lens, nsym, kind, lane);
  if (rc == 1) return 1;
  __builtin_amdgcn_wave_barrier();
  uint32_t lj[16];
#pragma unroll
  for (uint32_t v = 1; v <= 15; ++v) lj[v] = sm.pk[kind][v] >> 16;
#pragma unroll 4
  for (uint32_t i = lane; i < (1u << fast); i += WAVE)
    tab[i] = kind == 0 && fast == (uint32_t)LIT_FAST ? ptable_lit_entry(sm, lj, i) : ptable_entry(sm, lj, kind, fast, i);
  __builtin_amdgcn_wave_barrier();
  return rc;
}

template <bool PAR>
__device__ __forceinline__ uint32_t build_lit(WaveSmem &sm, const uint8_t *lens, uint32_t nsym, uint32_t lane) {
  return PAR ? build_ptable(sm, lens, nsym, 0, sm.lit, LIT_FAST, lane) : build_table(sm, lens, nsym, 0, sm.lit, LIT_FAST, lane);
}
template <bool PAR>
__device__ __forceinline__ uint32_t build_dist(WaveSmem &sm, const uint8_t *lens, uint32_t nsym, uint32_t lane) {
  return PAR ? build_ptable(sm, lens, nsym, 1, sm.dist, PDIST_FAST, lane)
             : build_table(sm, lens, nsym, 1, sm.dist, DIST_FAST, lane);
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

// Wave-uniform bit reader: 32-bit scalar loads (s_load_dword through the scalar
// cache) from the compressed bytes; LSB-first 64-bit bit buffer in SGPRs.
struct Bits {
  const uint32_t *__restrict__ c32;  // dword view of the compressed shard
  uint32_t idx;                      // next dword to load (absolute index)
  uint64_t buf;
  uint32_t cnt;
  uint32_t a0;     // dword index of the first dword holding the block's deflate data
  uint32_t limit;  // bits available, relative to a0 * 32: the Inflater input ends here

  __device__ __forceinline__ void refill() {  // guarantees cnt >= 32
    if (cnt <= 32) {
      buf |= (uint64_t)c32[idx] << cnt;
      ++idx;
      cnt += 32;
    }
  }
  __device__ __forceinline__ void seek(uint32_t bitpos) {
    idx = a0 + (bitpos >> 5);
    buf = 0;
    cnt = 0;
    refill();
    const uint32_t d = bitpos & 31;
    buf >>= d;
    cnt -= d;
  }
  __device__ __forceinline__ uint32_t pos() const { return (idx - a0) * 32 - cnt; }
  __device__ __forceinline__ void drop(uint32_t n) {
    buf >>= n;
    cnt -= n;
  }
  __device__ __forceinline__ uint32_t peek(uint32_t n) const { return (uint32_t)buf & ((1u << n) - 1u); }
  __device__ __forceinline__ uint32_t take(uint32_t n) {
    const uint32_t v = peek(n);
    drop(n);
    return v;
  }
  __device__ __forceinline__ bool avail(uint32_t n) const { return pos() + n <= limit; }
};

// Tokens are gathered one per lane in a VGPR and stored 64 at a time.
struct TokOut {
  uint32_t *__restrict__ dst;  // next unstored token slot (wave-uniform)
  uint32_t batch;              // VGPR: lane k = pending token k
  uint32_t pend;               // tokens pending in batch

  __device__ __forceinline__ void emit(uint32_t t, uint32_t lane) {
    batch = lane == pend ? t : batch;
    if (++pend == WAVE) {
      dst[lane] = batch;
      dst += WAVE;
      pend = 0;
    }
  }
  __device__ __forceinline__ void drain(uint32_t lane) {
    if (lane < pend) dst[lane] = batch;
    dst += pend;
    pend = 0;
  }
};

#ifndef SBH_HOT_ASM
#define SBH_HOT_ASM 1
#endif

// The symbol hot loop in hand-written SALU code.  The compiler's structurized version
// of the same loop spends ~60 scalar instructions per symbol on phi copies; the
// scalar unit is shared by the CU's four SIMDs, so scalar instructions per symbol
// are the decoder's throughput.  Runs while a whole symbol (<= 48 bits) is
// available and a whole match fits (idx <= hot, out <= olim); exits with
//   reason 0: bound reached, or a literal/length code that is not a plain
//             literal/length in the primary table (EOB, long code, invalid): nothing
//             of that symbol consumed;
//   reason 2: length consumed (plen), its distance code needs the careful path;
//   reason 3: distance too far back (DataFormatException).
// The bit buffer may hold valid stream bits above cnt (s_load_dwordx2 refill):
// later refills OR the same bits in again.  Fixed registers s[60:81] hold the loop
// state so 64-bit pairs can be addressed by halves.
__device__ __forceinline__ void hot_loop(uint64_t &buf, uint32_t &cnt, uint32_t &idx, uint32_t &out,
                                         TokOut &to, uint32_t &reason, uint32_t &plen, const uint32_t *c32,
                                         uint32_t hot, uint32_t olim, uint32_t litb, uint32_t distb,
                                         uint32_t lane4) {
  uint64_t dst = reinterpret_cast<uint64_t>(to.dst);
  uint32_t va, ve;
  uint32_t ve2;
  asm volatile(
      "s_mov_b64 s[60:61], %[buf]\n\t"
      "s_mov_b64 s[64:65], %[c32]\n\t"
      "s_mov_b64 s[66:67], %[dst]\n\t"
      "s_mov_b32 s68, %[cnt]\n\t"
      "s_mov_b32 s69, %[idx]\n\t"
      "s_mov_b32 s70, %[hot]\n\t"
      "s_mov_b32 s71, %[out]\n\t"
      "s_mov_b32 s72, %[olim]\n\t"
      "s_mov_b32 s81, m0\n\t"
      "s_add_u32 m0, %[pend], 0xffffffc0\n\t"  // pending count - 64: carry out at 64 tokens
      "s_mov_b32 s74, %[litb]\n\t"
      "s_mov_b32 s75, %[distb]\n\t"
      "s_mov_b32 s79, 0\n\t"
      "s_mov_b32 s80, 0\n"
      "L_top%=:\n\t"
      "s_cmp_gt_u32 s71, s72\n\t"  // out > olim: a match might not fit
      "s_cbranch_scc1 L_exit%=\n\t"
      "s_cmp_gt_u32 s68, 32\n\t"
      "s_cbranch_scc1 L_lit%=\n\t"
      "s_cmp_gt_u32 s69, s70\n\t"  // idx > hot: the next symbol may cross the input end
      "s_cbranch_scc1 L_exit%=\n\t"
      "s_lshl_b32 s77, s69, 2\n\t"
      "s_load_dwordx2 s[62:63], s[64:65], s77\n\t"
      "s_add_u32 s69, s69, 1\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_lshl_b64 s[62:63], s[62:63], s68\n\t"
      "s_or_b64 s[60:61], s[60:61], s[62:63]\n\t"
      "s_add_u32 s68, s68, 32\n"
      "L_lit%=:\n\t"
      "v_bfe_u32 %[va], s60, 0, %[lbits]\n\t"
      "v_lshl_add_u32 %[va], %[va], 2, s74\n\t"
      "ds_read_b32 %[ve], %[va]\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_nop 0\n\t"
      "v_readfirstlane_b32 s76, %[ve]\n\t"
      "s_and_b32 s77, s76, 31\n\t"
      "s_and_b32 s78, s76, 0xe0\n\t"
      "s_cbranch_scc1 L_nonlit%=\n\t"
      // literal: the entry is the token
      "s_lshr_b64 s[60:61], s[60:61], s77\n\t"
      "s_sub_u32 s68, s68, s77\n\t"
      "v_writelane_b32 %[batch], s76, m0\n\t"
      "s_add_u32 s71, s71, 1\n\t"
      "s_add_u32 m0, m0, 1\n\t"
      "s_cbranch_scc0 L_top%=\n"
      "L_store%=:\n\t"
      "global_store_dword %[lane4], %[batch], s[66:67]\n\t"
      "s_add_u32 s66, s66, 256\n\t"
      "s_addc_u32 s67, s67, 0\n\t"
      "s_mov_b32 m0, 0xffffffc0\n\t"
      "s_branch L_top%=\n"
      "L_nonlit%=:\n\t"
      "s_cmp_eq_u32 s78, 0x20\n\t"
      "s_cbranch_scc0 L_exit%=\n\t"
      // length: extra bits straight from the entry (offset L, width lx), then drop L + lx
      "s_bfe_u32 s78, s60, s76\n\t"
      "s_lshr_b32 s80, s76, 23\n\t"
      "s_add_u32 s80, s80, s78\n\t"
      "s_bfe_u32 s77, s76, 0x80008\n\t"
      "s_lshr_b64 s[60:61], s[60:61], s77\n\t"
      "s_sub_u32 s68, s68, s77\n\t"
      "s_cmp_gt_u32 s68, 32\n\t"
      "s_cbranch_scc1 L_dist%=\n\t"
      "s_lshl_b32 s77, s69, 2\n\t"
      "s_load_dwordx2 s[62:63], s[64:65], s77\n\t"
      "s_add_u32 s69, s69, 1\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_lshl_b64 s[62:63], s[62:63], s68\n\t"
      "s_or_b64 s[60:61], s[60:61], s[62:63]\n\t"
      "s_add_u32 s68, s68, 32\n\t"
      "s_cmp_gt_u32 s69, s70\n\t"  // past hot: finish this match, leave at the top
      "s_cselect_b32 s72, 0, s72\n"
      "L_dist%=:\n\t"
      "v_bfe_u32 %[va], s60, 0, %[dbits]\n\t"
      "v_lshl_add_u32 %[va], %[va], 3, s75\n\t"
      "ds_read_b32 %[ve], %[va]\n\t"
      "ds_read_b32 %[ve2], %[va] offset:4\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_nop 0\n\t"
      "v_readfirstlane_b32 s76, %[ve]\n\t"
      "v_readfirstlane_b32 s82, %[ve2]\n\t"
      "s_cmp_lt_i32 s76, 0\n\t"  // bit 31: a decoded distance
      "s_cbranch_scc0 L_pend%=\n\t"
      "s_bfe_u32 s78, s60, s76\n\t"
      "s_add_u32 s78, s82, s78\n\t"
      "s_bfe_u32 s77, s76, 0x80008\n\t"
      "s_lshr_b64 s[60:61], s[60:61], s77\n\t"
      "s_sub_u32 s68, s68, s77\n\t"
      "s_cmp_gt_u32 s78, s71\n\t"
      "s_cbranch_scc1 L_far%=\n\t"
      "s_lshl_b32 s77, s80, 16\n\t"
      "s_or_b32 s77, s77, s78\n\t"
      "s_bitset1_b32 s77, 31\n\t"
      "v_writelane_b32 %[batch], s77, m0\n\t"
      "s_add_u32 s71, s71, s80\n\t"
      "s_add_u32 m0, m0, 1\n\t"
      "s_cbranch_scc0 L_top%=\n\t"
      "s_branch L_store%=\n"
      "L_pend%=:\n\t"
      "s_mov_b32 s79, 2\n\t"
      "s_branch L_exit%=\n"
      "L_far%=:\n\t"
      "s_mov_b32 s79, 3\n"
      "L_exit%=:\n\t"
      "s_mov_b64 %[buf], s[60:61]\n\t"
      "s_mov_b64 %[dst], s[66:67]\n\t"
      "s_mov_b32 %[cnt], s68\n\t"
      "s_mov_b32 %[idx], s69\n\t"
      "s_mov_b32 %[out], s71\n\t"
      "s_add_u32 %[pend], m0, 64\n\t"
      "s_mov_b32 m0, s81\n\t"
      "s_mov_b32 %[reason], s79\n\t"
      "s_mov_b32 %[plen], s80\n\t"
      : [buf] "+s"(buf), [dst] "+s"(dst), [cnt] "+s"(cnt), [idx] "+s"(idx), [out] "+s"(out),
        [pend] "+s"(to.pend), [reason] "=s"(reason), [plen] "=s"(plen), [batch] "+v"(to.batch),
        [va] "=&v"(va), [ve] "=&v"(ve), [ve2] "=&v"(ve2)
      : [c32] "s"(c32), [hot] "s"(hot), [olim] "s"(olim), [litb] "s"(litb), [distb] "s"(distb),
        [lane4] "v"(lane4), [lbits] "i"(LIT_FAST), [dbits] "i"(DIST_FAST)
      : "memory", "scc", "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71",
        "s72", "s74", "s75", "s76", "s77", "s78", "s79", "s80", "s81", "s82");
  to.dst = reinterpret_cast<uint32_t *>(dst);
}

// Tables of a fixed (type 1) or dynamic (type 2) deflate block, read at br (just after
// the 3 block-header bits) and built in sm.  Wave-uniform; follows zlib inflate's
// TABLE / LENLENS / CODELENS states.  RT_STOP: the input ends inside the header (zlib
// waits for more input, so the block ends short); RT_ERR: DataFormatException.
constexpr uint32_t RT_OK = 0, RT_STOP = 1, RT_ERR = 2;

template <bool PAR>
__device__ __forceinline__ uint32_t read_tables(WaveSmem &sm, Bits &br, uint32_t type, bool &fixed_built,
                                                uint32_t lane) {
  if (type == 1) {
    if (!fixed_built) {
      for (uint32_t s = lane; s < 288; s += WAVE) sm.lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
      if (lane < 32) sm.lens[288 + lane] = 5;
      __builtin_amdgcn_wave_barrier();
      build_lit<PAR>(sm, sm.lens, 288, lane);
      build_dist<PAR>(sm, sm.lens + 288, 32, lane);
      fixed_built = true;
    }
    return RT_OK;
  }
  fixed_built = false;
  br.refill();
  if (!br.avail(14)) return RT_STOP;
  const uint32_t nlen = br.take(5) + 257, ndist = br.take(5) + 1, ncode = br.take(4) + 4;
  if (nlen > 286 || ndist > 30) return RT_ERR;
  if (!br.avail(ncode * 3)) return RT_STOP;
  if (lane < 20) sm.cl_lens[lane] = 0;
  __builtin_amdgcn_wave_barrier();
  for (uint32_t i = 0; i < ncode; ++i) {
    br.refill();
    const uint32_t v = br.take(3);
    if (lane == 0) sm.cl_lens[CL_ORDER[i]] = (uint8_t)v;
  }
  __builtin_amdgcn_wave_barrier();
  const uint32_t rc = uni(build_table(sm, sm.cl_lens, 19, 2, sm.lit, CL_FAST, lane));
  if (rc == 1) return RT_ERR;
  const uint32_t total = nlen + ndist;
  if (rc == 2) return br.avail(total) ? RT_ERR : RT_STOP;  // no code-length codes: each decodes as 0 (1 bit), then fails
  uint32_t i = 0, prevlen = 0;
  while (i < total) {
    br.refill();
    const uint32_t e = uni(sm.lit[br.peek(CL_FAST)]);
    const uint32_t L = e & 31;
    if (!br.avail(L)) return RT_STOP;
    br.drop(L);
    const uint32_t sym = (e >> 8) & 0xff;
    if (sym < 16) {
      if (lane == 0) sm.lens[i] = (uint8_t)sym;
      prevlen = sym;
      ++i;
      continue;
    }
    uint32_t rep, val;
    if (sym == 16) {
      if (i == 0) return RT_ERR;
      if (!br.avail(2)) return RT_STOP;
      rep = 3 + br.take(2);
      val = prevlen;
    } else if (sym == 17) {
      if (!br.avail(3)) return RT_STOP;
      rep = 3 + br.take(3);
      val = 0;
    } else {
      if (!br.avail(7)) return RT_STOP;
      rep = 11 + br.take(7);
      val = 0;
    }
    if (i + rep > total) return RT_ERR;
    for (uint32_t k = lane; k < rep; k += WAVE) sm.lens[i + k] = (uint8_t)val;
    prevlen = val;
    i += rep;
  }
  __builtin_amdgcn_wave_barrier();
  // split: lit lens [0,nlen) (+zeros to 288); dist lens -> [288, 288+ndist)
  const uint32_t dv = lane < ndist ? sm.lens[nlen + lane] : 0;
  __builtin_amdgcn_wave_barrier();
  for (uint32_t s = nlen + lane; s < 288; s += WAVE) sm.lens[s] = 0;
  __builtin_amdgcn_wave_barrier();
  if (lane < 32) sm.lens[288 + lane] = (uint8_t)dv;
  __builtin_amdgcn_wave_barrier();
  if (uni(sm.lens[256]) == 0) return RT_ERR;  // missing end-of-block
  if (uni(build_lit<PAR>(sm, sm.lens, nlen, lane)) == 1) return RT_ERR;
  if (uni(build_dist<PAR>(sm, sm.lens + 288, ndist, lane)) == 1) return RT_ERR;
  return RT_OK;
}

// Exact serial decode of block b by one wave (zlib semantics everywhere: stored blocks,
// long codes, every input/output edge, every error).  The lane-parallel k_huff falls
// back to it for any block its fast path does not prove well-formed.
__device__ __forceinline__ void inflate_serial(const uint8_t *__restrict__ comp, const DevBlocks &bl, uint64_t b,
                                            uint32_t *__restrict__ tok, WaveSmem &sm, uint32_t lane) {
  const uint64_t cstart = bl.cstart[b];
  const uint32_t csize = bl.csize[b], hsize = bl.hsize[b], usize = bl.usize[b];
  const uint64_t G = bl.ustart[b];
  const uint32_t bflags = bl.flags[b];
  uint32_t early = INF_OK;
  if (bflags & BLK_TRUNCATED) early = INF_SIZE;
  else if (usize > 65536u) early = INF_BAD_ISIZE;
  else if ((int32_t)csize - (int32_t)hsize - 8 < 0) early = INF_DATA;
  if (early != INF_OK) {
    if (lane == 0) {
      bl.status[b] = early;
      bl.ntok[b] = 0;
    }
    return;
  }
  const uint32_t data_len = csize - hsize - 8;

  Bits br;
  const uint64_t dbyte = cstart + hsize;
  // dword indices are relative to the block's first deflate dword (a 32-bit index into
  // the whole shard would wrap past 16 GiB of compressed bytes)
  br.c32 = reinterpret_cast<const uint32_t *>(comp + (dbyte & ~3ull));
  br.a0 = 0;
  const uint32_t skip = (uint32_t)(dbyte & 3) * 8;
  br.limit = skip + data_len * 8;
  br.seek(skip);
  // the hot loop needs no per-symbol input check while a whole symbol (<= 48 bits)
  // is guaranteed to be available: (idx - a0) * 32 + 48 <= limit
  const uint32_t hot_idx = br.limit >= 48 ? br.a0 + (br.limit - 48) / 32 : 0;

  TokOut to;
  to.dst = tok + G;
  to.batch = 0;
  to.pend = 0;
  const uint32_t lit_lds = (uint32_t)reinterpret_cast<uintptr_t>(sm.lit);
  const uint32_t dist_lds = (uint32_t)reinterpret_cast<uintptr_t>(sm.dist);
  const uint32_t olim = usize >= 258 ? usize - 258 : 0;

  uint32_t out = 0;  // bytes produced
  uint32_t status = INF_OK;
  bool fixed_built = false;
  bool last = false;
  bool done = false;

  while (!done) {  // deflate blocks inside the BGZF block
    br.refill();
    if (!br.avail(3)) break;  // needs input: stop
    last = br.take(1);
    const uint32_t type = br.take(2);
    if (type == 0) {
      // stored block: byte-align, LEN, NLEN; bytes become literal tokens
      br.drop((8 - (br.pos() & 7)) & 7);
      br.refill();
      if (!br.avail(32)) break;
      const uint32_t len = br.take(16), nlen = br.take(16);
      if (len != (~nlen & 0xffffu)) { status = INF_DATA; break; }
      const uint32_t p0 = br.pos();
      const uint32_t avail_bytes = (br.limit - p0) >> 3;
      uint32_t n = len;
      if (n > avail_bytes) n = avail_bytes;
      if (n > usize - out) n = usize - out;
      const uint8_t *src = reinterpret_cast<const uint8_t *>(br.c32) + (p0 >> 3);
      to.drain(lane);
      for (uint32_t i = lane; i < n; i += WAVE) to.dst[i] = (uint32_t)src[i] << 8;  // literal tokens
      to.dst += n;
      out += n;
      if (n < len) break;  // output full or input exhausted
      br.seek(p0 + len * 8);
      if (last) break;
      continue;
    }
    if (type == 3) { status = INF_DATA; break; }  // invalid block type
    const uint32_t rt = read_tables<false>(sm, br, type, fixed_built, lane);
    if (rt == RT_STOP) break;
    if (rt == RT_ERR) { status = INF_DATA; break; }

    // ---- symbols ----
    for (;;) {
      uint32_t mlen = 0;
      bool have_len = false;
#if SBH_HOT_ASM
      if (usize >= 258 && br.idx <= hot_idx) {
        uint32_t reason, plen;
        hot_loop(br.buf, br.cnt, br.idx, out, to, reason, plen, br.c32, uni(hot_idx), uni(olim), uni(lit_lds), uni(dist_lds),
                 lane * 4);
        if (reason == 3) { status = INF_DATA; done = true; break; }  // too far back
        if (reason == 2) {
          mlen = plen;
          have_len = true;
        }
      }
#else
      // C++ hot loop (A/B reference for the asm one): no input/output bound checks
      // while a whole symbol is available and a whole match fits
      while (br.idx <= hot_idx && out + 258 <= usize) {
        br.refill();
        const uint32_t e = uni(sm.lit[(uint32_t)br.buf & ((1u << LIT_FAST) - 1)]);
        const uint32_t kind = (e >> 5) & 7;
        if (kind == K_LIT) {
          br.drop(e & 31);
          to.emit(e, lane);
          ++out;
        } else if (kind == K_LEN) {
          br.drop(e & 31);
          const uint32_t ml = len_base(e) + br.take(len_extra(e));
          br.refill();
          uint32_t d = uni(sm.dist[2 * ((uint32_t)br.buf & ((1u << DIST_FAST) - 1))]);
          if (((d >> 5) & 7) != K_DIST) {
            mlen = ml;
            have_len = true;
            break;
          }
          br.drop(d & 31);
          const uint32_t dist = dist_base(d) + br.take(len_extra(d));
          if (dist > out) { status = INF_DATA; done = true; break; }  // too far back
          to.emit(TOK_MATCH | (ml << 16) | dist, lane);
          out += ml;
        } else {
          break;
        }
      }
      if (done) break;
#endif
      // careful path: one symbol with every bound checked (zlib semantics at the edges)
      if (!have_len) {
        br.refill();
        uint32_t e = uni(sm.lit[br.peek(LIT_FAST)]);
        uint32_t kind = (e >> 5) & 7;
        if (kind == K_SLOW) {
          e = uni(slow_decode(sm, br.buf, 0));
          kind = (e >> 5) & 7;
        }
        const uint32_t L = e & 31;
        if (kind == K_BAD) {
          if (br.avail(1)) status = INF_DATA;
          done = true;
          break;
        }
        if (!br.avail(L)) { done = true; break; }
        br.drop(L);
        if (kind == K_LIT) {
          if (out == usize) { done = true; break; }
          to.emit(e, lane);
          ++out;
          continue;
        }
        if (kind == K_EOB) break;
        const uint32_t lx = len_extra(e);
        if (!br.avail(lx)) { done = true; break; }
        mlen = len_base(e) + br.take(lx);
      }
      br.refill();
      uint32_t d = uni(sm.dist[2 * br.peek(DIST_FAST)]);
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
      const uint32_t dx = len_extra(d);
      if (!br.avail(dx)) { done = true; break; }
      const uint32_t dist = dist_base(d) + br.take(dx);
      if (out == usize) { done = true; break; }  // zlib stops at MATCH when full
      if (dist > out) { status = INF_DATA; done = true; break; }  // too far back
      const uint32_t n = mlen < usize - out ? mlen : usize - out;
      to.emit(TOK_MATCH | (n << 16) | dist, lane);
      out += n;
      if (n < mlen) { done = true; break; }  // output full mid-match
    }
    if (done || last) break;
  }
  to.drain(lane);
  if (status == INF_OK && out != usize) status = INF_SIZE;
  if (lane == 0) {
    bl.status[b] = status;
    bl.ntok[b] = (uint32_t)(to.dst - (tok + G));
  }
}

// Serial decoder kernel: one wave per block.  As the A/B baseline it decodes every block
// (SBH_HUFF_SERIAL); behind the lane-parallel k_huff it decodes only the blocks k_huff
// marked INF_SERIAL.
template <bool ONLY_MARKED>
__global__ __launch_bounds__(WAVES *WAVE) void k_huff_serial(const uint8_t *__restrict__ comp, DevBlocks bl,
                                                              uint64_t nblocks, uint32_t *__restrict__ tok) {
  __shared__ WaveSmem smem[WAVES];
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  const uint32_t wid = uni(threadIdx.x / WAVE);
  const uint64_t b = (uint64_t)blockIdx.x * WAVES + wid;
  if (b >= nblocks) return;
  if (ONLY_MARKED && uni(bl.status[b]) != INF_SERIAL) return;
  inflate_serial(comp, bl, b, tok, smem[wid], lane);
}

// Block-wide exclusive prefix sum over NT threads; *total gets the sum.  wsum: NT/64 words.
template <uint32_t NT>
__device__ __forceinline__ uint32_t block_scan(uint32_t v, uint32_t *wsum, uint32_t *total) {
  // (the wave index through readfirstlane: uniform, so the sums below are scalar work)
  const uint32_t lane = threadIdx.x & (WAVE - 1), w = uni(threadIdx.x / WAVE);
  const uint32_t x = wave_incl_scan(v);
  if (lane == WAVE - 1) wsum[w] = x;
  __syncthreads();
  uint32_t before = 0, all = 0;
#pragma unroll
  for (uint32_t k = 0; k < NT / WAVE; ++k) {
    const uint32_t s = wsum[k];
    before += k < w ? s : 0;
    all += s;
  }
  *total = all;
  return before + x - v;
}

// Block-wide minimum over NT threads (all threads get it).  wmin: NT/64 words, not
// read or written by anything else between two calls' barriers.
template <uint32_t NT>
__device__ __forceinline__ uint32_t block_min(uint32_t v, uint32_t *wmin) {
  const uint32_t lane = threadIdx.x & (WAVE - 1), w = uni(threadIdx.x / WAVE);
#pragma unroll
  for (uint32_t off = WAVE / 2; off > 0; off >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, (int)off, WAVE));
  if (lane == 0) wmin[w] = v;
  __syncthreads();
  uint32_t m = ~0u;
#pragma unroll
  for (uint32_t k = 0; k < NT / WAVE; ++k) m = min(m, wmin[k]);
  return m;
}

// ---------------------------------------------------------------------------------
// Lane-parallel Huffman decode (the k_huff fast path).
//
// A deflate block's symbol stream is serial only through its bit positions: decoding
// from a codeword boundary is deterministic, and Huffman/DEFLATE decoding
// self-synchronises -- a decode started at an arbitrary bit soon falls onto the true
// codeword boundaries.  So the HT lanes of the workgroup each take an equal slice of
// the bits, decode speculatively from the slice start to the first token boundary at or
// past the next slice (its exit), and then repair: a lane whose start differs from its
// left neighbour's exit redoes its slice from that exit, until no exit changes (round r
// fixes lane r at the latest; in practice one or two rounds).  The first lane whose
// chain ends (EOB, invalid code, input end) decides the deflate block; a prefix sum over
// the lanes' token/byte counts places every lane's tokens, and a third pass emits them
// and checks distances against the bytes produced so far.  Anything the fast path does
// not prove well-formed (stored blocks, an invalid code or too-far-back distance on the
// true chain, a stream that ends short/long, input end inside a symbol) falls back to
// the exact serial decoder above, so block status and tokens always equal zlib's.
// ---------------------------------------------------------------------------------
#ifndef SBH_HT
#define SBH_HT 256
#endif
#ifndef SBH_STAGE_DW
#define SBH_STAGE_DW 6144
#endif
#ifndef SBH_HUFF_OCC
#define SBH_HUFF_OCC 4  // waves per SIMD the register budget must allow
#endif
constexpr uint32_t HT = SBH_HT;              // k_huff lanes per BGZF block
constexpr uint32_t STAGE_DW = SBH_STAGE_DW;  // deflate bytes staged in LDS (24 KiB)
constexpr uint32_t PAR_MIN_USIZE = 4096;     // smaller blocks decode serially
#ifndef SBH_MIN_SLICE
#define SBH_MIN_SLICE 128
#endif
constexpr uint32_t MIN_SLICE = SBH_MIN_SLICE;  // bits per lane at least
constexpr uint32_t NOPOS = 0xffffffffu;
// k_hdr's output, at the end of a block's token region (dwords)
constexpr uint32_t HDR_SENT = (1u << LIT_FAST) + (1u << PDIST_FAST);  // after the PAR tables
constexpr uint32_t HDR_PK = HDR_SENT + 320;
constexpr uint32_t HDR_PSYM = HDR_PK + 32, HDR_LAST = HDR_PSYM + 1, HDR_STATUS = HDR_PSYM + 2;
constexpr uint32_t HDR_OUT_DW = HDR_PSYM + 4;
constexpr uint32_t HDR_OK = 0x48445231u;
constexpr uint32_t HDR_STAGE_DW = 160;  // deflate dwords k_hdr stages (a header is < 2.5 kbit)
static_assert(HDR_OUT_DW < PAR_MIN_USIZE, "the header record fits the token region of every parallel block");
static_assert(HDR_SENT % SBH_HT == 0, "k_huff copies the tables in whole rounds");
#ifndef SBH_CK1  // (A/B at 4 M records: 4/16, 6/24, 8/32, 10/40 within 2%)
#define SBH_CK1 8
#define SBH_CK2 32
#endif
#ifndef SBH_CK3
#define SBH_CK3 64
#endif
#ifndef SBH_MARGIN
#define SBH_MARGIN 0  // pass-1 warm-up bits before each slice (A/B: 128-384 bits measured neutral)
#endif
constexpr uint32_t CK1 = SBH_CK1, CK2 = SBH_CK2;  // pass-1 checkpoints (tokens)
constexpr uint32_t CK3 = SBH_CK3;                 // a third, for chains that sync late (0: none)
constexpr uint32_t LR_RUN = 0, LR_EOB = 1, LR_DEAD = 2, LR_PAST = 3;
#ifndef SBH_TAIL
#define SBH_TAIL 1  // short final deflate blocks left to k_huff_tail (0: k_huff decodes them)
#endif
constexpr uint32_t INF_TAIL = 0xfeu;  // (inside inflate only) k_huff_tail finishes the block
#ifdef SBH_HUFF_PROBE
// whole-kernel phase sums (cycles): 0 stage, 1 header, 2 pass 1, 3 repair, 4 emit, 5 repair
// rounds, 6 deflate blocks, 7 whole block, 8-10 header: CL table / walk / tables, 11 tokens
__device__ unsigned long long hp_acc[16];  // [14]: blocks timed
__device__ unsigned int hp_done;
#endif
template <uint32_t NT_, uint32_t SDW_>
struct HuffSmemT {
  static constexpr uint32_t NT = NT_, SDW = SDW_;
  WaveSmem t;               // tables (built by wave 0; the serial fallback's too)
  uint32_t stage[SDW + 8];  // the block's deflate dwords, from dword a0
  uint32_t exitv[NT];       // lane exits (NOPOS: the chain ended in the lane)
  uint32_t exitv2[NT];      // (the repair rounds alternate between the two)
  uint32_t wsum[NT / WAVE];
  uint32_t wsum2[NT / WAVE];
  uint32_t wk[NT / WAVE], wkt[NT / WAVE], wko[NT / WAVE], wke[NT / WAVE];  // per wave: first ended lane
  uint32_t ctl[8];
};
using HuffSmem = HuffSmemT<HT, STAGE_DW>;

// Bit source of a lane: the LDS stage or (blocks too large to stage) global memory.
template <bool LDS, uint32_t SDW = STAGE_DW>
struct Src {
  const uint32_t *p;
  __device__ __forceinline__ uint32_t operator()(uint32_t i) const {
    if (LDS) return p[i < SDW + 7 ? i : SDW + 7];
    return p[i];
  }
  // the dword at byte offset b (4-aligned; callers keep it inside the staged dwords)
  __device__ __forceinline__ uint32_t at_byte(uint32_t b) const {
    return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(p) + b);
  }
  // 32 stream bits starting at bit position `pos`
  // (no clamp: a lane never reads past dword (limit + 48) / 32 + 1, and staged blocks
  // leave that much of the STAGE_DW + 8 array)
  __device__ __forceinline__ uint32_t bits32(uint32_t pos) const {
    const uint32_t i = pos >> 5;
    return __builtin_amdgcn_alignbit(p[i + 1], p[i], pos & 31);
  }
};

// Long codes (> the table's bits) in the PAR format, decoded by left-justified limits:
// the length is one more than the number of lengths whose limit lies at or below the
// code, and the entry sits at sent[dl[len] + code].  lj/dl of lengths 10..15 are read
// together as packed (lj << 16 | dl) words, so a long code costs two LDS round trips.
__device__ __forceinline__ uint32_t slow_lane(const WaveSmem &sm, uint32_t bits, bool dist) {
  static_assert(LIT_FAST == 10 && PDIST_FAST == 10, "long codes are lengths 11..15");
  const uint32_t rev15 = __builtin_bitreverse32(bits) >> 17;
  const uint32_t *pk = sm.pk[dist ? 1 : 0];
  uint32_t len = 11, d = pk[11] & 0xffffu;
#pragma unroll
  for (uint32_t v = 12; v <= 15; ++v) {
    const uint32_t below = pk[v - 1], here = pk[v];
    if ((below >> 16) <= rev15) {
      len = v;
      d = here & 0xffffu;
    }
  }
  if (rev15 >= (pk[15] >> 16)) return 1u | PE_SPECIAL;
  return sm.sent[(dist ? 288 : 0) + ((d + (rev15 >> (15 - len))) & 0xffffu)];
}

struct LaneRun {
  uint32_t st;    // LR_*
  uint32_t exit;  // RUN: first token boundary >= stop; EOB: bit after the EOB code
  uint32_t ntok;  // tokens (EOB excluded)
  uint32_t nout;  // bytes
};

// Checkpoints of a lane's pass-1 chain: the boundaries after CK1, CK2 and CK3 tokens and
// the bytes produced up to them.  A repair run that lands on one of them has joined
// that chain, so the rest of the pass-1 result holds.  (A chain that synchronises with the
// true one only after CK2 tokens would otherwise be redone to its slice end, and the
// slowest lane of a wave sets the repair round's time.)
struct Ckpt {
  uint32_t p1, o1, p2, o2, p3, o3;
};
constexpr int RUN_SPEC = 0, RUN_REDO = 1, RUN_EMIT = 2;

// The bytes up to the checkpoint a redo joined, as register selects: written as
// `one ? ck.o1 : two ? ck.o2 : ck.o3` the compiler turned the select of fields into a select
// of addresses, kept the checkpoints in scratch and read them back with a scratch load.
__device__ __forceinline__ uint32_t ck_out(const Ckpt &ck, bool one, bool two) {
  uint32_t o1 = ck.o1, o2 = ck.o2, o3 = ck.o3;
  asm volatile("" : "+v"(o1), "+v"(o2), "+v"(o3));
  return one ? o1 : two ? o2 : o3;
}

// Decode tokens from bit A while the position is below `stop`, as a two-state machine
// (literal/length code, then distance code) so every lane runs the same instructions:
// one table lookup per code, the extra bits taken straight from the entry.
//   RUN_SPEC: record checkpoints in ck.
//   RUN_REDO: stop early on reaching one of ck's boundaries (sp: that chain's result).
//   RUN_EMIT: store tokens at dst, flag a distance reaching before the block's first
//             byte (out0: bytes before A).
// k_huff's passes are bound by VALU issue (each SIMD issues VALU on ~80% of its cycles at 4
// waves: r03n PMC), so the loop is written for few vector instructions per code:
//  * the decode state is the bit position and the two stream dwords under it (lo, hi): a
//    code's 32 bits come from them with one v_alignbit, enough for any code plus its extra
//    bits (<= 28); a code consumes < 32 bits, so the window moves by at most one dword per
//    code, and the dword after it is loaded at the top of every iteration beside the table
//    lookup (its byte address straight from the position: no dword index to maintain);
//  * `tsel` (0, or PE_LEN = the distance table's byte offset) is both the table select and
//    the state; a token is counted at its first code (a match at its length code), and the
//    bytes as acc = 4096 * sum(match length - 1), one v_mad_u32_u24 per code -- both equal
//    the per-token counts at every token boundary, where they are read;
//  * one sign test per code catches every special entry (EOB, invalid, long code);
//  * checkpoint recording and the loop exit are branches (scalar ops, off the VALU).
template <int MODE, class S>
__device__ __forceinline__ LaneRun lane_run(const WaveSmem &t, S src, uint32_t A, uint32_t stop,
                                            uint32_t limit, Ckpt &ck, const LaneRun &sp,
                                            uint32_t *__restrict__ dst, uint32_t out0, uint32_t &bad) {
  const uint32_t stop2 = stop < limit ? stop : limit;
  if (MODE == RUN_SPEC) ck = Ckpt{NOPOS, 0, NOPOS, 0, NOPOS, 0};
  // a lane starting at or past its stop ends there (a slice past the stream's end; its
  // stream reads would leave the stage)
  if (A >= stop2) return LaneRun{A >= limit ? LR_PAST : LR_RUN, A, 0, 0};
  const char *tab = reinterpret_cast<const char *>(t.tab);
  uint32_t pos = A;
  uint32_t lo = src((pos >> 5)), hi = src((pos >> 5) + 1);
  uint32_t tsel = 0;             // 0: at a token boundary (literal/length table); PE_LEN: a distance follows
  uint32_t ntok = 0, acc = 0;    // tokens started; 4096 * sum over matches of (length - 1)
  uint32_t ml = 0;               // RUN_EMIT: the pending match's length - 1
  uint32_t c1p = NOPOS, c1o = 0, c2p = NOPOS, c2o = 0, c3p = NOPOS, c3o = 0;
  uint32_t ck_next = CK1;  // RUN_SPEC: token count of the next checkpoint
  uint32_t e;
  bool cut;
  for (;;) {
    const uint32_t bits = __builtin_amdgcn_alignbit(hi, lo, pos);
    const uint32_t nx = src.at_byte(((pos >> 3) & ~3u) + 8);  // dword (pos >> 5) + 2
    e = *reinterpret_cast<const uint32_t *>(tab + (((bits & ((1u << LIT_FAST) - 1)) << 2) | tsel));
    bool special = (int32_t)e < 0;
    if (special && (e & PE_SLOW)) {  // rare: a code longer than the table
      e = slow_lane(t, bits, tsel != 0);
      special = (int32_t)e < 0;
    }
    const bool atb = tsel == 0;  // token boundary
    if (MODE == RUN_SPEC && atb && ntok == ck_next) {  // rare: a branch, not per-code selects
      // shift register: the newest checkpoint in c1 (the order is restored after the loop)
      c3p = c2p;
      c3o = c2o;
      c2p = c1p;
      c2o = c1o;
      c1p = pos;
      c1o = ntok + (acc >> 12);
      ck_next = ck_next == CK1 ? CK2 : ck_next == CK2 && CK3 > CK2 ? CK3 : ~0u;
    }
    cut = atb && (pos >= stop2 || (MODE == RUN_REDO && (pos == ck.p1 || pos == ck.p2 || pos == ck.p3)));
    if (cut || special) break;
    const uint32_t L = e & 31, x = __builtin_amdgcn_ubfe(e, 5, 4);
    const uint32_t val = (e >> 16) + __builtin_amdgcn_ubfe(bits, e, x);  // (offset: e's low 5 bits = L)
    const uint32_t np = pos + L + x;
    const bool adv = (np ^ pos) >= 32u;
    pos = np;
    lo = adv ? hi : lo;
    hi = adv ? nx : hi;
    const uint32_t tnew = e & PE_LEN;
    if (MODE == RUN_EMIT) {
      if (atb && !tnew) {
        dst[ntok] = (val << 8) | ((e & (PE_L2B7 | PE_PAIR)) << 14);  // a literal (or a pair: TOK_PAIR)
      } else if (!atb) {       // a distance completing a match (started at token ntok - 1)
        dst[ntok - 1] = TOK_MATCH | ((ml + 1) << 16) | val;
        // bytes before the match: out0 + tokens before it + the earlier matches' extra bytes
        bad |= val > out0 + ntok - 1 + ((acc >> 12) - ml) ? 1u : 0u;
      }
      ml = tnew ? val : ml;
    }
    ntok += atb ? 1u : 0u;
    acc += (uint32_t)__umul24(tnew, val);  // (tnew: 0 or 4096; one v_mad_u32_u24)
    acc += (e & PE_PAIR) << 2;              // a literal pair: one byte more than its token
    tsel = tnew;
  }
  if (MODE == RUN_SPEC) {  // oldest first: CK1's boundary in p1
    const uint32_t nck = ck_next == CK1 ? 0u : ck_next == CK2 ? 1u : ck_next == CK3 && CK3 > CK2 ? 2u : CK3 > CK2 ? 3u : 2u;
    ck = nck == 3 ? Ckpt{c3p, c3o, c2p, c2o, c1p, c1o}
       : nck == 2 ? Ckpt{c2p, c2o, c1p, c1o, NOPOS, 0}
       : nck == 1 ? Ckpt{c1p, c1o, NOPOS, 0, NOPOS, 0}
                  : Ckpt{NOPOS, 0, NOPOS, 0, NOPOS, 0};
  }
  const uint32_t nout = ntok + (acc >> 12);
  LaneRun r{LR_RUN, pos, ntok, nout};
  if (cut) {
    if (MODE == RUN_REDO && pos < stop2) {  // joined the pass-1 chain at a checkpoint
      const bool one = pos == ck.p1;
      const bool two = pos == ck.p2;
      r.ntok += sp.ntok - (one ? CK1 : two ? CK2 : CK3);
      r.nout += sp.nout - ck_out(ck, one, two);
      r.st = sp.st;
      r.exit = sp.exit;
    } else if (pos >= limit) {
      r.st = LR_PAST;
    }
  } else {  // end of block, or an invalid code
    r.st = (tsel == 0 && (e & PE_EOB)) ? LR_EOB : LR_DEAD;
    r.exit = pos + (e & 31);
  }
  return r;
}

#ifndef SBH_ASM_SPEC
#define SBH_ASM_SPEC 1  // pass 1 (RUN_SPEC over the LDS stage) as the hand-written loop below
#endif
// RUN_SPEC over the LDS stage as hand-written code: lane_run<RUN_SPEC>'s loop with the same
// results, in ~33 instructions per code instead of the compiler's ~57 (whose structurized loop
// spends ~25 scalar instructions per code on exit masks and phi copies, and waves of k_huff
// wait on their own issue: PMC r03n, 32% of wave cycles issuing, 54% parked).  Per code: the
// entry's LDS address from the stream bits, the next stream dword beside it; the token-boundary,
// checkpoint and cut tests as lane masks while the entry is in flight; lanes that reach their
// cut or a special entry leave the loop (exec shrinks) with their state as it was; long codes
// (> LIT_FAST bits) resolve in place through the PAR limits (slow_lane's arithmetic).  The
// checkpoints go into a shift register (newest in c1), reordered after the loop.
static_assert(CK1 == 8 && CK2 == 32 && CK3 == 64, "the asm pass-1 loop hard-codes the checkpoint schedule");
static_assert(LIT_FAST == 10 && PDIST_FAST == 10, "the asm pass-1 loop indexes 10-bit tables");
__device__ __forceinline__ LaneRun spec_asm(const WaveSmem &t, const uint32_t *stage, uint32_t A, uint32_t stop,
                                            uint32_t limit, Ckpt &ck) {
  const uint32_t stop2 = stop < limit ? stop : limit;
  ck = Ckpt{NOPOS, 0, NOPOS, 0, NOPOS, 0};
  if (A >= stop2) return LaneRun{A >= limit ? LR_PAST : LR_RUN, A, 0, 0};
  const uint32_t tabb = uni((uint32_t)reinterpret_cast<uintptr_t>(t.tab));
  const uint32_t stb = uni((uint32_t)reinterpret_cast<uintptr_t>(stage) + 8u);  // + dword 2 of the window
  const uint32_t pkb = uni((uint32_t)reinterpret_cast<uintptr_t>(&t.pk[0][11]));
  const uint32_t sentb = uni((uint32_t)reinterpret_cast<uintptr_t>(t.sent));
  const uint32_t sentd = sentb + 288u * 4u;
  uint32_t pos = A, lo = stage[A >> 5], hi = stage[(A >> 5) + 1];
  uint32_t vt = 0, tselb = tabb, ntok = 0, acc = 0, ckn = CK1;
  uint32_t c1p = NOPOS, c1o = 0, c2p = NOPOS, c2o = 0, c3p = NOPOS, c3o = 0;
  const uint32_t bad_e = 1u | PE_SPECIAL;
  uint32_t e = 0, bits, a, nx, x, ex, val, np, tmp, r15, q, p11, p12, p13, p14, p15, d, sh;
  uint64_t sA, sB, sC, sD, sE, sv;
  asm volatile(
      "s_mov_b64 %[sv], exec\n"
      "L_top%=:\n\t"
      "v_alignbit_b32 %[bits], %[hi], %[lo], %[pos]\n\t"
      "v_and_b32 %[a], 0x3ff, %[bits]\n\t"
      "v_lshl_add_u32 %[a], %[a], 2, %[tselb]\n\t"
      "ds_read_b32 %[e], %[a]\n\t"
      "v_lshrrev_b32 %[a], 5, %[pos]\n\t"
      "v_lshl_add_u32 %[a], %[a], 2, %[stb]\n\t"
      "ds_read_b32 %[nx], %[a]\n\t"
      // while the entry is in flight: token boundary (sA), cut (sC), checkpoint hit (sB)
      "v_cmp_eq_u32 %[sA], 0, %[vt]\n\t"
      "v_cmp_ge_u32 %[sC], %[pos], %[stop]\n\t"
      "s_and_b64 %[sC], %[sC], %[sA]\n\t"
      "v_cmp_eq_u32 %[sB], %[ntok], %[ckn]\n\t"
      "s_and_b64 %[sB], %[sB], %[sA]\n\t"
      "s_cbranch_scc0 L_nock%=\n\t"
      // checkpoint (hit lanes): shift in (pos, bytes), next threshold 8 -> 32 -> 64 -> never
      "s_and_saveexec_b64 %[sD], %[sB]\n\t"
      "v_mov_b32 %[c3p], %[c2p]\n\t"
      "v_mov_b32 %[c3o], %[c2o]\n\t"
      "v_mov_b32 %[c2p], %[c1p]\n\t"
      "v_mov_b32 %[c2o], %[c1o]\n\t"
      "v_mov_b32 %[c1p], %[pos]\n\t"
      "v_lshrrev_b32 %[c1o], 12, %[acc]\n\t"
      "v_add_u32 %[c1o], %[c1o], %[ntok]\n\t"
      "v_cmp_eq_u32 %[sB], 32, %[ckn]\n\t"
      "v_cmp_eq_u32 %[sE], 8, %[ckn]\n\t"
      "s_nop 1\n\t"
      "v_cndmask_b32_e64 %[tmp], -1, 64, %[sB]\n\t"
      "v_cndmask_b32_e64 %[ckn], %[tmp], 32, %[sE]\n\t"
      "s_mov_b64 exec, %[sD]\n"
      "L_nock%=:\n\t"
      "s_waitcnt lgkmcnt(1)\n\t"
      "v_cmp_gt_i32 %[sD], 0, %[e]\n\t"  // special entries
      "s_and_b64 %[sD], %[sD], exec\n\t"
      "s_cbranch_scc0 L_nosp%=\n\t"
      "v_and_b32 %[tmp], 0x4000, %[e]\n\t"  // PE_SLOW
      "v_cmp_ne_u32 %[sB], 0, %[tmp]\n\t"
      "s_and_b64 %[sB], %[sB], %[sD]\n\t"
      "s_cbranch_scc0 L_nosp%=\n\t"
      // long codes: the length is 11 + #{v in 11..14 : limit(v) <= rev15}; invalid past limit(15)
      "s_and_saveexec_b64 %[sB], %[sB]\n\t"
      "v_bfrev_b32 %[r15], %[bits]\n\t"
      "v_lshrrev_b32 %[r15], 17, %[r15]\n\t"
      "v_lshrrev_b32 %[q], 6, %[vt]\n\t"  // pk[kind]: 64 bytes per kind
      "v_add_u32 %[q], %[pkb], %[q]\n\t"
      "ds_read_b32 %[p11], %[q]\n\t"  // pk[kind][11..15]
      "ds_read_b32 %[p12], %[q] offset:4\n\t"
      "ds_read_b32 %[p13], %[q] offset:8\n\t"
      "ds_read_b32 %[p14], %[q] offset:12\n\t"
      "ds_read_b32 %[p15], %[q] offset:16\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "v_mov_b32 %[d], %[p11]\n\t"
      "v_mov_b32 %[sh], 4\n\t"
      "v_lshrrev_b32 %[tmp], 16, %[p11]\n\t"
      "v_cmp_le_u32 vcc, %[tmp], %[r15]\n\t"
      "s_nop 1\n\t"
      "v_cndmask_b32_e32 %[d], %[d], %[p12], vcc\n\t"
      "v_cndmask_b32_e64 %[sh], %[sh], 3, vcc\n\t"
      "v_lshrrev_b32 %[tmp], 16, %[p12]\n\t"
      "v_cmp_le_u32 vcc, %[tmp], %[r15]\n\t"
      "s_nop 1\n\t"
      "v_cndmask_b32_e32 %[d], %[d], %[p13], vcc\n\t"
      "v_cndmask_b32_e64 %[sh], %[sh], 2, vcc\n\t"
      "v_lshrrev_b32 %[tmp], 16, %[p13]\n\t"
      "v_cmp_le_u32 vcc, %[tmp], %[r15]\n\t"
      "s_nop 1\n\t"
      "v_cndmask_b32_e32 %[d], %[d], %[p14], vcc\n\t"
      "v_cndmask_b32_e64 %[sh], %[sh], 1, vcc\n\t"
      "v_lshrrev_b32 %[tmp], 16, %[p14]\n\t"
      "v_cmp_le_u32 vcc, %[tmp], %[r15]\n\t"
      "s_nop 1\n\t"
      "v_cndmask_b32_e32 %[d], %[d], %[p15], vcc\n\t"
      "v_cndmask_b32_e64 %[sh], %[sh], 0, vcc\n\t"
      "v_lshrrev_b32 %[tmp], %[sh], %[r15]\n\t"  // (d + (rev15 >> (15 - len))) & 0xffff
      "v_add_u32 %[tmp], %[tmp], %[d]\n\t"
      "v_and_b32 %[tmp], 0xffff, %[tmp]\n\t"
      "v_min_u32 %[tmp], 0x13f, %[tmp]\n\t"  // (inside sent[]; an index past it is an invalid code, replaced below)
      "v_cmp_ne_u32 vcc, 0, %[vt]\n\t"
      "v_mov_b32 %[q], %[sentd]\n\t"
      "v_mov_b32 %[d], %[sentb]\n\t"
      "v_cndmask_b32_e32 %[q], %[d], %[q], vcc\n\t"
      "v_lshl_add_u32 %[tmp], %[tmp], 2, %[q]\n\t"
      "ds_read_b32 %[e], %[tmp]\n\t"
      "v_lshrrev_b32 %[tmp], 16, %[p15]\n\t"
      "v_cmp_ge_u32 vcc, %[r15], %[tmp]\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_nop 1\n\t"
      "v_cndmask_b32_e32 %[e], %[e], %[bad_e], vcc\n\t"
      "s_mov_b64 exec, %[sB]\n\t"
      "v_cmp_gt_i32 %[sD], 0, %[e]\n"  // special after the long-code lookup
      "L_nosp%=:\n\t"
      // lanes at their cut or a special entry leave the loop
      "s_or_b64 %[sD], %[sD], %[sC]\n\t"
      "s_andn2_b64 exec, exec, %[sD]\n\t"
      "s_cbranch_execz L_end%=\n\t"
      "v_and_b32 %[tmp], 31, %[e]\n\t"
      "v_bfe_u32 %[x], %[e], 5, 4\n\t"
      "v_bfe_u32 %[ex], %[bits], %[e], %[x]\n\t"
      "v_add3_u32 %[np], %[pos], %[tmp], %[x]\n\t"
      "v_add_u32_sdwa %[val], %[ex], %[e] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
      "v_xor_b32 %[tmp], %[np], %[pos]\n\t"
      "v_cmp_lt_u32 vcc, 31, %[tmp]\n\t"
      "v_and_b32 %[vt], 0x1000, %[e]\n\t"
      "v_mov_b32 %[pos], %[np]\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "v_cndmask_b32_e32 %[lo], %[lo], %[hi], vcc\n\t"
      "v_cndmask_b32_e32 %[hi], %[hi], %[nx], vcc\n\t"
      "v_addc_co_u32_e64 %[ntok], vcc, 0, %[ntok], %[sA]\n\t"
      "v_add_u32 %[tselb], %[tabb], %[vt]\n\t"
      "v_mad_u32_u24 %[acc], %[vt], %[val], %[acc]\n\t"
#if SBH_HUFF_PAIRS
      "v_and_b32 %[tmp], 0x400, %[e]\n\t"  // a literal pair (PE_PAIR): one byte more than its token
      "v_lshl_add_u32 %[acc], %[tmp], 2, %[acc]\n\t"
#endif
      "s_branch L_top%=\n"
      "L_end%=:\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_mov_b64 exec, %[sv]"
      : [pos] "+v"(pos), [lo] "+v"(lo), [hi] "+v"(hi), [vt] "+v"(vt), [tselb] "+v"(tselb), [ntok] "+v"(ntok),
        [acc] "+v"(acc), [ckn] "+v"(ckn), [c1p] "+v"(c1p), [c1o] "+v"(c1o), [c2p] "+v"(c2p), [c2o] "+v"(c2o),
        [c3p] "+v"(c3p), [c3o] "+v"(c3o), [e] "+v"(e), [bits] "=&v"(bits), [a] "=&v"(a), [nx] "=&v"(nx),
        [x] "=&v"(x), [ex] "=&v"(ex), [val] "=&v"(val), [np] "=&v"(np), [tmp] "=&v"(tmp), [r15] "=&v"(r15),
        [q] "=&v"(q), [p11] "=&v"(p11), [p12] "=&v"(p12), [p13] "=&v"(p13), [p14] "=&v"(p14), [p15] "=&v"(p15),
        [d] "=&v"(d), [sh] "=&v"(sh), [sA] "=&s"(sA),
        [sB] "=&s"(sB), [sC] "=&s"(sC), [sD] "=&s"(sD), [sE] "=&s"(sE), [sv] "=&s"(sv)
      : [stop] "v"(stop2), [tabb] "s"(tabb), [stb] "s"(stb), [pkb] "s"(pkb), [sentb] "s"(sentb),
        [sentd] "s"(sentd), [bad_e] "v"(bad_e)
      : "vcc", "scc", "memory");
  const uint32_t nck = ckn == CK1 ? 0u : ckn == CK2 ? 1u : ckn == CK3 ? 2u : 3u;
  ck = nck == 3 ? Ckpt{c3p, c3o, c2p, c2o, c1p, c1o}
     : nck == 2 ? Ckpt{c2p, c2o, c1p, c1o, NOPOS, 0}
     : nck == 1 ? Ckpt{c1p, c1o, NOPOS, 0, NOPOS, 0}
                : Ckpt{NOPOS, 0, NOPOS, 0, NOPOS, 0};
  LaneRun r{LR_RUN, pos, ntok, ntok + (acc >> 12)};
  if (vt == 0 && pos >= stop2) {  // cut at a token boundary
    if (pos >= limit) r.st = LR_PAST;
  } else {  // end of block, or an invalid code
    r.st = (vt == 0 && (e & PE_EOB)) ? LR_EOB : LR_DEAD;
    r.exit = pos + (e & 31);
  }
  return r;
}

#ifndef SBH_ASM_REDO
#define SBH_ASM_REDO 1  // repair runs (RUN_REDO over the LDS stage) as the hand-written loop below
#endif
// RUN_REDO over the LDS stage as hand-written code (lane_run<RUN_REDO>'s results): spec_asm's
// loop with the checkpoint recording replaced by the join test -- a run also stops at a token
// boundary that is one of its pass-1 checkpoints (ck), and then takes that chain's rest (sp).
__device__ __forceinline__ LaneRun redo_asm(const WaveSmem &t, const uint32_t *stage, uint32_t A, uint32_t stop,
                                            uint32_t limit, const Ckpt &ck, const LaneRun &sp) {
  const uint32_t stop2 = stop < limit ? stop : limit;
  if (A >= stop2) return LaneRun{A >= limit ? LR_PAST : LR_RUN, A, 0, 0};
  const uint32_t tabb = uni((uint32_t)reinterpret_cast<uintptr_t>(t.tab));
  const uint32_t stb = uni((uint32_t)reinterpret_cast<uintptr_t>(stage) + 8u);
  const uint32_t pkb = uni((uint32_t)reinterpret_cast<uintptr_t>(&t.pk[0][11]));
  const uint32_t sentb = uni((uint32_t)reinterpret_cast<uintptr_t>(t.sent));
  const uint32_t sentd = sentb + 288u * 4u;
  uint32_t pos = A, lo = stage[A >> 5], hi = stage[(A >> 5) + 1];
  uint32_t vt = 0, tselb = tabb, ntok = 0, acc = 0;
  const uint32_t bad_e = 1u | PE_SPECIAL;
  const uint32_t k1 = ck.p1, k2 = ck.p2, k3 = ck.p3;
  uint32_t e = 0, bits, a, nx, x, ex, val, np, tmp, r15, q, p11, p12, p13, p14, p15, d, sh;
  uint64_t sA, sB, sC, sD, sE, sv;
  asm volatile(
      "s_mov_b64 %[sv], exec\n"
      "L_top%=:\n\t"
      "v_alignbit_b32 %[bits], %[hi], %[lo], %[pos]\n\t"
      "v_and_b32 %[a], 0x3ff, %[bits]\n\t"
      "v_lshl_add_u32 %[a], %[a], 2, %[tselb]\n\t"
      "ds_read_b32 %[e], %[a]\n\t"
      "v_lshrrev_b32 %[a], 5, %[pos]\n\t"
      "v_lshl_add_u32 %[a], %[a], 2, %[stb]\n\t"
      "ds_read_b32 %[nx], %[a]\n\t"
      // while the entry is in flight: token boundary (sA), cut (sC), checkpoint hit (sB)
      "v_cmp_eq_u32 %[sA], 0, %[vt]\n\t"
      "v_cmp_ge_u32 %[sC], %[pos], %[stop]\n\t"
      "v_cmp_eq_u32 %[sB], %[pos], %[k1]\n\t"
      "v_cmp_eq_u32 %[sE], %[pos], %[k2]\n\t"
      "s_or_b64 %[sC], %[sC], %[sB]\n\t"
      "v_cmp_eq_u32 %[sB], %[pos], %[k3]\n\t"
      "s_or_b64 %[sC], %[sC], %[sE]\n\t"
      "s_or_b64 %[sC], %[sC], %[sB]\n\t"
      "s_and_b64 %[sC], %[sC], %[sA]\n"
      "L_nock%=:\n\t"
      "s_waitcnt lgkmcnt(1)\n\t"
      "v_cmp_gt_i32 %[sD], 0, %[e]\n\t"  // special entries
      "s_and_b64 %[sD], %[sD], exec\n\t"
      "s_cbranch_scc0 L_nosp%=\n\t"
      "v_and_b32 %[tmp], 0x4000, %[e]\n\t"  // PE_SLOW
      "v_cmp_ne_u32 %[sB], 0, %[tmp]\n\t"
      "s_and_b64 %[sB], %[sB], %[sD]\n\t"
      "s_cbranch_scc0 L_nosp%=\n\t"
      // long codes: the length is 11 + #{v in 11..14 : limit(v) <= rev15}; invalid past limit(15)
      "s_and_saveexec_b64 %[sB], %[sB]\n\t"
      "v_bfrev_b32 %[r15], %[bits]\n\t"
      "v_lshrrev_b32 %[r15], 17, %[r15]\n\t"
      "v_lshrrev_b32 %[q], 6, %[vt]\n\t"  // pk[kind]: 64 bytes per kind
      "v_add_u32 %[q], %[pkb], %[q]\n\t"
      "ds_read_b32 %[p11], %[q]\n\t"  // pk[kind][11..15]
      "ds_read_b32 %[p12], %[q] offset:4\n\t"
      "ds_read_b32 %[p13], %[q] offset:8\n\t"
      "ds_read_b32 %[p14], %[q] offset:12\n\t"
      "ds_read_b32 %[p15], %[q] offset:16\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "v_mov_b32 %[d], %[p11]\n\t"
      "v_mov_b32 %[sh], 4\n\t"
      "v_lshrrev_b32 %[tmp], 16, %[p11]\n\t"
      "v_cmp_le_u32 vcc, %[tmp], %[r15]\n\t"
      "s_nop 1\n\t"
      "v_cndmask_b32_e32 %[d], %[d], %[p12], vcc\n\t"
      "v_cndmask_b32_e64 %[sh], %[sh], 3, vcc\n\t"
      "v_lshrrev_b32 %[tmp], 16, %[p12]\n\t"
      "v_cmp_le_u32 vcc, %[tmp], %[r15]\n\t"
      "s_nop 1\n\t"
      "v_cndmask_b32_e32 %[d], %[d], %[p13], vcc\n\t"
      "v_cndmask_b32_e64 %[sh], %[sh], 2, vcc\n\t"
      "v_lshrrev_b32 %[tmp], 16, %[p13]\n\t"
      "v_cmp_le_u32 vcc, %[tmp], %[r15]\n\t"
      "s_nop 1\n\t"
      "v_cndmask_b32_e32 %[d], %[d], %[p14], vcc\n\t"
      "v_cndmask_b32_e64 %[sh], %[sh], 1, vcc\n\t"
      "v_lshrrev_b32 %[tmp], 16, %[p14]\n\t"
      "v_cmp_le_u32 vcc, %[tmp], %[r15]\n\t"
      "s_nop 1\n\t"
      "v_cndmask_b32_e32 %[d], %[d], %[p15], vcc\n\t"
      "v_cndmask_b32_e64 %[sh], %[sh], 0, vcc\n\t"
      "v_lshrrev_b32 %[tmp], %[sh], %[r15]\n\t"  // (d + (rev15 >> (15 - len))) & 0xffff
      "v_add_u32 %[tmp], %[tmp], %[d]\n\t"
      "v_and_b32 %[tmp], 0xffff, %[tmp]\n\t"
      "v_min_u32 %[tmp], 0x13f, %[tmp]\n\t"  // (inside sent[]; an index past it is an invalid code, replaced below)
      "v_cmp_ne_u32 vcc, 0, %[vt]\n\t"
      "v_mov_b32 %[q], %[sentd]\n\t"
      "v_mov_b32 %[d], %[sentb]\n\t"
      "v_cndmask_b32_e32 %[q], %[d], %[q], vcc\n\t"
      "v_lshl_add_u32 %[tmp], %[tmp], 2, %[q]\n\t"
      "ds_read_b32 %[e], %[tmp]\n\t"
      "v_lshrrev_b32 %[tmp], 16, %[p15]\n\t"
      "v_cmp_ge_u32 vcc, %[r15], %[tmp]\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_nop 1\n\t"
      "v_cndmask_b32_e32 %[e], %[e], %[bad_e], vcc\n\t"
      "s_mov_b64 exec, %[sB]\n\t"
      "v_cmp_gt_i32 %[sD], 0, %[e]\n"  // special after the long-code lookup
      "L_nosp%=:\n\t"
      // lanes at their cut or a special entry leave the loop
      "s_or_b64 %[sD], %[sD], %[sC]\n\t"
      "s_andn2_b64 exec, exec, %[sD]\n\t"
      "s_cbranch_execz L_end%=\n\t"
      "v_and_b32 %[tmp], 31, %[e]\n\t"
      "v_bfe_u32 %[x], %[e], 5, 4\n\t"
      "v_bfe_u32 %[ex], %[bits], %[e], %[x]\n\t"
      "v_add3_u32 %[np], %[pos], %[tmp], %[x]\n\t"
      "v_add_u32_sdwa %[val], %[ex], %[e] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
      "v_xor_b32 %[tmp], %[np], %[pos]\n\t"
      "v_cmp_lt_u32 vcc, 31, %[tmp]\n\t"
      "v_and_b32 %[vt], 0x1000, %[e]\n\t"
      "v_mov_b32 %[pos], %[np]\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "v_cndmask_b32_e32 %[lo], %[lo], %[hi], vcc\n\t"
      "v_cndmask_b32_e32 %[hi], %[hi], %[nx], vcc\n\t"
      "v_addc_co_u32_e64 %[ntok], vcc, 0, %[ntok], %[sA]\n\t"
      "v_add_u32 %[tselb], %[tabb], %[vt]\n\t"
      "v_mad_u32_u24 %[acc], %[vt], %[val], %[acc]\n\t"
#if SBH_HUFF_PAIRS
      "v_and_b32 %[tmp], 0x400, %[e]\n\t"  // a literal pair (PE_PAIR): one byte more than its token
      "v_lshl_add_u32 %[acc], %[tmp], 2, %[acc]\n\t"
#endif
      "s_branch L_top%=\n"
      "L_end%=:\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_mov_b64 exec, %[sv]"
      : [pos] "+v"(pos), [lo] "+v"(lo), [hi] "+v"(hi), [vt] "+v"(vt), [tselb] "+v"(tselb), [ntok] "+v"(ntok),
        [acc] "+v"(acc), [e] "+v"(e), [bits] "=&v"(bits), [a] "=&v"(a), [nx] "=&v"(nx), [x] "=&v"(x),
        [ex] "=&v"(ex), [val] "=&v"(val), [np] "=&v"(np), [tmp] "=&v"(tmp), [r15] "=&v"(r15), [q] "=&v"(q),
        [p11] "=&v"(p11), [p12] "=&v"(p12), [p13] "=&v"(p13), [p14] "=&v"(p14), [p15] "=&v"(p15), [d] "=&v"(d),
        [sh] "=&v"(sh), [sA] "=&s"(sA), [sB] "=&s"(sB), [sC] "=&s"(sC), [sD] "=&s"(sD), [sE] "=&s"(sE),
        [sv] "=&s"(sv)
      : [stop] "v"(stop2), [k1] "v"(k1), [k2] "v"(k2), [k3] "v"(k3), [tabb] "s"(tabb), [stb] "s"(stb),
        [pkb] "s"(pkb), [sentb] "s"(sentb), [sentd] "s"(sentd), [bad_e] "v"(bad_e)
      : "vcc", "scc", "memory");
  LaneRun r{LR_RUN, pos, ntok, ntok + (acc >> 12)};
  if (vt == 0 && (pos >= stop2 || pos == k1 || pos == k2 || pos == k3)) {  // cut at a token boundary
    if (pos < stop2) {  // joined the pass-1 chain at a checkpoint
      const bool one = pos == k1;
      const bool two = pos == k2;
      r.ntok += sp.ntok - (one ? CK1 : two ? CK2 : CK3);
      r.nout += sp.nout - ck_out(ck, one, two);
      r.st = sp.st;
      r.exit = sp.exit;
    } else if (pos >= limit) {
      r.st = LR_PAST;
    }
  } else {  // end of block, or an invalid code
    r.st = (vt == 0 && (e & PE_EOB)) ? LR_EOB : LR_DEAD;
    r.exit = pos + (e & 31);
  }
  return r;
}

#ifndef SBH_ASM_EMIT
#define SBH_ASM_EMIT 1  // pass 3 (RUN_EMIT over the LDS stage) as the hand-written loop below
#endif
#ifndef SBH_EMIT_NOCHK
#define SBH_EMIT_NOCHK 1  // emit_asm: no too-far-back test per distance code (k_lz tests each match token once)
#endif
#ifndef SBH_EMIT_X4
#define SBH_EMIT_X4 1  // emit_asm: a lane's tokens stored four at a time (16-byte stores from v124..v127; A/B r05m/r05n: k_huff -7% E, +-0.2% B and D)
#endif
// RUN_EMIT over the LDS stage as hand-written code (lane_run<RUN_EMIT>'s results): the decode
// loop of spec_asm without the checkpoints, each token stored once (a literal at its code, a
// match at its distance code) through a 32-bit offset from the block's token base `tk` (wave-
// uniform), and the too-far-back test of every distance accumulated as a lane mask.
__device__ __forceinline__ void emit_asm(const WaveSmem &t, const uint32_t *stage, uint32_t A, uint32_t stop,
                                         uint32_t limit, uint32_t *tk, uint32_t tidx, uint32_t out0, uint32_t &bad) {
  const uint32_t stop2 = stop < limit ? stop : limit;
  if (A >= stop2) return;
  const uint32_t tabb = uni((uint32_t)reinterpret_cast<uintptr_t>(t.tab));
  const uint32_t stb = uni((uint32_t)reinterpret_cast<uintptr_t>(stage) + 8u);
  const uint32_t pkb = uni((uint32_t)reinterpret_cast<uintptr_t>(&t.pk[0][11]));
  const uint32_t sentb = uni((uint32_t)reinterpret_cast<uintptr_t>(t.sent));
  const uint32_t sentd = sentb + 288u * 4u;
  const uint64_t tkp = reinterpret_cast<uint64_t>(tk);
  const uint64_t tkb = (uint64_t)uni((uint32_t)tkp) | (uint64_t)uni((uint32_t)(tkp >> 32)) << 32;
  uint32_t pos = A, lo = stage[A >> 5], hi = stage[(A >> 5) + 1];
  uint32_t vt = 0, tselb = tabb, ntok = 0, acc = 0, ml = 0, voff = tidx * 4u, badv = 0, cnt = 0;
  const uint32_t om1 = out0 - 1u;
  const uint32_t bad_e = 1u | PE_SPECIAL;
  uint32_t e = 0, bits, a, nx, x, ex, val, np, tmp, r15, q, p11, p12, p13, p14, p15, d, sh, vtok, vb;
  uint64_t sA, sB, sC, sD, sE, sL, sBad, sv;
  asm volatile(
      "s_mov_b64 %[sv], exec\n\t"
      "s_mov_b64 %[sBad], 0\n"
      "L_top%=:\n\t"
      "v_alignbit_b32 %[bits], %[hi], %[lo], %[pos]\n\t"
      "v_and_b32 %[a], 0x3ff, %[bits]\n\t"
      "v_lshl_add_u32 %[a], %[a], 2, %[tselb]\n\t"
      "ds_read_b32 %[e], %[a]\n\t"
      "v_lshrrev_b32 %[a], 5, %[pos]\n\t"
      "v_lshl_add_u32 %[a], %[a], 2, %[stb]\n\t"
      "ds_read_b32 %[nx], %[a]\n\t"
      // while the entry is in flight: token boundary (sA), cut (sC), checkpoint hit (sB)
      "v_cmp_eq_u32 %[sA], 0, %[vt]\n\t"
      "v_cmp_ge_u32 %[sC], %[pos], %[stop]\n\t"
      "s_and_b64 %[sC], %[sC], %[sA]\n"
      "L_nock%=:\n\t"
      "s_waitcnt lgkmcnt(1)\n\t"
      "v_cmp_gt_i32 %[sD], 0, %[e]\n\t"  // special entries
      "s_and_b64 %[sD], %[sD], exec\n\t"
      "s_cbranch_scc0 L_nosp%=\n\t"
      "v_and_b32 %[tmp], 0x4000, %[e]\n\t"  // PE_SLOW
      "v_cmp_ne_u32 %[sB], 0, %[tmp]\n\t"
      "s_and_b64 %[sB], %[sB], %[sD]\n\t"
      "s_cbranch_scc0 L_nosp%=\n\t"
      // long codes: the length is 11 + #{v in 11..14 : limit(v) <= rev15}; invalid past limit(15)
      "s_and_saveexec_b64 %[sB], %[sB]\n\t"
      "v_bfrev_b32 %[r15], %[bits]\n\t"
      "v_lshrrev_b32 %[r15], 17, %[r15]\n\t"
      "v_lshrrev_b32 %[q], 6, %[vt]\n\t"  // pk[kind]: 64 bytes per kind
      "v_add_u32 %[q], %[pkb], %[q]\n\t"
      "ds_read_b32 %[p11], %[q]\n\t"  // pk[kind][11..15]
      "ds_read_b32 %[p12], %[q] offset:4\n\t"
      "ds_read_b32 %[p13], %[q] offset:8\n\t"
      "ds_read_b32 %[p14], %[q] offset:12\n\t"
      "ds_read_b32 %[p15], %[q] offset:16\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "v_mov_b32 %[d], %[p11]\n\t"
      "v_mov_b32 %[sh], 4\n\t"
      "v_lshrrev_b32 %[tmp], 16, %[p11]\n\t"
      "v_cmp_le_u32 vcc, %[tmp], %[r15]\n\t"
      "s_nop 1\n\t"
      "v_cndmask_b32_e32 %[d], %[d], %[p12], vcc\n\t"
      "v_cndmask_b32_e64 %[sh], %[sh], 3, vcc\n\t"
      "v_lshrrev_b32 %[tmp], 16, %[p12]\n\t"
      "v_cmp_le_u32 vcc, %[tmp], %[r15]\n\t"
      "s_nop 1\n\t"
      "v_cndmask_b32_e32 %[d], %[d], %[p13], vcc\n\t"
      "v_cndmask_b32_e64 %[sh], %[sh], 2, vcc\n\t"
      "v_lshrrev_b32 %[tmp], 16, %[p13]\n\t"
      "v_cmp_le_u32 vcc, %[tmp], %[r15]\n\t"
      "s_nop 1\n\t"
      "v_cndmask_b32_e32 %[d], %[d], %[p14], vcc\n\t"
      "v_cndmask_b32_e64 %[sh], %[sh], 1, vcc\n\t"
      "v_lshrrev_b32 %[tmp], 16, %[p14]\n\t"
      "v_cmp_le_u32 vcc, %[tmp], %[r15]\n\t"
      "s_nop 1\n\t"
      "v_cndmask_b32_e32 %[d], %[d], %[p15], vcc\n\t"
      "v_cndmask_b32_e64 %[sh], %[sh], 0, vcc\n\t"
      "v_lshrrev_b32 %[tmp], %[sh], %[r15]\n\t"  // (d + (rev15 >> (15 - len))) & 0xffff
      "v_add_u32 %[tmp], %[tmp], %[d]\n\t"
      "v_and_b32 %[tmp], 0xffff, %[tmp]\n\t"
      "v_min_u32 %[tmp], 0x13f, %[tmp]\n\t"  // (inside sent[]; an index past it is an invalid code, replaced below)
      "v_cmp_ne_u32 vcc, 0, %[vt]\n\t"
      "v_mov_b32 %[q], %[sentd]\n\t"
      "v_mov_b32 %[d], %[sentb]\n\t"
      "v_cndmask_b32_e32 %[q], %[d], %[q], vcc\n\t"
      "v_lshl_add_u32 %[tmp], %[tmp], 2, %[q]\n\t"
      "ds_read_b32 %[e], %[tmp]\n\t"
      "v_lshrrev_b32 %[tmp], 16, %[p15]\n\t"
      "v_cmp_ge_u32 vcc, %[r15], %[tmp]\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_nop 1\n\t"
      "v_cndmask_b32_e32 %[e], %[e], %[bad_e], vcc\n\t"
      "s_mov_b64 exec, %[sB]\n\t"
      "v_cmp_gt_i32 %[sD], 0, %[e]\n"  // special after the long-code lookup
      "L_nosp%=:\n\t"
      "s_or_b64 %[sD], %[sD], %[sC]\n\t"
      "s_andn2_b64 exec, exec, %[sD]\n\t"
      "s_cbranch_execz L_end%=\n\t"
      "v_and_b32 %[tmp], 31, %[e]\n\t"
      "v_bfe_u32 %[x], %[e], 5, 4\n\t"
      "v_bfe_u32 %[ex], %[bits], %[e], %[x]\n\t"
      "v_add3_u32 %[np], %[pos], %[tmp], %[x]\n\t"
      "v_add_u32_sdwa %[val], %[ex], %[e] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
      "v_and_b32 %[vt], 0x1000, %[e]\n\t"  // (the next code's state; this one's is in sA)
      "v_xor_b32 %[tmp], %[np], %[pos]\n\t"
      "v_cmp_ne_u32 %[sL], 0, %[vt]\n\t"  // a length code
      "v_cmp_lt_u32 vcc, 31, %[tmp]\n\t"
      "v_mov_b32 %[pos], %[np]\n\t"
      // the token: a literal (byte << 8) or the match completed by this distance code
      "v_lshlrev_b32 %[vtok], 8, %[val]\n\t"
#if SBH_HUFF_PAIRS
      "v_and_b32 %[tmp], 0x600, %[e]\n\t"  // (a literal pair: byte2's bit 7 and TOK_PAIR)
      "v_lshl_or_b32 %[vtok], %[tmp], 14, %[vtok]\n\t"
#endif
#if SBH_EMIT_NOCHK
      // (ml: the match token's upper half, TOK_MATCH | length << 16, set by every code -- only a
      // length code's is ever read, by the distance code after it)
      "v_or_b32 %[np], %[ml], %[val]\n\t"
      "v_lshl_add_u32 %[ml], %[val], 16, %[mlk]\n\t"
#else
      "v_add_u32 %[tmp], 1, %[ml]\n\t"
      "v_lshl_or_b32 %[np], %[tmp], 16, %[val]\n\t"
      "v_or_b32 %[np], 0x80000000, %[np]\n\t"
#endif
      "v_cndmask_b32_e64 %[vtok], %[np], %[vtok], %[sA]\n\t"
#if !SBH_EMIT_NOCHK
      // too far back: a distance past the bytes before its match
      "v_lshrrev_b32 %[vb], 12, %[acc]\n\t"
      "v_sub_u32 %[vb], %[vb], %[ml]\n\t"
      "v_add3_u32 %[vb], %[vb], %[ntok], %[om1]\n\t"
      "v_cmp_gt_u32 %[sB], %[val], %[vb]\n\t"
      "s_andn2_b64 %[sB], %[sB], %[sA]\n\t"
      "s_or_b64 %[sBad], %[sBad], %[sB]\n\t"
      "v_cndmask_b32_e64 %[ml], %[ml], %[val], %[sL]\n\t"
#endif
      "s_waitcnt lgkmcnt(0)\n\t"
      "v_cndmask_b32_e32 %[lo], %[lo], %[hi], vcc\n\t"
      "v_cndmask_b32_e32 %[hi], %[hi], %[nx], vcc\n\t"
      // store every code but a length code
      "s_and_b64 %[sE], %[sA], %[sL]\n\t"
      "s_mov_b64 %[sB], exec\n\t"
      "s_andn2_b64 exec, exec, %[sE]\n\t"
#if SBH_EMIT_X4
      // tokens gather in v124..v127 (oldest first) and leave four at a time in one 16-byte store
      "v_mov_b32 v124, v125\n\t"
      "v_mov_b32 v125, v126\n\t"
      "v_mov_b32 v126, v127\n\t"
      "v_mov_b32 v127, %[vtok]\n\t"
      "v_add_u32 %[cnt], 1, %[cnt]\n\t"
      "v_cmp_eq_u32 %[sE], 4, %[cnt]\n\t"
      "s_and_b64 exec, exec, %[sE]\n\t"
      "s_cbranch_execz L_nofl%=\n\t"
      "global_store_dwordx4 %[voff], v[124:127], %[tkb]\n\t"
      "s_nop 1\n\t"  // (a VALU write of a > 8-byte store's data VGPRs waits for the store to read them)
      "v_add_u32 %[voff], 16, %[voff]\n\t"
      "v_mov_b32 %[cnt], 0\n"
      "L_nofl%=:\n\t"
#else
      "global_store_dword %[voff], %[vtok], %[tkb]\n\t"
      "v_add_u32 %[voff], 4, %[voff]\n\t"
#endif
      "s_mov_b64 exec, %[sB]\n\t"
#if !SBH_EMIT_NOCHK  // (the token and byte counts feed the distance test only)
      "v_addc_co_u32_e64 %[ntok], vcc, 0, %[ntok], %[sA]\n\t"
      "v_mad_u32_u24 %[acc], %[vt], %[val], %[acc]\n\t"
#if SBH_HUFF_PAIRS
      "v_and_b32 %[tmp], 0x400, %[e]\n\t"
      "v_lshl_add_u32 %[acc], %[tmp], 2, %[acc]\n\t"
#endif
#endif
      "v_add_u32 %[tselb], %[tabb], %[vt]\n\t"
      "s_branch L_top%=\n"
      "L_end%=:\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_mov_b64 exec, %[sv]\n\t"
#if SBH_EMIT_X4
      // the last cnt (< 4) tokens of each lane: v127 (newest) at voff + 4 (cnt - 1), v126 before it, ...
      "v_cmp_le_u32 %[sE], 1, %[cnt]\n\t"
      "s_and_b64 exec, exec, %[sE]\n\t"
      "s_cbranch_execz L_fld%=\n\t"
      "v_lshl_add_u32 %[tmp], %[cnt], 2, %[voff]\n\t"
      "global_store_dword %[tmp], v127, %[tkb] offset:-4\n\t"
      "v_cmp_le_u32 %[sE], 2, %[cnt]\n\t"
      "s_and_b64 exec, exec, %[sE]\n\t"
      "global_store_dword %[tmp], v126, %[tkb] offset:-8\n\t"
      "v_cmp_le_u32 %[sE], 3, %[cnt]\n\t"
      "s_and_b64 exec, exec, %[sE]\n\t"
      "global_store_dword %[tmp], v125, %[tkb] offset:-12\n"
      "L_fld%=:\n\t"
      "s_mov_b64 exec, %[sv]\n\t"
#endif
      "v_cndmask_b32_e64 %[badv], 0, 1, %[sBad]"
      : [pos] "+v"(pos), [lo] "+v"(lo), [hi] "+v"(hi), [vt] "+v"(vt), [tselb] "+v"(tselb), [ntok] "+v"(ntok),
        [acc] "+v"(acc), [ml] "+v"(ml), [voff] "+v"(voff), [badv] "+v"(badv), [cnt] "+v"(cnt), [e] "+v"(e),
        [bits] "=&v"(bits),
        [a] "=&v"(a), [nx] "=&v"(nx), [x] "=&v"(x), [ex] "=&v"(ex), [val] "=&v"(val), [np] "=&v"(np),
        [tmp] "=&v"(tmp), [r15] "=&v"(r15), [q] "=&v"(q), [p11] "=&v"(p11), [p12] "=&v"(p12), [p13] "=&v"(p13),
        [p14] "=&v"(p14), [p15] "=&v"(p15), [d] "=&v"(d), [sh] "=&v"(sh), [vtok] "=&v"(vtok),
        [vb] "=&v"(vb), [sA] "=&s"(sA), [sB] "=&s"(sB), [sC] "=&s"(sC), [sD] "=&s"(sD), [sE] "=&s"(sE),
        [sL] "=&s"(sL), [sBad] "=&s"(sBad), [sv] "=&s"(sv)
      : [stop] "v"(stop2), [tabb] "s"(tabb), [stb] "s"(stb), [pkb] "s"(pkb), [sentb] "s"(sentb),
        [sentd] "s"(sentd), [bad_e] "v"(bad_e), [om1] "v"(om1), [tkb] "s"(tkb), [mlk] "s"(0x80010000u)
      : "vcc", "scc", "memory"
#if SBH_EMIT_X4
      , "v124", "v125", "v126", "v127"
#endif
  );
  bad |= badv;
}

// The code-length part of a dynamic block header (RFC 1951 3.2.7) by one wave: the
// code-length code, then the nlen + ndist lengths into t.lens ([0, 288) lit/len, [288,
// 320) dist).  The code-length symbols are decoded 64 bit positions at a time -- lane i
// decodes the symbol that would start at q + i -- and the wave walks the chain through
// those with v_readlane, writing each run of lengths with one vector store.  Returns
// (uniformly) whether the lengths are well formed and include an end-of-block code;
// q: the bit after the header.  `p` is the block's first bit (BFINAL).
template <class SM, class S>
__device__ __forceinline__ bool hdr_walk(SM &t, const S &src, uint32_t p, uint32_t limit, uint32_t nlen,
                                         uint32_t ndist, uint32_t ncode, uint32_t lane, uint32_t &q_out,
                                         uint64_t *h1, uint64_t *h2) {
  if (lane < 19) t.cl_lens[CL_ORDER[lane]] = lane < ncode ? (uint8_t)(src.bits32(p + 17 + 3 * lane) & 7) : 0;
  __builtin_amdgcn_wave_barrier();
  bool ok = uni(build_table(t, t.cl_lens, 19, 2, t.lit, CL_FAST, lane)) == 0;
  if (h1) *h1 = __builtin_readcyclecounter();
  for (uint32_t w = lane; w < 320 / 4; w += WAVE) reinterpret_cast<uint32_t *>(t.lens)[w] = 0;
  __builtin_amdgcn_wave_barrier();
  const uint32_t total = nlen + ndist;
  uint32_t i = 0, prev = 0, q = p + 17 + 3 * ncode;
  const uint64_t below = (1ull << lane) - 1;  // lanes under this one
  while (ok && i < total && q <= limit) {
    // every lane decodes the symbol that would start at q + lane
    const uint32_t b = src.bits32(q + lane);
    const uint32_t e = t.lit[b & ((1u << CL_FAST) - 1)];
    const uint32_t L = e & 31, sym = (e >> 8) & 31;
    const uint32_t xb = sym < 16 ? 0 : sym == 16 ? 2 : sym == 17 ? 3 : 7;
    const uint32_t xv = __builtin_amdgcn_ubfe(b, L, xb);
    const uint32_t rep = sym < 16 ? 1 : sym == 16 ? 3 + xv : sym == 17 ? 3 + xv : 11 + xv;
    const uint32_t pack = (L + xb) | (rep << 8);
    // serial part: the chain of symbol starts through this window.  (symbol index << 8 | bit
    // offset) advances by one scalar add per symbol (pack = bits | rep << 8; the offset stays
    // below 256), and both exit tests read that one word -- the walk is k_hdr's scalar hot loop
    uint64_t M = 0;
    const uint32_t i0 = i, tot8 = uni(total << 8);
    uint32_t oi = uni(i0 << 8), inf, tw;
    // (v_readlane and s_bitset1_b64 take the offset's low 6 bits; the loop leaves once the
    // offset reaches 64 or the symbols reach `total`; 7 scalar-unit instructions per symbol
    // against the compiler's 12)
    asm volatile(
        "s_nop 3\n"  // (a lane select written by a VALU just before needs 4 wait states)
        "L_walk%=:\n\t"
        "v_readlane_b32 %[inf], %[pack], %[oi]\n\t"
        "s_bitset1_b64 %[M], %[oi]\n\t"
        "s_add_u32 %[oi], %[oi], %[inf]\n\t"
        "s_and_b32 %[tw], %[oi], 0xc0\n\t"
        "s_cbranch_scc1 L_wend%=\n\t"
        "s_cmp_lt_u32 %[oi], %[tot8]\n\t"
        "s_cbranch_scc1 L_walk%=\n"
        "L_wend%=:"
        : [M] "+s"(M), [oi] "+s"(oi), [inf] "=&s"(inf), [tw] "=&s"(tw)
        : [pack] "v"(pack), [tot8] "s"(tot8)
        : "scc");
    const uint32_t o = oi & 0xffu;
    i = oi >> 8;
    // parallel part: output index and value of each symbol, then its run of lengths
    const bool mine = (M >> lane) & 1;
    uint32_t ex;  // exclusive prefix of rep over the window's symbols
    {
      const uint32_t x = wave_incl_scan(mine ? rep : 0);
      ex = x - (mine ? rep : 0);
    }
    const uint32_t start = i0 + ex;
    const uint64_t N = M & __ballot(sym != 16);  // symbols with a value of their own
    const uint64_t lowN = N & below;
    const uint32_t own = sym < 16 ? sym : 0;
    const uint32_t src_lane = lowN ? 63 - (uint32_t)__builtin_clzll(lowN) : 0;
    const uint32_t from = __shfl(own, src_lane, WAVE);
    const uint32_t val = sym == 16 ? (lowN ? from : prev) : own;
    if (M & 1 && __builtin_amdgcn_readfirstlane(sym) == 16 && i0 == 0) ok = false;  // repeat with no previous length
    if (mine && val != 0) {  // the run [start, start + rep) of lengths (zeros: pre-set); distances at 288
      const uint32_t e = min(start + rep, total);
      const uint32_t v4 = val * 0x01010101u;
      for (uint32_t j = start; j < e;) {
        const uint32_t d = j < nlen ? j : 288 + j - nlen;
        const uint32_t seg_end = j < nlen ? min(e, nlen) : e;  // don't cross the lit/dist split
        if ((d & 3) == 0 && j + 4 <= seg_end) {
          *reinterpret_cast<uint32_t *>(&t.lens[d]) = v4;
          j += 4;
        } else {
          t.lens[d] = (uint8_t)val;
          ++j;
        }
      }
    }
    const uint32_t top = 63 - (uint32_t)__builtin_clzll(M);
    prev = __builtin_amdgcn_readlane(val, top);
    q += o;
  }
  if (i != total || q > limit) ok = false;  // a repeat past the end, or input ran out
  __builtin_amdgcn_wave_barrier();
  if (h2) *h2 = __builtin_readcyclecounter();
  if (ok && uni(t.lens[256]) == 0) ok = false;  // no end-of-block code
  q_out = q;
  return ok;
}

// Both PAR decode tables from ptable_meta's limits (pk) and order (sent), by the NT
// threads of a k_huff workgroup.
template <uint32_t NT>
__device__ __forceinline__ void fill_ptables(WaveSmem &t, uint32_t tid) {
  uint32_t lj0[16], lj1[16];
#pragma unroll
  for (uint32_t v = 1; v <= 15; ++v) {
    lj0[v] = t.pk[0][v] >> 16;
    lj1[v] = t.pk[1][v] >> 16;
  }
#pragma unroll 4
  for (uint32_t i = tid; i < (1u << LIT_FAST); i += NT) t.lit[i] = ptable_lit_entry(t, lj0, i);
#pragma unroll 4
  for (uint32_t i = tid; i < (1u << PDIST_FAST); i += NT) t.dist[i] = ptable_entry(t, lj1, 1, PDIST_FAST, i);
}

// Deflate block header and tables for the lane-parallel path, read from the bit source
// (sm.ctl[5..6] carry wave 0's result to the workgroup).  The code-length symbols are
// decoded 64 bit positions at a time -- lane i decodes the symbol that would start at
// q + i -- and wave 0 walks the chain through those with v_readlane, writing each run
// of lengths with one vector store.  Then wave 0 builds the literal/length table and
// wave 1 the distance table, concurrently.  Returns false (uniformly) for anything
// the serial decoder must judge: stored/invalid block types, invalid or incomplete
// codes, a header running past the input.
template <class SM, class S>
__device__ __forceinline__ bool par_header(SM &sm, S src, uint32_t p, uint32_t limit, bool &fixed_built,
                                           uint32_t wid, uint32_t lane, uint32_t &psym, uint32_t &last) {
  constexpr uint32_t NT = SM::NT;
  WaveSmem &t = sm.t;
  // both decode tables from ptable_meta's limits and order, filled by the whole workgroup
  auto fill_tables = [&]() { fill_ptables<NT>(t, wid * WAVE + lane); };
  const uint32_t hb = uni(src.bits32(p));
  last = hb & 1;
  const uint32_t type = (hb >> 1) & 3;
  if (p + 3 > limit || type == 0 || type == 3) return false;
  if (type == 1) {
    psym = p + 3;
    if (!fixed_built) {
      if (wid == 0) {
        for (uint32_t s = lane; s < 288; s += WAVE) t.lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
        __builtin_amdgcn_wave_barrier();
        ptable_meta(t, t.lens, 288, 0, lane);
      }
      if (wid == (NT > WAVE ? 1u : 0u)) {  // (one wave: it builds both)
        if (lane < 32) t.lens[288 + lane] = 5;
        __builtin_amdgcn_wave_barrier();
        ptable_meta(t, t.lens + 288, 32, 1, lane);
      }
      __syncthreads();
      fill_tables();
      __syncthreads();
      fixed_built = true;
    }
    return true;
  }
  fixed_built = false;
  const uint32_t nlen = ((hb >> 3) & 31) + 257, ndist = ((hb >> 8) & 31) + 1, ncode = ((hb >> 13) & 15) + 4;
  if (nlen > 286 || ndist > 30) return false;
#ifdef SBH_HUFF_PROBE
  const uint64_t h0 = __builtin_readcyclecounter();
  uint64_t h1 = 0, h2 = 0;
#endif
  if (wid == 0) {
    uint32_t q;
#ifdef SBH_HUFF_PROBE
    const bool ok = hdr_walk(t, src, p, limit, nlen, ndist, ncode, lane, q, &h1, &h2);
#else
    const bool ok = hdr_walk(t, src, p, limit, nlen, ndist, ncode, lane, q, nullptr, nullptr);
#endif
    if (lane == 0) {
      sm.ctl[5] = ok;
      sm.ctl[6] = q;
    }
  }
  __syncthreads();
  if (!uni(sm.ctl[5])) return false;
  psym = uni(sm.ctl[6]);
  bool bad = false;
  if (wid == 0) bad = ptable_meta(t, t.lens, nlen, 0, lane) == 1;
  if (wid == (NT > WAVE ? 1u : 0u)) bad = bad || ptable_meta(t, t.lens + 288, ndist, 1, lane) == 1;
  if (__syncthreads_or(bad)) return false;
  fill_tables();
  __syncthreads();
#ifdef SBH_HUFF_PROBE
  if (NT == HT && wid == 0 && lane == 0) {
    atomicAdd(&hp_acc[8], h1 - h0);
    atomicAdd(&hp_acc[9], h2 - h1);
    atomicAdd(&hp_acc[10], __builtin_readcyclecounter() - h2);
  }
#endif
  return true;
}

// The deflate blocks of one BGZF block (from bit `skip` of dbase's dwords), lane-parallel
// over SM::NT lanes.  Returns (uniformly) PAR_OK, PAR_FAIL when the block must be decoded
// by the serial path instead, or -- with `tail_ok` -- PAR_TAIL after a non-final deflate
// block when the bits left are few (< a quarter of the block's): *tail_p / *tail_out get
// the next block's first bit and the bytes produced, and k_huff_tail finishes the block
// with one wave, instead of this workgroup decoding a short final block (zlib's level-6
// BGZF member: 16383 symbols, then ~1 k) with most of its lanes idle.  `out_before`:
// bytes of the BGZF block before this call (for the too-far-back distance check).
constexpr uint32_t PAR_OK = 0, PAR_FAIL = 1, PAR_TAIL = 2;
template <bool LDS, class SM>
__device__ __forceinline__ uint32_t inflate_par(SM &sm, const uint8_t *__restrict__ dbase, uint32_t skip,
                            uint32_t limit, uint32_t usize, uint32_t *__restrict__ tk, uint32_t tid, uint32_t lane,
                            uint32_t wid, uint32_t &ntok_out, bool pre, uint32_t pre_psym, uint32_t pre_last,
                            uint32_t out_before, bool tail_ok, uint32_t *tail_p, uint32_t *tail_out) {
  constexpr uint32_t NT = SM::NT;
  const Src<LDS, SM::SDW> src{LDS ? sm.stage : reinterpret_cast<const uint32_t *>(dbase)};
  uint32_t p = skip, out = 0, ntok = 0;
  bool fixed_built = false;  // the tables in sm.t are the fixed code's
  for (;;) {
#ifdef SBH_HUFF_PROBE
    const uint64_t tp0 = __builtin_readcyclecounter();
#endif
    uint32_t p0, last;
    if (pre) {  // the first deflate block's tables came from k_hdr (already in sm.t)
      p0 = pre_psym;
      last = pre_last;
      pre = false;
    } else if (!par_header(sm, src, p, limit, fixed_built, wid, lane, p0, last)) {
      return PAR_FAIL;
    }

#ifdef SBH_HUFF_PROBE
    const uint64_t tph = __builtin_readcyclecounter();
#endif
    // pass 1: speculative decode of every lane's slice
    uint32_t S = (limit > p0 ? limit - p0 : 0) / NT + 1;
    if (S < MIN_SLICE) S = MIN_SLICE;  // short streams: fewer, longer slices (sync needs bits)
    const uint32_t s = p0 + tid * S, stop = s + S;
    uint32_t A = s, nobad = 0;
    Ckpt ck;
    const LaneRun none{};
#if SBH_MARGIN
    // warm-up: decode from SBH_MARGIN bits before the slice, so that by the slice start the
    // chain has (very likely) fallen onto the true token boundaries; the speculative start is
    // then the first boundary at or past the slice start -- usually exactly where the left
    // neighbour's chain exits, so the first repair round has nothing to redo for that lane
    if (tid) {
      Ckpt nock{NOPOS, 0, NOPOS, 0, NOPOS, 0};
      const uint32_t w0 = s - p0 > SBH_MARGIN ? s - SBH_MARGIN : p0;
      const LaneRun rw = lane_run<RUN_REDO>(sm.t, src, w0, s, limit, nock, none, nullptr, 0, nobad);
      if (rw.st == LR_RUN && rw.exit < stop) A = rw.exit;
    }
#endif
#if SBH_ASM_SPEC
    LaneRun r = LDS ? spec_asm(sm.t, sm.stage, A, stop, limit, ck)
                    : lane_run<RUN_SPEC>(sm.t, src, A, stop, limit, ck, none, nullptr, 0, nobad);
#else
    LaneRun r = lane_run<RUN_SPEC>(sm.t, src, A, stop, limit, ck, none, nullptr, 0, nobad);
#endif
    const LaneRun r1 = r;  // the pass-1 chain's result: a redo that joins it at a checkpoint takes its rest
    // exits alternate between two arrays: a round reads one and writes the other, so the
    // round's closing barrier (__syncthreads_or) is its only one
    uint32_t *xa = sm.exitv, *xb = sm.exitv2;
    xa[tid] = r.st == LR_RUN ? r.exit : NOPOS;
    __syncthreads();
    // pass 2: repair rounds until every lane starts where its left neighbour exits.
    // A repair run stops as soon as it joins the lane's pass-1 chain (in any round: the
    // pass-1 result from a checkpoint on holds for every chain that reaches it).
#ifdef SBH_HUFF_PROBE
    uint32_t nrounds = 0;
    __syncthreads();
    const uint64_t tp1 = __builtin_readcyclecounter();
#endif
#if defined(SBH_HUFF_TIMING) && (SBH_HUFF_TIMING & 1)
    if (false)  // timing probe: no repair rounds
#endif
    for (;;) {
#ifdef SBH_HUFF_PROBE
      ++nrounds;
#endif
      // a lane keeps its speculation while its left neighbour's chain has ended (that
      // neighbour is then past the true end, or itself speculating and not yet repaired)
      const uint32_t nA = tid == 0 ? p0 : xa[tid - 1];
      const bool changed = nA != NOPOS && nA != A;
      if (changed) {
        A = nA;
#if SBH_ASM_REDO
        r = LDS ? redo_asm(sm.t, sm.stage, A, stop, limit, ck, r1)
                : lane_run<RUN_REDO>(sm.t, src, A, stop, limit, ck, r1, nullptr, 0, nobad);
#else
        r = lane_run<RUN_REDO>(sm.t, src, A, stop, limit, ck, r1, nullptr, 0, nobad);
#endif
      }
      xb[tid] = r.st == LR_RUN ? r.exit : NOPOS;
      const bool again = __syncthreads_or(changed);
      uint32_t *const xt = xa;
      xa = xb;
      xb = xt;
#ifdef SBH_HUFF_PROBE
      if (SM::NT == HT && tid == 0 && nrounds == 1) atomicAdd(&hp_acc[12], __builtin_readcyclecounter() - tp1);
      if (SM::NT == HT && tid == 0 && nrounds == 2) atomicAdd(&hp_acc[13], __builtin_readcyclecounter() - tp1);
#endif
      if (!again) break;
    }
    // The first lane whose chain ends (k) decides the deflate block: the lanes up to it hold its
    // tokens and bytes.  One barrier gives k, every lane's exclusive token / byte prefix (for
    // tid <= k the same as a prefix over those lanes alone) and the block's totals (lane k's
    // inclusive prefix): each wave posts its sums and its first ended lane with that lane's
    // inclusive prefixes and end.
    uint32_t k, tpre, opre, ttot, otot, eob_end;
    {
      const uint64_t em = __ballot(r.st != LR_RUN);
      const uint32_t wf = em ? uni((uint32_t)__builtin_ctzll(em)) : (uint32_t)WAVE;
      const uint32_t it = wave_incl_scan(r.ntok), io = wave_incl_scan(r.nout);
      if (lane == WAVE - 1) {
        sm.wsum[wid] = it;
        sm.wsum2[wid] = io;
      }

      if (lane == (wf < WAVE ? wf : 0u)) {
        sm.wk[wid] = wf < WAVE ? tid : NT;
        sm.wkt[wid] = it;
        sm.wko[wid] = io;
        sm.wke[wid] = (r.st == LR_EOB && r.exit <= limit) ? r.exit : NOPOS;
      }
      __syncthreads();
      uint32_t bt = 0, bo = 0, at = 0, ao = 0;
      k = NT;
      ttot = otot = 0;
      eob_end = NOPOS;
#pragma unroll
      for (uint32_t w = 0; w < NT / WAVE; ++w) {
        const uint32_t st = sm.wsum[w], so = sm.wsum2[w], wkw = sm.wk[w];
        if (k == NT) {
          if (wkw < NT) {
            k = wkw;
            ttot = at + sm.wkt[w];
            otot = ao + sm.wko[w];
            eob_end = sm.wke[w];
          } else {
            at += st;
            ao += so;
          }
        }
        if (w < wid) {
          bt += st;
          bo += so;
        }
      }
      k = uni(k);
      ttot = uni(ttot);
      otot = uni(otot);
      eob_end = uni(eob_end);
      tpre = bt + it - r.ntok;
      opre = bo + io - r.nout;
    }
#ifdef SBH_HUFF_PROBE
    const uint64_t tp3 = __builtin_readcyclecounter();
    if (SM::NT == HT && tid == 0) {  // (k_huff only: the tail kernel's passes are not in the report)
      atomicAdd(&hp_acc[1], tph - tp0);
      atomicAdd(&hp_acc[2], tp1 - tph);
      atomicAdd(&hp_acc[3], tp3 - tp1);
      atomicAdd(&hp_acc[5], (unsigned long long)nrounds);
      atomicAdd(&hp_acc[6], 1ull);
      atomicAdd(&hp_acc[11], (unsigned long long)ttot);
    }
#endif
#ifdef SBH_HUFF_TIMING  // A/B phase-cost probe (timing only, results wrong): the first deflate block's
                        // passes, none of the checks; bit 0: no repair rounds, bit 1: no emit pass
    {
      uint32_t bad = 0;
      if ((SBH_HUFF_TIMING & 2) == 0)
        lane_run<RUN_EMIT>(sm.t, src, A, stop, limit, ck, none, tk + ((tid * 16) & 2047), opre, bad);  // (in bounds)
      __syncthreads();
      ntok_out = 0;
      return PAR_OK;
    }
#endif
    if (k >= NT || eob_end == NOPOS || otot > usize - out) return PAR_FAIL;
    // pass 3: emit
    uint32_t bad = 0;
    if (tid <= k) {
#if SBH_ASM_EMIT
      if (LDS)
        emit_asm(sm.t, sm.stage, A, stop, limit, tk + ntok, tpre, out_before + out + opre, bad);
      else
#endif
        lane_run<RUN_EMIT>(sm.t, src, A, stop, limit, ck, none, tk + ntok + tpre, out_before + out + opre, bad);
    }
    if (__syncthreads_or(bad)) return PAR_FAIL;
#ifdef SBH_HUFF_PROBE
    if (SM::NT == HT && tid == 0) atomicAdd(&hp_acc[4], __builtin_readcyclecounter() - tp3);
#endif
    ntok += ttot;
    out += otot;
    p = eob_end;
#ifdef SBH_HUFF_FIRST_ONLY  // A/B probe (timing only, results wrong): the first deflate block alone
    ntok_out = ntok;
    return PAR_OK;
#endif
    if (last) break;
    // (the tail's two words go where its tokens will start: ntok + 2 <= usize keeps them
    // inside the block's token region)
    if (tail_ok && (limit - p) * 4 < limit && ntok + 2 <= usize) {
      *tail_p = p;
      *tail_out = out;
      ntok_out = ntok;
      return PAR_TAIL;
    }
  }
  if (out != usize) return PAR_FAIL;
  ntok_out = ntok;
  return PAR_OK;
}

// First-header pre-pass: the first deflate block of every BGZF block starts at the
// block's first data bit, so its dynamic header (code-length walk, canonical tables) can
// be decoded before k_huff runs, by one small wave per block at high occupancy (3.7 KB of
// LDS: HdrSmem), instead of on k_huff's critical path with three of its four waves idle.  The PAR tables, the
// sorted entries / limits slow_lane reads, the bit after the header and BFINAL go to
// the end of the block's token region (k_huff copies them into LDS before it writes a
// token).  Anything this pass does not accept (fixed / stored first block, a header
// longer than the staged bits, any invalid code) leaves HDR_STATUS != HDR_OK and k_huff
// decodes that header itself, so results are unchanged.
struct HdrSrc {  // bits of the staged dwords [0, n) (clamped reads past them are never used)
  const uint32_t *p;
  uint32_t n;
  __device__ __forceinline__ uint32_t bits32(uint32_t pos) const {
    const uint32_t i = pos >> 5;
    const uint32_t a = p[i < n ? i : n - 1], b = p[i + 1 < n ? i + 1 : n - 1];
    return __builtin_amdgcn_alignbit(b, a, pos & 31);
  }
};

// k_hdr's LDS: WaveSmem's header-time members only (the code-length-code table instead of
// the 8 KB decode tables, which go straight to HBM), so many more headers are in flight.
struct HdrSmem {
  uint32_t lit[1 << CL_FAST];  // the code-length-code table (build_table's CL format)
  uint16_t sorted[320];
  uint8_t lens[320];
  uint8_t cl_lens[20];
  uint32_t cnt[2][16];
  uint32_t pk[2][16];
  uint32_t sent[320];
};

__device__ __forceinline__ bool huff_serial_block(const DevBlocks &bl, uint64_t b) {
  const uint32_t csize = bl.csize[b], hsize = bl.hsize[b], usize = bl.usize[b];
  return (bl.flags[b] & BLK_TRUNCATED) || usize > 65536u || usize < PAR_MIN_USIZE ||
         (int32_t)csize - (int32_t)hsize - 8 < 0;
}

#ifndef SBH_HDR_WAVES
#define SBH_HDR_WAVES 4
#endif
constexpr uint32_t HDR_WAVES = SBH_HDR_WAVES;  // blocks (one per wave) per k_hdr workgroup
#ifndef SBH_TAIL_HDR
#define SBH_TAIL_HDR 1  // the tails' headers decoded and tabled by k_hdr<true> between k_huff and k_huff_tail
#endif

// A tail's header record fits between its two leading words (tok[G + n1 ..]) and the end of the
// block's token region; k_huff_tail reads it there, before any tail token is written over it.
__device__ __forceinline__ bool tail_hdr_room(uint32_t n1, uint32_t usize) {
  return SBH_TAIL_HDR && n1 <= usize && usize - n1 >= HDR_OUT_DW + 2;
}

// TAIL: the header of a tail k_huff left (INF_TAIL), at the bit its two leading words give --
// the same record, in the same place, in the bit coordinates k_huff_tail decodes in (its stage
// starts at the dword holding the tail's first bit).
template <bool TAIL>
__global__ __launch_bounds__(WAVE * HDR_WAVES) void k_hdr(const uint8_t *__restrict__ comp, DevBlocks bl,
                                                         uint64_t nblocks, uint32_t *__restrict__ tok) {
  __shared__ HdrSmem tw[HDR_WAVES];
  __shared__ uint32_t stagew[HDR_WAVES][HDR_STAGE_DW];
  const uint32_t lane = threadIdx.x & (WAVE - 1), wid = uni(threadIdx.x / WAVE);
  const uint64_t b = (uint64_t)blockIdx.x * HDR_WAVES + wid;  // waves work alone: no workgroup barriers
  if (b >= nblocks) return;
  if (TAIL ? uni(bl.status[b]) != INF_TAIL : huff_serial_block(bl, b)) return;
  HdrSmem &t = tw[wid];
  uint32_t *stage = stagew[wid];
  const uint64_t cstart = bl.cstart[b];
  const uint32_t csize = bl.csize[b], hsize = bl.hsize[b], usize = bl.usize[b];
  const uint32_t data_len = csize - hsize - 8;
  const uint64_t dbyte = cstart + hsize;
  uint32_t skip = (uint32_t)(dbyte & 3) * 8;
  uint32_t limit = skip + data_len * 8;
  // 64-bit byte address of the block's first deflate dword (no 32-bit dword index)
  const uint8_t *dbase = comp + (dbyte & ~3ull);
  if (TAIL) {
    const uint32_t n1 = uni(bl.ntok[b]);
    if (!tail_hdr_room(n1, usize)) return;  // (k_huff_tail decodes this header itself)
    const uint32_t p = uni(tok[bl.ustart[b] + n1]), pd = p >> 5;
    dbase += 4ull * pd;
    skip = p & 31;
    limit -= 32 * pd;
  }
  const uint32_t ndw = min((limit + 31) / 32 + 2, HDR_STAGE_DW);
  const uint32_t *g = reinterpret_cast<const uint32_t *>(dbase);
  {
    // every load before any store (index clamped: a load in the loop was waited for before the next)
    constexpr uint32_t R = (HDR_STAGE_DW + WAVE - 1) / WAVE;
    uint32_t v[R];
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) v[r] = g[min(lane + r * WAVE, ndw - 1)];
#pragma unroll
    for (uint32_t r = 0; r < R; ++r)
      if (lane + r * WAVE < ndw) stage[lane + r * WAVE] = v[r];
  }
  __builtin_amdgcn_wave_barrier();  // (a wave's LDS accesses complete in order)
  uint32_t *out = tok + bl.ustart[b] + usize - HDR_OUT_DW;
  const HdrSrc src{stage, ndw};
  // every code-length symbol start the walk visits keeps its 32-bit reads inside the stage
  const uint32_t lim = min(limit, ndw * 32 > 96 ? ndw * 32 - 96 : 0u);
  const uint32_t hb = uni(src.bits32(skip));
  const uint32_t nlen = ((hb >> 3) & 31) + 257, ndist = ((hb >> 8) & 31) + 1, ncode = ((hb >> 13) & 15) + 4;
  bool ok = ((hb >> 1) & 3) == 2 && skip + 17 <= lim && nlen <= 286 && ndist <= 30;
  uint32_t q = 0;
  if (ok) ok = hdr_walk(t, src, skip, lim, nlen, ndist, ncode, lane, q, nullptr, nullptr);
  if (ok) {
    const uint32_t r0 = ptable_meta(t, t.lens, nlen, 0, lane);
    const uint32_t r1 = ptable_meta(t, t.lens + 288, ndist, 1, lane);
    ok = r0 != 1 && r1 != 1;
  }
  __builtin_amdgcn_wave_barrier();
  if (ok) {
    uint32_t lj0[16], lj1[16];
#pragma unroll
    for (uint32_t v = 1; v <= 15; ++v) {
      lj0[v] = t.pk[0][v] >> 16;
      lj1[v] = t.pk[1][v] >> 16;
    }
#pragma unroll 4
    for (uint32_t i = lane; i < (1u << LIT_FAST); i += WAVE) out[i] = ptable_lit_entry(t, lj0, i);
#pragma unroll 4
    for (uint32_t i = lane; i < (1u << PDIST_FAST); i += WAVE)
      out[(1u << LIT_FAST) + i] = ptable_entry(t, lj1, 1, PDIST_FAST, i);
    for (uint32_t i = lane; i < 320; i += WAVE) out[HDR_SENT + i] = t.sent[i];
    if (lane < 32) out[HDR_PK + lane] = t.pk[lane >> 4][lane & 15];
    if (lane == 0) {
      out[HDR_PSYM] = q;
      out[HDR_LAST] = hb & 1;
    }
  }
  if (lane == 0) out[HDR_STATUS] = ok ? HDR_OK : 0u;
}

#ifdef SBH_HUFF_PROBE
// (probe) one BGZF block done: its whole-block cycles when `timed` (the parallel path; tails
// counted up to the hand-off), and the per-launch report once every block of the launch is done
__device__ void huff_probe_done(uint32_t tid, uint64_t nblocks, uint64_t hk0, bool timed) {
  if (tid != 0) return;
  if (timed) {
    atomicAdd(&hp_acc[7], __builtin_readcyclecounter() - hk0);
    atomicAdd(&hp_acc[14], 1ull);
  }
  __threadfence();
  if (atomicAdd(&hp_done, 1u) == (uint32_t)nblocks - 1) {
    unsigned long long a[15];
    for (int k = 0; k < 15; ++k) a[k] = atomicExch(&hp_acc[k], 0ull);
    hp_done = 0;
    const double n = (double)(a[14] ? a[14] : 1), d = (double)(a[6] ? a[6] : 1);
    printf("huffprobe blocks %llu (parallel %.0f) deflate %.0f per-BGZF-block cycles: stage %.0f hdr %.0f (cl %.0f walk %.0f tables %.0f) p1 %.0f p2 %.0f (rounds/defl %.2f) p3 %.0f whole %.0f tokens/defl %.0f | p2 to end of round1 %.0f round2 %.0f\n",
           (unsigned long long)nblocks, n, d, a[0] / n, a[1] / n, a[8] / n, a[9] / n, a[10] / n, a[2] / n, a[3] / n,
           a[5] / d, a[4] / n, a[7] / n, a[11] / d, a[12] / n, a[13] / n);
  }
}
#endif

__global__ __launch_bounds__(HT, SBH_HUFF_OCC) void k_huff(const uint8_t *__restrict__ comp, DevBlocks bl, uint64_t nblocks,
                                              uint32_t *__restrict__ tok) {
  __shared__ HuffSmem sm;
  const uint32_t tid = threadIdx.x, lane = tid & (WAVE - 1), wid = uni(tid / WAVE);
  const uint64_t b = blockIdx.x;
  if (b >= nblocks) return;
  const uint64_t cstart = bl.cstart[b];
  const uint32_t csize = bl.csize[b], hsize = bl.hsize[b], usize = bl.usize[b];
  const uint64_t G = bl.ustart[b];
  // The payload is one final stored deflate block exactly (BGZF level 0): zlib's output is
  // the LEN stored bytes, so k_lz copies them (ntok = NTOK_STORED) instead of resolving a
  // literal token per byte from the serial decoder.
  if (!(bl.flags[b] & BLK_TRUNCATED) && usize - 1u < 65535u && (int32_t)csize - (int32_t)hsize - 8 == (int32_t)usize + 5) {
    const uint64_t d = cstart + hsize;
    const uint32_t b0 = comp[d], len = comp[d + 1] | (uint32_t)comp[d + 2] << 8;
    const uint32_t nlen = comp[d + 3] | (uint32_t)comp[d + 4] << 8;
    if ((b0 & 7u) == 1u && len == usize && (len ^ nlen) == 0xffffu) {
      if (tid == 0) {
        bl.status[b] = INF_OK;
        bl.ntok[b] = NTOK_STORED;
      }
#ifdef SBH_HUFF_PROBE
      huff_probe_done(tid, nblocks, 0, false);
#endif
      return;
    }
  }
  const bool serial = huff_serial_block(bl, b);
#ifdef SBH_HUFF_PROBE
  const uint64_t hk0 = __builtin_readcyclecounter();
#endif
  if (!serial) {
    const uint32_t data_len = csize - hsize - 8;
    const uint64_t dbyte = cstart + hsize;
    // the block's deflate dwords, addressed from a 64-bit byte base (a 32-bit dword index
    // into the shard would wrap past 16 GiB of compressed bytes)
    const uint8_t *dbase = comp + (dbyte & ~3ull);
    const uint32_t skip = (uint32_t)(dbyte & 3) * 8;
    const uint32_t limit = skip + data_len * 8;
    const uint32_t ndw = (limit + 31) / 32 + 2;
    uint32_t ntok = 0, rc, tail_p = 0, tail_out = 0;
    // the first deflate block's header, decoded and tabled by k_hdr at the end of this
    // block's token region (read here before any token is written over it)
    const uint32_t *hd = tok + G + usize - HDR_OUT_DW;
    // the record's dwords go to registers first, loaded before its status is known (its place is
    // inside the token region whatever the status: PAR_MIN_USIZE > HDR_OUT_DW), so the record,
    // its status and the stage are one round trip and only the LDS stores wait
    constexpr uint32_t NTV = HDR_SENT / HT, NSV = (320 + 32 + HT - 1) / HT;
    uint32_t tv[NTV], sv[NSV];
#pragma unroll
    for (uint32_t k = 0; k < NTV; ++k) tv[k] = hd[tid + k * HT];
#pragma unroll
    for (uint32_t k = 0; k < NSV; ++k) sv[k] = hd[HDR_SENT + min(tid + k * HT, 351u)];
    const uint32_t h_st = hd[HDR_STATUS], h_psym = hd[HDR_PSYM], h_last = hd[HDR_LAST];
    bool pre = false;
    uint32_t pre_psym = 0, pre_last = 0;
    auto take_record = [&]() {  // (after the stage's loads are issued: its wait covers the record's)
      pre = uni(h_st) == HDR_OK;
      pre_psym = pre ? uni(h_psym) : 0u;
      pre_last = pre ? uni(h_last) : 0u;
    };
    auto put_tables = [&]() {
#pragma unroll
      for (uint32_t k = 0; k < NTV; ++k) sm.t.tab[tid + k * HT] = tv[k];
#pragma unroll
      for (uint32_t k = 0; k < NSV; ++k) {  // sent[320] then pk[2][16]
        const uint32_t i = tid + k * HT;
        if (i < 320) sm.t.sent[i] = sv[k];
        else if (i < 352) sm.t.pk[(i - 320) >> 4][(i - 320) & 15] = sv[k];
      }
    };
    if (ndw <= STAGE_DW) {
      const uint32_t *g = reinterpret_cast<const uint32_t *>(dbase);
      // every stage load before any store (the index clamped): a loop of loads and stores left a
      // remainder whose loads were each waited for before the next
      constexpr uint32_t RS = (STAGE_DW + HT - 1) / HT;
      uint32_t sg[RS];
#pragma unroll
      for (uint32_t r = 0; r < RS; ++r) sg[r] = g[min(tid + r * HT, ndw - 1)];
#pragma unroll
      for (uint32_t r = 0; r < RS; ++r)
        if (tid + r * HT < ndw) sm.stage[tid + r * HT] = sg[r];
      take_record();
      if (pre) put_tables();
      __syncthreads();
#ifdef SBH_HUFF_PROBE
      if (tid == 0) atomicAdd(&hp_acc[0], __builtin_readcyclecounter() - hk0);
#endif
      rc = inflate_par<true>(sm, dbase, skip, limit, usize, tok + G, tid, lane, wid, ntok, pre, pre_psym, pre_last, 0,
                             SBH_TAIL != 0, &tail_p, &tail_out);
    } else {
      take_record();
      if (pre) {
        put_tables();
        __syncthreads();
      }
      rc = inflate_par<false>(sm, dbase, skip, limit, usize, tok + G, tid, lane, wid, ntok, pre, pre_psym, pre_last,
                              0, SBH_TAIL != 0, &tail_p, &tail_out);
    }
    if (uni(rc) == PAR_TAIL) {  // k_huff_tail decodes the rest: its start bit and bytes so far at tok[ntok..]
      if (tid == 0) {
        tok[G + ntok] = tail_p;
        tok[G + ntok + 1] = tail_out;
        bl.ntok[b] = ntok;
        bl.status[b] = INF_TAIL;
      }
#ifdef SBH_HUFF_PROBE
      huff_probe_done(tid, nblocks, hk0, true);
#endif
      return;
    }
    if (uni(rc) == PAR_OK) {
      if (tid == 0) {
        bl.status[b] = INF_OK;
        bl.ntok[b] = ntok;
      }
#ifdef SBH_HUFF_PROBE
      huff_probe_done(tid, nblocks, hk0, true);
#endif
      return;
    }
  }
  if (tid == 0) bl.status[b] = INF_SERIAL;  // k_huff_serial<true> decodes it
#ifdef SBH_HUFF_PROBE
  huff_probe_done(tid, nblocks, hk0, false);
#endif
}

// The rest of a block k_huff deferred (INF_TAIL: a short final deflate block, typically),
// by one wave per block: that block's header and the lane-parallel passes over 64 lanes,
// with the remaining compressed bytes staged from the tail's first dword (1 KiB; longer
// tails read global memory).  The tokens continue at tok[ntok]; anything the fast path
// does not prove leaves INF_SERIAL, and the serial decoder redoes the whole block.
#ifndef SBH_TAIL_DW
#define SBH_TAIL_DW 256  // (A/B: 1024 -> 256 dwords: k_huff incl. tail 2.324 -> 2.214 ms at 4 M records; more tails per CU)
#endif
#ifndef SBH_TAIL_NT
#define SBH_TAIL_NT 64  // lanes per tail (one wave; 128: the header's two tables built by two waves)
#endif
constexpr uint32_t TAIL_DW = SBH_TAIL_DW, TAIL_NT = SBH_TAIL_NT;
static_assert(TAIL_NT % WAVE == 0 && TAIL_NT <= 256, "whole waves per tail");
using TailSmem = HuffSmemT<TAIL_NT, TAIL_DW>;
__global__ __launch_bounds__(TAIL_NT) void k_huff_tail(const uint8_t *__restrict__ comp, DevBlocks bl, uint64_t nblocks,
                                                       uint32_t *__restrict__ tok) {
  __shared__ TailSmem sm;
  const uint64_t b = blockIdx.x;
  if (b >= nblocks || uni(bl.status[b]) != INF_TAIL) return;
  const uint32_t tid = threadIdx.x, lane = tid & (WAVE - 1), wid = uni(tid / WAVE);
  const uint64_t cstart = bl.cstart[b];
  const uint32_t csize = bl.csize[b], hsize = bl.hsize[b], usize = bl.usize[b];
  const uint64_t G = bl.ustart[b];
  const uint32_t n1 = uni(bl.ntok[b]);
  uint32_t *tk = tok + G + n1;
  const uint32_t p = uni(tk[0]), out1 = uni(tk[1]);  // (read before any token overwrites them)
  const uint64_t dbyte = cstart + hsize;
  const uint32_t limit0 = (uint32_t)(dbyte & 3) * 8 + (csize - hsize - 8) * 8;
  // rebased at the dword holding the tail's first bit
  const uint32_t pd = p >> 5;
  const uint8_t *dbase = comp + (dbyte & ~3ull) + 4ull * pd;
  const uint32_t skip = p & 31, limit = limit0 - 32 * pd;
  const uint32_t ndw = (limit + 31) / 32 + 2;
  // the tail's first header, from k_hdr<true> (same place and format as k_huff's first one)
  // (the record is read whatever its status -- its place is inside the token region, usize >=
  // PAR_MIN_USIZE -- so the record, its status and the stage are loaded in one round trip)
  const uint32_t *hd = tok + G + usize - HDR_OUT_DW;
  constexpr uint32_t NTV = HDR_SENT / TAIL_NT, NSV = (352 + TAIL_NT - 1) / TAIL_NT;
  uint32_t tv[NTV], sv[NSV];
#pragma unroll
  for (uint32_t k = 0; k < NTV; ++k) tv[k] = hd[tid + k * TAIL_NT];
#pragma unroll
  for (uint32_t k = 0; k < NSV; ++k) sv[k] = hd[HDR_SENT + min(tid + k * TAIL_NT, 351u)];
  const uint32_t h_st = hd[HDR_STATUS], h_psym = hd[HDR_PSYM], h_last = hd[HDR_LAST];
  bool pre = false;
  uint32_t pre_psym = 0, pre_last = 0;
  auto take_record = [&]() {
    pre = tail_hdr_room(n1, usize) && uni(h_st) == HDR_OK;
    if (!pre) return;
    pre_psym = uni(h_psym);
    pre_last = uni(h_last);
#pragma unroll
    for (uint32_t k = 0; k < NTV; ++k) sm.t.tab[tid + k * TAIL_NT] = tv[k];
#pragma unroll
    for (uint32_t k = 0; k < NSV; ++k) {  // sent[320] then pk[2][16]
      const uint32_t i = tid + k * TAIL_NT;
      if (i < 320) sm.t.sent[i] = sv[k];
      else if (i < 352) sm.t.pk[(i - 320) >> 4][(i - 320) & 15] = sv[k];
    }
  };
  uint32_t n2 = 0, rc;
  if (ndw <= TAIL_DW) {
    const uint32_t *g = reinterpret_cast<const uint32_t *>(dbase);
    constexpr uint32_t R = (TAIL_DW + TAIL_NT - 1) / TAIL_NT;
    uint32_t v[R];  // (every load before any store, the index clamped)
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) v[r] = g[min(tid + r * TAIL_NT, ndw - 1)];
#pragma unroll
    for (uint32_t r = 0; r < R; ++r)
      if (tid + r * TAIL_NT < ndw) sm.stage[tid + r * TAIL_NT] = v[r];
    take_record();
    __syncthreads();
    rc = inflate_par<true>(sm, dbase, skip, limit, usize - out1, tk, tid, lane, wid, n2, pre, pre_psym, pre_last, out1,
                           false, nullptr, nullptr);
  } else {
    take_record();
    __syncthreads();
    rc = inflate_par<false>(sm, dbase, skip, limit, usize - out1, tk, tid, lane, wid, n2, pre, pre_psym, pre_last,
                            out1, false, nullptr, nullptr);
  }
  if (tid == 0) {
    bl.status[b] = uni(rc) == PAR_OK ? INF_OK : INF_SERIAL;
    bl.ntok[b] = n1 + n2;
  }
}

#ifndef SBH_LZ_TPT
#define SBH_LZ_TPT 3
#endif
constexpr uint32_t LZ_TPT = SBH_LZ_TPT;                       // tokens per thread per chunk
constexpr uint32_t LZ_CHUNK = LZ_THREADS * LZ_TPT;      // tokens per chunk
constexpr uint32_t PTR_HALF = 8;                        // pointer slots per thread and pass
#ifndef SBH_LZ_RING
// k_lz's block image as a ring of 32 KiB of history + one pass, flushed to U pass by pass, so that
// three workgroups fit a CU (6656-byte passes, 80 VGPRs: 6 waves per SIMD) instead of two with the
// whole 64 KiB image (A/B r05y, output identical: k_lz -13% B, -15% D, -11% E)
#define SBH_LZ_RING 1
#endif
#ifndef SBH_LZ_PTR_CAP
#define SBH_LZ_PTR_CAP (SBH_LZ_RING ? 6656 : 7552)
#endif
constexpr uint32_t PTR_CAP = SBH_LZ_PTR_CAP;            // bytes one pointer-chasing pass resolves
constexpr uint32_t SB_WORDS = PTR_CAP / 32;             // token-start bitmap words
constexpr uint32_t NHP = 2;                             // half granules (8 slots) per k_lz thread, at most
static_assert(PTR_CAP <= NHP * LZ_THREADS * PTR_HALF, "slot pass covers the slots");

// image bytes: the whole block, or (ring) the deflate window before a pass plus the pass itself
// (a pass's pointers reach at most 32768 bytes before its first byte), a multiple of 16 so
// granules stay whole; image position q lives at q mod LZ_IMG (q < 2 LZ_IMG always)
constexpr uint32_t LZ_IMG = SBH_LZ_RING ? (32768u + PTR_CAP + 16u + 15u) / 16u * 16u : 65536u + 16u;
static_assert(!SBH_LZ_RING || 65536u + 16u < 2 * LZ_IMG, "one subtraction maps an image position into the ring");
__device__ __forceinline__ uint32_t lz_ri(uint32_t q) {
  if (!SBH_LZ_RING) return q;
  const uint32_t r = q - LZ_IMG;
  return r < q ? r : q;  // (q < LZ_IMG: r wraps above q)
}
struct LzSmem {
  uint8_t img[LZ_IMG];  // block image (or its ring), placed at (ustart & 15) so granules align with HBM
  struct {
    uint16_t p16[PTR_CAP];     // per pass byte: its source pointer (token starts first)
    uint32_t sbits[SB_WORDS];  // per pass byte: starts a token (every byte of a long match)
    uint32_t wsum[LZ_THREADS / WAVE];  // block_scan scratch
    uint32_t wmin[LZ_THREADS / WAVE];  // block_min scratch (a pass cut)
  } pp;
};
// two workgroups per CU (three with the ring), counting the 256 B of LDS the compiler adds
static_assert(sizeof(LzSmem) * 2 + 512 <= 160 * 1024, "two k_lz workgroups per CU");
static_assert(!SBH_LZ_RING || sizeof(LzSmem) * 3 + 768 <= 160 * 1024, "three k_lz workgroups per CU with the ring");

// k mod d for k < 2^17, d >= 1 (one reciprocal, one correction).
__device__ __forceinline__ uint32_t mod_small(uint32_t k, uint32_t d) {
  const uint32_t q = (uint32_t)((float)k * __builtin_amdgcn_rcpf((float)d));
  int32_t r = (int32_t)(k - q * d);
  r = r < 0 ? r + (int32_t)d : r;
  return (uint32_t)(r >= (int32_t)d ? r - (int32_t)d : r);
}

// Eight u16 slot values (positions; ones before the block may have wrapped) as a uint4.
__device__ __forceinline__ uint4 pack8_u16(const uint32_t *c) {
  return make_uint4(__builtin_amdgcn_perm(c[1], c[0], 0x05040100u), __builtin_amdgcn_perm(c[3], c[2], 0x05040100u),
                    __builtin_amdgcn_perm(c[5], c[4], 0x05040100u), __builtin_amdgcn_perm(c[7], c[6], 0x05040100u));
}

#ifndef SBH_LZ_NO_END_BAR
#define SBH_LZ_NO_END_BAR 1  // k_lz: no barrier at a chunk's end (the next chunk's scan barrier orders it; A/B: k_lz -3% B, -2% D, -3% E)
#endif
#ifndef SBH_ASM_CHASE
#define SBH_ASM_CHASE 1  // k_lz's pointer chase as the hand-written loop below
#endif
#ifndef SBH_LZ_SLOT128
#define SBH_LZ_SLOT128 1  // k_lz slot pass: a thread's 8 start values from one 16-byte read of its own slots
#endif
#ifndef SBH_LZ_SBMASK
#define SBH_LZ_SBMASK 0  // 1: k_lz marks OR a thread's start bits per word (A/B r04e: +0.5..3% k_lz: kept off)
#endif
#ifndef SBH_LZ_LMARK_MIN
#define SBH_LZ_LMARK_MIN 1  // k_lz: long matches per wave and token slot from which their threads mark them (A/B r04f: 1 best; 99 = wave-serial only: D +11%)
#endif
constexpr uint32_t LZ_LMARK_MIN = SBH_LZ_LMARK_MIN;
#ifndef SBH_LZ_OVL_WAVE
#define SBH_LZ_OVL_WAVE 0  // 1: overlapping short matches (dist < len) marked byte by byte by the wave (A/B r04c: k_lz +5% B, +26% D, +10% E: kept off)
#endif
#ifndef SBH_LZ_CARRY
#define SBH_LZ_CARRY 1  // k_lz: a chunk that overflows its pass ends at the cut; the next chunk starts there
#endif
#ifndef SBH_LZ_NOCLAMP
#define SBH_LZ_NOCLAMP 1  // the chase reads settled pointers' slots unclamped: one VALU + one SALU fewer per pointer (A/B r04v: k_lz -2.7% B, -2.8% D, -3.4% E)
#endif
#ifndef SBH_LZ_NOHOIST
#define SBH_LZ_NOHOIST 1  // keep the long-match marker mod inside its branch (see k_lz)
#endif
#ifndef SBH_LZ_RUN1
#define SBH_LZ_RUN1 1  // distance-1 matches point every byte at the source byte (no mod branch)
#endif

#ifndef SBH_LZ_MOD2
#define SBH_LZ_MOD2 1  // (with RUN1) overlaps at distance >= 2 chased instead of taking the mod
#endif
#ifndef SBH_LZ_MOD
#define SBH_LZ_MOD 1  // 1: a byte of an overlapping short match points at v + (j mod distance) (0: at v + j, a longer chase: A/B r04p k_lz +4% B, +2% D)
#endif
// (r04n-r04p, measured and removed -- profiles/r04_ab/: each lane's 8 pointers rotated by
// 2 ((h >> 3) & 3) slots so the chase's u16 reads of lanes h, h + 8, h + 16, h + 24 (16 bytes
// apart, one bank) hit four distinct dwords: k_lz +5% B, +4% D, +2.5% E; a thread's two half
// granules chased in one loop (16 reads per round, a single-granule thread chasing a copy):
// +17% B, +19% D, +17% E, and only in the waves that have two (waves 0-3): +10% B, +8% D, +7% E
// (chasing the lower granule first shortens the chains of the higher one); the slot pass's two
// half granules as one straight-line body: +30% B, and only in the waves that have two, every
// LDS read of both issued before either is waited for: +5% B, +3.5% D (the slot pass's time did
// not move: not its round trips); an all-literal half granule skipping its
// gather: +3% B; the slot pass without its range test in waves wholly inside the pass: +0.7% B,
// -1% E; one pending flag per half granule instead of a bit per slot: +0.6% B, -4% E; full
// chunks without the per-token bound tests: +0.3% B, +2.4% D, +1.6% E; beyond distance 1,
// overlap bytes with j < 2 d pointed one period back / power-of-two distances by a mask, both
// without the mod: +5% / +2% B;
// 1024-token chunks (SBH_LZ_TPT=2): +10% B, +6% D.  Each variant that added LDS instructions or
// VALU work per byte lost more than the latency it overlapped or the conflicts it removed.)

// k_lz's pointer chase for one half granule (8 slots) as hand-written code, the same rounds as
// the C++ loop: every pointer at or past the pass start pb is replaced by its target's slot
// value (u16 LDS reads at 2 c + p16 - 2 * abase, all 8 issued before the first is
// waited for), the 8 slots written back as 16 bytes at w0, until no pointer of the lane moved to
// another in-pass position.  4 vector + 2 scalar instructions per pointer and round besides
// the read (SBH_LZ_NOCLAMP; the compiler's version: ~9 and ~3, plus a register rotation of the
// 8 pointers every round); a read's address register takes its result (8 VGPRs fewer: k_lz -1% B).
#if SBH_LZ_NOCLAMP
// (no clamp to the pass start: a settled pointer c < pb reads whatever LDS word 2 c + off names
// -- the image below the slots, or nothing (an out-of-range LDS read returns 0) -- and the
// value is dropped: c moves only when pb <= c.  A pointer moves on in the pass when
// pb <= r < c: slot values never exceed their slot, so r != c is r < c)
#define SBH_CH_ADDR(k) "v_lshl_add_u32 %[a" #k "], %[c" #k "], 1, %[off]\n\t" \
                       "ds_read_u16 %[a" #k "], %[a" #k "]\n\t"
#define SBH_CH_STEP(k, w) "s_waitcnt lgkmcnt(" #w ")\n\t" \
                          "v_cmp_le_u32 vcc, %[pb], %[c" #k "]\n\t" \
                          "v_cmp_lt_u32 %[sx], %[a" #k "], %[c" #k "]\n\t" \
                          "v_cmp_le_u32 %[sy], %[pb], %[a" #k "]\n\t" \
                          "s_and_b64 %[sx], %[sx], %[sy]\n\t" \
                          "s_or_b64 %[sc], %[sc], %[sx]\n\t" \
                          "v_cndmask_b32_e32 %[c" #k "], %[c" #k "], %[a" #k "], vcc\n\t"
#else
#define SBH_CH_ADDR(k) "v_max_u32 %[a" #k "], %[pb], %[c" #k "]\n\t" \
                       "v_lshl_add_u32 %[a" #k "], %[a" #k "], 1, %[off]\n\t" \
                       "ds_read_u16 %[a" #k "], %[a" #k "]\n\t"
#define SBH_CH_STEP(k, w) "s_waitcnt lgkmcnt(" #w ")\n\t" \
                          "v_cmp_le_u32 vcc, %[pb], %[c" #k "]\n\t" \
                          "v_cmp_ne_u32 %[sx], %[a" #k "], %[c" #k "]\n\t" \
                          "v_cmp_le_u32 %[sy], %[pb], %[a" #k "]\n\t" \
                          "s_and_b64 %[sx], %[sx], vcc\n\t" \
                          "s_and_b64 %[sx], %[sx], %[sy]\n\t" \
                          "s_or_b64 %[sc], %[sc], %[sx]\n\t" \
                          "v_cndmask_b32_e32 %[c" #k "], %[c" #k "], %[a" #k "], vcc\n\t"
#endif
#define SBH_CH_WB(w, k0, k1, k2, k3, k4, k5, k6, k7) \
  "v_perm_b32 %[a" #k0 "], %[c" #k1 "], %[c" #k0 "], %[sel]\n\t" \
  "v_perm_b32 %[a" #k1 "], %[c" #k3 "], %[c" #k2 "], %[sel]\n\t" \
  "v_perm_b32 %[a" #k2 "], %[c" #k5 "], %[c" #k4 "], %[sel]\n\t" \
  "v_perm_b32 %[a" #k3 "], %[c" #k7 "], %[c" #k6 "], %[sel]\n\t" \
  "ds_write2_b32 %[" #w "], %[a" #k0 "], %[a" #k1 "] offset1:1\n\t" \
  "ds_write2_b32 %[" #w "], %[a" #k2 "], %[a" #k3 "] offset0:2 offset1:3\n\t"
#define SBH_CH_HEAD "s_mov_b64 %[sv], exec\n\t" \
                    "v_cmp_ne_u32 %[sm], 0, %[pend]\n\t" \
                    "s_and_b64 exec, exec, %[sm]\n\t" \
                    "s_cbranch_execz L_chend%=\n" \
                    "L_round%=:\n\t"
#define SBH_CH_TAIL "s_and_b64 exec, exec, %[sc]\n\t" \
                    "s_cbranch_execnz L_round%=\n" \
                    "L_chend%=:\n\t" \
                    "s_mov_b64 exec, %[sv]"
__device__ __forceinline__ void chase8_asm(uint32_t (&c)[8], uint32_t pend, uint32_t pb, uint32_t off,
                                           uint32_t w0) {
  const uint32_t sel = 0x05040100u;  // v_perm: the low halves of two dwords
  uint32_t a0, a1, a2, a3, a4, a5, a6, a7;
  uint64_t sv, sm, sx, sy, sc;
  asm volatile(SBH_CH_HEAD
      SBH_CH_ADDR(0) SBH_CH_ADDR(1) SBH_CH_ADDR(2) SBH_CH_ADDR(3)
      SBH_CH_ADDR(4) SBH_CH_ADDR(5) SBH_CH_ADDR(6) SBH_CH_ADDR(7)
      "s_mov_b64 %[sc], 0\n\t"
      SBH_CH_STEP(0, 7) SBH_CH_STEP(1, 6) SBH_CH_STEP(2, 5) SBH_CH_STEP(3, 4)
      SBH_CH_STEP(4, 3) SBH_CH_STEP(5, 2) SBH_CH_STEP(6, 1) SBH_CH_STEP(7, 0)
      SBH_CH_WB(w0, 0, 1, 2, 3, 4, 5, 6, 7)
      SBH_CH_TAIL
      : [c0] "+v"(c[0]), [c1] "+v"(c[1]), [c2] "+v"(c[2]), [c3] "+v"(c[3]), [c4] "+v"(c[4]), [c5] "+v"(c[5]),
        [c6] "+v"(c[6]), [c7] "+v"(c[7]), [a0] "=&v"(a0), [a1] "=&v"(a1), [a2] "=&v"(a2), [a3] "=&v"(a3),
        [a4] "=&v"(a4), [a5] "=&v"(a5), [a6] "=&v"(a6), [a7] "=&v"(a7),
        [sv] "=&s"(sv), [sm] "=&s"(sm), [sx] "=&s"(sx), [sy] "=&s"(sy), [sc] "=&s"(sc)
      : [pend] "v"(pend), [pb] "s"(pb), [off] "s"(off), [w0] "v"(w0), [sel] "s"(sel)
      : "vcc", "scc", "memory");
}
#undef SBH_CH_ADDR
#undef SBH_CH_STEP
#undef SBH_CH_WB
#undef SBH_CH_HEAD
#undef SBH_CH_TAIL

// LZ77 resolution of one block per workgroup, LZ_CHUNK tokens per chunk (LZ_TPT consecutive
// tokens per thread); bytes before the chunk are final.  A chunk whose output fits PTR_CAP
// bytes (the common case) is resolved by pointer chasing: every byte gets the position it
// copies from (itself for a literal; match byte k: off - dist + k mod dist, always
// earlier), written by its own token; then each thread follows its 16 bytes' pointers to
// final bytes -- rewriting its slots with the results, which shortens other threads'
// chases -- and gathers.  A longer chunk (long matches) is resolved the same way in
// passes of at most PTR_CAP bytes, each cut at a token start, so every chunk takes the
// pointer path (the dependency-rounds fallback this replaced cost ~100 k cycles per
// overflowing chunk: 2-4 per block of long-read data).
#ifndef SBH_LZ_WAVES_PER_EU
#define SBH_LZ_WAVES_PER_EU (SBH_LZ_RING ? 6 : 4)  // (the register budget: 512 VGPRs / waves per SIMD)
#endif
#ifndef SBH_LZ_SIEVE
// 1: k_lz leaves k_eager's first filter as a bitmap (launch_lz's sieve; run with SBH_SIEVE=1).
// Measured and not kept: k_eager -0.55 ms, k_lz +0.95 ms on config B -- the
// filter's ~180 vector instructions per 16-byte granule are issue time k_lz does not have spare
#define SBH_LZ_SIEVE 0
#endif
// k_eager's first filter at the 16 positions of a granule: eager.Checker reads refID, pos, next
// refID and next pos first (PosChecker.getRefPosError, check/.../PosChecker.scala:43-63; the
// refID / next refID in [-1, n) and pos / next pos >= -1 parts need no contig length), so a
// position failing one of them is false; d[] = the 48 bytes from the granule's first.
__device__ __forceinline__ uint32_t sieve16(const uint32_t (&d)[12], uint32_t nref1) {
  uint32_t m = 0;
#pragma unroll
  for (uint32_t j = 0; j < 16; ++j) {
    const uint32_t q = j >> 2, k = j & 3;
    const uint32_t ref = __builtin_amdgcn_alignbyte(d[q + 2], d[q + 1], k);
    const uint32_t pos = __builtin_amdgcn_alignbyte(d[q + 3], d[q + 2], k);
    const uint32_t nrf = __builtin_amdgcn_alignbyte(d[q + 7], d[q + 6], k);
    const uint32_t nps = __builtin_amdgcn_alignbyte(d[q + 8], d[q + 7], k);
    m |= (ref + 1u < nref1 && nrf + 1u < nref1 && (int32_t)pos >= -1 && (int32_t)nps >= -1) ? 1u << j : 0u;
  }
  return m;
}

__global__ __launch_bounds__(LZ_THREADS, SBH_LZ_WAVES_PER_EU) void k_lz(const uint8_t *__restrict__ comp, DevBlocks bl, uint64_t nblocks,
                                                    const uint32_t *__restrict__ tok, uint8_t *__restrict__ U,
                                                    uint32_t *__restrict__ sieve, uint32_t nref1) {
  __shared__ LzSmem sm;
  uint32_t *wsum = sm.pp.wsum;
  const uint64_t b = blockIdx.x;
  if (b >= nblocks) return;
  const uint32_t t = threadIdx.x;
  [[maybe_unused]] const uint32_t lane = t & (WAVE - 1);
  const uint32_t n = bl.ntok[b];
  const uint64_t G = bl.ustart[b];
  const uint32_t sh = (uint32_t)(G & 15);
  if (n == NTOK_STORED) {  // a stored payload: copy it in 16-byte granules aligned to the flat address
    const uint64_t src = bl.cstart[b] + bl.hsize[b] + 5;
    const uint32_t usize = bl.usize[b];
    const uint64_t g0 = G & ~15ull;
    if (SBH_LZ_SIEVE && sieve) {  // (no ring here: the whole block is "undecided" for k_eager's filter)
      uint16_t *sv = reinterpret_cast<uint16_t *>(sieve) + (g0 >> 4);
      for (uint32_t q = t; q < (sh + usize + 15) / 16; q += LZ_THREADS) sv[q] = 0xffffu;
    }
    // the thread's whole granules: every load first (a granule past the payload reads the
    // first one again and is not stored), then the stores -- one round trip, not one per granule
    constexpr uint32_t NG = (65536u + 16u + 16u * LZ_THREADS - 1u) / (16u * LZ_THREADS);
    uint32_t d[NG][5];
#pragma unroll
    for (uint32_t r = 0; r < NG; ++r) {
      const uint32_t lo = 16 * t + 16 * LZ_THREADS * r;
      const bool whole = lo >= sh && lo + 16 <= sh + usize;
      const uint64_t a = src + (whole ? lo - sh : 0u);
      const uint32_t *w = reinterpret_cast<const uint32_t *>(comp + (a & ~3ull));
#pragma unroll
      for (uint32_t j = 0; j < 5; ++j) d[r][j] = w[j];
    }
#pragma unroll
    for (uint32_t r = 0; r < NG; ++r) {
      const uint32_t lo = 16 * t + 16 * LZ_THREADS * r;
      if (lo >= sh + usize) break;
      if (lo >= sh && lo + 16 <= sh + usize) {
        const uint32_t k = (uint32_t)(src + (lo - sh)) & 3u;
        *reinterpret_cast<uint4 *>(U + g0 + lo) =
            make_uint4(__builtin_amdgcn_alignbyte(d[r][1], d[r][0], k), __builtin_amdgcn_alignbyte(d[r][2], d[r][1], k),
                       __builtin_amdgcn_alignbyte(d[r][3], d[r][2], k), __builtin_amdgcn_alignbyte(d[r][4], d[r][3], k));
      } else {  // the block's partial first / last granule
        for (uint32_t j = 0; j < 16; ++j) {
          const uint32_t x = lo + j;
          if (x >= sh && x < sh + usize) U[g0 + x] = comp[src + (x - sh)];
        }
      }
    }
    return;
  }
  [[maybe_unused]] uint8_t *img = sm.img + sh;
  const uint32_t *tk = tok + G;
  const uint64_t g0u = G & ~15ull;  // flat address of image position 0
#if SBH_LZ_RING
  uint32_t fl = 0;  // image position of the first granule not yet in U (uniform)
  // granules [fl, to) of the ring to U (the first one partial: the image starts at sh)
  auto lz_flush = [&](uint32_t &from, uint32_t to) {
    for (uint32_t q = from / 16 + t; q < to / 16; q += LZ_THREADS) {
      const uint32_t lo = q * 16;
      if (lo >= sh) {
        *reinterpret_cast<uint4 *>(U + g0u + lo) = *reinterpret_cast<const uint4 *>(sm.img + lz_ri(lo));
      } else {
        for (uint32_t k = sh; k < 16; ++k) U[g0u + k] = sm.img[k];
      }
    }
    from = to > from ? to : from;
  };
#endif
#if SBH_LZ_RING && SBH_LZ_SIEVE
  // k_eager's first filter on the bytes in the ring: granule G's 16 positions need image bytes
  // [16 G, 16 G + 48), so its sieve word is written once granule G + 2 is final (flushed); a
  // granule holding another block's positions (the first, when the block does not start on a
  // granule) or positions whose 48 bytes run past the block is all ones -- k_eager decides those
  // itself (both blocks write 0xffff to a shared granule)
  uint16_t *const sv16 = sieve ? reinterpret_cast<uint16_t *>(sieve) + (g0u >> 4) : nullptr;
  uint32_t svf = 0;  // first granule whose sieve word is not written yet (uniform)
  auto lz_sieve = [&](uint32_t upto, uint32_t end_img) {
    for (uint32_t q = svf + t; q < upto; q += LZ_THREADS) {
      const uint32_t lo = q * 16;
      uint32_t m = 0xffffu;
      if (lo >= sh && lo + 48 <= end_img) {
        const uint4 a = *reinterpret_cast<const uint4 *>(sm.img + lz_ri(lo));
        const uint4 b2 = *reinterpret_cast<const uint4 *>(sm.img + lz_ri(lo + 16));
        const uint4 c2 = *reinterpret_cast<const uint4 *>(sm.img + lz_ri(lo + 32));
        const uint32_t d[12] = {a.x, a.y, a.z, a.w, b2.x, b2.y, b2.z, b2.w, c2.x, c2.y, c2.z, c2.w};
        m = sieve16(d, nref1);
      }
      sv16[q] = (uint16_t)m;
    }
    svf = upto > svf ? upto : svf;
  };
#endif

  uint32_t base = 0;  // output offset of the chunk's first token
#ifdef SBH_LZ_PROBE
  uint64_t tp0 = __builtin_readcyclecounter(), t_pre = 0, t_rounds = 0, t_init = 0, t_w = 0, t_ch = 0, t_mk = 0, t_b1 = 0;
  uint32_t nrounds = 0, njumps = 0, nlong = 0;
#endif
#ifndef SBH_LZ_TOUCH
#define SBH_LZ_TOUCH 1  // k_lz: the next chunk's tokens touched into L2 while this chunk's load
#endif
#ifndef SBH_LZ_PREFETCH
// the next chunk's tokens loaded one chunk ahead (0: at the chunk's top).  At the ring's 80 VGPRs
// the prefetched tokens were spilled to scratch right after their load (which then waited for
// them): off for the ring (A/B r05za: k_lz -5% B, -6% D, -5% E, output identical)
#define SBH_LZ_PREFETCH (!SBH_LZ_RING)
#endif
static_assert(!(SBH_LZ_CARRY && SBH_LZ_PREFETCH), "the token prefetch assumes chunks of LZ_CHUNK tokens");
  uint32_t xn[LZ_TPT];  // next chunk's tokens, loaded one chunk ahead
#pragma unroll
  for (uint32_t k = 0; k < LZ_TPT; ++k) xn[k] = LZ_TPT * t + k < n ? tk[LZ_TPT * t + k] : 0;
#if SBH_LZ_CARRY
  uint32_t c0n = 0;  // the next chunk's first token
  for (uint32_t c0 = 0; c0 < n; c0 = c0n) {
    c0n = c0 + LZ_CHUNK;
#else
  for (uint32_t c0 = 0; c0 < n; c0 += LZ_CHUNK) {
#endif
#ifdef SBH_LZ_PROBE
    uint64_t ta = __builtin_readcyclecounter();
#endif
    // this thread's LZ_TPT tokens
    const uint32_t i0 = c0 + LZ_TPT * t;
    uint32_t x[LZ_TPT], len[LZ_TPT], dist[LZ_TPT], off[LZ_TPT];
    bool match[LZ_TPT];
    uint32_t mysum = 0;
#if !SBH_LZ_PREFETCH
    // all of the thread's token loads first, every lane loading (the index clamped): a load under
    // a branch, or one after the previous token's decoding, was waited for before the next one
    // was issued -- LZ_TPT HBM round trips per chunk instead of one
#pragma unroll
    for (uint32_t k = 0; k < LZ_TPT; ++k) x[k] = tk[min(i0 + k, n - 1)];
#if SBH_LZ_TOUCH
    // the next chunk's tokens (as if this chunk is not cut) touched into L2, a dword per 128-byte
    // line, behind this chunk's own loads: their wait covers the touch, and the next chunk's
    // loads then come from L2 instead of HBM
    uint32_t tch = 0;
    {
      const uint32_t nx0 = c0 + LZ_CHUNK + 32 * t;
      if (t < LZ_CHUNK / 32 && nx0 < n)
        asm volatile("global_load_dword %0, %1, off" : "=v"(tch) : "v"(tk + nx0) : "memory");
    }
#endif
#endif
#pragma unroll
    for (uint32_t k = 0; k < LZ_TPT; ++k) {
#if SBH_LZ_PREFETCH
      x[k] = xn[k];
      xn[k] = i0 + LZ_CHUNK + k < n ? tk[i0 + LZ_CHUNK + k] : 0;
#endif
      match[k] = i0 + k < n && (x[k] & TOK_MATCH) != 0;
      len[k] = i0 + k >= n ? 0 : match[k] ? (x[k] >> 16) & 0x1ff : 1 + ((x[k] >> 24) & 1u);  // (TOK_PAIR: 2)
      dist[k] = x[k] & 0xffff;
      mysum += len[k];
    }
#if !SBH_LZ_PREFETCH && SBH_LZ_TOUCH
    asm volatile("" ::"v"(tch));  // (live until the tokens' wait above has covered it)
#endif
    for (uint32_t w = t; w < SB_WORDS; w += LZ_THREADS) sm.pp.sbits[w] = 0;  // ordered by the scan's barrier
    uint32_t chunk_len;
    off[0] = base + block_scan<LZ_THREADS>(mysum, wsum, &chunk_len);
#pragma unroll
    for (uint32_t k = 1; k < LZ_TPT; ++k) off[k] = off[k - 1] + len[k - 1];
    const uint32_t chunk_end = base + chunk_len;
#if SBH_EMIT_NOCHK
    // too far back (zlib's "invalid distance too far back"): a match reaching before the block's
    // first byte fails the block as the serial decoder would (INF_DATA); the Huffman passes no
    // longer test each distance code (a block another path already failed keeps its status)
    {
      bool far = false;
#pragma unroll
      for (uint32_t k = 0; k < LZ_TPT; ++k) {
        const bool fk = match[k] && dist[k] > off[k];
        far = far || fk;
        // the block's bytes no longer matter, but its pointers must stay well formed: the bad
        // match copies from itself (distance 0: every byte's pointer is its own slot, a final
        // pointer), never from before the block (a wrapped u16 the chase would follow)
        dist[k] = fk ? 0u : dist[k];
      }
      if (far && bl.status[b] == INF_OK) bl.status[b] = INF_DATA;
    }
#endif
#ifdef SBH_LZ_PROBE
    const uint64_t tb = __builtin_readcyclecounter();
    t_pre += tb - ta;
#endif
    // Passes over the chunk's output, each at most PTR_CAP bytes (from its 16-byte granule):
    // a pass takes the tokens that START in [pb, pe) and pe is the start of the first token
    // that would end past the pass's slots.  One pass when the chunk fits (the common
    // case); long-match chunks take a few instead of a slower resolution.
    uint32_t pb = base;
    [[maybe_unused]] uint32_t cend = chunk_end;  // (SBH_LZ_CARRY) where this chunk's pass ended
    for (;;) {
#if SBH_LZ_RING
      // every byte before pb is final (the scan's or the last pass's barrier): its whole granules
      // leave the ring for U before the ring wraps onto them
      lz_flush(fl, (sh + pb) & ~15u);
#if SBH_LZ_SIEVE
      if (sv16 && fl >= 48) lz_sieve(fl / 16 - 2, ~0u);
#endif
#endif
      // slots start at the 16-byte LDS granule holding `pb`, so that each thread's 16
      // slots are one granule of the image
      const uint32_t lead = (sh + pb) & 15, abase = pb - lead;
      uint32_t pe = chunk_end;
#if SBH_LZ_CARRY
      // (carry: a chunk is one pass; the tokens from the cut on start the next chunk, so every
      // chunk but the last of a block fills its pass instead of leaving a short second one)
      static_assert(LZ_CHUNK <= 2048 && 65536u + 16u + 258u < (1u << 21), "cut keys: offset << 11 | token");
      if (chunk_end - abase > PTR_CAP) {  // uniform: cut the chunk
        uint32_t cut = ~0u;
#pragma unroll
        for (uint32_t k = 0; k < LZ_TPT; ++k)
          if (i0 + k < n && off[k] + len[k] - abase > PTR_CAP) cut = min(cut, off[k] << 11 | (LZ_TPT * t + k));
        const uint32_t key = block_min<LZ_THREADS>(cut, sm.pp.wmin);
        pe = key >> 11;
        c0n = c0 + (key & 0x7ffu);
      }
#else
      if (chunk_end - abase > PTR_CAP) {  // uniform: cut the chunk
        uint32_t cut = chunk_end;
#pragma unroll
        for (uint32_t k = 0; k < LZ_TPT; ++k)
          if (i0 + k < n && off[k] >= pb && off[k] + len[k] - abase > PTR_CAP) cut = min(cut, off[k]);
        pe = block_min<LZ_THREADS>(cut, sm.pp.wmin);
      }
#endif
      const uint32_t plen = pe - pb;
#ifdef SBH_LZ_PROBE
      nrounds += pe != chunk_end || pb != base;
#endif
      uint16_t *p16 = sm.pp.p16;
      uint32_t *sbits = sm.pp.sbits;
      // Tokens mark their starts: one slot write (a literal points at itself, a short
      // match at its source) and one start bit each; the bytes inside a short match get
      // their pointers in the slot pass below, from the nearest start.
      // a match the wave marks byte by byte: longer than LZ_SHORT, or overlapping itself
      // (dist < len: its bytes repeat a period shorter than the match, a mod per byte)
      bool wide[LZ_TPT];
#pragma unroll
      for (uint32_t k = 0; k < LZ_TPT; ++k)
        wide[k] = match[k] && (len[k] > LZ_SHORT || (SBH_LZ_OVL_WAVE && dist[k] < len[k]));
#if SBH_LZ_SBMASK
      // start bits gathered per word first: a thread's short tokens span at most 3 words (2 x 32
      // bytes), so 3 atomics at most (one when they share a word) instead of one per token
      uint32_t wA = ~0u, mA = 0, mB = 0, mC = 0;
#endif
#pragma unroll
      for (uint32_t k = 0; k < LZ_TPT; ++k) {
        if (i0 + k >= n || wide[k] || !(off[k] - pb < plen)) continue;
        const uint32_t d = off[k] - abase;
        p16[d] = (uint16_t)(match[k] ? off[k] - dist[k] : off[k]);
        if (!match[k]) {
          const uint32_t ia = lz_ri(sh + off[k]);
          sm.img[ia] = (uint8_t)(x[k] >> 8);
          // a literal pair's second byte: no start of its own (the slot pass points it at v + 1,
          // itself); its image index from the first's (the ring wraps at LZ_IMG), computed here
          if (x[k] & TOK_PAIR) {
            uint32_t ib = ia + 1;
            asm volatile("" : "+v"(ib));
            sm.img[SBH_LZ_RING && ib == LZ_IMG ? 0u : ib] = (uint8_t)(x[k] >> 16);
          }
        }
#if SBH_LZ_SBMASK
        const uint32_t w = d >> 5, bit = 1u << (d & 31);
        wA = wA == ~0u ? w : wA;
        const uint32_t r = w - wA;
        mA |= r == 0 ? bit : 0u;
        mB |= r == 1 ? bit : 0u;
        mC |= r == 2 ? bit : 0u;
        if (r > 2)  // (a long match between this thread's short tokens)
          __hip_atomic_fetch_or(&sbits[w], bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#else
        __hip_atomic_fetch_or(&sbits[d >> 5], 1u << (d & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
      }
#if SBH_LZ_SBMASK
      if (mA) __hip_atomic_fetch_or(&sbits[wA], mA, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (mB) __hip_atomic_fetch_or(&sbits[wA + 1], mB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (mC) __hip_atomic_fetch_or(&sbits[wA + 2], mC, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
      // long matches.  Few in a wave (short-read data: one or two): the wave writes every byte's
      // pointer, match by match.  Many (long reads): each thread marks its own with a start every
      // 32 bytes (a pointer and a start bit each), so the slot pass finds every byte's start
      // within 31 slots back as for a short match; a marker at 32 m copies from
      // o - dist + (32 m mod dist) (for an overlapping match the same byte periods earlier).
      // (A/B r04e, k_lz: lane markers -12% on config D, +2.5% on B; wave-serial the reverse.)
#pragma unroll
      for (uint32_t k = 0; k < LZ_TPT; ++k) {
        const bool mine = i0 + k < n && wide[k] && off[k] - pb < plen;
        uint64_t lm = __ballot(mine);
#ifdef SBH_LZ_PROBE
        nlong += __builtin_popcountll(lm);
#endif
        if ((uint32_t)__builtin_popcountll(lm) >= LZ_LMARK_MIN) {
          if (mine) {
            uint32_t D = dist[k];
#if SBH_LZ_NOHOIST
            // (opaque to the compiler, which otherwise computes the mod below for every token of
            // every chunk, ahead of this branch: ~36 VALU per chunk and wave)
            asm volatile("" : "+v"(D));
#endif
            const uint32_t d0 = off[k] - abase, L = len[k];
            const bool ov = D != 0 && D < L;  // (D = 0: a too-far-back match, marked at itself)
            uint32_t r = 0;  // 32 m mod D (ov)
            const uint32_t r32 = ov ? (D > 32 ? 32 : mod_small(32, D)) : 0;
            for (uint32_t m = 0; m < L; m += 32) {
              const uint32_t d = d0 + m;
              p16[d] = (uint16_t)(off[k] - D + (ov ? r : m));
              __hip_atomic_fetch_or(&sbits[d >> 5], 1u << (d & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              r += r32;
              r = r >= D ? r - D : r;
            }
          }
          continue;
        }
        while (lm) {
          const uint32_t l = (uint32_t)__builtin_ctzll(lm);
          lm &= lm - 1;
          const uint32_t o = __builtin_amdgcn_readlane(off[k], l), d = __builtin_amdgcn_readlane(dist[k], l);
          const uint32_t L = __builtin_amdgcn_readlane(len[k], l);
          // (d = 0: a too-far-back match, every byte pointing at itself)
          uint32_t s = lane < d || d == 0 ? lane : mod_small(lane, d);
          const uint32_t step = WAVE < d || d == 0 ? WAVE : mod_small(WAVE, d);
          for (uint32_t j = lane; j < L; j += WAVE) {
            p16[o - abase + j] = (uint16_t)(o - d + s);
            s += step;
            s = s >= d ? s - d : s;
          }
          const uint32_t sa = o - abase, se = sa + L;  // every byte is a start
          for (uint32_t wi = (sa >> 5) + lane; wi <= ((se - 1) >> 5); wi += WAVE) {
            const uint32_t lo = max(sa, wi * 32), hi = min(se, wi * 32 + 32);
            const uint32_t m = (hi - lo == 32 ? ~0u : (1u << (hi - lo)) - 1) << (lo & 31);
            __hip_atomic_fetch_or(&sbits[wi], m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
        }
      }
#ifdef SBH_LZ_PROBE
      t_mk += __builtin_readcyclecounter() - tb;
#endif
      __syncthreads();
#ifdef SBH_LZ_PROBE
      t_b1 += __builtin_readcyclecounter() - tb;
#endif
      // slot pass: every byte's pointer from its token's start (at most LZ_SHORT - 1
      // slots back): byte j of a match that starts at slot s and copies from v points at
      // v + j, or v + (j mod (s - v)) when the match overlaps itself (rare); a literal
      // start points at itself.  Each thread owns up to NHP half granules (8 slots) and
      // keeps their pointers in registers for the chase below.
      const uint32_t nh = (plen + lead + PTR_HALF - 1) / PTR_HALF;
      uint32_t c[NHP][PTR_HALF], pend[NHP];
#pragma unroll
      for (uint32_t hh = 0; hh < NHP; ++hh) {
        const uint32_t h = t + hh * LZ_THREADS;
        pend[hh] = 0;
        if (h >= nh) continue;
        const uint32_t s0 = PTR_HALF * h, g0 = abase + s0;  // first slot, its position
        const uint32_t wi = h >> 2, sh8 = (h & 3) * PTR_HALF;
        const uint32_t cur = sbits[wi], prev = wi ? sbits[wi - 1] : 0u;
        // the window's slots inside the pass: [klo, khi)
        const int32_t rlo = (int32_t)lead - (int32_t)s0, rhi = rlo + (int32_t)plen;
        const uint32_t klo = (uint32_t)min(max(rlo, 0), (int32_t)PTR_HALF);
        const uint32_t khi = (uint32_t)min(max(rhi, 0), (int32_t)PTR_HALF);
        // nearest start before the window, then walk the window's start bits
        const uint32_t low = cur & ((1u << sh8) - 1u);
        uint32_t st = low ? wi * 32 + 31 - __builtin_clz(low) : prev ? wi * 32 - 1 - __builtin_clz(prev) : s0;
        const uint32_t wb = cur >> sh8;
        uint32_t sidx[PTR_HALF], v[PTR_HALF];
#if SBH_LZ_SLOT128
        // the start values: the window's own 8 slots in one 16-byte read (lane h at 16 h bytes: no
        // bank conflicts, where 8 u16 reads at a 16-byte lane stride were 4-way), the nearest start
        // before the window in one u16 read; each slot takes its last start's value
        const uint4 ow = reinterpret_cast<const uint4 *>(p16)[h];
        const uint32_t od[4] = {ow.x, ow.y, ow.z, ow.w};
        uint32_t vl = p16[st];
#pragma unroll
        for (uint32_t k = 0; k < PTR_HALF; ++k) {
          const bool s = (wb >> k) & 1u;
          st = s ? s0 + k : st;
          sidx[k] = st;
          vl = s ? (k & 1 ? od[k >> 1] >> 16 : od[k >> 1] & 0xffffu) : vl;
          v[k] = vl;
        }
#else
#pragma unroll
        for (uint32_t k = 0; k < PTR_HALF; ++k) {
          st = (wb >> k) & 1u ? s0 + k : st;
          sidx[k] = st;
        }
#pragma unroll
        for (uint32_t k = 0; k < PTR_HALF; ++k) v[k] = p16[sidx[k]];
#endif
#if SBH_LZ_OVL_WAVE
        // (no byte of a short start-marked match reaches past its distance: overlapping matches
        // had every byte marked with its final offset by the wave)
#pragma unroll
        for (uint32_t k = 0; k < PTR_HALF; ++k) {
          const bool in = k - klo < khi - klo;
          c[hh][k] = in ? v[k] + (s0 + k - sidx[k]) : g0 + k;
        }
#elif !SBH_LZ_MOD
        // byte j of every match points at v + j = its position - distance: inside the match
        // itself when the match overlaps (j >= distance), which is still an earlier byte of the
        // same value; the chase follows it
#pragma unroll
        for (uint32_t k = 0; k < PTR_HALF; ++k) {
          const bool in = k - klo < khi - klo;
          c[hh][k] = in ? v[k] + (s0 + k - sidx[k]) : g0 + k;
        }
#else
        uint32_t ovl = 0;  // slots of overlapping matches
#pragma unroll
        for (uint32_t k = 0; k < PTR_HALF; ++k) {
          const uint32_t j = s0 + k - sidx[k], dd = abase + sidx[k] - v[k];
          const bool in = k - klo < khi - klo;
#if SBH_LZ_RUN1 && SBH_LZ_MOD2
          // distance 1 (a run of one byte value): every byte points at the source byte (A/B r04h:
          // k_lz -9.1% B, -6.2% D, -4.6% E); a longer overlap (d >= 2) keeps v + j, an earlier
          // byte of the match itself, which the chase follows -- no mod at all (A/B r04m2: k_lz
          // -6.5% B, -6.4% D, -9.2% E; v + j is position - d, always an earlier byte of equal value)
          c[hh][k] = in ? v[k] + (dd == 1 ? 0u : j) : g0 + k;
#elif SBH_LZ_RUN1
          // a match at distance 1 (a run of one byte value): every byte copies its source byte,
          // no mod needed
          const bool one = dd == 1;
          // (dd = 0: a literal pair's second byte or a too-far-back match -- its own slot, final)
          ovl |= (in && j != 0 && dd != 0 && j >= dd && !one) ? 1u << k : 0u;
          c[hh][k] = in ? v[k] + (one ? 0u : j) : g0 + k;
#else
          ovl |= (in && j != 0 && dd != 0 && j >= dd) ? 1u << k : 0u;
          c[hh][k] = in ? v[k] + j : g0 + k;
#endif
        }
        if (ovl) {
#pragma unroll
          for (uint32_t k = 0; k < PTR_HALF; ++k)
            if ((ovl >> k) & 1u) c[hh][k] = v[k] + mod_small(s0 + k - sidx[k], abase + sidx[k] - v[k]);
        }
#endif
#pragma unroll
        for (uint32_t k = 0; k < PTR_HALF; ++k)  // in the pass, not a literal, not final yet
          pend[hh] |= (c[hh][k] != g0 + k && c[hh][k] >= pb) ? 1u << k : 0u;
        reinterpret_cast<uint4 *>(p16)[h] = pack8_u16(c[hh]);
      }
#ifdef SBH_LZ_PROBE
      t_w += __builtin_readcyclecounter() - tb;
#endif
      __syncthreads();
#ifdef SBH_LZ_PROBE
      const uint64_t tc = __builtin_readcyclecounter();
      t_init += tc - tb;
#endif
      // chase the pointers of each half granule together, one LDS round trip per round,
      // writing shortened pointers back (other threads' chains pass through them); no
      // barriers.  A pointer is final when it is before the pass or names a literal (a
      // slot pointing at itself).  Then gather the bytes and store them.
      // Plain loads: another thread may rewrite a slot concurrently, and either value (u16 LDS
      // accesses are single-copy atomic) is a valid pointer.  Rounds are branch-free; settled
      // slots reread their own final pointer's slot harmlessly.  Each round replaces every
      // in-pass pointer by the one stored at its target (a final slot -- a literal -- stores
      // itself, so it stays); a lane stops once no pointer of its own moved to another in-pass
      // position.
      auto gather8 = [&](const uint32_t *cp, uint32_t g0) {
        uint32_t w[2];
#if SBH_LZ_RING
        const uint8_t *rb = sm.img;
#pragma unroll
        for (uint32_t q = 0; q < 2; ++q)
          w[q] = (uint32_t)rb[lz_ri(sh + cp[4 * q])] | (uint32_t)rb[lz_ri(sh + cp[4 * q + 1])] << 8 |
                 (uint32_t)rb[lz_ri(sh + cp[4 * q + 2])] << 16 | (uint32_t)rb[lz_ri(sh + cp[4 * q + 3])] << 24;
        *reinterpret_cast<uint2 *>(sm.img + lz_ri(sh + g0)) = make_uint2(w[0], w[1]);
#else
#pragma unroll
        for (uint32_t q = 0; q < 2; ++q)
          w[q] = (uint32_t)img[cp[4 * q]] | (uint32_t)img[cp[4 * q + 1]] << 8 | (uint32_t)img[cp[4 * q + 2]] << 16 |
                 (uint32_t)img[cp[4 * q + 3]] << 24;
        *reinterpret_cast<uint2 *>(img + g0) = make_uint2(w[0], w[1]);
#endif
      };
      const uint32_t p16a = (uint32_t)reinterpret_cast<uintptr_t>(p16);
      [[maybe_unused]] const uint32_t choff = uni(p16a) - 2u * abase;  // LDS address of pointer c: choff + 2 c
#pragma unroll
      for (uint32_t hh = 0; hh < NHP; ++hh) {
        const uint32_t h = t + hh * LZ_THREADS;
        if (h >= nh) continue;
        const uint32_t g0 = abase + PTR_HALF * h;  // image position of the half granule
#ifdef SBH_LZ_DEBUG
        uint32_t guard = 0;
#endif
#if SBH_ASM_CHASE && !defined(SBH_LZ_DEBUG) && !defined(SBH_LZ_PROBE)
        chase8_asm(c[hh], pend[hh], pb, choff, p16a + 16u * h);
#else
        bool more = pend[hh] != 0;
        while (__builtin_expect(more, 0)) {
#ifdef SBH_LZ_DEBUG
          if (++guard > 300) {
            for (uint32_t k = 0; k < PTR_HALF; ++k)
              printf("lz chase stuck blk %llu pos %u c %u base %u plen %u lead %u\n", (unsigned long long)b,
                     g0 + k, c[hh][k], pb, plen, lead);
            break;
          }
#endif
          uint32_t v[PTR_HALF];
#pragma unroll
          for (uint32_t k = 0; k < PTR_HALF; ++k) v[k] = p16[(c[hh][k] >= pb ? c[hh][k] : pb) - abase];
#ifdef SBH_LZ_PROBE
          if (__builtin_amdgcn_readfirstlane(lane) == lane) ++njumps;  // rounds this wave ran
#endif
          more = false;
#pragma unroll
          for (uint32_t k = 0; k < PTR_HALF; ++k) {
            const uint32_t nc = c[hh][k] >= pb ? v[k] : c[hh][k];
            more = more || (nc != c[hh][k] && nc >= pb);
            c[hh][k] = nc;
          }
          // write back: settled and shortened pointers alike (literal and out-of-pass
          // slots keep pointing at themselves)
          reinterpret_cast<uint4 *>(p16)[h] = pack8_u16(c[hh]);
        }
#endif
        gather8(c[hh], g0);
      }
#ifdef SBH_LZ_PROBE
      t_ch += __builtin_readcyclecounter() - tc;
#endif
#if SBH_LZ_CARRY
      cend = pe;
      break;  // (one pass per chunk)
#endif
      if (pe == chunk_end) break;
      __syncthreads();  // the pass's slots and start bits are reused by the next pass
      for (uint32_t w = t; w < SB_WORDS; w += LZ_THREADS) sm.pp.sbits[w] = 0;
      pb = pe;
      __syncthreads();
    }
#if SBH_LZ_CARRY
    base = cend;  // (chunk_end unless cut: the cut token starts the next chunk)
#else
    base += chunk_len;
#endif
#if !SBH_LZ_NO_END_BAR
    __syncthreads();  // slots / wsum are reused by the next chunk
#endif
    // (without it: the next chunk's slot writes all come after its scan's barrier, which every
    // wave reaches only once done with this chunk; its wsum / sbits writes before that barrier
    // touch nothing this chunk still reads -- wsum was read before this chunk's marks, sbits
    // before its chase)
#ifdef SBH_LZ_PROBE
    t_rounds += __builtin_readcyclecounter() - tb;
#endif
  }
#if SBH_LZ_NO_END_BAR
  __syncthreads();  // the image is complete
#endif
#ifdef SBH_LZ_PROBE
  {
    uint32_t tot = 0;
    for (uint32_t l = 0; l < WAVE; ++l) tot += __builtin_amdgcn_readlane(njumps, l);
    njumps = tot;
  }
  if (lane == 0 && (b == 1000 || (b == 1 && t < WAVE)))
    printf("lz blk %llu wave %u ntok %u cyc %llu pre %llu marks %llu marks+bar %llu marks+slots %llu init+bar %llu chase %llu resolve+bar %llu fallback %u chase_rounds %u long %u\n",
           (unsigned long long)b, t / WAVE, n, (unsigned long long)(__builtin_readcyclecounter() - tp0),
           (unsigned long long)t_pre, (unsigned long long)t_mk, (unsigned long long)t_b1, (unsigned long long)t_w,
           (unsigned long long)t_init, (unsigned long long)t_ch, (unsigned long long)t_rounds, nrounds, njumps, nlong);
#endif
  const uint32_t usize = base;
  // write the image: 16-byte granules aligned to the flat address (the ring: those not yet written)
  const uint64_t g0 = g0u;
  const uint32_t ngran = (sh + usize + 15) / 16;
#if SBH_LZ_RING
  const uint32_t q0 = fl / 16;
#else
  const uint32_t q0 = 0;
#endif
  for (uint32_t q = q0 + t; q < ngran; q += LZ_THREADS) {
    const uint32_t lo = q * 16;  // image offset (relative to sm.img) of the granule
    if (lo >= sh && lo + 16 <= sh + usize) {
      *reinterpret_cast<uint4 *>(U + g0 + lo) = *reinterpret_cast<const uint4 *>(sm.img + lz_ri(lo));
    } else {
      for (uint32_t k = 0; k < 16; ++k) {
        const uint32_t a = lo + k;
        if (a >= sh && a < sh + usize) U[g0 + a] = sm.img[lz_ri(a)];
      }
    }
  }
#if SBH_LZ_RING && SBH_LZ_SIEVE
  if (sv16) lz_sieve(ngran, sh + usize);  // (the image is complete: the last barrier above)
#endif
}

// The first block whose inflate status is not INF_OK (atomicMin; *first preset to ~0):
// the host reads 8 bytes instead of every block's status.
__global__ void k_first_bad(const uint32_t *status, uint64_t n, unsigned long long *first) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && status[i] != INF_OK) atomicMin(first, (unsigned long long)i);
}

}  // namespace

hipError_t launch_first_bad(const uint32_t *status, uint64_t n, unsigned long long *first, hipStream_t stream,
                            bool init) {
  hipError_t e = init ? hipMemsetAsync(first, 0xff, sizeof(unsigned long long), stream) : hipSuccess;
  if (e != hipSuccess || n == 0) return e;
  hipLaunchKernelGGL(k_first_bad, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, stream, status, n, first);
  return hipGetLastError();
}

hipError_t launch_huff(const uint8_t *comp, DevBlocks blocks, uint64_t nblocks, uint32_t *tok_buf, uint64_t tok_base,
                       hipStream_t stream) {
  if (nblocks == 0) return hipSuccess;
  // the kernels index tokens by flat offset: tok[ustart_b] is block b's first token slot
  uint32_t *tok = reinterpret_cast<uint32_t *>(reinterpret_cast<uintptr_t>(tok_buf) - tok_base * 4);
#ifdef SBH_HUFF_SERIAL
  const uint64_t grid = (nblocks + WAVES - 1) / WAVES;
  hipLaunchKernelGGL(k_huff_serial<false>, dim3((uint32_t)grid), dim3(WAVES * WAVE), 0, stream, comp, blocks, nblocks,
                     tok);
#else
  const dim3 hdr_grid((uint32_t)((nblocks + HDR_WAVES - 1) / HDR_WAVES)), hdr_wg(WAVE * HDR_WAVES);
  hipLaunchKernelGGL(k_hdr<false>, hdr_grid, hdr_wg, 0, stream, comp, blocks, nblocks, tok);
  hipLaunchKernelGGL(k_huff, dim3((uint32_t)nblocks), dim3(HT), 0, stream, comp, blocks, nblocks, tok);
#if SBH_TAIL
#if SBH_TAIL_HDR
  hipLaunchKernelGGL(k_hdr<true>, hdr_grid, hdr_wg, 0, stream, comp, blocks, nblocks, tok);
#endif
  hipLaunchKernelGGL(k_huff_tail, dim3((uint32_t)nblocks), dim3(TAIL_NT), 0, stream, comp, blocks, nblocks, tok);
#endif
  const uint64_t grid = (nblocks + WAVES - 1) / WAVES;
  hipLaunchKernelGGL(k_huff_serial<true>, dim3((uint32_t)grid), dim3(WAVES * WAVE), 0, stream, comp, blocks, nblocks,
                     tok);
#endif
  return hipGetLastError();
}

hipError_t launch_lz(const uint8_t *comp, DevBlocks blocks, uint64_t nblocks, const uint32_t *tok_buf,
                     uint64_t tok_base, uint8_t *U, hipStream_t stream, uint32_t *sieve, uint32_t nref1) {
  if (nblocks == 0) return hipSuccess;
  const uint32_t *tok = reinterpret_cast<const uint32_t *>(reinterpret_cast<uintptr_t>(tok_buf) - tok_base * 4);
  if (!SBH_LZ_SIEVE || !SBH_LZ_RING) sieve = nullptr;
#ifdef SBH_LZ_PAD  // occupancy probe: dynamic LDS that leaves one workgroup per CU
  hipLaunchKernelGGL(k_lz, dim3((uint32_t)nblocks), dim3(LZ_THREADS), SBH_LZ_PAD, stream, comp, blocks, nblocks, tok, U,
                     sieve, nref1);
#else
  hipLaunchKernelGGL(k_lz, dim3((uint32_t)nblocks), dim3(LZ_THREADS), 0, stream, comp, blocks, nblocks, tok, U, sieve,
                     nref1);
#endif
  return hipGetLastError();
}

}  // namespace sbh
