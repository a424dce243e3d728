// check.hip -- BAM record-boundary checkers at every uncompressed position (CDNA4).
//
// Replaces, for every flat position of a range at once:
//  * eager.Checker.apply  (check/.../bam/check/eager/Checker.scala:24-126)
//  * full.Checker.apply   (check/.../bam/check/full/Checker.scala:22-184) + the
//    FullCheck Counts aggregation (cli/.../check/full/FullCheck.scala:142-192)
//  * PosChecker.getRefPosError (check/.../bam/check/PosChecker.scala:43-63)
// and the record-chain bookkeeping behind split/count computation
// (check/.../iterator/PosStream.scala:14-22, load/.../CanLoadBam.scala:346-355).
//
// Layout: a workgroup owns a tile of positions (eager: 16 Ki, full: 8 Ki).  Eager: it stages
// the tile plus a 4.5 KiB look-ahead into LDS with coalesced 16-byte loads, evaluates the
// single-record predicate at every position of the window (97% reject on refID), then walks
// each surviving position's record chain through those LDS bits; only chains that leave the
// window (long reads) or touch an EOF edge re-read HBM/L2.  Full: byte-class bitmaps of the
// staged window make each position's first record O(1) LDS work, histograms are counted by
// wave ballots.  Results are a bit per position (2 KiB per tile, 16-byte stores) or a word
// per position.
#include <algorithm>
#include <cstdlib>

#include "sbh_internal.h"

namespace sbh {
namespace {

constexpr uint32_t T = 256;

constexpr uint32_t FULL_SUCCESS = 0x80000000u;
constexpr uint32_t FULL_UNKNOWN = 0x40000000u;  // depends on bytes past an open end
constexpr uint32_t N_SHIFT = 20;

struct Src {
  const uint8_t *U;
  const uint32_t *lds32;  // staged dwords; lds byte i <-> flat s0 + i
  uint64_t s0;            // dword-aligned flat start of the staged window
  uint32_t sn;            // staged bytes (multiple of 4)

  __device__ __forceinline__ uint32_t word_at(uint64_t q) const {  // little-endian u32 at q
    const uint64_t w = q - s0;
    if (q >= s0 && w + 8 <= sn) {
      const uint32_t i = (uint32_t)w >> 2;
      return __builtin_amdgcn_alignbyte(lds32[i + 1], lds32[i], (uint32_t)w & 3);
    }
    const uint32_t *g = reinterpret_cast<const uint32_t *>(U + (q & ~3ull));
    return __builtin_amdgcn_alignbyte(g[1], g[0], (uint32_t)q & 3);
  }
  __device__ __forceinline__ uint8_t byte_at(uint64_t q) const {
    const uint64_t w = q - s0;
    if (q >= s0 && w < sn) return (uint8_t)(lds32[w >> 2] >> (8 * (w & 3)));
    return U[q];
  }
};

struct Ctg {
  const int32_t *len;
  int32_t n;
};

// PosChecker.getRefPosError: bits {0 negIdx, 1 bigIdx, 2 negPos, 3 bigPos}
__device__ __forceinline__ uint32_t ref_pos_error(int32_t idx, int32_t pos, const Ctg &c) {
  if (idx < -1) return pos < -1 ? 5u : 1u;
  if (idx >= c.n) return pos < -1 ? 6u : 2u;
  if (pos < -1) return 4u;
  if (idx >= 0 && (int64_t)pos > (int64_t)c.len[idx]) return 8u;
  return 0;
}

__device__ __forceinline__ bool name_char_ok(uint32_t ch) {
  return (ch >= 0x21 && ch <= 0x3F) || (ch >= 0x41 && ch <= 0x7E);
}

// Every byte of [q, q + nn) a valid read-name character (name_char_ok), 16 bytes per
// step from 4 independent dword reads with SWAR range tests (bytes past nn count as 'A').
__device__ __forceinline__ bool name_bytes_ok(const Src &s, uint64_t q, uint32_t nn) {
  for (uint32_t i = 0; i < nn; i += 16) {
    uint32_t w[4];
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) w[k] = s.word_at(q + i + 4 * k);
    uint32_t bad = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      const uint32_t b0 = i + 4 * k;
      uint32_t x = w[k];
      if (b0 + 4 > nn) {
        const uint32_t keep = b0 >= nn ? 0u : (1u << (8 * (nn - b0))) - 1u;
        x = (x & keep) | (0x41414141u & ~keep);
      }
      bad |= (x - 0x21212121u) & ~x & 0x80808080u;        // a byte < 0x21
      bad |= ((x + 0x01010101u) | x) & 0x80808080u;        // a byte > 0x7e
      const uint32_t y = x ^ 0x40404040u;
      bad |= (y - 0x01010101u) & ~y & 0x80808080u;         // a byte == 0x40 ('@')
    }
    if (bad) return false;
  }
  return true;
}

__device__ __forceinline__ int32_t implied_min_remaining(int32_t rnl, int32_t nc, int32_t seq_len) {
  int32_t s1 = (int32_t)((uint32_t)seq_len + 1u);
  int32_t nsq = (int32_t)((uint32_t)(s1 / 2) + (uint32_t)seq_len);
  return (int32_t)(32u + (uint32_t)rnl + 4u * (uint32_t)nc + (uint32_t)nsq);
}

// The first CIGAR op k < nc (ops at q + 4k) that does not fit below `bound`
// (q + 4k + 4 > bound) or is invalid ((byte & 0xf) > 8); nc if none.  Eight op bytes are
// loaded per step before any test, so a long run of valid ops costs one load latency per
// eight ops rather than per op (op bytes past `bound` are loaded but never decide).
__device__ __forceinline__ uint32_t first_bad_op(const Src &s, uint64_t q, uint32_t nc, uint64_t bound) {
  const uint64_t fit = bound >= q ? (bound - q) / 4 : 0;
  const uint32_t lim = fit < (uint64_t)nc ? (uint32_t)fit : nc;
  for (uint32_t k = 0; k < lim; k += 8) {
    uint8_t b[8];
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) b[j] = s.byte_at(q + 4ull * (k + j));
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j)
      if (k + j < lim && (b[j] & 0xf) > 8) return k + j;
  }
  return lim;
}

// Bad-CIGAR-op index for the full checker over flat bytes [base, end) (base 1024-aligned):
// ob word w holds one bit per byte of [base + 32 w, +32) -- (b & 0xf) > 8, an op code no CIGAR
// has -- and os[r] (r = flat position mod 4) one bit per ob word that holds such a byte at a
// position of residue r.  A record's first invalid op is the first set bit at stride 4 from its
// CIGAR start: a scan across kilobytes of valid-looking op bytes (the packed bases of a long
// read, whose low nibbles are all valid op codes) costs a few summary words instead of one
// byte per op.
struct OpIdx {
  const uint32_t *ob;
  const uint32_t *os;  // four arrays of nsw words, residue-major
  uint64_t base, end;
  uint64_t nsw;
};

// First y in [x, lim) with y = x (mod 4) and a bad op byte at y; lim if none
// (base <= x, lim <= end).
__device__ __forceinline__ uint64_t op_scan(const OpIdx &oi, uint64_t x, uint64_t lim) {
  if (x >= lim) return lim;
  const uint32_t pat = 0x11111111u << ((uint32_t)x & 3);
  uint64_t w = (x - oi.base) >> 5;
  uint32_t m = oi.ob[w] & pat & (~0u << ((uint32_t)(x - oi.base) & 31));
  if (!m) {
    const uint32_t *os = oi.os + ((uint32_t)x & 3) * oi.nsw;
    const uint64_t gl = (lim - oi.base + 31) >> 5;  // ob words below lim
    uint64_t g = w + 1;
    for (;;) {
      if (g >= gl) return lim;
      const uint32_t sm = os[g >> 5] & (~0u << (g & 31));
      if (sm) {
        w = (g & ~31ull) + __builtin_ctz(sm);
        break;
      }
      g = (g | 31) + 1;
    }
    if (w >= gl) return lim;
    m = oi.ob[w] & pat;
  }
  const uint64_t y = oi.base + 32 * w + __builtin_ctz(m);
  return y < lim ? y : lim;
}

// first_bad_op through the index when it covers the ops, else byte by byte
__device__ __forceinline__ uint32_t first_bad_op_ix(const Src &s, const OpIdx &oi, uint64_t q, uint32_t nc,
                                                    uint64_t bound) {
  const uint64_t fit = bound >= q ? (bound - q) / 4 : 0;
  const uint32_t lim = fit < (uint64_t)nc ? (uint32_t)fit : nc;
  if (oi.ob && q >= oi.base && q + 4ull * lim <= oi.end)
    return (uint32_t)((op_scan(oi, q, q + 4ull * lim) - q + 3) / 4);
  return first_bad_op(s, q, nc, bound);
}

// Eager check at p: 0 false, 1 true, 2 unknown (needs bytes past an open end), 3 deferred
// (needs flat bytes at or past `front`, which are not inflated yet: the pipelined run
// re-checks the position once they are).
constexpr uint32_t EAGER_DEFER = 3;
// Src / Ctg by value: passed in registers (a reference would materialize them in scratch
// memory at every launch of the calling kernel)
__device__ uint32_t eager_at(const Src s, uint64_t p, uint64_t total, bool open, const Ctg c,
                             int32_t rtc, uint64_t front = ~0ull) {
  uint64_t cur = p, start = p;
  for (int32_t n = 0;; ++n) {
    if (n == rtc) return 1;
    if (cur + 36 > total) {
      if (open) return 2;
      return (total == start && n > 0) ? 1 : 0;
    }
    if (cur + 36 > front) return EAGER_DEFER;
    const int32_t rem = (int32_t)s.word_at(cur);
    const uint64_t nominal = start + 4 + (int64_t)rem;
    if (ref_pos_error((int32_t)s.word_at(cur + 4), (int32_t)s.word_at(cur + 8), c)) return 0;
    const int32_t rnl = (int32_t)(s.word_at(cur + 12) & 0xff);
    if (rnl < 2) return 0;
    const uint32_t fnc = s.word_at(cur + 16);
    const uint32_t flags = fnc >> 16;
    const int32_t nc = (int32_t)(fnc & 0xffff);
    const int32_t seq_len = (int32_t)s.word_at(cur + 20);
    if ((flags & 4) == 0 && (seq_len == 0 || nc == 0)) return 0;
    if (rem < implied_min_remaining(rnl, nc, seq_len)) return 0;
    if (ref_pos_error((int32_t)s.word_at(cur + 24), (int32_t)s.word_at(cur + 28), c)) return 0;
    cur += 36;
    if (cur + (uint64_t)rnl > total) return open ? 2 : 0;
    if (cur + (uint64_t)rnl > front) return EAGER_DEFER;
    if (s.byte_at(cur + rnl - 1) != 0) return 0;
    if (!name_bytes_ok(s, cur, (uint32_t)rnl - 1)) return 0;
    cur += rnl;
    {  // the op loop's outcome order: past total, past front, invalid op
      const uint32_t kb = first_bad_op(s, cur, (uint32_t)nc, total < front ? total : front);
      if (kb < (uint32_t)nc) {
        const uint64_t e = cur + 4ull * kb + 4;
        if (e > total) return open ? 2 : 0;
        if (e > front) return EAGER_DEFER;
        return 0;
      }
      cur += 4ull * (uint32_t)nc;
    }
    if ((int64_t)(nominal - cur) > 0) {
      if (nominal > total) {
        if (open) return 2;
        cur = total;
      } else {
        cur = nominal;
      }
    }
    start = nominal;
  }
}

// Full check at p: result word (see include/sparkbam.h), or FULL_UNKNOWN.
__device__ uint32_t full_at(const Src s, uint64_t p, uint64_t total, bool open, const Ctg c,
                            int32_t rtc, const OpIdx oi) {
  uint64_t cur = p, start = p;
  for (int32_t n = 0;; ++n) {
    if (n == rtc) return FULL_SUCCESS | ((uint32_t)n << N_SHIFT);
    if (cur + 36 > total) {
      if (open) return FULL_UNKNOWN;
      if (total == start && n > 0) return FULL_SUCCESS | ((uint32_t)n << N_SHIFT);
      return 1u | ((uint32_t)n << N_SHIFT);
    }
    const int32_t rem = (int32_t)s.word_at(cur);
    const uint64_t nominal = start + 4 + (int64_t)rem;
    uint32_t f = ref_pos_error((int32_t)s.word_at(cur + 4), (int32_t)s.word_at(cur + 8), c) << 1;
    const int32_t rnl = (int32_t)(s.word_at(cur + 12) & 0xff);
    const uint32_t fnc = s.word_at(cur + 16);
    const uint32_t flags = fnc >> 16;
    const int32_t nc = (int32_t)(fnc & 0xffff);
    const int32_t seq_len = (int32_t)s.word_at(cur + 20);
    if (rem < implied_min_remaining(rnl, nc, seq_len)) f |= 1u << 18;
    f |= ref_pos_error((int32_t)s.word_at(cur + 24), (int32_t)s.word_at(cur + 28), c) << 5;
    cur += 36;
    bool name_eof = false;
    if (rnl == 0) {
      f |= 1u << 12;
    } else if (rnl == 1) {
      f |= 1u << 13;
    } else if (cur + (uint64_t)rnl > total) {
      if (open) return FULL_UNKNOWN;
      f |= 1u << 9;
      name_eof = true;
    } else {
      if (s.byte_at(cur + rnl - 1) != 0) {
        f |= 1u << 10;
      } else {
        if (!name_bytes_ok(s, cur, (uint32_t)rnl - 1)) f |= 1u << 11;
      }
      cur += rnl;
    }
    if (!name_eof) {
      bool cig_err = false;
      const uint32_t kb = first_bad_op_ix(s, oi, cur, (uint32_t)nc, total);
      if (kb < (uint32_t)nc) {  // past the stream end first, else an invalid op
        cig_err = true;
        if (cur + 4ull * kb + 4 > total) {
          if (open) return FULL_UNKNOWN;
          f |= 1u << 14;
        } else {
          f |= 1u << 15;
        }
      } else {
        cur += 4ull * (uint32_t)nc;
      }
      if (!cig_err && (flags & 4) == 0 && (seq_len == 0 || nc == 0)) {
        if (seq_len == 0) f |= 1u << 16;  // EmptyMapped(emptySeq, emptyCigar) field swap
        if (nc == 0) f |= 1u << 17;
      }
    }
    if (f) return f | ((uint32_t)n << N_SHIFT);
    if ((int64_t)(nominal - cur) > 0) {
      if (nominal > total) {
        if (open) return FULL_UNKNOWN;
        cur = total;
      } else {
        cur = nominal;
      }
    }
    start = nominal;
  }
}

struct Segs {
  const uint64_t *end;  // sorted; last entry = resident flat size
  uint32_t n;
  uint32_t open_last;  // last segment ends at the resident end, not at a stream end
};

// Stage NV 16-byte vectors of U from s0 (16-aligned) into LDS: every load is issued
// before any LDS store (one HBM latency per workgroup, not one per iteration).
// Vectors not wholly below u_pad stage as zeros (u_pad - u_total >= 16: only pad).
template <uint32_t NV>
__device__ __forceinline__ void stage_vec(uint4 *lds, const uint8_t *U, uint64_t s0, uint64_t u_pad) {
  constexpr uint32_t R = (NV + T - 1) / T;
  const uint4 *g = reinterpret_cast<const uint4 *>(U + s0);
  // every lane loads in every round (a vector out of range reads U's first one instead, and is
  // zeroed after): a load under a branch made the compiler wait for each one before the next
  uint4 v[R];
  bool in[R];
#pragma unroll
  for (uint32_t r = 0; r < R; ++r) {
    const uint32_t i = threadIdx.x + r * T;
    in[r] = i < NV && s0 + 16ull * i + 16 <= u_pad;
    v[r] = *(in[r] ? g + i : reinterpret_cast<const uint4 *>(U));
  }
#pragma unroll
  for (uint32_t r = 0; r < R; ++r) {
    const uint32_t i = threadIdx.x + r * T;
    if (i < NV) lds[i] = in[r] ? v[r] : make_uint4(0, 0, 0, 0);
  }
}

// One dword of every 128-byte line of [p, p + n) (a lane per line) loaded into a register that
// nothing waits for: the lines come into L2 / MALL for the workgroup that stages them later.
// The caller keeps the result live (l2_keep) past a wait the compiler places for its own later
// loads -- vector loads return in order, so that wait covers this one too and the register is
// never reused while the load is in flight.
__device__ __forceinline__ uint32_t l2_touch(const uint8_t *p, uint64_t n) {
  uint32_t v = 0;
  const uint64_t off = (uint64_t)threadIdx.x * 128;
  if (off < n) asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(p + off) : "memory");
  return v;
}
__device__ __forceinline__ void l2_keep(uint32_t v) { asm volatile("" ::"v"(v)); }

__device__ __forceinline__ uint32_t seg_index(const Segs &sg, uint64_t p, uint32_t from) {
  uint32_t k = from;
  while (k + 1 < sg.n && sg.end[k] <= p) ++k;
  return k;
}

__device__ __forceinline__ uint32_t seg_first(const Segs &sg, uint64_t p) {
  uint32_t lo = 0, hi = sg.n - 1;
  while (lo < hi) {
    uint32_t m = (lo + hi) >> 1;
    if (sg.end[m] <= p) lo = m + 1; else hi = m;
  }
  return lo;
}

struct EagerOut {
  uint32_t *bits;                 // bit i <-> position begin + i
  unsigned long long *n_true;
  unsigned long long *n_unknown;
  unsigned long long *min_unknown;
  uint64_t front;                 // flat bytes at/after front are not inflated yet (pipelined run)
  uint64_t *defer_pos;            // positions whose exact check needs them (re-checked later)
  unsigned long long *defer_n;
  uint64_t defer_cap;
  uint64_t *xq_pos;               // long-record candidates for the wave-cooperative exact pass
  unsigned long long *xq_n;
  uint64_t xq_cap;                // 0: every exact check runs inline
  unsigned long long *true_spread;  // k_eager: per-wave true counts, folded into n_true by k_fold_true
  TileSum *tsum;                  // per tile: the chain proof's summary (nullptr: none)
  const uint32_t *sieve = nullptr;  // k_lz's first-filter bitmap, bit p = flat position p (nullptr: sweep here)
};

// k_eager's true count goes to TRUE_SLOTS counters TRUE_STRIDE u64 apart (one atomic per
// wave), not to n_true itself: one address takes every workgroup's atomic in turn at one
// L2 channel, and the barrier a per-workgroup sum needs waits for the bitmap stores.
constexpr uint32_t TRUE_SLOTS = 64, TRUE_STRIDE = 16;
constexpr uint32_t TRUE_SPREAD_OFF = CTR_TRUE_SPREAD;  // u64 offset of the slots in the counter buffer
static_assert(TRUE_SLOTS * TRUE_STRIDE == CTR_TRUE_WORDS, "true-count slots fill their region");

// A candidate whose first record is at least this long (block_size) leaves its exact check
// to k_eager_xq: its name / CIGAR bytes are read by a whole wave instead of one lane.
constexpr int32_t XQ_MIN_REC = 2048;
constexpr int32_t XQ_MIN_OPS = 32;
constexpr uint32_t EAGER_XQ = 4;

// A plausible long first record at p (its fixed fields pass and it carries >= XQ_MIN_OPS
// CIGAR ops): the candidates worth a whole wave.
__device__ __forceinline__ bool long_candidate(const Src &s, uint64_t p, const Ctg &c) {
  const int32_t rem = (int32_t)s.word_at(p);
  if (rem < XQ_MIN_REC) return false;
  const uint32_t fnc = s.word_at(p + 16);
  const int32_t nc = (int32_t)(fnc & 0xffff), rnl = (int32_t)(s.word_at(p + 12) & 0xff);
  if (nc < XQ_MIN_OPS || rnl < 2) return false;
  if (rem < implied_min_remaining(rnl, nc, (int32_t)s.word_at(p + 20))) return false;
  if (ref_pos_error((int32_t)s.word_at(p + 4), (int32_t)s.word_at(p + 8), c) ||
      ref_pos_error((int32_t)s.word_at(p + 24), (int32_t)s.word_at(p + 28), c))
    return false;
  return true;
}

constexpr uint32_t ETILE = SBH_ETILE;     // eager tile: positions per workgroup
#ifndef SBH_ELA
#define SBH_ELA 4096
#endif
constexpr uint32_t ELA = SBH_ELA;         // look-ahead: chains of short reads stay inside
constexpr uint32_t EW = ETILE + ELA;      // eager window: single-record predicate evaluated here
constexpr uint32_t ESTAGE = EW + 512;     // staged bytes (records near the end fit)
#ifndef SBH_EQ_CHUNK
#define SBH_EQ_CHUNK 4096
#endif
constexpr uint32_t EQ_CHUNK = SBH_EQ_CHUNK;  // survivor-queue capacity
#ifndef SBH_EAGER_PF
#define SBH_EAGER_PF 0  // k_eager: the tile this many workgroups ahead is touched into L2 (A/B r06zb: 1024 slower, k_eager 2.42 -> 2.50 ms)
#endif
#ifndef SBH_EAGER_SHIFT_SWEEP
#define SBH_EAGER_SHIFT_SWEEP 1  // k_eager's refID sweep: tests shifted into each word (see k_eager)
#endif
static_assert(EAGER_REACH >= ESTAGE + 32 + 16, "EAGER_REACH covers the staged window");

// PosChecker.getRefPosError with the contig length already loaded (len_idx: len[idx]
// when 0 <= idx < n, else unused).
__device__ __forceinline__ uint32_t ref_pos_error_l(int32_t idx, int32_t pos, int32_t len_idx, const Ctg &c) {
  if (idx < -1) return pos < -1 ? 5u : 1u;
  if (idx >= c.n) return pos < -1 ? 6u : 2u;
  if (pos < -1) return 4u;
  if (idx >= 0 && (int64_t)pos > (int64_t)len_idx) return 8u;
  return 0;
}

// Single-record eager predicate at q, with cur == start == q, reading only the
// staged window: 0 fail, 1 pass, 2 cannot decide from the window (or EOF edge).
// On pass, *succ = the next record start (nominal), *normal = nominal >= cursor
// after name + cigar (so the next record is read at nominal).
// Latency-shaped: the fixed fields and the first 32 read-name bytes come from one batch
// of 18 LDS dword reads, and both contig lengths are loaded beside them, so a record
// costs about three dependent round trips (fields, then CIGAR op bytes) instead of one
// per field; the tests run in the reference's order on the loaded values.
// With `cig` set, a record whose CIGAR has more than CIG_WAVE ops returns ONE_CIGAR after
// every other test passed, with *cig = its first op byte and *ncig = nc: the caller
// checks those op bytes with the whole wave (one lane walking hundreds of ops would hold
// the workgroup at its next barrier).
constexpr uint32_t ONE_CIGAR = 3, CIG_WAVE = 16;
__device__ __forceinline__ uint32_t one_record(const Src &s, uint64_t q, uint64_t total, const Ctg &c,
                                               uint64_t *succ, bool *normal, uint64_t *cig = nullptr,
                                               uint32_t *ncig = nullptr) {
  if (q + 36 > total) return 2;                       // EOF rules: exact path
  if (q - s.s0 + 36 + 8 > s.sn) return 2;
  const uint32_t w = (uint32_t)(q - s.s0), i = w >> 2, k = w & 3;
  // dwords [i, i + 18): bytes [w, w + 68) (the staged array holds sn + 32 bytes, and
  // w + 44 <= sn); bytes past sn are read but only used below need <= sn
  uint32_t d[18];
#pragma unroll
  for (uint32_t j = 0; j < 18; ++j) d[j] = s.lds32[i + j];
  auto fld = [&](uint32_t j) { return __builtin_amdgcn_alignbyte(d[j + 1], d[j], k); };
  const int32_t ref = (int32_t)fld(1), pos = (int32_t)fld(2), nrf = (int32_t)fld(6), nps = (int32_t)fld(7);
  const int32_t l1 = ref >= 0 && ref < c.n ? c.len[ref] : 0;
  const int32_t l2 = nrf >= 0 && nrf < c.n ? c.len[nrf] : 0;
  // most selective predicate first: refID / pos (99% of positions fail here)
  if (ref_pos_error_l(ref, pos, l1, c)) return 0;
  const int32_t rnl = (int32_t)(fld(3) & 0xff);
  if (rnl < 2) return 0;
  const uint32_t fnc = fld(4);
  const int32_t nc = (int32_t)(fnc & 0xffff);
  const int32_t seq_len = (int32_t)fld(5);
  if (((fnc >> 16) & 4) == 0 && (seq_len == 0 || nc == 0)) return 0;
  const int32_t rem = (int32_t)fld(0);
  if (rem < implied_min_remaining(rnl, nc, seq_len)) return 0;
  if (ref_pos_error_l(nrf, nps, l2, c)) return 0;
  uint64_t cur = q + 36;
  const uint64_t need = cur + (uint64_t)rnl + 4ull * (uint64_t)nc;
  if (need > total || need - s.s0 > s.sn) return 2;
  // the name: NUL at rnl - 1, then every byte before it a valid name character
  const uint32_t nn = (uint32_t)rnl - 1;
  uint32_t nul;
  if (nn < 32) {
    const uint32_t m = nn >> 2;
    uint32_t x = 0;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) x = j == m ? fld(9 + j) : x;
    nul = (x >> (8 * (nn & 3))) & 0xff;
  } else {
    nul = s.byte_at(cur + nn);
  }
  if (nul != 0) return 0;
  {
    const uint32_t n0 = nn < 32 ? nn : 32u;
    uint32_t bad = 0;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
      const uint32_t b0 = 4 * j;
      uint32_t x = fld(9 + j);
      if (b0 + 4 > n0) {
        const uint32_t keep = b0 >= n0 ? 0u : (1u << (8 * (n0 - b0))) - 1u;
        x = (x & keep) | (0x41414141u & ~keep);
      }
      bad |= (x - 0x21212121u) & ~x & 0x80808080u;        // a byte < 0x21
      bad |= ((x + 0x01010101u) | x) & 0x80808080u;        // a byte > 0x7e
      const uint32_t y = x ^ 0x40404040u;
      bad |= (y - 0x01010101u) & ~y & 0x80808080u;         // a byte == 0x40 ('@')
    }
    if (bad) return 0;
    if (nn > 32 && !name_bytes_ok(s, cur + 32, nn - 32)) return 0;
  }
  cur += rnl;
  const uint64_t nominal = q + 4 + (int64_t)rem;
  *succ = nominal;
  *normal = (int64_t)(nominal - (cur + 4ull * (uint32_t)nc)) >= 0;
  if (cig && (uint32_t)nc > CIG_WAVE) {
    *cig = cur;
    *ncig = (uint32_t)nc;
    return ONE_CIGAR;
  }
  if (first_bad_op(s, cur, (uint32_t)nc, cur + 4ull * (uint32_t)nc) < (uint32_t)nc) return 0;
  return 1;
}

// Two phases per 4096-position tile, all in LDS:
//  A. the single-record predicate for every position of the tile and of the
//     following 4096-position look-ahead -> `ok` bits + `normal` bits;
//  B. for each passing tile position, walk the record chain through the `ok` bits
//     (next = nominal); chains that leave the window, hit an EOF edge, or meet an
//     abnormal (cursor > nominal) record are finished by the exact eager_at() reading
//     HBM/L2.  Semantics are exactly eager.Checker.apply's.
__global__ __launch_bounds__(T) void k_eager(const uint8_t *__restrict__ U, uint64_t u_pad, uint64_t begin,
                                             uint64_t end, Segs sg, Ctg c, int32_t rtc, EagerOut o) {
  constexpr uint32_t NV = (ESTAGE + 32) / 16;
  constexpr uint32_t NWV = T / WAVE, SEGCAP = EQ_CHUNK / NWV;
  __shared__ uint4 ldsv[NV];
  __shared__ uint32_t ok[EW / 32], nrm[EW / 32], und[EW / 32];
  __shared__ __attribute__((aligned(16))) uint32_t res[ETILE / 32];
  __shared__ uint32_t lnk[EQ_CHUNK / 32], lfail[EQ_CHUNK / 32];  // per sorted candidate: LINK / FAIL step
  __shared__ uint32_t seg0, nq, wcnt[NWV];
  __shared__ uint64_t seg_end0;
  __shared__ uint32_t ts_dirty;  // a result settled after this kernel (no chain summary)
  __shared__ uint16_t queue[EQ_CHUNK];
  const uint32_t *lds32 = reinterpret_cast<const uint32_t *>(ldsv);
  const uint64_t t0 = begin + (uint64_t)blockIdx.x * ETILE;
  const uint64_t s0 = t0 & ~15ull;
#ifdef SBH_EPROBE
  const uint64_t c0 = __builtin_readcyclecounter();
  uint32_t nsurv = 0, ncand = 0, nexact = 0;
#endif
  // the window of the tile SBH_EAGER_PF workgroups on (the one that starts about when this one
  // ends, on the same XCD) into L2 / MALL while this one stages its own
  uint32_t pfv = 0;
  if (SBH_EAGER_PF) {
    const uint64_t tn = begin + ((uint64_t)blockIdx.x + SBH_EAGER_PF) * ETILE;
    const uint64_t sn = tn & ~15ull;
    if (tn < end && sn < u_pad) pfv = l2_touch(U + sn, std::min<uint64_t>(ESTAGE + 32, u_pad - sn));
  }
  stage_vec<NV>(ldsv, U, s0, u_pad);
  for (uint32_t i = threadIdx.x; i < EW / 32; i += T) { ok[i] = 0; nrm[i] = 0; und[i] = 0; }
  for (uint32_t i = threadIdx.x; i < ETILE / 32; i += T) res[i] = 0;
  for (uint32_t i = threadIdx.x; i < EQ_CHUNK / 32; i += T) { lnk[i] = 0; lfail[i] = 0; }
  if (threadIdx.x == 0) {
    const uint32_t k = seg_first(sg, t0);
    seg0 = k;
    seg_end0 = sg.end[k];
    nq = 0;
    ts_dirty = 0;
  }
  __syncthreads();
  l2_keep(pfv);
  Src s{U, lds32, s0, ESTAGE};  // >= EW + 15 + 44: every phase-A read is staged
  const uint32_t k0 = seg0;
  const uint64_t e0 = seg_end0;  // positions below e0 are in segment k0 (nearly all)
  // window-relative end of the positions whose first record is wholly inside segment k0
  const uint32_t fast_end = e0 - t0 >= 36 + (uint64_t)EW ? EW : e0 - t0 >= 36 ? (uint32_t)(e0 - t0 - 36) + 1 : 0;
  const uint32_t sa = (uint32_t)(t0 - s0);
  const uint32_t nref1 = (uint32_t)c.n + 1u;
  const uint32_t lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
#ifdef SBH_EPROBE
  const uint64_t c1 = __builtin_readcyclecounter();
  uint64_t c1a = 0, c1b = 0, c2 = 0, c3 = 0, c4 = 0;
#endif
  // single-record predicate at window position i -> ok / nrm / und bits
  auto eval_one = [&](uint32_t i) {
    const uint64_t q = t0 + i;
    const uint64_t total = q < e0 ? e0 : sg.end[seg_index(sg, q, k0)];
    uint64_t succ;
    bool normal;
    const uint32_t r = one_record(s, q, total, c, &succ, &normal);
    if (r == 1) {
      atomicOr(&ok[i >> 5], 1u << (i & 31));
      if (normal) atomicOr(&nrm[i >> 5], 1u << (i & 31));
    } else if (r == 2) {
      atomicOr(&und[i >> 5], 1u << (i & 31));
    }
  };
  // the same for the wave's lanes together (every lane of the wave must call it; lanes
  // with has == false only help): long CIGARs are checked 64 ops per step by the wave
  auto eval_one_w = [&](uint32_t i, bool has) {
    const uint64_t q = t0 + i;
    uint64_t succ = 0, cig = 0;
    uint32_t ncig = 0;
    bool normal = false;
    uint32_t r = 0;
    if (has) {
      const uint64_t total = q < e0 ? e0 : sg.end[seg_index(sg, q, k0)];
      r = one_record(s, q, total, c, &succ, &normal, &cig, &ncig);
    }
    uint64_t pend = __ballot(r == ONE_CIGAR);
    while (pend) {
      const uint32_t l = (uint32_t)__builtin_ctzll(pend);
      pend &= pend - 1;
      // (readlane returns int: widen through uint32_t, or a flat offset >= 2^31 sign-extends)
      const uint64_t cl = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(cig >> 32), l) << 32) |
                          (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)cig, l);
      const uint32_t nl = (uint32_t)__builtin_amdgcn_readlane(ncig, l);
      bool bad = false;
      for (uint32_t k = lane; k < nl; k += WAVE) bad = bad || (s.byte_at(cl + 4ull * k) & 0xf) > 8;
      const bool any = __ballot(bad) != 0;
      if (lane == l) r = any ? 0u : 1u;
    }
    if (r == 1) {
      atomicOr(&ok[i >> 5], 1u << (i & 31));
      if (normal) atomicOr(&nrm[i >> 5], 1u << (i & 31));
    } else if (r == 2) {
      atomicOr(&und[i >> 5], 1u << (i & 31));
    }
  };
  // the fixed fields other than refID at window position i < fast_end (refID / next
  // refID in [-1, n), pos / next pos >= -1, l_read_name >= 2, the empty-mapped rule, the
  // remaining-length floor); failing one implies one_record fails, so the filter is exact
  auto fixed_ok = [&](uint32_t i) -> bool {
    const uint32_t gb = i + sa, g = gb >> 2, k = gb & 3;
    const uint32_t *dw = lds32 + g;
    const uint32_t rem = __builtin_amdgcn_alignbyte(dw[1], dw[0], k);
    const uint32_t pos = __builtin_amdgcn_alignbyte(dw[3], dw[2], k);
    const uint32_t bmn = __builtin_amdgcn_alignbyte(dw[4], dw[3], k);
    const uint32_t fnc = __builtin_amdgcn_alignbyte(dw[5], dw[4], k);
    const uint32_t lsq = __builtin_amdgcn_alignbyte(dw[6], dw[5], k);
    const uint32_t nrf = __builtin_amdgcn_alignbyte(dw[7], dw[6], k);
    const uint32_t nps = __builtin_amdgcn_alignbyte(dw[8], dw[7], k);
    const int32_t rnl = (int32_t)(bmn & 0xff), nc = (int32_t)(fnc & 0xffff);
    return nrf + 1u < nref1 && (int32_t)pos >= -1 && (int32_t)nps >= -1 && rnl >= 2 &&
           (((fnc >> 16) & 4) != 0 || ((int32_t)lsq != 0 && nc != 0)) &&
           (int32_t)rem >= implied_min_remaining(rnl, nc, (int32_t)lsq);
  };
  // phase B helpers.  r: 1 true, 0 false, 2 unknown (needs bytes past an open end)
  uint32_t mytrue = 0;
  const uint64_t wbase = (uint64_t)blockIdx.x * (ETILE / 32);
  const uint64_t nwords = (end - begin + 31) / 32;
  // exact check of a candidate: inline (one lane), or queued for k_eager_xq when its first
  // record is long (CIGARs of hundreds of ops: a lane-serial walk would dominate the tile)
  auto exact = [&](uint64_t p, uint64_t total, bool open) -> uint32_t {
    if (o.xq_cap && rtc > 0 && p + 36 <= total && long_candidate(s, p, c)) {
      const unsigned long long x = atomicAdd(o.xq_n, 1ull);
      if (x < o.xq_cap) {
        o.xq_pos[x] = p;
        return EAGER_XQ;
      }
    }
    return eager_at(s, p, total, open, c, rtc, o.front);
  };
  auto call_at = [&](uint32_t i) -> uint32_t {
    const uint64_t p = t0 + i;
    const uint32_t k = p < e0 ? k0 : seg_index(sg, p, k0);
    const uint64_t total = sg.end[k];
    const bool open = sg.open_last && k == sg.n - 1;
    const bool und_p = (und[i >> 5] >> (i & 31)) & 1;
#ifdef SBH_EPROBE
    ++ncand;
#endif
    if (rtc <= 0 || und_p) return exact(p, total, open);  // exact path (HBM/L2 reads)
    // walk the chain through the window's ok bits (next record read at nominal)
    uint64_t q = p;
    int32_t n = 1;
    for (;;) {
      if (n == rtc) return 1;
      const uint32_t iq = (uint32_t)(q - t0);
      if (!((nrm[iq >> 5] >> (iq & 31)) & 1)) break;  // cursor past nominal: exact path
      const uint64_t nxt = q + 4 + (int64_t)(int32_t)s.word_at(q);
      if (nxt + 36 > total || nxt < t0 || nxt - t0 >= EW) break;  // EOF edge / outside window
      const uint32_t jn = (uint32_t)(nxt - t0);
      if ((und[jn >> 5] >> (jn & 31)) & 1) break;
      if (!((ok[jn >> 5] >> (jn & 31)) & 1)) return 0;
      q = nxt;
      ++n;
    }
#ifdef SBH_EPROBE
    ++nexact;
#endif
    return exact(p, total, open);
  };
  auto defer = [&](uint32_t i) {
    const unsigned long long x = atomicAdd(o.defer_n, 1ull);
    if (x < o.defer_cap) o.defer_pos[x] = t0 + i;
  };
  auto settle = [&](uint32_t i, uint32_t r) {  // a candidate's result (queue-driven paths)
    if (r > 1) ts_dirty = 1;  // its bit is settled later (k_eager_xq / k_eager_defer) or unknown
    if (r == 1) {
      atomicOr(&res[i >> 5], 1u << (i & 31));
    } else if (r == EAGER_DEFER) {
      defer(i);
    } else if (r == 2) {
      atomicAdd(o.n_unknown, 1ull);
      atomicMin(o.min_unknown, (unsigned long long)(t0 + i));
    }
  };
  auto write_res = [&]() {  // 16 B per lane: the tile's 2 KiB of bits in one wave-store per 1 KiB
    static_assert(ETILE % 128 == 0, "whole uint4 groups of result words");
    for (uint32_t w4 = threadIdx.x; w4 < ETILE / 128; w4 += T) {
      const uint64_t w = wbase + 4ull * w4;
      if (w >= nwords) break;
      const uint4 v = reinterpret_cast<const uint4 *>(res)[w4];
      if (w + 4 <= nwords) {
        *reinterpret_cast<uint4 *>(o.bits + w) = v;
      } else {
        const uint32_t x[4] = {v.x, v.y, v.z, v.w};
        for (uint32_t k = 0; w + k < nwords; ++k) o.bits[w + k] = x[k];
      }
      mytrue += __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);
    }
  };

  // ---- phase A, stage 1: refID in [-1, n) (the most selective field; ~3% pass) for
  // every position of the window, 4 positions per thread and step from staged dwords
  // with v_alignbyte.  This thread's groups of 4 positions: [g0, g0 + EG); group g
  // covers staged bytes 4g..4g+3. ----
  constexpr uint32_t EG = (EW / 4 + 4 + T - 1) / T;
  constexpr uint32_t EMW = (EG * 4 + 31) / 32;
  const uint32_t ngroups = (EW + sa + 3) / 4;
  const uint32_t g0 = threadIdx.x * EG;
  uint32_t msk[EMW];
#pragma unroll
  for (uint32_t w = 0; w < EMW; ++w) msk[w] = 0;
  // bit b of msk[w] <-> window index ib + 32 w + b; the bits a word keeps: in the window [0, EW),
  // group < ngroups and < EG; from fast_end on every in-window position is kept (decided below)
  const int32_t ib = (int32_t)(4 * g0) - (int32_t)sa;
  const int32_t gl = 4 * ((int32_t)ngroups - (int32_t)g0);
  auto upto = [](int32_t k) -> uint32_t { return k <= 0 ? 0u : k >= 32 ? ~0u : (1u << k) - 1u; };
  auto word_keep = [&](uint32_t w, uint32_t m) -> uint32_t {
    const int32_t i0 = ib + 32 * (int32_t)w;
    const uint32_t in = ~upto(-i0) & upto((int32_t)EW - i0) & upto(gl - 32 * (int32_t)w) &
                        upto(4 * (int32_t)EG - 32 * (int32_t)w);
    return (m | ~upto((int32_t)fast_end - i0)) & in;
  };
  if (o.sieve) {
    // k_lz evaluated this filter (and the next refID / pos signs) on the bytes in its LDS ring:
    // the thread's bits are the sieve's bits [s0 + 4 g0, + 4 EG), masked to the window, plus every
    // position from fast_end on (near a segment end, decided below)
    const uint64_t A = s0 + 4ull * g0;
    const uint32_t *sw = o.sieve + (A >> 5);
    const uint32_t sft = (uint32_t)(A & 31);
    uint32_t lo_w = sw[0];
#pragma unroll
    for (uint32_t w = 0; w < EMW; ++w) {
      const uint32_t hi_w = sw[w + 1];
      const uint32_t m = sft ? (lo_w >> sft) | (hi_w << (32 - sft)) : lo_w;
      lo_w = hi_w;
      msk[w] = word_keep(w, m);
    }
  } else if (SBH_EAGER_SHIFT_SWEEP) {
    // each word's 32 refID tests shifted into it last position first (m = 2 m + test: one
    // add-with-carry per position, no per-position range logic); the word's range after
    static_assert(EMW * 8 >= EG, "the words cover the thread's groups");
#pragma unroll
    for (uint32_t w = 0; w < EMW; ++w) {
      constexpr uint32_t GW = 8;  // groups (of 4 positions) per word
      uint32_t d[GW + 1];         // staged dwords g0 + 8 w + 1 .. + 9: bytes 4..7 of every position's record
#pragma unroll
      for (uint32_t j = 0; j <= GW; ++j) d[j] = 8 * w + j <= EG ? lds32[g0 + 8 * w + j + 1] : 0u;
      uint32_t m = 0;
#pragma unroll
      for (int32_t j = GW - 1; j >= 0; --j) {
        if (8 * w + (uint32_t)j >= EG) continue;
#pragma unroll
        for (int32_t k = 3; k >= 0; --k) {
          const uint32_t ref = __builtin_amdgcn_alignbyte(d[j + 1], d[j], (uint32_t)k);
          m = m + m + (ref + 1u < nref1 ? 1u : 0u);
        }
      }
      msk[w] = word_keep(w, m);
    }
  } else {
    uint32_t a = lds32[g0 + 1];
#pragma unroll
    for (uint32_t gi = 0; gi < EG; ++gi) {
      const uint32_t g = g0 + gi;
      const uint32_t b = lds32[g + 2];
      uint32_t m4 = 0;
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t ref = __builtin_amdgcn_alignbyte(b, a, k);
        const uint32_t ii = 4 * g + k - sa;  // wraps for positions before the window
        const bool in = ii < EW && g < ngroups;
        m4 |= (in && (ref + 1u < nref1 || ii >= fast_end)) ? 1u << k : 0u;
      }
      msk[(gi * 4) / 32] |= m4 << ((gi * 4) % 32);
      a = b;
    }
  }
#ifdef SBH_EPROBE
  const uint64_t c1x = __builtin_readcyclecounter();
#endif
  // ---- survivor lists: each wave compacts its refID survivors, in position order, into
  // its own queue segment and filters them in place (fixed fields, then the whole
  // single-record predicate), so every step runs one survivor per lane.  The candidate
  // list comes out sorted, which lets phase B link each record to the next candidate. ----
  uint16_t *wq = queue + wid * SEGCAP;
  uint32_t n1 = 0;
#pragma unroll
  for (uint32_t w = 0; w < EMW; ++w) n1 += __popc(msk[w]);
  const uint32_t incl1 = wave_incl_scan(n1);
  const uint32_t wtot1 = __builtin_amdgcn_readlane(incl1, WAVE - 1);
  if (wtot1 <= SEGCAP) {
    uint32_t o1 = incl1 - n1;
#pragma unroll
    for (uint32_t w = 0; w < EMW; ++w) {
      uint32_t mw = msk[w];
      while (mw) {
        const uint32_t bit = __builtin_ctz(mw);
        mw &= mw - 1;
        const uint32_t gk = w * 32 + bit;
        wq[o1++] = (uint16_t)(4 * (g0 + gk / 4) + gk % 4 - sa);
      }
    }
  }
  // in-place, order-keeping wave compaction of wq[0, n) by pred; returns the kept count
  // (a lane's store never reaches an entry another lane has yet to load)
  auto compact = [&](uint32_t n, auto pred) -> uint32_t {
    uint32_t kept = 0;
    for (uint32_t x = 0; x < n; x += WAVE) {
      const bool has = x + lane < n;
      const uint32_t i = has ? wq[x + lane] : 0u;
      const bool keep = has && pred(i);
      const uint64_t bal = __ballot(keep);
      const uint32_t rank =
          __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
      if (keep) wq[kept + rank] = (uint16_t)i;
      kept += (uint32_t)__popcll(bal);
    }
    return kept;
  };
  uint32_t n2 = 0;
#ifdef SBH_EPROBE
  const uint64_t c1y = __builtin_readcyclecounter();
#endif
  if (wtot1 <= SEGCAP) n2 = compact(wtot1, [&](uint32_t i) { return i >= fast_end || fixed_ok(i); });
  if (lane == 0) wcnt[wid] = wtot1 <= SEGCAP ? n2 : ~0u;
#ifdef SBH_EPROBE
  c1a = __builtin_readcyclecounter();
#endif
  __syncthreads();
  bool fast = rtc > 0;
#pragma unroll
  for (uint32_t w = 0; w < NWV; ++w) fast = fast && wcnt[w] != ~0u;
  if (fast) {
    // entries of the concatenated segment lists (sorted by position)
    uint32_t pre[NWV + 1];
    pre[0] = 0;
#pragma unroll
    for (uint32_t w = 0; w < NWV; ++w) pre[w + 1] = pre[w] + wcnt[w];
    auto entry = [&](uint32_t g) -> uint32_t {
      uint32_t w = 0;
#pragma unroll
      for (uint32_t k = 1; k < NWV; ++k) w += g >= pre[k] ? 1u : 0u;
      return queue[w * SEGCAP + g - pre[w]];
    };
#ifdef SBH_EPROBE
    if (threadIdx.x == 0) nsurv = pre[NWV];
#endif
    for (uint32_t xb = 0; xb < pre[NWV]; xb += T) {  // uniform trip count: eval_one_w uses the whole wave
      const uint32_t x = xb + threadIdx.x;
      eval_one_w(x < pre[NWV] ? entry(x) : 0u, x < pre[NWV]);
    }
#ifdef SBH_EPROBE
    c1b = __builtin_readcyclecounter();
#endif
    __syncthreads();
    // candidates: ok or undecidable
    const uint32_t n3 = compact(n2, [&](uint32_t i) { return (((ok[i >> 5] | und[i >> 5]) >> (i & 31)) & 1) != 0; });
    __syncthreads();  // every thread has read wcnt
    if (lane == 0) wcnt[wid] = n3;
    __syncthreads();
#pragma unroll
    for (uint32_t w = 0; w < NWV; ++w) pre[w + 1] = pre[w] + wcnt[w];
    const uint32_t nc3 = pre[NWV];
#ifdef SBH_EPROBE
    c2 = __builtin_readcyclecounter();
#endif
    // ---- phase B.  One step of call_at's chain walk per candidate: from an ok, normal
    // record whose successor lies in the window, is decidable and is ok, the step LINKs
    // when that successor is the next candidate; it FAILs when the successor is not ok;
    // anything else leaves the candidate to call_at.  A candidate is true when the
    // rtc - 1 steps from it and its successors all LINK. ----
    for (uint32_t g = threadIdx.x; g < nc3; g += T) {
      const uint32_t i = entry(g);
      if ((und[i >> 5] >> (i & 31)) & 1) continue;
      if (!((nrm[i >> 5] >> (i & 31)) & 1)) continue;  // cursor past nominal
      const uint64_t q = t0 + i;
      const uint64_t total = q < e0 ? e0 : sg.end[seg_index(sg, q, k0)];
      const uint64_t nxt = q + 4 + (int64_t)(int32_t)s.word_at(q);
      if (nxt + 36 > total || nxt < t0 || nxt - t0 >= EW) continue;  // EOF edge / outside window
      const uint32_t jn = (uint32_t)(nxt - t0);
      if ((und[jn >> 5] >> (jn & 31)) & 1) continue;
      if (!((ok[jn >> 5] >> (jn & 31)) & 1)) atomicOr(&lfail[g >> 5], 1u << (g & 31));
      else if (g + 1 < nc3 && entry(g + 1) == jn) atomicOr(&lnk[g >> 5], 1u << (g & 31));
    }
    __syncthreads();
#ifdef SBH_EPROBE
    c3 = __builtin_readcyclecounter();
#endif
    const uint32_t need = (uint32_t)rtc - 1;  // steps from a candidate to its rtc-th record
    for (uint32_t g = threadIdx.x; g < nc3; g += T) {
      const uint32_t i = entry(g);
      if (i >= ETILE || t0 + i >= end) continue;
      uint32_t r;
      if ((und[i >> 5] >> (i & 31)) & 1) {
        r = call_at(i);
      } else {
        uint32_t m = 0;  // first non-LINK step among [g, g + need)
        bool all = true;
        while (m < need) {
          const uint32_t gg = g + m, b = gg & 31;
          const uint32_t span = min(32u - b, need - m);
          const uint32_t gap = ~(gg < EQ_CHUNK ? lnk[gg >> 5] : 0u) >> b;
          const uint32_t mk = span == 32 ? ~0u : (1u << span) - 1u;
          if (gap & mk) {
            m += __builtin_ctz(gap & mk);
            all = false;
            break;
          }
          m += span;
        }
        if (all) r = 1;
        else if (g + m < EQ_CHUNK && ((lfail[(g + m) >> 5] >> ((g + m) & 31)) & 1)) r = 0;
        else r = call_at(i);
      }
      settle(i, r);
    }
    __syncthreads();
#ifdef SBH_EPROBE
    c4 = __builtin_readcyclecounter();
#endif
    if (SBH_TSUM_CODE && o.tsum) {
      // each wave's quarter of the tile (EAGER_SUB positions, its lanes' result words): each true
      // position's record step (its length field, staged) against the next true position of the
      // quarter; the last one's step for k_verify_chain_w.  Wave-local: no barrier.
      constexpr uint32_t TW = ETILE / 32 / T;  // result words per thread
      static_assert(TW * T * 32 == ETILE && ETILE / NWV == EAGER_SUB, "whole result words per thread");
      const uint32_t wt0 = threadIdx.x * TW;
      uint32_t rw[TW];
      bool any = false;
#pragma unroll
      for (uint32_t k = 0; k < TW; ++k) {
        rw[k] = res[wt0 + k];
        any = any || rw[k] != 0;
      }
      const uint64_t bal = __ballot(any);
      uint32_t an = 0, af = ~0u;
      uint64_t mystep = TS_NONE;
      bool last = false;
      if (any) {
        uint32_t nx = ETILE;  // the first true position after this thread's words in the quarter
        const uint64_t after = lane == WAVE - 1 ? 0ull : bal & (~0ull << (lane + 1));
        if (after) {
          const uint32_t tn = wid * WAVE + (uint32_t)__builtin_ctzll(after);
#pragma unroll
          for (uint32_t k = TW; k-- > 0;) {
            const uint32_t x = res[tn * TW + k];
            if (x) nx = 32 * (tn * TW + k) + __builtin_ctz(x);
          }
        }
#pragma unroll
        for (uint32_t k = 0; k < TW; ++k) {
          uint32_t x = rw[k];
          while (x) {
            const uint32_t i = 32 * (wt0 + k) + __builtin_ctz(x);
            x &= x - 1;
            uint32_t nxt = nx;
            if (x) {
              nxt = 32 * (wt0 + k) + __builtin_ctz(x);
            } else {
#pragma unroll
              for (uint32_t k2 = k + 1; k2 < TW; ++k2)
                if (rw[k2] && nxt == nx) nxt = 32 * (wt0 + k2) + __builtin_ctz(rw[k2]);
            }
            const uint64_t q = t0 + i;
            const uint64_t total = q < e0 ? e0 : sg.end[seg_index(sg, q, k0)];
            const uint64_t step = q + 4 > total ? TS_NONE : q + 4 + (int64_t)(int32_t)s.word_at(q);
            if (nxt < ETILE) {
              if (step != t0 + nxt) {
                ++an;
                af = min(af, i - wid * EAGER_SUB);
              }
            } else {
              mystep = step;
              last = true;
            }
          }
        }
      }
      an = __builtin_amdgcn_readlane(wave_incl_scan(an), WAVE - 1);
#pragma unroll
      for (uint32_t o2 = 1; o2 < WAVE; o2 <<= 1) af = min(af, (uint32_t)__shfl_xor(af, o2, WAVE));
      const uint64_t lb = __ballot(last);
      uint64_t sl = TS_NONE;
      if (lb) {
        const uint32_t l = (uint32_t)__builtin_ctzll(lb);
        sl = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(mystep >> 32), l) << 32 |
             (uint32_t)__builtin_amdgcn_readlane((uint32_t)mystep, l);
      }
      if (lane == 0) o.tsum[blockIdx.x * NWV + wid] = TileSum{ts_dirty ? TS_DIRTY : sl, an, af};
    }
    write_res();
  } else {
    // ---- fallback (a survivor list overflowed, or rtc <= 0): per-thread survivor loop
    // (fixed fields), shared queue, word-wise phase B ----
#pragma unroll
    for (uint32_t w = 0; w < EMW; ++w) {
      uint32_t mw = msk[w];
      while (mw) {
        const uint32_t bit = __builtin_ctz(mw);
        mw &= mw - 1;
        const uint32_t gk = w * 32 + bit;
        const uint32_t i = 4 * (g0 + gk / 4) + gk % 4 - sa;
        if (i < fast_end && !fixed_ok(i)) continue;
#ifdef SBH_EPROBE
        ++nsurv;
#endif
        const uint32_t x = atomicAdd(&nq, 1u);
        if (x < EQ_CHUNK) queue[x] = (uint16_t)i;
        else eval_one(i);  // queue full: evaluate in place
      }
    }
    __syncthreads();
    {
      const uint32_t nsv = nq < EQ_CHUNK ? nq : EQ_CHUNK;
      for (uint32_t x = threadIdx.x; x < nsv; x += T) eval_one(queue[x]);
    }
    __syncthreads();
    if (rtc > 0 && nq <= EQ_CHUNK) {
      // every candidate is in the survivor queue: one candidate per thread, balanced
      for (uint32_t x = threadIdx.x; x < nq; x += T) {
        const uint32_t i = queue[x];
        if (i >= ETILE || t0 + i >= end) continue;
        if (!(((ok[i >> 5] | und[i >> 5]) >> (i & 31)) & 1)) continue;
        settle(i, call_at(i));
      }
      __syncthreads();
      write_res();
    } else {
      for (uint32_t w = threadIdx.x; w < ETILE / 32; w += T) {
        if (wbase + w >= nwords) break;
        uint32_t cand = rtc <= 0 ? ~0u : (ok[w] | und[w]);
        uint32_t rw = 0;
        while (cand) {
          const uint32_t bit = __builtin_ctz(cand);
          cand &= cand - 1;
          const uint32_t i = 32 * w + bit;
          if (t0 + i >= end) break;
          const uint32_t r = call_at(i);
          if (r == 1) {
            rw |= 1u << bit;
          } else if (r == EAGER_DEFER) {
            defer(i);
          } else if (r == 2) {
            atomicAdd(o.n_unknown, 1ull);
            atomicMin(o.min_unknown, (unsigned long long)(t0 + i));
          }
        }
        o.bits[wbase + w] = rw;
        mytrue += __popc(rw);
      }
    }
  }
  {
    const uint32_t wt = (uint32_t)__builtin_amdgcn_readlane(wave_incl_scan(mytrue), WAVE - 1);
    if (lane == 0 && wt)
      atomicAdd(o.true_spread + ((blockIdx.x * NWV + wid) % TRUE_SLOTS) * TRUE_STRIDE, (unsigned long long)wt);
  }
  if (SBH_TSUM_CODE && o.tsum && !fast && lane == 0)  // (the fallback path leaves no summaries)
    o.tsum[blockIdx.x * NWV + wid] = TileSum{TS_DIRTY, 0, ~0u};
#ifdef SBH_EPROBE
  __shared__ uint32_t psurv, pcand, pexact, ntrue;
  if (threadIdx.x == 0) { psurv = 0; pcand = 0; pexact = 0; ntrue = 0; }
  __syncthreads();
  atomicAdd(&ntrue, mytrue);
  atomicAdd(&psurv, nsurv);
  atomicAdd(&pcand, ncand);
  atomicAdd(&pexact, nexact);
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x >= 3000 && blockIdx.x < 3008)
    printf("eager wg %u fast %d stage %llu sweep %llu lists %llu A1+2 %llu eval %llu cand %llu B %llu (links %llu calls %llu tail %llu) surv %u exactcalls %u true %u exact %u\n",
           blockIdx.x, (int)fast, (unsigned long long)(c1 - c0), (unsigned long long)(c1x - c1),
           (unsigned long long)(c1y - c1x), (unsigned long long)(c1a - c1),
           (unsigned long long)(c1b - c1a), (unsigned long long)(c2 - c1b),
           (unsigned long long)(__builtin_readcyclecounter() - c2), (unsigned long long)(c3 - c2),
           (unsigned long long)(c4 - c3), (unsigned long long)(__builtin_readcyclecounter() - c4), psurv, pcand, ntrue,
           pexact);
#endif
}

struct FullOut {
  uint32_t *words;                 // optional: word per position
  unsigned long long *counts;      // [21][19]
  unsigned long long *rbe;         // [21][64]
  unsigned long long *n_success;
  unsigned long long *n_unknown;
  unsigned long long *min_unknown;
  unsigned long long *close_n;     // positions with numNonZeroFields <= 2
  uint64_t *close_pos;
  uint32_t *close_word;
  uint64_t close_cap;
};

// ---- full check, one tile per workgroup, O(1) LDS work per position for the first record ----
// Tiles are 16-byte aligned (tile b covers flat [B + b * FTILE, B + (b + 1) * FTILE), B =
// begin rounded down to 16; positions before `begin` are skipped), so the staged window
// starts at the tile's first position and lane t owns 16 consecutive positions: three
// 16-byte LDS reads give the fixed fields of all 16 (v_alignbyte on neighbouring dwords).
// Per staged window two byte-class bitmaps are built once: `bad name byte` (outside
// [0x21..0x3F] u [0x41..0x7E]) and `bad CIGAR op byte` ((b & 0xf) > 8); a position's read
// name is valid iff no bad name byte lies in [name, name + l_read_name - 1), and its first
// invalid op is the first bad op byte at a stride of 4 from the CIGAR start -- one or two
// word reads each.  Positions whose first record passes (record starts: the chain must be
// followed) or whose CIGAR runs past the window are queued and decided by the exact full_at()
// after the tile's sweep, one per lane (no wave waits on another lane's chain).  Histograms
// are LDS adds into 4 replicas (lane mod 4, stride coprime to the 32 banks), so lanes
// counting the same (numNonZeroFields, flag) rarely meet on one address; close calls are
// collected in LDS and appended with one global atomic per workgroup.
constexpr uint32_t FTILE = 8192;              // positions per workgroup
constexpr uint32_t FPL = 16;                  // positions per lane and step
constexpr uint32_t FNV = FTILE / 16 + 256;    // staged 16-byte vectors: tile + 4 KiB look-ahead (chains of
                                              // 10 short records stay in LDS)
constexpr uint32_t FSN = FNV * 16;            // staged bytes
constexpr uint32_t FBW = FSN / 32;            // bitmap words
#ifndef SBH_FULL_FCCAP
#define SBH_FULL_FCCAP 256
#endif
constexpr uint32_t FCCAP = SBH_FULL_FCCAP;    // close calls buffered per workgroup
#ifndef SBH_FULL_CTG_LDS
#define SBH_FULL_CTG_LDS 1
#endif
#ifndef SBH_FULL_RUN
#define SBH_FULL_RUN 0  // 1: Counts rows of equal consecutive failure words added once per run (A/B: 7.44 -> 7.50 ms, off)
#endif
#ifndef SBH_FULL_ACCF
#define SBH_FULL_ACCF 1  // fast tiles: failures accounted without the success / unknown / rbe cases
#endif
#ifndef SBH_FULL_FAST
#define SBH_FULL_FAST 1  // tiles far from a segment end: full_first_win (no end-of-stream cases)
#endif
#ifndef SBH_FULL_HOT
#define SBH_FULL_HOT 0  // 1: fast tiles count the wave's most shared failure word by ballot (A/B r04o: 7.40 -> 7.89 ms at 4 M records: off)
#endif
constexpr uint32_t FCTG = 1024;               // contig lengths staged in LDS (more: read from global)
constexpr uint32_t FULL_SLOW = 0xFFFFFFFFu;   // "take the exact path" (no valid word has all bits)
constexpr uint32_t FULL_PASS = 0xFFFFFFFEu;   // the first record passes: the chain decides
static_assert(FTILE % (FPL * T) == 0 && FSN % 32 == 0 && FSN >= FTILE + 36 + 255 + 16, "full tile layout");

// exact per-byte classes of the 4 bytes of x, as 4 bits (bit k = byte k)
__device__ __forceinline__ uint32_t pack4(uint32_t hi_bits) {  // bit 7 of each byte -> 4 bits
  return (((hi_bits >> 7) & 0x01010101u) * 0x01020408u) >> 24;
}
__device__ __forceinline__ uint32_t bad_name4(uint32_t x) {
  const uint32_t lo7 = x & 0x7f7f7f7fu;
  const uint32_t lt21 = ~((lo7 + 0x5f5f5f5fu) | x) & 0x80808080u;  // b < 0x21
  const uint32_t gt7e = (x | (lo7 + 0x01010101u)) & 0x80808080u;   // b > 0x7e
  const uint32_t y = x ^ 0x40404040u;
  const uint32_t eq40 = ~(((y & 0x7f7f7f7fu) + 0x7f7f7f7fu) | y) & 0x80808080u;  // b == 0x40
  return pack4(lt21 | gt7e | eq40);
}
__device__ __forceinline__ uint32_t bad_op4(uint32_t x) {  // (b & 0xf) > 8
  return pack4((((x & 0x0f0f0f0fu) + 0x07070707u) & 0x10101010u) << 3);
}

// first set bit y in [x, lim) of an LDS bitmap (bit positions = staged byte offsets), masked
// per word by `pat` (all ones, or every 4th bit from x's residue); lim if none
__device__ __forceinline__ uint32_t next_set(const uint32_t *bm, uint32_t x, uint32_t lim, uint32_t pat) {
  if (x >= lim) return lim;
  uint32_t w = x >> 5;
  const uint32_t wl = (lim + 31) >> 5;
  uint32_t m = bm[w] & pat & (~0u << (x & 31));
  while (!m) {
    if (++w >= wl) return lim;
    m = bm[w] & pat;
  }
  const uint32_t y = 32 * w + __builtin_ctz(m);
  return y < lim ? y : lim;
}

struct Fixed {  // the 36-byte fixed part of a record (tlen unused by the checkers)
  int32_t rem, idx, pos, seq_len, nidx, npos;
  uint32_t bmn, fnc;
};

// The full check's first record at p (window offset q) from its fixed fields, the staged
// window and its bitmaps: the result word when the first record fails (or at EOF / open-end
// rules), FULL_PASS when it passes, FULL_SLOW when the window cannot decide it.
__device__ __forceinline__ uint32_t full_first(const Src &s, const uint32_t *bname, const uint32_t *bop, uint64_t p,
                                               uint32_t q, const Fixed &x, uint64_t total, bool open, const Ctg &c,
                                               int32_t rtc, const OpIdx &oi) {
  if (rtc == 0) return FULL_SUCCESS;
  if (p + 36 > total) return open ? FULL_UNKNOWN : 1u;
  const int32_t rnl = (int32_t)(x.bmn & 0xff), nc = (int32_t)(x.fnc & 0xffff);
  uint32_t f = ref_pos_error(x.idx, x.pos, c) << 1;
  if (x.rem < implied_min_remaining(rnl, nc, x.seq_len)) f |= 1u << 18;
  f |= ref_pos_error(x.nidx, x.npos, c) << 5;
#ifdef SBH_FULL_FIXEDONLY  // A/B probe (timing only, results wrong): no read-name / CIGAR tests
  if (f) return f;
#endif
  uint64_t cur = p + 36;
  uint32_t a = q + 36;  // window offset of cur
  if (rnl == 0) {
    f |= 1u << 12;
  } else if (rnl == 1) {
    f |= 1u << 13;
  } else if (cur + (uint64_t)rnl > total) {
    if (open) return FULL_UNKNOWN;
    return f | (1u << 9);  // tooFewBytesForReadName: the CIGAR is not read
  } else {
    const uint32_t z = a + (uint32_t)rnl - 1;  // name bytes [a, z), its NUL at z
    if ((uint8_t)(s.lds32[z >> 2] >> (8 * (z & 3))) != 0) f |= 1u << 10;
    else if (next_set(bname, a, z, ~0u) < z) f |= 1u << 11;
    cur += rnl;
    a = z + 1;
  }
  // CIGAR: the first op k < lim = min(nc, ops that fit below total) with a bad op byte
  const uint64_t fit = total >= cur ? (total - cur) / 4 : 0;
  const uint32_t lim = fit < (uint64_t)nc ? (uint32_t)fit : (uint32_t)nc;
  const uint64_t stop = (uint64_t)a + 4ull * lim;  // window offset past the ops to test
  const uint32_t hi = stop < FSN ? (uint32_t)stop : FSN;
  const uint32_t y = next_set(bop, a, hi, 0x11111111u << (a & 3));
  bool cig_err = false, beyond = false;
  if (y >= hi && stop > hi) {  // ops past the window: the op index, else the exact path
    if (!(oi.ob && s.s0 + a >= oi.base && s.s0 + stop <= oi.end)) return FULL_SLOW;
    beyond = op_scan(oi, s.s0 + a, s.s0 + stop) < s.s0 + stop;
  }
  if (y < hi || beyond) {
    cig_err = true;
    f |= 1u << 15;
  } else if (lim < (uint32_t)nc) {
    if (open) return FULL_UNKNOWN;
    cig_err = true;
    f |= 1u << 14;
  }
  if (!cig_err && (x.fnc & (4u << 16)) == 0 && (x.seq_len == 0 || nc == 0)) {
    if (x.seq_len == 0) f |= 1u << 16;  // EmptyMapped(emptySeq, emptyCigar) field swap
    if (nc == 0) f |= 1u << 17;
  }
  return f ? f : FULL_PASS;  // a passing first record: the chain decides
}

// getRefPosError without branches (PosChecker.scala:43-63): the four error bits are
// independent tests -- idx < -1, idx >= n, pos < -1, and pos past the contig of a valid idx --
// which is exactly the reference's if/else chain (each earlier case rules the later bits out).
__device__ __forceinline__ uint32_t ref_pos_error_bf(int32_t idx, int32_t pos, const Ctg &c) {
  const bool inr = (uint32_t)idx < (uint32_t)c.n;
  const int32_t L = c.len[inr ? idx : 0];
  return (idx < -1 ? 1u : 0u) | (idx >= c.n ? 2u : 0u) | (pos < -1 ? 4u : 0u) | (inr && pos > L ? 8u : 0u);
}

// Bytes past a position that full_first may read or judge against the stream end: fixed
// fields, the longest name, the longest CIGAR.  A tile all of whose positions lie at least
// this far before their segment's end (and inside [begin, end)) never meets an end-of-stream
// rule, so full_first reduces to full_first_win there.
constexpr uint64_t FULL_FAST_REACH = 36 + 255 + 4ull * 65535 + 4;

// full_first for a position of a fast tile (see FULL_FAST_REACH): the same word, from 32-bit
// window offsets and no end-of-stream cases (every read of the name is inside the staged
// window: q < FTILE, q + 36 + 255 < FSN).
__device__ __forceinline__ uint32_t full_first_win(const Src &s, const uint32_t *bname, const uint32_t *bop,
                                                   uint32_t q, const Fixed &x, const Ctg &c, const OpIdx &oi) {
  const int32_t rnl = (int32_t)(x.bmn & 0xff), nc = (int32_t)(x.fnc & 0xffff);
  uint32_t f = ref_pos_error_bf(x.idx, x.pos, c) << 1;
  f |= x.rem < implied_min_remaining(rnl, nc, x.seq_len) ? 1u << 18 : 0u;
  f |= ref_pos_error_bf(x.nidx, x.npos, c) << 5;
#ifdef SBH_FULL_FIXEDONLY  // A/B probe (timing only, results wrong): no read-name / CIGAR tests
  if (f) return f;
#endif
  uint32_t a = q + 36;  // window offset of the name / CIGAR
  if (rnl < 2) {
    f |= rnl == 0 ? 1u << 12 : 1u << 13;
  } else {
    const uint32_t z = a + (uint32_t)rnl - 1;  // name bytes [a, z), its NUL at z
    if ((uint8_t)(s.lds32[z >> 2] >> (8 * (z & 3))) != 0) f |= 1u << 10;
    else if (next_set(bname, a, z, ~0u) < z) f |= 1u << 11;
    a = z + 1;
  }
  const uint32_t stop = a + 4u * (uint32_t)nc;  // (no stream end within reach: lim = nc)
  const uint32_t hi = stop < FSN ? stop : FSN;
  const uint32_t y = next_set(bop, a, hi, 0x11111111u << (a & 3));
  bool cig_err = y < hi;
  if (!cig_err && stop > hi) {  // ops past the window: the op index, else the exact path
    if (!(oi.ob && s.s0 + a >= oi.base && s.s0 + stop <= oi.end)) return FULL_SLOW;
    cig_err = op_scan(oi, s.s0 + a, s.s0 + stop) < s.s0 + stop;
  }
  if (cig_err) {
    f |= 1u << 15;
  } else if ((x.fnc & (4u << 16)) == 0 && (x.seq_len == 0 || nc == 0)) {
    if (x.seq_len == 0) f |= 1u << 16;  // EmptyMapped(emptySeq, emptyCigar) field swap
    if (nc == 0) f |= 1u << 17;
  }
  return f ? f : FULL_PASS;
}

__device__ __forceinline__ Fixed fixed_at(const uint32_t *lds32, uint32_t q) {
  const uint32_t *d = lds32 + (q >> 2);
  const uint32_t k = q & 3;
  Fixed x;
  x.rem = (int32_t)__builtin_amdgcn_alignbyte(d[1], d[0], k);
  x.idx = (int32_t)__builtin_amdgcn_alignbyte(d[2], d[1], k);
  x.pos = (int32_t)__builtin_amdgcn_alignbyte(d[3], d[2], k);
  x.bmn = __builtin_amdgcn_alignbyte(d[4], d[3], k);
  x.fnc = __builtin_amdgcn_alignbyte(d[5], d[4], k);
  x.seq_len = (int32_t)__builtin_amdgcn_alignbyte(d[6], d[5], k);
  x.nidx = (int32_t)__builtin_amdgcn_alignbyte(d[7], d[6], k);
  x.npos = (int32_t)__builtin_amdgcn_alignbyte(d[8], d[7], k);
  return x;
}

// full.Checker.apply at p through the window (full/Checker.scala:22-184): record n of the
// chain sits at the previous record's nominal end, so while records stay normal (their name
// and CIGAR end at or before the nominal end) and inside the window, each one is the
// first-record check at its own start (full_first), with readsBeforeError = n and the clean
// end rule (the stream ends exactly at a record boundary after n > 0 records) in between.
// Anything else -- an abnormal record, a nominal end past the stream, a record the window
// does not hold -- returns FULL_SLOW for the exact full_at().
__device__ uint32_t chain_full(const Src &s, const uint32_t *bname, const uint32_t *bop, uint64_t p, uint64_t total,
                               bool open, const Ctg &c, int32_t rtc, const OpIdx &oi) {
  uint64_t q = p;
  for (uint32_t n = 0;; ++n) {
    if ((int32_t)n == rtc) return FULL_SUCCESS | (n << N_SHIFT);
    if (q + 36 > total) {
      if (open) return FULL_UNKNOWN;
      return n > 0 && q == total ? FULL_SUCCESS | (n << N_SHIFT) : 1u | (n << N_SHIFT);
    }
    if (q - s.s0 + 36 + 255 + 8 > FSN) return FULL_SLOW;  // fixed fields + the longest name staged
    const uint32_t qw = (uint32_t)(q - s.s0);
    const Fixed x = fixed_at(s.lds32, qw);
    const uint32_t r = full_first(s, bname, bop, q, qw, x, total, open, c, 1, oi);
    if (r == FULL_SLOW || r == FULL_UNKNOWN) return r;
    if (r != FULL_PASS) return r | (n << N_SHIFT);
    const uint64_t nominal = q + 4 + (int64_t)x.rem;
    const uint64_t cur = q + 36 + (x.bmn & 0xff) + 4ull * (x.fnc & 0xffff);
    if ((int64_t)(nominal - cur) < 0 || nominal > total) return FULL_SLOW;
    q = nominal;
  }
}

#ifndef SBH_FULL_WGS
#define SBH_FULL_WGS 5  // workgroups per CU the register budget allows
#endif
__global__ __launch_bounds__(T, SBH_FULL_WGS) void k_full(const uint8_t *__restrict__ U, uint64_t u_pad, uint64_t begin,
                                            uint64_t end, Segs sg, Ctg c, int32_t rtc, FullOut o, OpIdx oi) {
#ifndef SBH_FULL_PACKED
#define SBH_FULL_PACKED 0  // 1: Counts replicas as 16-bit counter pairs (A/B: 7.53 -> 7.72 ms, not kept)
#endif
#ifndef SBH_FULL_NREP
#define SBH_FULL_NREP (SBH_FULL_PACKED ? 8 : 4)
#endif
  // Counts histogram replicas, one per lane residue.  Packed: a row of 10 words per nnz, flags 2w
  // and 2w + 1 as the low / high 16 bits of word w (a replica counts at most FTILE positions, so
  // 16 bits hold it): the same LDS as 4 unpacked replicas gives 8, halving the lanes that add to
  // one address in one instruction, and a failing position adds once per flag pair, not per flag.
  constexpr uint32_t RW = SBH_FULL_PACKED ? 10 : 19;  // words per nnz row
  static_assert(!SBH_FULL_PACKED || FTILE < 65536, "16-bit replica counters");
  constexpr uint32_t NREP = SBH_FULL_NREP, REP = 21 * RW + (SBH_FULL_PACKED ? 1 : 2);  // (odd stride: replica
                                                                 // bases on distinct banks)
  constexpr uint32_t SLOWCAP = 512;
  __shared__ uint4 ldsv[FNV];
  __shared__ uint32_t bname[FBW], bop[FBW];
  __shared__ uint32_t hist[NREP * REP];   // [lane % NREP][nnz * 19 + flag]
  __shared__ uint64_t cpos[FCCAP];
  __shared__ uint32_t cword[FCCAP];
  __shared__ uint32_t slowq[SLOWCAP];     // tile offsets of positions for the exact path
  __shared__ uint32_t seg0, nsucc, ncl, nslow;
  __shared__ uint64_t e0;
  __shared__ unsigned long long cbase;
#if SBH_FULL_CTG_LDS
  // contig lengths in LDS (getRefPosError reads one for every position whose refID is valid:
  // inside records that is several per record, each an L1/L2 round trip from global memory)
  __shared__ int32_t ctgl[FCTG];
  if (c.n <= (int32_t)FCTG) {
    for (int32_t i = threadIdx.x; i < c.n; i += T) ctgl[i] = c.len[i];
    c.len = ctgl;
  }
#endif
  const uint32_t *lds32 = reinterpret_cast<const uint32_t *>(ldsv);
  const uint64_t s0 = (begin & ~15ull) + (uint64_t)blockIdx.x * FTILE;  // 16-aligned tile start
  stage_vec<FNV>(ldsv, U, s0, u_pad);
  for (uint32_t i = threadIdx.x; i < NREP * REP; i += T) hist[i] = 0;
  if (threadIdx.x == 0) {
    seg0 = seg_first(sg, s0 > begin ? s0 : begin);
    e0 = sg.end[seg0];
    nsucc = ncl = nslow = 0;
  }
  __syncthreads();
  for (uint32_t w = threadIdx.x; w < FBW; w += T) {  // byte classes of staged bytes 32w..32w+31
    uint32_t bn = 0, bo = 0;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
      const uint32_t x = lds32[8 * w + j];
      bn |= bad_name4(x) << (4 * j);
      bo |= bad_op4(x) << (4 * j);
    }
    bname[w] = bn;
    bop[w] = bo;
  }
  __syncthreads();
  const Src s{U, lds32, s0, FSN};
  uint32_t *myhist = hist + (threadIdx.x % NREP) * REP;
  uint32_t mysucc = 0;
  // one position's result into the counters (FullCheck.scala:142-192): Success, unknown, or a
  // failure counted per (numNonZeroFields, flag) unless it is TooFewFixedBlockBytes alone
  auto account = [&](uint64_t p, uint32_t r) {
    if (o.words) o.words[p - begin] = r;
    if (r & FULL_SUCCESS) {
      ++mysucc;
      return;
    }
    if (r & FULL_UNKNOWN) {
      atomicAdd(o.n_unknown, 1ull);
      atomicMin(o.min_unknown, (unsigned long long)p);
      return;
    }
    uint32_t f = r & 0x7FFFFu;
    const uint32_t rbe = (r >> N_SHIFT) & 0x3FFu;
    if (f == 1u && rbe == 0) return;
    const uint32_t nnz = __popc(f) + (rbe > 0);
#ifdef SBH_FULL_NOHIST  // A/B: the check without its aggregation (tools/full_ab.py)
    if (nnz != 77) return;
#endif
    uint32_t *row = myhist + nnz * RW;
#if SBH_FULL_PACKED
    while (f) {
      const uint32_t w = __builtin_ctz(f) >> 1;
      const uint32_t pr = (f >> (2 * w)) & 3u;
      atomicAdd(&row[w], (pr & 1u) | (pr >> 1) << 16);
      f &= ~(3u << (2 * w));
    }
#else
    while (f) {
      atomicAdd(&row[__builtin_ctz(f)], 1u);
      f &= f - 1;
    }
#endif
    if (rbe > 0 && rbe < 64) atomicAdd(&o.rbe[nnz * 64 + rbe], 1ull);  // rare: positions past a record
    if (nnz <= 2) {
      const uint32_t slot = atomicAdd(&ncl, 1u);
      if (slot < FCCAP) {
        cpos[slot] = p;
        cword[slot] = r;
      } else {
        const unsigned long long gs = atomicAdd(o.close_n, 1ull);
        if (gs < o.close_cap) { o.close_pos[gs] = p; o.close_word[gs] = r; }
      }
    }
  };
  // account() for a first-record failure of a fast tile: never success, unknown, TooFewFixed-
  // BlockBytes alone or a readsBeforeError count, so only the Counts row and close calls
  // Counts rows of a run of equal failure words are added once with the run's length: inside
  // quality strings consecutive positions mostly fail the same checks (every field is ASCII)
#if SBH_FULL_RUN
  uint32_t run_f = 0, run_n = 0;
  auto run_flush = [&]() {
    if (run_n) {
      uint32_t f = run_f;
      uint32_t *row = myhist + __popc(f) * RW;
      while (f) {
        atomicAdd(&row[__builtin_ctz(f)], run_n);
        f &= f - 1;
      }
    }
  };
#endif
  auto account_fail = [&](uint64_t p, uint32_t r) {
    if (o.words) o.words[p - begin] = r;
    const uint32_t nnz = __popc(r);  // (a fast tile's failure word has no high bits)
#ifdef SBH_FULL_NOHIST
    if (nnz != 77) return;
#endif
#if SBH_FULL_RUN
    if (r == run_f) {
      ++run_n;
    } else {
      run_flush();
      run_f = r;
      run_n = 1;
    }
#else
    uint32_t f = r;
    uint32_t *row = myhist + nnz * RW;
    while (f) {
      atomicAdd(&row[__builtin_ctz(f)], 1u);
      f &= f - 1;
    }
#endif
    if (nnz <= 2) {
      const uint32_t slot = atomicAdd(&ncl, 1u);
      if (slot < FCCAP) {
        cpos[slot] = p;
        cword[slot] = r;
      } else {
        const unsigned long long gs = atomicAdd(o.close_n, 1ull);
        if (gs < o.close_cap) { o.close_pos[gs] = p; o.close_word[gs] = r; }
      }
    }
  };
  auto where = [&](uint64_t p, uint64_t *total, bool *open) {
    const uint32_t kseg = p < e0 ? seg0 : seg_index(sg, p, seg0);
    *total = p < e0 ? e0 : sg.end[kseg];
    *open = sg.open_last && kseg == sg.n - 1;
  };
  // a tile inside [begin, end) whose every position is FULL_FAST_REACH before its segment's
  // end meets no end-of-stream rule: its positions take full_first_win
  const bool fast = SBH_FULL_FAST && rtc > 0 && s0 >= begin && s0 + FTILE <= end &&
                    s0 + FTILE + FULL_FAST_REACH <= e0;
  if (fast) {
    // queue overflows (more record starts in the tile than slowq holds) are kept as bits and
    // decided after the sweep, so the exact path is not inlined into every unrolled position
    uint32_t ovf = 0;
#if SBH_FULL_HOT
    // The wave's hot failure word: inside quality strings and sequences most of a wave's 64
    // positions fail with one and the same word, and their per-flag LDS adds all land on the
    // same counters (a same-address atomic serialises: the bulk of k_full's bank conflicts).
    // Lanes whose word equals the hot word only count (one ballot popcount per wave); the count
    // goes into the word's Counts row when the hot word changes (to a word more lanes share) and
    // after the sweep.  Words with <= 2 flags (close calls, listed per position) are never hot.
    uint32_t hotw = 0, hotn = 0;  // wave-uniform; 0 is no failure word
    const uint32_t lane = threadIdx.x & (WAVE - 1);
    auto hot_flush = [&]() {
      if (hotn && lane == 0) {
        uint32_t f = hotw;
        uint32_t *row = myhist + __popc(f) * RW;
        while (f) {
          atomicAdd(&row[__builtin_ctz(f)], hotn);
          f &= f - 1;
        }
      }
    };
#endif
    for (uint32_t step = 0; step < FTILE / (FPL * T); ++step) {
      const uint32_t j = threadIdx.x + step * T;
      const uint4 v0 = ldsv[j], v1 = ldsv[j + 1], v2 = ldsv[j + 2];
      const uint32_t D[12] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w, v2.x, v2.y, v2.z, v2.w};
#pragma unroll
      for (uint32_t b = 0; b < 4; ++b) {  // dword b of the lane's 16 bytes (register-indexed: unrolled)
#pragma unroll 1
        for (uint32_t sh = 0; sh < 4; ++sh) {  // byte in the dword (a shift: rolled)
          const uint32_t q = 16 * j + 4 * b + sh;
          Fixed x;
          x.rem = (int32_t)__builtin_amdgcn_alignbyte(D[b + 1], D[b], sh);
          x.idx = (int32_t)__builtin_amdgcn_alignbyte(D[b + 2], D[b + 1], sh);
          x.pos = (int32_t)__builtin_amdgcn_alignbyte(D[b + 3], D[b + 2], sh);
          x.bmn = __builtin_amdgcn_alignbyte(D[b + 4], D[b + 3], sh);
          x.fnc = __builtin_amdgcn_alignbyte(D[b + 5], D[b + 4], sh);
          x.seq_len = (int32_t)__builtin_amdgcn_alignbyte(D[b + 6], D[b + 5], sh);
          x.nidx = (int32_t)__builtin_amdgcn_alignbyte(D[b + 7], D[b + 6], sh);
          x.npos = (int32_t)__builtin_amdgcn_alignbyte(D[b + 8], D[b + 7], sh);
          const uint32_t r = full_first_win(s, bname, bop, q, x, c, oi);
          const bool queued = r == FULL_SLOW || r == FULL_PASS;
#if SBH_FULL_HOT
          uint64_t hm = __ballot(!queued && r == hotw);
          const uint64_t om = __ballot(!queued && r != hotw);
          if (__builtin_popcountll(om) > __builtin_popcountll(hm)) {  // uniform: try another hot word
            const uint32_t cw = __builtin_amdgcn_readlane(r, (uint32_t)__builtin_ctzll(om));
            const uint64_t cm = __ballot(!queued && r == cw);
            if (__popc(cw) > 2 && __builtin_popcountll(cm) > __builtin_popcountll(hm)) {
              hot_flush();
              hotw = cw;
              hotn = 0;
              hm = cm;
            }
          }
          hotn += (uint32_t)__builtin_popcountll(hm);
#endif
          if (queued) {  // record starts, long CIGARs: the balanced pass below
            const uint32_t qi = atomicAdd(&nslow, 1u);
            if (qi < SLOWCAP) slowq[qi] = q;
            else ovf |= 1u << (16 * step + 4 * b + sh);
            continue;
          }
#if SBH_FULL_HOT
          if ((hm >> lane) & 1ull) {
            if (o.words) o.words[s0 + q - begin] = r;
            continue;
          }
#endif
#if SBH_FULL_ACCF
          account_fail(s0 + q, r);
#else
          account(s0 + q, r);
#endif
        }
      }
    }
#if SBH_FULL_RUN
    run_flush();
#endif
#if SBH_FULL_HOT
    hot_flush();
#endif
    static_assert(FTILE / (FPL * T) * FPL <= 32, "overflow bits fit a word");
    while (ovf) {
      const uint32_t i = __builtin_ctz(ovf);
      ovf &= ovf - 1;
      const uint32_t q = 16 * (threadIdx.x + (i / 16) * T) + (i & 15);
      const uint64_t p = s0 + q;
      uint64_t total;
      bool open;
      where(p, &total, &open);
      const uint32_t rc = chain_full(s, bname, bop, p, total, open, c, rtc, oi);
      account(p, rc == FULL_SLOW ? full_at(s, p, total, open, c, rtc, oi) : rc);
    }
  }
  for (uint32_t step = 0; step < (fast ? 0u : FTILE / (FPL * T)); ++step) {
    const uint32_t j = threadIdx.x + step * T;  // this lane's 16 positions: window bytes 16j..16j+15
    const uint4 v0 = ldsv[j], v1 = ldsv[j + 1], v2 = ldsv[j + 2];
    const uint32_t D[12] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w, v2.x, v2.y, v2.z, v2.w};
#pragma unroll
    for (uint32_t k = 0; k < FPL; ++k) {
      const uint32_t q = 16 * j + k;
      const uint64_t p = s0 + q;
      if (p < begin || p >= end) continue;
      const uint32_t b = k >> 2, sh = k & 3;
      Fixed x;
      x.rem = (int32_t)__builtin_amdgcn_alignbyte(D[b + 1], D[b], sh);
      x.idx = (int32_t)__builtin_amdgcn_alignbyte(D[b + 2], D[b + 1], sh);
      x.pos = (int32_t)__builtin_amdgcn_alignbyte(D[b + 3], D[b + 2], sh);
      x.bmn = __builtin_amdgcn_alignbyte(D[b + 4], D[b + 3], sh);
      x.fnc = __builtin_amdgcn_alignbyte(D[b + 5], D[b + 4], sh);
      x.seq_len = (int32_t)__builtin_amdgcn_alignbyte(D[b + 6], D[b + 5], sh);
      x.nidx = (int32_t)__builtin_amdgcn_alignbyte(D[b + 7], D[b + 6], sh);
      x.npos = (int32_t)__builtin_amdgcn_alignbyte(D[b + 8], D[b + 7], sh);
      uint64_t total;
      bool open;
      where(p, &total, &open);
      const uint32_t r = full_first(s, bname, bop, p, q, x, total, open, c, rtc, oi);
      if (r == FULL_SLOW || r == FULL_PASS) {  // record starts, long CIGARs: the balanced pass below
        const uint32_t qi = atomicAdd(&nslow, 1u);
        if (qi < SLOWCAP) {
          slowq[qi] = q;
          continue;
        }
        const uint32_t rc = chain_full(s, bname, bop, p, total, open, c, rtc, oi);
        account(p, rc == FULL_SLOW ? full_at(s, p, total, open, c, rtc, oi) : rc);
        continue;
      }
      account(p, r);
    }
  }
  __syncthreads();
#ifdef SBH_FULL_NOCHAIN  // A/B probe (timing only, results wrong): queued record starts not walked
  const uint32_t ns = 0;
#else
  const uint32_t ns = nslow < SLOWCAP ? nslow : SLOWCAP;
#endif
  for (uint32_t i = threadIdx.x; i < ns; i += T) {
    const uint64_t p = s0 + slowq[i];
    uint64_t total;
    bool open;
    where(p, &total, &open);
    const uint32_t rc = chain_full(s, bname, bop, p, total, open, c, rtc, oi);
    account(p, rc == FULL_SLOW ? full_at(s, p, total, open, c, rtc, oi) : rc);
  }
  if (mysucc) atomicAdd(&nsucc, mysucc);
  __syncthreads();
  const uint32_t nc = ncl < FCCAP ? ncl : FCCAP;
  if (threadIdx.x == 0) cbase = nc ? atomicAdd(o.close_n, (unsigned long long)nc) : 0;
  for (uint32_t i = threadIdx.x; i < 21 * 19; i += T) {
    uint32_t t = 0;
#pragma unroll
    for (uint32_t r = 0; r < NREP; ++r)
#if SBH_FULL_PACKED
      t += (hist[r * REP + (i / 19) * RW + (i % 19) / 2] >> (16 * ((i % 19) & 1))) & 0xffffu;
#else
      t += hist[r * REP + i];
#endif
    if (t) atomicAdd(&o.counts[i], (unsigned long long)t);
  }
  if (threadIdx.x == 0 && nsucc) atomicAdd(o.n_success, (unsigned long long)nsucc);
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nc; i += T) {
    const unsigned long long g = cbase + i;
    if (g < o.close_cap) { o.close_pos[g] = cpos[i]; o.close_word[g] = cword[i]; }
  }
}

// ---------------------------------------------------------------- bitmap utilities
// First set bit at or after `from` and before `to` (positions; bit i <-> begin + i).
// A persistent grid walks FS_SPAN-word chunks in order (chunk i by workgroup i mod grid)
// and stops as soon as a hit before its next chunk is known: records start every few
// hundred bytes, so the search normally ends within the first round of chunks.
constexpr uint32_t FS_SPAN = 1024;  // words per chunk (4 per thread)
__global__ __launch_bounds__(256) void k_first_set(const uint32_t *bits, uint64_t begin, uint64_t from,
                                                   uint64_t to, unsigned long long *best) {
  const uint64_t w0 = (from - begin) / 32, w_end = (to - begin + 31) / 32;
  __shared__ unsigned long long wbest[256 / WAVE];
  __shared__ uint32_t stop;
  for (uint64_t c = blockIdx.x;; c += gridDim.x) {
    const uint64_t cw = w0 + c * FS_SPAN;
    if (cw >= w_end) return;  // (uniform)
    if (threadIdx.x == 0) stop = __hip_atomic_load(best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < begin + 32 * cw;
    __syncthreads();
    if (stop) return;  // (uniform: read before the loop's closing barrier)
    const uint64_t w = cw + 4 * threadIdx.x;
    uint32_t v[4];
    if (w + 4 <= w_end && (w & 3) == 0) {
      const uint4 q = *reinterpret_cast<const uint4 *>(bits + w);
      v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    } else {
      for (uint32_t k = 0; k < 4; ++k) v[k] = w + k < w_end ? bits[w + k] : 0u;
    }
    unsigned long long hit = ~0ull;
    for (uint32_t k = 0; k < 4; ++k) {
      uint32_t x = v[k];
      const uint64_t p0 = begin + 32 * (w + k);
      if (p0 < from) x &= ~0u << (uint32_t)(from - p0);
      if (p0 + 32 > to) x &= (to - p0) >= 32 ? ~0u : ((1u << (uint32_t)(to - p0)) - 1u);
      if (x) {
        hit = p0 + __builtin_ctz(x);
        break;
      }
    }
    // positions grow with the lane and the wave, so the workgroup's lowest hitting lane holds
    // its minimum: one atomic per workgroup, and none when an earlier chunk already hit (the
    // atomics of all workgroups on one address serialise: one per wave cost ~60 us per call)
    const uint64_t m = __ballot(hit != ~0ull);
    if ((threadIdx.x & (WAVE - 1)) == 0) wbest[threadIdx.x / WAVE] = ~0ull;
    if (m && (threadIdx.x & (WAVE - 1)) == (uint32_t)__builtin_ctzll(m)) wbest[threadIdx.x / WAVE] = hit;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long h = ~0ull;
      for (uint32_t k = 0; k < 256 / WAVE && h == ~0ull; ++k) h = wbest[k];
      if (h != ~0ull && h < __hip_atomic_load(best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(best, h);
    }
    __syncthreads();
  }
}

// Chain verification over eager-true positions s in [from, E): the record chain
// (PosStream: next = s + 4 + block_size) must step exactly from each true position
// to the next true one (or leave [from, E) / reach the stream end).  Any other
// step is an anomaly (a false positive inside the chain, or a chain record the
// eager checker rejects); those ranges fall back to an exact sequential walk.
// Wave-cooperative, with the popcount of [from, E) folded in (one pass over the bitmap,
// one host round trip).  A wave covers 64 consecutive 4-word groups: the successor of a lane's last set bit is the first set bit
// of the next non-empty lane (a readlane), and only the wave's last one looks past the
// wave -- the whole wave scanning 64 words per step -- so each set bit costs one bitmap
// load and one U load, and sparse bitmaps (long records) no longer scan word by word.
__global__ __launch_bounds__(256) void k_verify_chain_w(const uint8_t *U, const uint32_t *bits, uint64_t begin,
                                                         uint64_t bits_end, uint64_t from, uint64_t E, uint64_t total,
                                                         unsigned long long *n_anom, unsigned long long *first_anom,
                                                         unsigned long long *exit_pos, unsigned long long *n_set,
                                                         const TileSum *tsum, const unsigned long long *from_dev,
                                                         uint32_t *chunk_cnt) {
  // chunk_cnt (optional): the set bits of [from, E) per wave chunk of VC_CHUNK words, chunk k =
  // words [VC_CHUNK k, VC_CHUNK (k + 1)) from `begin` (the chunks are aligned to that grid): the
  // split counts (sbh_split_starts) then read the bitmap only at their ends
  // from_dev: the chain's first record as another kernel left it on the device (k_first_set's
  // answer; ~0: none, nothing to prove)
  if (from_dev) {
    from = *from_dev;
    if (from >= E) return;
  }
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  constexpr uint32_t TWORDS = EAGER_SUB / 32;  // bitmap words per summarised quarter tile (from `begin`)
  const uint64_t W0 = (from - begin) / 32 / VC_CHUNK * VC_CHUNK;  // (chunk-aligned; earlier words are masked)
  const uint64_t w_end = (E - begin + 31) / 32;
  const uint64_t w_lim = (bits_end - begin + 31) / 32;
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x / WAVE);
  uint32_t tot = 0;  // set bits this lane saw (the popcount; one atomic per workgroup)
  // wave chunks of 64 x 4 words, grid-stride
  for (uint64_t wc = (uint64_t)blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE;; wc += nwaves) {
    const uint64_t wave_w0 = W0 + 4 * WAVE * wc;
    if (wave_w0 >= w_end) break;
    const uint64_t w = wave_w0 + 4 * lane;
    uint32_t v[4] = {0, 0, 0, 0};
    if (w < w_end) {
      if (w + 4 <= w_lim) {
        const uint4 q = *reinterpret_cast<const uint4 *>(bits + w);
        v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
      } else {
        for (uint32_t k = 0; k < 4; ++k) v[k] = w + k < w_lim ? bits[w + k] : 0u;
      }
      for (uint32_t k = 0; k < 4; ++k) {  // positions outside [from, E)
        const uint64_t p0 = begin + 32 * (w + k);
        if (p0 + 32 <= from || p0 >= E) v[k] = 0;
        else {
          if (p0 < from) v[k] &= ~0u << (uint32_t)(from - p0);
          if (p0 + 32 > E) v[k] &= (E - p0) >= 32 ? ~0u : ((1u << (uint32_t)(E - p0)) - 1u);
        }
      }
    }
    const uint32_t cnt = __popc(v[0]) + __popc(v[1]) + __popc(v[2]) + __popc(v[3]);
    tot += cnt;
    if (chunk_cnt) {  // (a wave chunk is VC_CHUNK words: its sum by one lane)
      uint32_t cs = cnt;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) cs += __shfl_xor(cs, off, WAVE);
      if (lane == 0) chunk_cnt[wave_w0 / VC_CHUNK] = cs;
    }
    // a tile wholly inside [from, E) with a summary: its own pairs were checked by k_eager (their
    // anomalies added once, by the lane of its first word); only its last true position's step
    // is needed, from the summary, not from U
    bool cov = false;
    uint64_t tstep = TS_NONE, thi = 0;
    if (SBH_TSUM_CODE && tsum && w < w_end) {
      const uint64_t tile = w / TWORDS, tlo = begin + tile * EAGER_SUB;
      thi = tlo + EAGER_SUB;
      if (tlo >= from && thi <= E) {
        const TileSum ts = tsum[tile];
        cov = ts.step_last != TS_DIRTY;
        tstep = ts.step_last;
        if (cov && w % TWORDS == 0 && ts.n_anom) {
          atomicAdd(n_anom, (unsigned long long)ts.n_anom);
          atomicMin(first_anom, (unsigned long long)(tlo + ts.first_anom));
        }
      }
    }
    // the lane's first set position (successor of the previous non-empty lane's last bit)
    uint64_t f = ~0ull;
    for (int k = 3; k >= 0; --k)
      if (v[k]) f = begin + 32 * (w + (uint32_t)k) + __builtin_ctz(v[k]);
    const uint64_t has = __ballot(cnt != 0);
    if (!has) continue;
    // next non-empty lane after this one, in this wave
    const uint64_t after = lane == WAVE - 1 ? 0ull : has & (~0ull << (lane + 1));
    const uint32_t nl = after ? (uint32_t)__builtin_ctzll(after) : 0u;
    const uint32_t f_lo = __shfl((uint32_t)f, nl, WAVE), f_hi = __shfl((uint32_t)(f >> 32), nl, WAVE);
    uint64_t lane_next = after ? ((uint64_t)f_hi << 32 | f_lo) : ~0ull;
    // past the wave: the first set bit at or after the wave's end (uniform scan; bounded by E)
    const uint32_t top = 63 - (uint32_t)__builtin_clzll(has);
    uint64_t past = ~0ull;
    for (uint64_t ww = wave_w0 + 4 * WAVE; ww < w_end && ww < w_lim; ww += WAVE) {
      const uint64_t wl = ww + lane;
      uint32_t x = wl < w_end && wl < w_lim ? bits[wl] : 0u;
      const uint64_t p0 = begin + 32 * wl;
      if (x && p0 + 32 > E) x &= (E - p0) >= 32 ? ~0u : ((1u << (uint32_t)(E - p0)) - 1u);
      const uint64_t b = __ballot(x != 0);
      if (b) {
        const uint32_t l = (uint32_t)__builtin_ctzll(b);
        const uint32_t xl = __shfl(x, l, WAVE);
        past = begin + 32 * (ww + l) + __builtin_ctz(xl);
        break;
      }
    }
    if (past >= E) past = ~0ull;
    if (lane == top) lane_next = past;
    // walk this lane's set bits in order
    uint32_t k = 0;
    while (k < 4 && !v[k]) ++k;
    while (k < 4) {
      const uint32_t b = __builtin_ctz(v[k]);
      v[k] &= v[k] - 1;
      const uint64_t s = begin + 32 * (w + k) + b;
      uint32_t kn = k;
      while (kn < 4 && !v[kn]) ++kn;
      const uint64_t nxt_set = kn < 4 ? begin + 32 * (w + kn) + __builtin_ctz(v[kn]) : lane_next;
      uint64_t step;
      if (cov && nxt_set != ~0ull && nxt_set < thi) {  // a pair inside a summarised tile
        k = kn;
        continue;
      }
      if (cov) {
        step = tstep;  // the tile's last true position
      } else if (s + 4 > total) {
        step = ~0ull;  // getInt at EOF: the chain ends here
      } else {
        const uint32_t *g = reinterpret_cast<const uint32_t *>(U + (s & ~3ull));
        const int32_t rem = (int32_t)__builtin_amdgcn_alignbyte(g[1], g[0], (uint32_t)s & 3);
        step = s + 4 + (int64_t)rem;
      }
      bool ok;
      if (nxt_set != ~0ull) ok = step == nxt_set;
      else ok = step >= E || step + 4 > total;  // leaves the counted range or hits EOF
      if (!ok) {
        atomicAdd(n_anom, 1ull);
        atomicMin(first_anom, (unsigned long long)s);
      } else if (nxt_set == ~0ull) {
        atomicMin(exit_pos, (unsigned long long)(step > total ? total : step));
      }
      k = kn;
    }
  }
  __shared__ uint32_t part[4];
  for (int off = 32; off > 0; off >>= 1) tot += __shfl_down(tot, off);
  if (lane == 0) part[threadIdx.x / WAVE] = tot;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long t = (unsigned long long)part[0] + part[1] + part[2] + part[3];
    if (t) atomicAdd(n_set, t);
  }
}

// ---- chain marking by pointer doubling (the parallel replacement of k_chain_walk when
// the eager bitmap holds false positives or misses chain records) ----
// Nodes are the n set bits of [from, E) in order (pos[], group prefix counts wpre from word
// (from - begin) / 32).  J[i] = index of the node the chain steps to from node i
// (next = s + 4 + block_size), or CM_TERM when the step leaves [from, E) / reaches the
// stream end (a valid end of the counted range), or CM_BROKEN when it lands on a
// position whose bit is clear or does not move forward (the exact walk must decide).
// Since every step moves forward, the nodes reachable from node 0 are exactly the chain.
__global__ void k_cm_succ(const uint8_t *U, const uint32_t *bits, uint64_t begin, uint64_t from, uint64_t E,
                          uint64_t total, const uint64_t *pos, const uint64_t *wpre, uint64_t n, uint32_t *J,
                          uint32_t *J0, uint64_t *mark, uint32_t *indeg) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t s = pos[i];
  const uint32_t term = (uint32_t)n, broken = (uint32_t)n + 1;
  uint32_t j;
  if (s + 4 > total) {
    j = term;
  } else {
    const int32_t rem = (int32_t)((uint32_t)U[s] | ((uint32_t)U[s + 1] << 8) | ((uint32_t)U[s + 2] << 16) |
                                  ((uint32_t)U[s + 3] << 24));
    const int64_t nx = (int64_t)s + 4 + rem;
    if (nx <= (int64_t)s) {
      j = broken;
    } else if ((uint64_t)nx >= E || (uint64_t)nx + 4 > total) {
      j = term;
    } else {
      const uint64_t q = (uint64_t)nx - begin, w = q >> 5;
      const uint32_t v = bits[w], b = (uint32_t)(q & 31);
      if (!((v >> b) & 1u)) {
        j = broken;
      } else {
        const uint64_t w0 = (from - begin) >> 5;
        const uint32_t lo = ~0u << (uint32_t)((from - begin) & 31);  // bits before `from` are not nodes
        uint32_t below = v & ((1u << b) - 1u);
        if (w == w0) below &= lo;
        // the group's prefix plus the set bits of its words before w
        const uint64_t r = w - w0, g0 = r - r % WPRE_GROUP;
        uint64_t c = wpre[r / WPRE_GROUP];
        for (uint64_t k = g0; k < r; ++k) c += __popc(k == 0 ? bits[w0] & lo : bits[w0 + k]);
        j = (uint32_t)(c + __popc(below));
      }
    }
  }
  J[i] = j;
  J0[i] = j;
  if (indeg) {  // (the peeling path: every node starts marked, predecessors counted)
    mark[i] = 1;
    if (j < n) atomicAdd(&indeg[j], 1u);
  } else {
    mark[i] = i == 0;
  }
}

// Chain marking by peeling instead of doubling (launch_chain_mark).  Edges only go forward, so a
// node other than node 0 is off the chain exactly when every predecessor is: the nodes nobody
// steps to are the roots of the off-chain set (k_cm_roots), and each root walks forward,
// taking one predecessor off each successor and continuing while it took the last one
// (k_cm_peel).  False positives are roots whose walks end at once (their successor is a chain
// record with a chained predecessor), so this is ~3 passes where doubling took log2(n) rounds
// over every node.  A walk longer than CM_PEEL_MAX (the chain itself breaking: everything after
// the break is off) gives up and marks the result unusable, so the host takes the exact walk
// as it does for a broken chain.
constexpr uint32_t CM_PEEL_MAX = 4096;
__global__ void k_cm_roots(const uint32_t *indeg, uint64_t *mark, uint64_t n, uint32_t *code) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) *code = (uint32_t)n;
  if (i == 0 || i >= n) return;
  if (indeg[i] == 0) mark[i] = 2;
}
__global__ void k_cm_peel(const uint32_t *J0, uint32_t *indeg, uint64_t *mark, uint64_t n, uint32_t *code) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || mark[i] != 2) return;
  mark[i] = 0;
  uint32_t j = J0[i];
  for (uint32_t steps = 0; j < n; ++steps) {
    if (steps == CM_PEEL_MAX) {
      atomicMax(code, (uint32_t)n + 2);  // (not n: the host walks exactly)
      return;
    }
    if (atomicSub(&indeg[j], 1u) != 1u) return;  // j keeps a predecessor
    mark[j] = 0;
    j = J0[j];
  }
}

// One doubling round: nodes at distance < 2^k are marked; mark their 2^k-successors
// (Jin) and square the jump (Jout = Jin o Jin; terminal codes stay).  Marks written by
// other threads during the round are reachable nodes too, so the race only marks early.
__global__ void k_cm_round(const uint32_t *Jin, uint32_t *Jout, uint64_t *mark, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t j = Jin[i];
  if (j < n) {
    if (mark[i]) mark[j] = 1;
    Jout[i] = Jin[j];
  } else {
    Jout[i] = j;
  }
}

// The chain's last counted node (marked, J0 terminal): its successor is the exit.  (code: the
// peeling path's verdict -- a chained node whose step leaves the set bits makes it unusable.)
__global__ void k_cm_exit(const uint8_t *U, const uint64_t *pos, const uint32_t *J0, const uint64_t *mark,
                          uint64_t n, uint64_t total, unsigned long long *exit_pos, uint32_t *code) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !mark[i] || J0[i] < n) return;
  if (code && J0[i] != (uint32_t)n) atomicMax(code, J0[i]);  // (broken: n + 1)
  const uint64_t s = pos[i];
  uint64_t x = total;
  if (s + 4 <= total) {
    const int32_t rem = (int32_t)((uint32_t)U[s] | ((uint32_t)U[s + 1] << 8) | ((uint32_t)U[s + 2] << 16) |
                                  ((uint32_t)U[s + 3] << 24));
    const int64_t nx = (int64_t)s + 4 + rem;
    x = nx > (int64_t)total ? total : (uint64_t)nx;
  }
  atomicMin(exit_pos, (unsigned long long)x);
}

// Exact sequential chain walk (fallback): counts records r in [first, E) following
// next = r + 4 + block_size, stopping at the stream end.
__global__ void k_chain_walk(const uint8_t *U, uint64_t first, uint64_t E, uint64_t total,
                             unsigned long long *count, unsigned long long *exit_pos) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint64_t r = first, n = 0;
  while (r < E && r + 4 <= total) {
    ++n;
    const int32_t rem = (int32_t)((uint32_t)U[r] | ((uint32_t)U[r + 1] << 8) | ((uint32_t)U[r + 2] << 16) |
                                  ((uint32_t)U[r + 3] << 24));
    const int64_t nx = (int64_t)r + 4 + rem;
    if (nx <= (int64_t)r) break;  // malformed: htsjdk would fail; stop the walk
    r = (uint64_t)nx;
  }
  *count = n;
  *exit_pos = r > total ? total : r;  // first record at/after E (or where the walk stopped)
}

// eager.Checker.apply at p by one wave (k_eager_xq): the control flow of eager_at is
// wave-uniform; the read-name bytes and the CIGAR ops of each record are tested by all
// 64 lanes at once (ballots), preserving eager_at's outcome order: the bound checks
// (unknown / false at the stream end) against the first invalid byte or op before them.
__device__ uint32_t eager_at_wave(const uint8_t *__restrict__ U, uint64_t p, uint64_t total, bool open, const Ctg c,
                                  int32_t rtc, uint32_t lane) {
  auto word = [&](uint64_t q) -> uint32_t {
    const uint32_t *g = reinterpret_cast<const uint32_t *>(U + (q & ~3ull));
    return __builtin_amdgcn_alignbyte(g[1], g[0], (uint32_t)q & 3);
  };
  uint64_t cur = p, start = p;
  for (int32_t n = 0;; ++n) {
    if (n == rtc) return 1;
    if (cur + 36 > total) {
      if (open) return 2;
      return (total == start && n > 0) ? 1 : 0;
    }
    const int32_t rem = (int32_t)word(cur);
    const uint64_t nominal = start + 4 + (int64_t)rem;
    if (ref_pos_error((int32_t)word(cur + 4), (int32_t)word(cur + 8), c)) return 0;
    const int32_t rnl = (int32_t)(word(cur + 12) & 0xff);
    if (rnl < 2) return 0;
    const uint32_t fnc = word(cur + 16);
    const uint32_t flags = fnc >> 16;
    const int32_t nc = (int32_t)(fnc & 0xffff);
    const int32_t seq_len = (int32_t)word(cur + 20);
    if ((flags & 4) == 0 && (seq_len == 0 || nc == 0)) return 0;
    if (rem < implied_min_remaining(rnl, nc, seq_len)) return 0;
    if (ref_pos_error((int32_t)word(cur + 24), (int32_t)word(cur + 28), c)) return 0;
    cur += 36;
    if (cur + (uint64_t)rnl > total) return open ? 2 : 0;
    // one round trip for the name bytes and the first 512 CIGAR op bytes: every load is
    // issued before any test
    const uint64_t avail = total > cur + rnl ? (total - cur - rnl) / 4 : 0;
    const uint64_t lim = (uint64_t)nc < avail ? (uint64_t)nc : avail;
    const uint64_t qc = cur + (uint64_t)rnl;
    const uint8_t term = U[cur + rnl - 1];
    uint8_t nb[4], ob[8];
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
      const uint32_t k = lane + WAVE * j;
      nb[j] = k < (uint32_t)rnl ? U[cur + k] : (uint8_t)'A';
    }
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
      const uint64_t k = lane + WAVE * j;
      ob[j] = k < lim ? U[qc + 4 * k] : (uint8_t)0;
    }
    if (term != 0) return 0;
    bool bad = false;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) bad |= lane + WAVE * j + 1 < (uint32_t)rnl && !name_char_ok(nb[j]);
    if (__ballot(bad)) return 0;
    cur = qc;
    bool badop = false;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) badop |= (ob[j] & 0xf) > 8;
    if (__ballot(badop)) return 0;
    for (uint64_t b = 8 * WAVE; b < lim; b += WAVE) {  // CIGARs longer than 512 ops
      const uint64_t k = b + lane;
      const bool bo = k < lim && (U[cur + 4 * k] & 0xf) > 8;
      if (__ballot(bo)) return 0;
    }
    if ((uint64_t)nc > avail) return open ? 2 : 0;
    cur += 4ull * (uint64_t)nc;
    if ((int64_t)(nominal - cur) > 0) {
      if (nominal > total) {
        if (open) return 2;
        cur = total;
      } else {
        cur = nominal;
      }
    }
    start = nominal;
  }
}

// The queued long-record candidates, pass 1 (a lane each): the read name and the first
// XQ_MIN_OPS CIGAR ops must hold (random bytes fail there: an op byte passes with
// probability 9/16); survivors go to the second queue.
__global__ __launch_bounds__(256) void k_eager_xq_pre(const uint8_t *__restrict__ U, Segs sg, const uint64_t *pos,
                                                      const unsigned long long *n, uint64_t cap, uint64_t *pos2,
                                                      unsigned long long *n2) {
  const uint64_t cnt = *n < cap ? *n : cap;
  const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x < cnt; x += nt) {
    const uint64_t p = pos[x];
    const uint64_t total = sg.end[seg_first(sg, p)];
    const uint64_t q = p + 36;
    const uint32_t rnl = U[p + 12];
    bool alive = true;
    if (q + rnl + 4ull * XQ_MIN_OPS <= total) {  // else: leave the EOF rules to the exact walk
      const Src s{U, nullptr, 0, 0};
      alive = U[q + rnl - 1] == 0 && name_bytes_ok(s, q, rnl - 1);
      for (uint32_t k = 0; alive && k < (uint32_t)XQ_MIN_OPS; ++k) alive = (U[q + rnl + 4 * k] & 0xf) <= 8;
    }
    if (alive) pos2[atomicAdd(n2, 1ull)] = p;
  }
}

// Pass 2: one wave per surviving candidate (grid-stride over the device count).
__global__ __launch_bounds__(256) void k_eager_xq(const uint8_t *__restrict__ U, uint64_t begin, Segs sg, Ctg c,
                                                  int32_t rtc, const uint64_t *pos, const unsigned long long *n,
                                                  uint64_t cap, EagerOut o) {
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  const uint64_t cnt = *n < cap ? *n : cap;
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x / WAVE);
  for (uint64_t x = (uint64_t)blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE; x < cnt; x += nw) {
    const uint64_t p = pos[x];
    const uint32_t k = seg_first(sg, p);
    const uint64_t total = sg.end[k];
    const bool open = sg.open_last && k == sg.n - 1;
    const uint32_t r = eager_at_wave(U, p, total, open, c, rtc, lane);
    if (lane == 0) {
      if (r == 1) {
        atomicOr(&o.bits[(p - begin) >> 5], 1u << ((p - begin) & 31));
        atomicAdd(o.n_true, 1ull);
      } else if (r == 2) {
        atomicAdd(o.n_unknown, 1ull);
        atomicMin(o.min_unknown, (unsigned long long)p);
      }
    }
  }
}

// Positions the pipelined eager pass deferred (their exact check reached flat bytes that
// were not inflated yet), re-checked once everything is: bit set atomically over the
// tile's word, counters as in k_eager.
// n_true += k_eager's per-wave slots, which are left zero for the next launch (the shard
// zeroes them once when it allocates the counter buffer).
__global__ void k_fold_true(unsigned long long *spread, unsigned long long *n_true) {
  const uint32_t t = threadIdx.x;
  unsigned long long v = t < TRUE_SLOTS ? spread[t * TRUE_STRIDE] : 0ull;
  if (t < TRUE_SLOTS) spread[t * TRUE_STRIDE] = 0ull;
#pragma unroll
  for (uint32_t d = WAVE / 2; d > 0; d >>= 1) v += __shfl_down(v, d, WAVE);
  if (t == 0 && v) atomicAdd(n_true, v);
}

__global__ void k_eager_defer(const uint8_t *__restrict__ U, uint64_t begin, Segs sg, Ctg c, int32_t rtc,
                              const uint64_t *pos, const unsigned long long *n, EagerOut o) {
  const uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= *n) return;
  const uint64_t p = pos[x];
  const uint32_t k = seg_first(sg, p);
  const uint64_t total = sg.end[k];
  const bool open = sg.open_last && k == sg.n - 1;
  Src s{U, nullptr, 0, 0};
  const uint32_t r = eager_at(s, p, total, open, c, rtc);
  if (r == 1) {
    atomicOr(&o.bits[(p - begin) >> 5], 1u << ((p - begin) & 31));
    atomicAdd(o.n_true, 1ull);
  } else if (r == 2) {
    atomicAdd(o.n_unknown, 1ull);
    atomicMin(o.min_unknown, (unsigned long long)p);
  }
}

// The full checker's bad-CIGAR-op index (OpIdx) over [base, base + 32 nw): a thread per
// 32-byte group (two 16-byte loads, SWAR byte classes), the residue summaries from ballots
// (a wave's 64 groups are two summary words per residue).
__global__ __launch_bounds__(256) void k_op_index(const uint8_t *__restrict__ U, uint64_t u_pad, uint64_t base,
                                                 uint64_t nw, uint32_t *__restrict__ ob, uint32_t *__restrict__ os,
                                                 uint64_t nsw) {
  const uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t v = 0;
  if (w < nw) {
    const uint64_t p = base + 32 * w;
    const uint4 *g = reinterpret_cast<const uint4 *>(U + p);
    const uint4 z = make_uint4(0, 0, 0, 0);
    const uint4 a = p + 16 <= u_pad ? g[0] : z, b = p + 32 <= u_pad ? g[1] : z;
    v = bad_op4(a.x) | bad_op4(a.y) << 4 | bad_op4(a.z) << 8 | bad_op4(a.w) << 12 | bad_op4(b.x) << 16 |
        bad_op4(b.y) << 20 | bad_op4(b.z) << 24 | bad_op4(b.w) << 28;
    ob[w] = v;
  }
  const uint64_t w0 = w & ~63ull;  // the wave's first group
#pragma unroll
  for (uint32_t r = 0; r < 4; ++r) {
    const uint64_t m = __ballot((v & (0x11111111u << r)) != 0);
    if ((threadIdx.x & 63) == 0 && w0 < nw) {
      os[r * nsw + w0 / 32] = (uint32_t)m;
      if (w0 / 32 + 1 < nsw) os[r * nsw + w0 / 32 + 1] = (uint32_t)(m >> 32);
    }
  }
}

}  // namespace

static inline uint32_t ngrid(uint64_t n, uint32_t t) { return (uint32_t)((n + t - 1) / t); }

// counters: a shard's counter buffer (CTR_WORDS u64, layout in sbh_internal.h) -- the
// true-count slots at CTR_TRUE_SPREAD must be zero on entry; k_fold_true leaves them zero.
hipError_t launch_eager(const uint8_t *U, uint64_t u_pad, uint64_t begin, uint64_t end, const uint64_t *seg_end,
                        uint32_t nseg, uint32_t open_last, const int32_t *ctg, int32_t nctg, int32_t rtc,
                        uint32_t *bits, unsigned long long *counters, hipStream_t st, uint64_t front,
                        uint64_t *defer_pos, uint64_t defer_cap, uint64_t *xq_pos, uint64_t xq_cap, TileSum *tsum,
                        const uint32_t *sieve) {
  if (end <= begin) return hipSuccess;
  Segs sg{seg_end, nseg, open_last};
  Ctg c{ctg, nctg};
  EagerOut o{bits,   counters,     counters + 1, counters + 2, front, defer_pos, counters + 3, defer_cap,
             xq_pos, counters + 4, xq_cap,       counters + TRUE_SPREAD_OFF, tsum, sieve};
  hipLaunchKernelGGL(k_eager, dim3(ngrid(end - begin, ETILE)), dim3(T), 0, st, U, u_pad, begin, end, sg, c,
                     rtc, o);
  hipLaunchKernelGGL(k_fold_true, dim3(1), dim3(WAVE), 0, st, counters + TRUE_SPREAD_OFF, counters);
  return hipGetLastError();
}

// Re-check of deferred positions (launched with a grid for `cap` entries; threads past
// the device-side count exit).  bits is the bitmap of the whole range from `begin`.
hipError_t launch_eager_defer(const uint8_t *U, uint64_t begin, const uint64_t *seg_end, uint32_t nseg,
                              uint32_t open_last, const int32_t *ctg, int32_t nctg, int32_t rtc, uint32_t *bits,
                              unsigned long long *counters, const uint64_t *defer_pos, uint64_t cap,
                              hipStream_t st) {
  if (cap == 0) return hipSuccess;
  Segs sg{seg_end, nseg, open_last};
  Ctg c{ctg, nctg};
  EagerOut o{bits, counters, counters + 1, counters + 2, ~0ull, nullptr, nullptr, 0, nullptr, nullptr, 0};
  hipLaunchKernelGGL(k_eager_defer, dim3(ngrid(cap, 256)), dim3(256), 0, st, U, begin, sg, c, rtc, defer_pos,
                     counters + 3, o);
  return hipGetLastError();
}

hipError_t launch_full(const uint8_t *U, uint64_t u_pad, uint64_t begin, uint64_t end, const uint64_t *seg_end,
                       uint32_t nseg, uint32_t open_last, const int32_t *ctg, int32_t nctg, int32_t rtc,
                       uint32_t *words, unsigned long long *counters /* [2+21*19+21*64+2] */,
                       uint64_t *close_pos, uint32_t *close_word, uint64_t close_cap, uint32_t *op_words,
                       uint64_t op_cap_words, hipStream_t st) {
  if (end <= begin) return hipSuccess;
  Segs sg{seg_end, nseg, open_last};
  Ctg c{ctg, nctg};
  // the op index over [begin rounded down to 1 KiB, the last byte a CIGAR of a position
  // before `end` can reach), clipped to the resident bytes and to op_cap_words
  OpIdx oi{nullptr, nullptr, 0, 0, 0};
#ifdef SBH_FULL_NOOPIX  // A/B: every CIGAR past the staged window takes the exact path
  op_words = nullptr;
#endif
  if (op_words) {
    const uint64_t base = begin & ~1023ull;
    uint64_t top = end + 36 + 255 + 4ull * 65535 + 4;
    const uint64_t u_total = u_pad;  // (bytes past the stream are padding: never bad ops)
    if (top > u_total) top = u_total;
    uint64_t nw = (top - base + 31) / 32;
    nw = (nw + 63) & ~63ull;
    const uint64_t nsw = nw / 32;
    if (nw + 4 * nsw <= op_cap_words) {
      uint32_t *ob = op_words, *os = op_words + nw;
      hipLaunchKernelGGL(k_op_index, dim3(ngrid(nw, 256)), dim3(256), 0, st, U, u_pad, base, nw, ob, os, nsw);
      oi = OpIdx{ob, os, base, base + 32 * nw, nsw};
    }
  }
  FullOut o;
  o.words = words;
  o.n_success = counters + 0;
  o.n_unknown = counters + 1;
  o.min_unknown = counters + 2;
  o.close_n = counters + 3;
  o.counts = counters + 4;
  o.rbe = counters + 4 + 21 * 19;
  o.close_pos = close_pos;
  o.close_word = close_word;
  o.close_cap = close_cap;
  hipLaunchKernelGGL(k_full, dim3(ngrid(end - (begin & ~15ull), FTILE)), dim3(T), 0, st, U, u_pad, begin, end, sg, c, rtc,
                     o, oi);
  return hipGetLastError();
}

hipError_t launch_first_set(const uint32_t *bits, uint64_t begin, uint64_t from, uint64_t to,
                            unsigned long long *best, hipStream_t st) {
  if (to <= from) return hipSuccess;
  const uint64_t nw = (to - begin + 31) / 32 - (from - begin) / 32;
  const uint32_t grid = (uint32_t)std::min<uint64_t>(ngrid(nw, FS_SPAN), 256);
  hipLaunchKernelGGL(k_first_set, dim3(grid), dim3(256), 0, st, bits, begin, from, to, best);
  return hipGetLastError();
}

hipError_t launch_verify_chain_count(const uint8_t *U, const uint32_t *bits, uint64_t begin, uint64_t bits_end,
                                     uint64_t from, uint64_t E, uint64_t total, unsigned long long *n_anom,
                                     unsigned long long *first_anom, unsigned long long *exit_pos,
                                     unsigned long long *n_set, const TileSum *tsum, hipStream_t st,
                                     const unsigned long long *from_dev, uint32_t *chunk_cnt) {
  if (E <= from) return hipSuccess;  // (with from_dev: from is a lower bound of *from_dev)
  const uint64_t nw = (E - begin + 31) / 32 - (from - begin) / 32 / VC_CHUNK * VC_CHUNK;
  const uint32_t grid = (uint32_t)std::min<uint64_t>(ngrid(nw, 1024), 2048);
  hipLaunchKernelGGL(k_verify_chain_w, dim3(grid), dim3(256), 0, st, U, bits, begin, bits_end, from, E, total,
                     n_anom, first_anom, exit_pos, n_set, tsum, from_dev, chunk_cnt);
  return hipGetLastError();
}

hipError_t launch_chain_walk(const uint8_t *U, uint64_t first, uint64_t E, uint64_t total,
                             unsigned long long *count, unsigned long long *exit_pos, hipStream_t st) {
  hipLaunchKernelGGL(k_chain_walk, dim3(1), dim3(64), 0, st, U, first, E, total, count, exit_pos);
  return hipGetLastError();
}

// pos, wpre: from launch_rec_positions_bits over [from, E); J, J2, J0: n + 1 u32; mark: n + 1 u64.
// *final_code = the chain's terminal code after doubling (n: ended validly, n + 1: broken).
hipError_t launch_chain_mark(const uint8_t *U, const uint32_t *bits, uint64_t begin, uint64_t from, uint64_t E,
                             uint64_t total, const uint64_t *pos, const uint64_t *wpre, uint64_t n, uint32_t *J,
                             uint32_t *J2, uint32_t *J0, uint64_t *mark, unsigned long long *exit_pos,
                             uint32_t *final_code, hipStream_t st) {
  if (!n) return hipSuccess;
  const uint32_t g = ngrid(n, 256);
  const char *dbl = std::getenv("SBH_CM_DOUBLING");  // 1: the pointer-doubling marking (A/B, tests)
  if (dbl && dbl[0] == '1') {
    hipLaunchKernelGGL(k_cm_succ, dim3(g), dim3(256), 0, st, U, bits, begin, from, E, total, pos, wpre, n, J, J0,
                       mark, nullptr);
    uint32_t *a = J, *b = J2;
    for (uint64_t span = 1; span < n; span <<= 1) {
      hipLaunchKernelGGL(k_cm_round, dim3(g), dim3(256), 0, st, a, b, mark, n);
      std::swap(a, b);
    }
    hipLaunchKernelGGL(k_cm_exit, dim3(g), dim3(256), 0, st, U, pos, J0, mark, n, total, exit_pos, nullptr);
    hipError_t e = hipMemcpyAsync(final_code, a, 4, hipMemcpyDeviceToHost, st);
    if (e != hipSuccess) return e;
    return hipGetLastError();
  }
  // peeling: J2 holds the predecessor counts, the word after exit_pos the verdict (n: usable)
  uint32_t *indeg = J2, *code = reinterpret_cast<uint32_t *>(exit_pos + 1);
  hipError_t e = hipMemsetAsync(indeg, 0, n * sizeof(uint32_t), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_cm_succ, dim3(g), dim3(256), 0, st, U, bits, begin, from, E, total, pos, wpre, n, J, J0, mark,
                     indeg);
  hipLaunchKernelGGL(k_cm_roots, dim3(g), dim3(256), 0, st, indeg, mark, n, code);
  hipLaunchKernelGGL(k_cm_peel, dim3(g), dim3(256), 0, st, J0, indeg, mark, n, code);
  hipLaunchKernelGGL(k_cm_exit, dim3(g), dim3(256), 0, st, U, pos, J0, mark, n, total, exit_pos, code);
  e = hipMemcpyAsync(final_code, code, 4, hipMemcpyDeviceToHost, st);
  if (e != hipSuccess) return e;
  return hipGetLastError();
}

// The wave-cooperative exact pass over the long-record queue (counters[4] = its device
// count, counters[5] = the survivors of the lane pre-test in xq_pos[cap, 2 cap)); fixed
// grids stride over the device counts, so no host round trip is needed.  bits: the bitmap
// from `begin`.  xq_pos holds 2 * cap entries.
hipError_t launch_eager_xq(const uint8_t *U, uint64_t begin, const uint64_t *seg_end, uint32_t nseg,
                           uint32_t open_last, const int32_t *ctg, int32_t nctg, int32_t rtc, uint32_t *bits,
                           unsigned long long *counters, uint64_t *xq_pos, uint64_t cap, hipStream_t st) {
  if (cap == 0) return hipSuccess;
  Segs sg{seg_end, nseg, open_last};
  Ctg c{ctg, nctg};
  EagerOut o{bits, counters, counters + 1, counters + 2, ~0ull, nullptr, nullptr, 0, nullptr, nullptr, 0};
  hipLaunchKernelGGL(k_eager_xq_pre, dim3(512), dim3(256), 0, st, U, sg, xq_pos, counters + 4, cap, xq_pos + cap,
                     counters + 5);
  hipLaunchKernelGGL(k_eager_xq, dim3(8192), dim3(256), 0, st, U, begin, sg, c, rtc, xq_pos + cap, counters + 5,
                     cap, o);
  return hipGetLastError();
}

}  // namespace sbh
