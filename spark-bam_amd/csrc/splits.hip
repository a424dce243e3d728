// splits.hip -- every split of a shard in one batch, and check-bam's truth comparison,
// on the device.
//
//  * k_split_prologue: one wave per Hadoop split runs the per-split prologue of
//    CanLoadBam.loadReadsAndPositions (load/.../CanLoadBam.scala:316-356):
//    FindBlockStart(start) (bgzf/.../block/FindBlockStart.scala:8-36) over the shard's
//    header-candidate list, the block's flat start, FindRecordStart
//    (check/.../spark/FindRecordStart.scala:30-63) as the first set bit of the eager
//    bitmap, and the flat bound of Pos(end, 0).  Anything off the common path (a search
//    that fails or leaves the resident bytes, an empty block, a record start outside the
//    bitmap) is flagged for the exact per-split host path (sbh_split), so the batch never
//    decides a case differently from it.
//  * k_split_popcount / k_split_cm_count: the record count of every split from the
//    chain proof count_records_impl left (the bitmap verified equal to the record chain,
//    or the chain marked by pointer doubling): a popcount of the split's flat range, or a
//    difference of the mark prefix.
//  * k_truth_scatter / k_truth_compare: CheckerApp's TP/FP/FN (cli/.../CheckerApp.scala:65-227)
//    -- the `.records` truth as a bitmap, compared word by word with the eager bitmap over
//    the selected flat ranges; mismatching positions are compacted (unordered) up to a cap.
#include <algorithm>

#include "sbh_internal.h"

namespace sbh {
namespace {

__device__ __forceinline__ bool header_at(const uint8_t *c, uint64_t p) {
  // gzip magic 31 139 8 4 and 'B' 'C' 2 (Header.scala:61-75; byte 15 unchecked)
  return c[p] == 31 && c[p + 1] == 139 && c[p + 2] == 8 && c[p + 3] == 4 && c[p + 12] == 66 &&
         c[p + 13] == 67 && c[p + 14] == 2;
}
__device__ __forceinline__ uint32_t u16_at(const uint8_t *c, uint64_t p) {
  return (uint32_t)c[p] | ((uint32_t)c[p + 1] << 8);
}

// MetadataStream.take(k).size from q (FindBlockStart's attempt): 0 ok, 1 HeaderParseException
// (the search moves on), 2 another exception (escapes), 3 needs bytes past the resident range.
// Same decision as k_find_block_start (bgzf_index.hip).
__device__ uint32_t fbs_outcome(const uint8_t *comp, uint64_t n, uint64_t q, int32_t k_check, int at_eof) {
  for (int32_t k = 0; k < k_check; ++k) {
    if (q + 18 > n) return at_eof ? 0u : 3u;
    if (!header_at(comp, q)) return 1u;
    const int32_t hs = 18 + (int32_t)u16_at(comp, q + 10) - 6;
    const int32_t cs = (int32_t)u16_at(comp, q + 16) + 1;
    const int32_t remaining = cs - hs;
    if (remaining - 4 < 0) return 2u;
    if (q + (uint64_t)cs > n) return at_eof ? 2u : 3u;
    if (remaining - 8 == 2) return 0u;
    q += (uint64_t)cs;
  }
  return 0u;
}

template <typename T>
__device__ __forceinline__ uint64_t lower_bound(const T *a, uint64_t n, T v) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t m = (lo + hi) >> 1;
    if (a[m] < v) lo = m + 1;
    else hi = m;
  }
  return lo;
}

struct SplitIn {
  const uint8_t *comp;
  uint64_t n;  // resident compressed bytes
  int at_eof;
  const uint64_t *cand;  // header candidates (shard-relative, ascending), from sbh_index
  uint64_t ncand;
  uint64_t cand_from;  // candidates exist only at/after this offset
  int32_t k_check;
  const uint64_t *cstart;
  const uint64_t *ustart;
  const uint32_t *flags;
  uint64_t nblocks;
  uint64_t utotal;
  uint64_t last_start;  // shard-relative start of the last resident block
  const uint64_t *seg_end;
  uint32_t nseg;
  const uint32_t *bits;
  uint64_t bits_begin, bits_end;
  int64_t mrs;
};

// One wave per split.  starts/ends shard-relative.  Output: first_flat, E (flat bound of
// the end), code (SPLIT_OK / SPLIT_HOST).
__global__ __launch_bounds__(64) void k_split_prologue(SplitIn in, const uint64_t *starts, const uint64_t *ends,
                                                       uint64_t nsplit, uint64_t *first_out, uint64_t *E_out,
                                                       uint32_t *code_out) {
  const uint64_t i = blockIdx.x;
  if (i >= nsplit) return;
  const uint32_t lane = threadIdx.x;
  const uint64_t s = starts[i];
  // off the common path: SPLIT_HOST | why << 4 (why: the step that gave up, for diagnostics)
  uint32_t code = SPLIT_HOST | 1u << 4;
  uint64_t first = 0, E = 0;
  do {
    if (s < in.cand_from) break;
    code = SPLIT_HOST | 2u << 4;
    // FindBlockStart: the first candidate in [s, s + 64 KiB) whose attempt is not a
    // HeaderParseException; positions within 18 bytes of the resident end are attempts
    // that never parse a header, so they end the search too (host path decides them).
    uint64_t best = ~0ull;
    if (lane == 0) {
      const uint64_t lim = s + 65536;
      for (uint64_t j = lower_bound(in.cand, in.ncand, s); j < in.ncand && in.cand[j] < lim; ++j) {
        const uint32_t o = fbs_outcome(in.comp, in.n, in.cand[j], in.k_check, in.at_eof);
        if (o != 1u) {
          best = o == 0u ? in.cand[j] : ~1ull;
          break;
        }
      }
      const uint64_t tail = in.n >= 17 ? in.n - 17 : 0;
      if (lim > tail && (best == ~0ull || best >= tail) && best != ~1ull) best = ~1ull;
    }
    // readfirstlane returns int: widen both halves through uint32_t, or a shard-relative
    // offset with bit 31 set would sign-extend into the high word
    best = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(best >> 32)) << 32) |
           (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)best);
    if (best >= ~1ull) break;
    code = SPLIT_HOST | 3u << 4;
    const uint64_t bi = lower_bound(in.cstart, in.nblocks, best);
    if (bi >= in.nblocks || in.cstart[bi] != best) break;
    if (in.flags[bi] & BLK_EMPTY) {  // the stream from an empty block ends at once (sbh_split)
      code = SPLIT_NOREAD;
      break;
    }
    const uint64_t from = in.ustart[bi];
    // the stream segment holding `from` (an empty block ends the stream) and maxReadSize
    uint64_t seg = in.seg_end[in.nseg - 1];
    for (uint32_t k = 0; k < in.nseg; ++k)
      if (in.seg_end[k] > from) { seg = in.seg_end[k]; break; }
    const uint64_t limit = min(seg, from + (uint64_t)in.mrs);
    code = SPLIT_HOST | 4u << 4;
    if (from < in.bits_begin) break;
    code = SPLIT_HOST | 5u << 4;
    const uint64_t hi = min(limit, in.bits_end);
    // FindRecordStart: first set bit in [from, hi), 64 words per step
    uint64_t found = ~0ull;
    for (uint64_t w = (from - in.bits_begin) >> 5; in.bits_begin + 32 * w < hi; w += 64) {
      const uint64_t ww = w + lane;
      const uint64_t p0 = in.bits_begin + 32 * ww;
      uint32_t x = p0 < hi ? in.bits[ww] : 0u;
      if (p0 < from) x &= p0 + 32 <= from ? 0u : ~0u << (uint32_t)(from - p0);
      if (p0 + 32 > hi) x &= p0 >= hi ? 0u : (hi - p0 >= 32 ? ~0u : (1u << (uint32_t)(hi - p0)) - 1u);
      const uint64_t m = __ballot(x != 0);
      if (m) {
        const uint32_t l = (uint32_t)__builtin_ctzll(m);
        const uint32_t xl = __builtin_amdgcn_readlane(x, l);
        found = in.bits_begin + 32 * (w + l) + (uint32_t)__builtin_ctz(xl);
        break;
      }
    }
    if (found == ~0ull) break;  // no read start in the bitmap: the host path decides
    first = found;
    code = SPLIT_HOST | 6u << 4;
    // flat bound of Pos(end, 0): the first block starting at/after end
    const uint64_t e = ends[i];
    const uint64_t bj = lower_bound(in.cstart, in.nblocks, e);
    E = bj >= in.nblocks ? in.utotal : in.ustart[bj];
    if (bj >= in.nblocks && e > in.last_start && !in.at_eof) break;  // past the resident blocks
    code = SPLIT_OK;
  } while (false);
  if (lane == 0) {
    first_out[i] = first;
    E_out[i] = E;
    code_out[i] = code;
  }
}

// counts[i] += set bits of [first[i], E[i]) (the bitmap verified equal to the chain there).
constexpr uint32_t PC_WORDS = 8192;  // words per workgroup (32 per thread)
__global__ __launch_bounds__(256) void k_split_popcount(const uint32_t *bits, uint64_t begin, const uint64_t *first,
                                                        const uint64_t *E, const uint32_t *code, uint64_t nsplit,
                                                        unsigned long long *counts) {
  const uint64_t i = blockIdx.y;
  if (i >= nsplit || code[i] != SPLIT_OK) return;
  const uint64_t from = first[i], to = E[i];
  if (from >= to) return;
  const uint64_t w0 = (from - begin) / 32, w_end = (to - begin + 31) / 32;
  const uint64_t c0 = w0 + (uint64_t)blockIdx.x * PC_WORDS;
  if (c0 >= w_end) return;
  const uint64_t c1 = min(c0 + PC_WORDS, w_end);
  uint32_t c = 0;
  auto count = [&](uint64_t w, uint32_t v) {
    const uint64_t p0 = begin + 32 * w;
    if (p0 < from) v &= ~0u << (uint32_t)(from - p0);
    if (p0 + 32 > to) v &= (to - p0) >= 32 ? ~0u : ((1u << (uint32_t)(to - p0)) - 1u);
    c += __popc(v);
  };
  const uint64_t a0 = (c0 + 3) & ~3ull, a1 = c1 & ~3ull;  // 16-byte loads over the aligned middle
  if (a0 < a1) {
    for (uint64_t w = c0 + threadIdx.x; w < a0; w += 256) count(w, bits[w]);
#pragma unroll 4
    for (uint64_t w = a0 + 4 * threadIdx.x; w < a1; w += 4 * 256) {
      const uint4 q = *reinterpret_cast<const uint4 *>(bits + w);
      count(w, q.x);
      count(w + 1, q.y);
      count(w + 2, q.z);
      count(w + 3, q.w);
    }
    for (uint64_t w = a1 + threadIdx.x; w < c1; w += 256) count(w, bits[w]);
  } else {
    for (uint64_t w = c0 + threadIdx.x; w < c1; w += 256) count(w, bits[w]);
  }
  for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off);
  __shared__ uint32_t part[4];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t = part[0] + part[1] + part[2] + part[3];
    if (t) atomicAdd(&counts[i], (unsigned long long)t);
  }
}

// Chain marked by pointer doubling: nodes pos[0..n) (ascending), mark prefix mpre[0..n].
// A split whose first record is a marked node counts the marked nodes in [first, E); any
// other split goes to the host path.
__global__ void k_split_cm_count(const uint64_t *pos, const uint64_t *mark, const uint64_t *mpre, uint64_t n,
                                 const uint64_t *first, const uint64_t *E, uint32_t *code, uint64_t nsplit,
                                 unsigned long long *counts) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nsplit || code[i] != SPLIT_OK) return;
  const uint64_t a = lower_bound(pos, n, first[i]);
  if (a >= n || pos[a] != first[i] || !mark[a]) {
    code[i] = SPLIT_HOST;
    return;
  }
  const uint64_t b = first[i] < E[i] ? lower_bound(pos, n, E[i]) : a;
  counts[i] = mpre[b] - mpre[a];
}

// `.records` truth: Pos(blockPos, offset) = vpos -> flat via the block table; bits set in
// the truth bitmap over [begin, end).  Unknown block positions are counted in *bad.
__global__ void k_truth_scatter(const uint64_t *vpos, uint64_t n, const uint64_t *cstart, const uint64_t *ustart,
                                uint64_t nblocks, uint64_t file_off, uint64_t begin, uint64_t end, uint32_t *tbits,
                                unsigned long long *bad) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t v = vpos[i], bp = v >> 16, off = v & 0xffff;
  if (bp < file_off) {
    atomicAdd(bad, 1ull);
    return;
  }
  const uint64_t rel = bp - file_off;
  const uint64_t b = lower_bound(cstart, nblocks, rel);
  if (b >= nblocks || cstart[b] != rel) {
    atomicAdd(bad, 1ull);
    return;
  }
  const uint64_t f = ustart[b] + off;
  if (f < begin || f >= end) return;
  atomicOr(&tbits[(f - begin) >> 5], 1u << ((f - begin) & 31));
}

// Per 32-position word of [begin, end): the mask of positions inside the selected ranges
// (sorted, disjoint), then TP / FP / FN counts and the mismatching positions.  Grid-stride over
// the words with a bounded grid, the counts reduced per workgroup (one atomic per counter and
// workgroup: one per wave on a single address serialised in L2 -- 1.5 M of them per 3 GB
// window took 17.6 ms, r05c)
constexpr uint32_t TC_THREADS = 256, TC_MAX_BLOCKS = 2048;
__global__ __launch_bounds__(TC_THREADS) void k_truth_compare(const uint32_t *ebits, uint64_t ebegin,
                                                              const uint32_t *tbits, uint64_t begin, uint64_t end,
                                                              const uint64_t *rb, const uint64_t *re, uint64_t nr,
                                                              unsigned long long *acc, uint64_t *fp_pos,
                                                              uint64_t fp_cap, uint64_t *fn_pos, uint64_t fn_cap) {
  __shared__ uint32_t red[3][TC_THREADS / WAVE];
  const uint64_t nw = (end - begin + 31) / 32;
  uint32_t tp = 0, fp = 0, fn = 0;
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t p0 = begin + 32 * w, p1 = min(p0 + 32, end);
    uint32_t m = 0;
    for (uint64_t r = lower_bound(re, nr, p0 + 1); r < nr && rb[r] < p1; ++r) {
      const uint64_t a = max(rb[r], p0), b = min(re[r], p1);
      if (a < b) {
        const uint32_t lo = (uint32_t)(a - p0), len = (uint32_t)(b - a);
        m |= (len >= 32 ? ~0u : ((1u << len) - 1u)) << lo;
      }
    }
    // the eager bitmap word for positions p0..p0+31 (ebegin may differ from begin by a
    // multiple of 32 only: begin - ebegin is checked on the host)
    const uint64_t ew = (p0 - ebegin) >> 5;
    const uint32_t e = ebits[ew] & m, t = tbits[w] & m;
    tp += __popc(e & t);
    uint32_t f = e & ~t, g = t & ~e;
    fp += __popc(f);
    fn += __popc(g);
    if (f) {
      const unsigned long long o = atomicAdd(&acc[3], (unsigned long long)__popc(f));
      for (uint64_t k = o; f; f &= f - 1, ++k)
        if (k < fp_cap) fp_pos[k] = p0 + __builtin_ctz(f);
    }
    if (g) {
      const unsigned long long o = atomicAdd(&acc[4], (unsigned long long)__popc(g));
      for (uint64_t k = o; g; g &= g - 1, ++k)
        if (k < fn_cap) fn_pos[k] = p0 + __builtin_ctz(g);
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    tp += __shfl_down(tp, off);
    fp += __shfl_down(fp, off);
    fn += __shfl_down(fn, off);
  }
  const uint32_t wv = threadIdx.x / WAVE;
  if ((threadIdx.x & (WAVE - 1)) == 0) red[0][wv] = tp, red[1][wv] = fp, red[2][wv] = fn;
  __syncthreads();
  if (threadIdx.x < 3) {
    unsigned long long s = 0;
    for (uint32_t k = 0; k < TC_THREADS / WAVE; ++k) s += red[threadIdx.x][k];
    if (s) atomicAdd(&acc[threadIdx.x], s);
  }
}


// counts[i] += set bits of [first[i], E[i]) from the chain proof's per-chunk counts: the chunks
// strictly inside the range (neither holds the range's first or last word) are summed, the
// bitmap is popcounted only over the words before and after them.  One workgroup per split.
// (chain_E != 0: every split's count is written, not added -- 0 when it has no range, and
// SPLIT_NOCOUNT when its range leaves the proven [chain_first, chain_E): the host then decides)
__global__ __launch_bounds__(256) void k_split_count_cc(const uint32_t *bits, uint64_t begin, const uint32_t *cc,
                                                        const uint64_t *first, const uint64_t *E, const uint32_t *code,
                                                        uint64_t nsplit, unsigned long long *counts,
                                                        uint64_t chain_first, uint64_t chain_E) {
  const uint64_t i = blockIdx.x;
  if (i >= nsplit) return;
  const bool direct = chain_E != 0;
  const uint64_t from = first[i], to = E[i];
  if (code[i] != SPLIT_OK || from >= to) {
    if (direct && threadIdx.x == 0) counts[i] = 0;
    return;
  }
  if (direct && (from < chain_first || to > chain_E)) {
    if (threadIdx.x == 0) counts[i] = SPLIT_NOCOUNT;
    return;
  }
  const uint64_t wa = (from - begin) / 32, wb = (to - begin + 31) / 32;  // words [wa, wb)
  const uint64_t ca = wa / VC_CHUNK + 1, cb = (wb - 1) / VC_CHUNK;          // inner chunks [ca, cb)
  uint32_t c = 0;
  auto count = [&](uint64_t w) {
    uint32_t v = bits[w];
    const uint64_t p0 = begin + 32 * w;
    if (p0 < from) v &= ~0u << (uint32_t)(from - p0);
    if (p0 + 32 > to) v &= (to - p0) >= 32 ? ~0u : ((1u << (uint32_t)(to - p0)) - 1u);
    c += __popc(v);
  };
  if (ca < cb) {
    for (uint64_t k = ca + threadIdx.x; k < cb; k += 256) c += cc[k];
    for (uint64_t w = wa + threadIdx.x; w < ca * VC_CHUNK; w += 256) count(w);
    for (uint64_t w = cb * VC_CHUNK + threadIdx.x; w < wb; w += 256) count(w);
  } else {
    for (uint64_t w = wa + threadIdx.x; w < wb; w += 256) count(w);
  }
  __shared__ uint32_t part[256 / 64];
  for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x / 64] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long t = (unsigned long long)part[0] + part[1] + part[2] + part[3];
    if (direct)
      counts[i] = t;
    else if (t)
      atomicAdd(&counts[i], t);
  }
}
}  // namespace

static inline uint32_t nblk(uint64_t n, uint32_t t) { return (uint32_t)((n + t - 1) / t); }

hipError_t launch_split_prologue(const SplitArgs &a, const uint64_t *starts, const uint64_t *ends, uint64_t nsplit,
                                 uint64_t *first, uint64_t *E, uint32_t *code, hipStream_t st) {
  if (!nsplit) return hipSuccess;
  SplitIn in{a.comp, a.n, a.at_eof, a.cand, a.ncand, a.cand_from, a.k_check, a.cstart, a.ustart, a.flags,
             a.nblocks, a.utotal, a.last_start, a.seg_end, a.nseg, a.bits, a.bits_begin, a.bits_end, a.mrs};
  hipLaunchKernelGGL(k_split_prologue, dim3((uint32_t)nsplit), dim3(64), 0, st, in, starts, ends, nsplit, first, E,
                     code);
  return hipGetLastError();
}

hipError_t launch_split_popcount(const uint32_t *bits, uint64_t begin, const uint64_t *first, const uint64_t *E,
                                 const uint32_t *code, uint64_t nsplit, uint64_t max_span,
                                 unsigned long long *counts, hipStream_t st) {
  if (!nsplit) return hipSuccess;
  const uint64_t gx = (max_span / 32 + 2 + PC_WORDS - 1) / PC_WORDS;
  // grid.y is limited to 65535: launch in slices of splits
  for (uint64_t s0 = 0; s0 < nsplit; s0 += 65535) {
    const uint64_t ns = std::min<uint64_t>(65535, nsplit - s0);
    hipLaunchKernelGGL(k_split_popcount, dim3((uint32_t)gx, (uint32_t)ns), dim3(256), 0, st, bits, begin, first + s0,
                       E + s0, code + s0, ns, counts + s0);
  }
  return hipGetLastError();
}

hipError_t launch_split_count_cc(const uint32_t *bits, uint64_t begin, const uint32_t *chunk_cnt, const uint64_t *first,
                                 const uint64_t *E, const uint32_t *code, uint64_t nsplit, unsigned long long *counts,
                                 hipStream_t st, uint64_t chain_first, uint64_t chain_E) {
  if (!nsplit) return hipSuccess;
  for (uint64_t s0 = 0; s0 < nsplit; s0 += 1u << 30)  // (grid.x holds 2^31 - 1 workgroups)
    hipLaunchKernelGGL(k_split_count_cc, dim3((uint32_t)std::min<uint64_t>(nsplit - s0, 1u << 30)), dim3(256), 0, st,
                       bits, begin, chunk_cnt, first + s0, E + s0, code + s0, std::min<uint64_t>(nsplit - s0, 1u << 30),
                       counts + s0, chain_first, chain_E);
  return hipGetLastError();
}

hipError_t launch_split_cm_count(const uint64_t *pos, const uint64_t *mark, const uint64_t *mpre, uint64_t n,
                                 const uint64_t *first, const uint64_t *E, uint32_t *code, uint64_t nsplit,
                                 unsigned long long *counts, hipStream_t st) {
  if (!nsplit) return hipSuccess;
  hipLaunchKernelGGL(k_split_cm_count, dim3(nblk(nsplit, 256)), dim3(256), 0, st, pos, mark, mpre, n, first, E, code,
                     nsplit, counts);
  return hipGetLastError();
}

hipError_t launch_truth_scatter(const uint64_t *vpos, uint64_t n, const uint64_t *cstart, const uint64_t *ustart,
                                uint64_t nblocks, uint64_t file_off, uint64_t begin, uint64_t end, uint32_t *tbits,
                                unsigned long long *bad, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_truth_scatter, dim3(nblk(n, 256)), dim3(256), 0, st, vpos, n, cstart, ustart, nblocks,
                     file_off, begin, end, tbits, bad);
  return hipGetLastError();
}

hipError_t launch_truth_compare(const uint32_t *ebits, uint64_t ebegin, const uint32_t *tbits, uint64_t begin,
                                uint64_t end, const uint64_t *rb, const uint64_t *re, uint64_t nr,
                                unsigned long long *acc, uint64_t *fp_pos, uint64_t fp_cap, uint64_t *fn_pos,
                                uint64_t fn_cap, hipStream_t st) {
  if (end <= begin) return hipSuccess;
  const uint64_t nw = (end - begin + 31) / 32;
  hipLaunchKernelGGL(k_truth_compare, dim3((uint32_t)std::min<uint64_t>(nblk(nw, TC_THREADS), TC_MAX_BLOCKS)),
                     dim3(TC_THREADS), 0, st, ebits, ebegin, tbits, begin, end, rb, re, nr, acc, fp_pos, fp_cap,
                     fn_pos, fn_cap);
  return hipGetLastError();
}

// A few words from the host into device memory through the kernel's arguments instead of a
// host-to-device copy: a copy on a kernel stream queues behind any large copy in flight on the
// same DMA engine (sbh_run_stream2 prefetches the next window while this one's kernels run).
namespace {
constexpr uint32_t SET_WORDS_MAX = 128;
struct Words {
  uint64_t w[SET_WORDS_MAX];
};
__global__ __launch_bounds__(SET_WORDS_MAX) void k_set_words(uint64_t *dst, Words v, uint32_t n) {
  if (threadIdx.x < n) dst[threadIdx.x] = v.w[threadIdx.x];
}
}  // namespace

hipError_t set_words(uint64_t *dst, const uint64_t *src, uint64_t n, hipStream_t st) {
  if (!n) return hipSuccess;
  if (n > SET_WORDS_MAX) return hipMemcpyAsync(dst, src, n * 8, hipMemcpyHostToDevice, st);
  Words v;
  for (uint64_t i = 0; i < n; ++i) v.w[i] = src[i];
  hipLaunchKernelGGL(k_set_words, dim3(1), dim3(SET_WORDS_MAX), 0, st, dst, v, (uint32_t)n);
  return hipGetLastError();
}

}  // namespace sbh
