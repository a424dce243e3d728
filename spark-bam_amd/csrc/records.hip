// records.hip -- BAM record field extraction on CDNA4.
//
// Replaces, for every record of a flat range at once, the decode behind RecordStream
// (check/.../iterator/RecordStream.scala:16-41) and CanLoadBam.loadReads
// (load/.../CanLoadBam.scala:244-264): htsjdk BAMRecordCodec.decode of the fixed fields,
// read name, CIGAR, 4-bit sequence, qualities and the raw tag bytes.  Record starts come
// from the chain (next = start + 4 + block_size): the verified eager bitmap when it
// covers the range, otherwise a sequential walk.  Output is columnar: fixed fields as
// arrays, variable-length fields packed into arenas addressed by exclusive prefix sums.
#include <algorithm>

#include "sbh_internal.h"

namespace sbh {
namespace {

__device__ __forceinline__ uint32_t rd_u32(const uint8_t *U, uint64_t p) {
  return (uint32_t)U[p] | (uint32_t)U[p + 1] << 8 | (uint32_t)U[p + 2] << 16 | (uint32_t)U[p + 3] << 24;
}

// Per-word prefix counts in two levels: a workgroup covers WP_CHUNK words (WP_WPT per
// thread); k_chunk_popcounts sums each chunk, the chunk sums are scanned (a few thousand
// values), and k_word_prefix re-counts its words, scans them inside the workgroup and
// writes wpre -- one write pass over the words instead of a multi-pass global scan.
constexpr uint32_t WP_T = 256, WP_WPT = WPRE_GROUP, WP_CHUNK = WP_T * WP_WPT;

__device__ __forceinline__ uint32_t masked_word(const uint32_t *bits, uint64_t begin, uint64_t first, uint64_t E,
                                                uint64_t w) {
  if (w >= (E - begin + 31) / 32) return 0;
  uint32_t v = bits[w];
  const uint64_t p0 = begin + 32 * w;
  if (p0 < first) v &= ~0u << (uint32_t)(first - p0);
  if (p0 + 32 > E) v &= (E - p0) >= 32 ? ~0u : ((1u << (uint32_t)(E - p0)) - 1u);
  return v;
}

// Record starts = set bits of [first, E): a thread per group of WPRE_GROUP bitmap words,
// positions written from the group's prefix (wpre) on.
__global__ void k_bits_positions(const uint32_t *bits, uint64_t begin, uint64_t first, uint64_t E,
                                 const uint64_t *wpre, uint64_t *pos) {
  const uint64_t w0 = (first - begin) / 32, wend = (E - begin + 31) / 32;
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t wg = w0 + g * WPRE_GROUP;
  if (wg >= wend) return;
  uint64_t o = wpre[g];
  for (uint32_t k = 0; k < WPRE_GROUP; ++k) {
    uint32_t v = masked_word(bits, begin, first, E, wg + k);
    const uint64_t p0 = begin + 32 * (wg + k);
    while (v) {
      pos[o++] = p0 + __builtin_ctz(v);
      v &= v - 1;
    }
  }
}

__global__ __launch_bounds__(WP_T) void k_chunk_popcounts(const uint32_t *bits, uint64_t begin, uint64_t first,
                                                          uint64_t E, uint64_t *ccnt) {
  __shared__ uint32_t part[WP_T / WAVE];
  const uint64_t w0 = (first - begin) / 32 + (uint64_t)blockIdx.x * WP_CHUNK + (uint64_t)threadIdx.x * WP_WPT;
  uint32_t c = 0;
#pragma unroll
  for (uint32_t k = 0; k < WP_WPT; ++k) c += __popc(masked_word(bits, begin, first, E, w0 + k));
  for (int off = WAVE / 2; off > 0; off >>= 1) c += __shfl_down(c, off);
  if ((threadIdx.x & (WAVE - 1)) == 0) part[threadIdx.x / WAVE] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (uint32_t k = 0; k < WP_T / WAVE; ++k) t += part[k];
    ccnt[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(WP_T) void k_word_prefix(const uint32_t *bits, uint64_t begin, uint64_t first,
                                                      uint64_t E, const uint64_t *cpre, uint64_t *wpre) {
  __shared__ uint32_t wsum[WP_T / WAVE];
  const uint64_t wb = (first - begin) / 32;
  const uint64_t nw = (E - begin + 31) / 32 - wb;
  const uint64_t r0 = (uint64_t)blockIdx.x * WP_CHUNK + (uint64_t)threadIdx.x * WP_WPT;  // relative word
  uint32_t mine = 0;
#pragma unroll
  for (uint32_t k = 0; k < WP_WPT; ++k) mine += __popc(masked_word(bits, begin, first, E, wb + r0 + k));
  const uint32_t lane = threadIdx.x & (WAVE - 1), wv = threadIdx.x / WAVE;
  const uint32_t incl = wave_incl_scan(mine);
  if (lane == WAVE - 1) wsum[wv] = incl;
  __syncthreads();
  uint32_t before = 0;
  for (uint32_t k = 0; k < wv; ++k) before += wsum[k];
  if (r0 < nw) wpre[r0 / WP_WPT] = cpre[blockIdx.x] + before + incl - mine;  // (the group's prefix)
}

// Sequential chain from first while the start is < E (fallback when no verified bitmap).
__global__ void k_chain_positions(const uint8_t *U, uint64_t first, uint64_t E, uint64_t total, uint64_t cap,
                                  uint64_t *pos) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint64_t r = first, n = 0;
  while (r < E && r + 4 <= total && n < cap) {
    pos[n++] = r;
    const int64_t nx = (int64_t)r + 4 + (int32_t)rd_u32(U, r);
    if (nx <= (int64_t)r) break;
    r = (uint64_t)nx;
  }
}

// Per record: name bytes (l_read_name, with the NUL), CIGAR ops, bases, tag bytes
// (block_size + 4 minus everything before the tags).  bad: a record whose parts do not
// fit its block or the stream (htsjdk would throw).
__global__ void k_rec_sizes(const uint8_t *U, const uint64_t *pos, uint64_t n, uint64_t total, uint64_t *nm,
                            uint64_t *cg, uint64_t *sq, uint64_t *ax, unsigned long long *bad) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t p = pos[i];
  uint64_t l_name = 0, n_cig = 0, l_seq = 0, l_aux = 0;
  if (p + 36 > total) {
    atomicMin(bad, (unsigned long long)i);
  } else {
    const int64_t bsz = (int32_t)rd_u32(U, p);
    l_name = U[p + 12];
    n_cig = rd_u32(U, p + 16) & 0xffff;
    const int64_t ls = (int32_t)rd_u32(U, p + 20);
    const int64_t fixed = 32 + (int64_t)l_name + 4 * (int64_t)n_cig + (ls + 1) / 2 + ls;
    if (ls < 0 || bsz < fixed || p + 4 + (uint64_t)bsz > total) {
      atomicMin(bad, (unsigned long long)i);
      l_name = n_cig = 0;
    } else {
      l_seq = (uint64_t)ls;
      l_aux = (uint64_t)(bsz - fixed);
    }
  }
  nm[i] = l_name;
  cg[i] = n_cig;
  sq[i] = l_seq;
  ax[i] = l_aux;
}


// loadBamIntervals' record filter (load/.../CanLoadBam.scala:137-152, region() at :446-454):
// keep[i] = 1 when the record's reference span overlaps one of the query intervals.
// Region(contig, getStart - 1, getEnd) is [pos, pos + reference length of the CIGAR)
// (ops M D N = X consume the reference); no contig (refID < 0), an unmapped read
// (htsjdk getAlignmentEnd = 0) or an empty span never intersects.  Intervals are the
// LociSet's merged half-open ranges as (ref, begin, end), sorted by (ref, begin), so
// ends are sorted too: binary search for the first interval of the record's ref whose
// end exceeds pos.  A record whose fields run past `total` is kept, so the size pass
// reports it as malformed (htsjdk would throw on it).
__global__ void k_region_keep(const uint8_t *__restrict__ U, const uint64_t *pos, uint64_t n, uint64_t total,
                              const int32_t *iv_ref, const int64_t *iv_begin, const int64_t *iv_end, uint32_t n_iv,
                              uint64_t *keep) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t p = pos[i];
  uint64_t k = 0;
  if (p + 36 > total) {
    k = 1;
  } else {
    const int32_t ref = (int32_t)rd_u32(U, p + 4), rp = (int32_t)rd_u32(U, p + 8);
    const uint32_t fnc = rd_u32(U, p + 16), nc = fnc & 0xffff;
    const uint64_t q = p + 36 + U[p + 12];
    if (q + 4ull * nc > total) {
      k = 1;
    } else if (ref >= 0 && !((fnc >> 16) & 4) && rp >= 0) {
      int64_t span = 0;
      for (uint32_t c = 0; c < nc; ++c) {
        const uint32_t op = rd_u32(U, q + 4ull * c);
        const uint32_t t = op & 15;
        if (t == 0 || t == 2 || t == 3 || t == 7 || t == 8) span += op >> 4;
      }
      if (span > 0) {
        const int64_t b = rp, e = b + span;
        uint32_t lo = 0, hi = n_iv;  // first interval with (ref, end) > (ref, b)
        while (lo < hi) {
          const uint32_t m = (lo + hi) >> 1;
          if (iv_ref[m] < ref || (iv_ref[m] == ref && iv_end[m] <= b)) lo = m + 1; else hi = m;
        }
        k = lo < n_iv && iv_ref[lo] == ref && iv_begin[lo] < e;
      }
    }
  }
  keep[i] = k;
}

__global__ void k_compact_u64(const uint64_t *in, const uint64_t *keep, const uint64_t *kpre, uint64_t n,
                              uint64_t *out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && keep[i]) out[kpre[i]] = in[i];
}

// Record start (flat) -> htsjdk virtual position, canonical as Pos is (bgzf/.../Pos.scala,
// UncompressedBytes.curPos): the LAST block of the chain whose first flat byte is <= the start,
// so a start at a block's end is Pos(next block, 0); empty blocks (usize 0) hold no position.
__global__ void k_rec_vpos(const uint64_t *pos, uint64_t n, const uint64_t *ustart, const uint64_t *cstart,
                           const uint32_t *usize, uint64_t nblocks, uint64_t file_off, uint64_t *vpos) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t f = pos[i];
  uint64_t lo = 0, hi = nblocks;  // first block with ustart > f
  while (lo < hi) {
    const uint64_t m = (lo + hi) / 2;
    if (ustart[m] <= f) lo = m + 1;
    else hi = m;
  }
  uint64_t k = lo ? lo - 1 : 0;
  while (k > 0 && usize[k] == 0) --k;
  vpos[i] = (file_off + cstart[k]) << 16 | (f - ustart[k]);
}
}  // namespace

namespace {

// One wave per record (grid-stride): lane 0 the fixed fields, all lanes the variable
// parts -- name, CIGAR (unaligned u32 ops), bases (4-bit codes -> "=ACMGRSVTWYHKDBN"),
// qualities and tag bytes, each at its prefix-sum offset.
__global__ __launch_bounds__(256) void k_rec_fields(const uint8_t *__restrict__ U, const uint64_t *pos, uint64_t n,
                                                    const uint64_t *nm_off, const uint64_t *cg_off,
                                                    const uint64_t *sq_off, const uint64_t *ax_off, RecCols c) {
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x / WAVE);
  for (uint64_t i = (uint64_t)blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE; i < n; i += nw) {
    const uint64_t p = pos[i];
    if (lane == 0) {
      c.ref_id[i] = (int32_t)rd_u32(U, p + 4);
      c.pos[i] = (int32_t)rd_u32(U, p + 8);
      const uint32_t bmn = rd_u32(U, p + 12), fnc = rd_u32(U, p + 16);
      c.mapq[i] = (uint8_t)(bmn >> 8);
      c.bin[i] = (uint16_t)(bmn >> 16);
      c.flag[i] = (uint16_t)(fnc >> 16);
      c.next_ref_id[i] = (int32_t)rd_u32(U, p + 24);
      c.next_pos[i] = (int32_t)rd_u32(U, p + 28);
      c.tlen[i] = (int32_t)rd_u32(U, p + 32);
    }
    const uint64_t l_name = nm_off[i + 1] - nm_off[i], n_cig = cg_off[i + 1] - cg_off[i];
    const uint64_t l_seq = sq_off[i + 1] - sq_off[i], l_aux = ax_off[i + 1] - ax_off[i];
    const uint64_t q_name = p + 36, q_cig = q_name + l_name, q_seq = q_cig + 4 * n_cig;
    const uint64_t q_qual = q_seq + (l_seq + 1) / 2, q_aux = q_qual + l_seq;
    for (uint64_t k = lane; k < l_name; k += WAVE) c.names[nm_off[i] + k] = (char)U[q_name + k];
    for (uint64_t k = lane; k < n_cig; k += WAVE) c.cigar[cg_off[i] + k] = rd_u32(U, q_cig + 4 * k);
    for (uint64_t k = lane; k < l_seq; k += WAVE) {
      const uint8_t b = U[q_seq + k / 2];
      c.seq[sq_off[i] + k] = "=ACMGRSVTWYHKDBN"[(k & 1) ? (b & 15) : (b >> 4)];
      c.qual[sq_off[i] + k] = U[q_qual + k];
    }
    for (uint64_t k = lane; k < l_aux; k += WAVE) c.aux[ax_off[i] + k] = U[q_aux + k];
  }
}

}  // namespace

hipError_t scan_exclusive_u64(const uint64_t *in, uint64_t *out, uint64_t n, uint64_t *tmp, hipStream_t st);

// cnt: 2 u64 per WP_CHUNK words (chunk sums and their prefix); wpre: one u64 per WPRE_GROUP
// words of [first, E); tmp: scan_tmp_words(words)
hipError_t launch_rec_positions_bits(const uint32_t *bits, uint64_t begin, uint64_t first, uint64_t E, uint64_t *cnt,
                                     uint64_t *wpre, uint64_t *tmp, uint64_t *pos, hipStream_t st) {
  const uint64_t nw = (E - begin + 31) / 32 - (first - begin) / 32;
  if (!nw) return hipSuccess;
  const uint32_t g = (uint32_t)(((nw + WPRE_GROUP - 1) / WPRE_GROUP + 255) / 256);
  const uint64_t nch = (nw + WP_CHUNK - 1) / WP_CHUNK;  // cnt: chunk sums, then (cnt + nch) their prefix
  hipLaunchKernelGGL(k_chunk_popcounts, dim3((uint32_t)nch), dim3(WP_T), 0, st, bits, begin, first, E, cnt);
  hipError_t e = scan_exclusive_u64(cnt, cnt + nch, nch, tmp, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_word_prefix, dim3((uint32_t)nch), dim3(WP_T), 0, st, bits, begin, first, E, cnt + nch, wpre);
  hipLaunchKernelGGL(k_bits_positions, dim3(g), dim3(256), 0, st, bits, begin, first, E, wpre, pos);
  return hipGetLastError();
}

hipError_t launch_rec_positions_chain(const uint8_t *U, uint64_t first, uint64_t E, uint64_t total, uint64_t cap,
                                      uint64_t *pos, hipStream_t st) {
  hipLaunchKernelGGL(k_chain_positions, dim3(1), dim3(64), 0, st, U, first, E, total, cap, pos);
  return hipGetLastError();
}

hipError_t launch_rec_sizes(const uint8_t *U, const uint64_t *pos, uint64_t n, uint64_t total, uint64_t *nm,
                            uint64_t *cg, uint64_t *sq, uint64_t *ax, unsigned long long *bad, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_rec_sizes, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, U, pos, n, total, nm, cg, sq,
                     ax, bad);
  return hipGetLastError();
}

hipError_t launch_rec_fields(const uint8_t *U, const uint64_t *pos, uint64_t n, const uint64_t *nm_off,
                             const uint64_t *cg_off, const uint64_t *sq_off, const uint64_t *ax_off, const RecCols &c,
                             hipStream_t st) {
  if (!n) return hipSuccess;
  const uint32_t g = (uint32_t)std::min<uint64_t>((n + 3) / 4, 65536);  // 4 records (waves) per workgroup
  hipLaunchKernelGGL(k_rec_fields, dim3(g), dim3(256), 0, st, U, pos, n, nm_off, cg_off, sq_off, ax_off, c);
  return hipGetLastError();
}

hipError_t launch_region_keep(const uint8_t *U, const uint64_t *pos, uint64_t n, uint64_t total, const int32_t *iv_ref,
                              const int64_t *iv_begin, const int64_t *iv_end, uint32_t n_iv, uint64_t *keep,
                              hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_region_keep, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, U, pos, n, total, iv_ref,
                     iv_begin, iv_end, n_iv, keep);
  return hipGetLastError();
}

hipError_t launch_compact_u64(const uint64_t *in, const uint64_t *keep, const uint64_t *kpre, uint64_t n,
                              uint64_t *out, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_compact_u64, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, in, keep, kpre, n, out);
  return hipGetLastError();
}

hipError_t launch_rec_vpos(const uint64_t *pos, uint64_t n, DevBlocks bl, uint64_t nblocks, uint64_t file_off,
                           uint64_t *vpos, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_rec_vpos, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, pos, n, bl.ustart, bl.cstart,
                     bl.usize, nblocks, file_off, vpos);
  return hipGetLastError();
}

}  // namespace sbh
