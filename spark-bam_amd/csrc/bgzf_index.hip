// bgzf_index.hip -- BGZF header scan, FindBlockStart and block-chain indexing on CDNA4.
//
// Replaces, for a whole shard at once:
//  * Header.make            (bgzf/.../block/Header.scala:48-83)
//  * MetadataStream         (bgzf/.../block/MetadataStream.scala:23-54)
//  * FindBlockStart.apply   (bgzf/.../block/FindBlockStart.scala:8-36)
// Compressed bytes are resident in HBM.  The scan is byte-parallel (one thread per 16
// candidate offsets, coalesced 16 B loads); the block chain from a known start is
// recovered exactly with pointer jumping over the (sparse) candidate list, so a
// false header pattern inside stored (level-0) data can never enter the chain.
#include "sbh_internal.h"

namespace sbh {
namespace {

constexpr int SCAN_T = 256;       // threads per workgroup
constexpr int SCAN_PER = 8;       // elements per thread in the scans
constexpr uint64_t CHUNK = 16384;  // bytes per candidate-scan workgroup (256 x 4 x 16)
static_assert(CHUNK % 4096 == 0 && CHUNK / 256 <= 64, "chunk layout");

__device__ __forceinline__ bool header_at(const uint8_t *c, uint64_t p) {
  // gzip magic 31 139 8 4 and 'B' 'C' 2 (Header.scala:61-75; byte 15 unchecked)
  return c[p] == 31 && c[p + 1] == 139 && c[p + 2] == 8 && c[p + 3] == 4 && c[p + 12] == 66 &&
         c[p + 13] == 67 && c[p + 14] == 2;
}
__device__ __forceinline__ uint32_t u16_at(const uint8_t *c, uint64_t p) {
  return (uint32_t)c[p] | ((uint32_t)c[p + 1] << 8);
}
__device__ __forceinline__ uint32_t u32_at(const uint8_t *c, uint64_t p) {
  return (uint32_t)c[p] | ((uint32_t)c[p + 1] << 8) | ((uint32_t)c[p + 2] << 16) |
         ((uint32_t)c[p + 3] << 24);
}

// ---------------------------------------------------------------- exclusive scan
__global__ __launch_bounds__(SCAN_T) void k_scan_local(const uint64_t *in, uint64_t *out,
                                                       uint64_t *sums, uint64_t n) {
  __shared__ uint64_t s[SCAN_T];
  const uint64_t base = ((uint64_t)blockIdx.x * SCAN_T + threadIdx.x) * SCAN_PER;
  uint64_t v[SCAN_PER];
  uint64_t t = 0;
#pragma unroll
  for (int k = 0; k < SCAN_PER; ++k) {
    v[k] = base + k < n ? in[base + k] : 0;
    t += v[k];
  }
  s[threadIdx.x] = t;
  __syncthreads();
  for (int off = 1; off < SCAN_T; off <<= 1) {
    uint64_t x = threadIdx.x >= (unsigned)off ? s[threadIdx.x - off] : 0;
    __syncthreads();
    s[threadIdx.x] += x;
    __syncthreads();
  }
  uint64_t run = s[threadIdx.x] - t;  // exclusive prefix of this thread
#pragma unroll
  for (int k = 0; k < SCAN_PER; ++k) {
    if (base + k < n) out[base + k] = run;
    run += v[k];
  }
  if (threadIdx.x == SCAN_T - 1) sums[blockIdx.x] = s[SCAN_T - 1];
}

__global__ __launch_bounds__(SCAN_T) void k_scan_add(uint64_t *out, const uint64_t *pref, uint64_t n) {
  const uint64_t base = ((uint64_t)blockIdx.x * SCAN_T + threadIdx.x) * SCAN_PER;
  const uint64_t add = pref[blockIdx.x];
#pragma unroll
  for (int k = 0; k < SCAN_PER; ++k)
    if (base + k < n) out[base + k] += add;
}

// ---------------------------------------------------------------- FindBlockStart
// For each pos in [0, 65536): the MetadataStream.take(k).size attempt from start+pos.
// Outcome per pos: 0 ok, 1 HeaderParseException (retry), 2 other exception (escapes),
// 3 needs bytes beyond the resident range.  The smallest non-1 pos wins.
__global__ void k_find_block_start(const uint8_t *comp, uint64_t n, uint64_t start, int32_t k_check,
                                   int at_eof, unsigned long long *best) {
  const uint64_t pos = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (pos >= 65536) return;
  uint64_t q = start + pos;
  uint32_t outcome = 0;
  for (int32_t k = 0; k < k_check; ++k) {
    if (q + 18 > n) {  // readFully(18) would hit the end of the resident bytes
      outcome = at_eof ? 0 : 3;
      break;
    }
    if (!header_at(comp, q)) { outcome = 1; break; }
    const uint32_t xlen = u16_at(comp, q + 10);
    const int32_t hs = 18 + (int32_t)xlen - 6;
    const int32_t cs = (int32_t)u16_at(comp, q + 16) + 1;
    const int32_t remaining = cs - hs;
    if (remaining - 4 < 0) { outcome = 2; break; }
    if (q + (uint64_t)cs > n) { outcome = at_eof ? 2 : 3; break; }  // getInt EOF
    if (remaining - 8 == 2) break;  // empty block ends the stream: success
    q += (uint64_t)cs;
  }
  if (outcome != 1) atomicMin(best, (unsigned long long)((pos << 8) | outcome));
}

// ---------------------------------------------------------------- candidate scan
// Pass 1 streams every byte once with coalesced 16 B loads (lane t of segment i reads
// chunk + i*4096 + 16t) and finds the BGZF magic (31 139 8 4) with exact SWAR byte tests
// in registers; only those offsets get the full header check.  Per chunk it records the candidate count and
// the first candidate's offset.  Pass 2 then needs the bytes again only for the rare
// chunks holding two or more candidates (blocks are ~20-65 KB apart).

// 4-bit mask of the bytes of w equal to the byte replicated in b4 (exact per byte), and
// the 16-bit mask over a 16-byte vector.
__device__ __forceinline__ uint32_t eq4(uint32_t w, uint32_t b4) {
  const uint32_t t = w ^ b4;
  const uint32_t z = ~(((t & 0x7f7f7f7fu) + 0x7f7f7f7fu) | t) & 0x80808080u;
  return ((z >> 7) * 0x204081u >> 21) & 0xfu;  // bits 7/15/23/31 -> 0..3
}
__device__ __forceinline__ uint32_t eq16(const uint4 &v, uint32_t b4) {
  return eq4(v.x, b4) | eq4(v.y, b4) << 4 | eq4(v.z, b4) << 8 | eq4(v.w, b4) << 12;
}

__device__ __forceinline__ bool cand_at(const uint8_t *comp, uint64_t n, uint64_t from, uint64_t p) {
  return p >= from && p + 18 <= n && header_at(comp, p);
}

#ifndef SBH_CAND_CPW
#define SBH_CAND_CPW 1  // chunks per k_cand_count workgroup (A/B r06o: 4 chunks, all loads in flight, index +0.045 ms on config B)
#endif
constexpr uint32_t CAND_CPW = SBH_CAND_CPW;

__global__ __launch_bounds__(256) void k_cand_count(const uint8_t *comp, uint64_t n, uint64_t from,
                                                     uint64_t *counts, uint32_t *first, uint64_t nchunks) {
  __shared__ uint32_t c[CAND_CPW], f[CAND_CPW];
  if (threadIdx.x < CAND_CPW) {
    c[threadIdx.x] = 0;
    f[threadIdx.x] = ~0u;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) counts[nchunks] = 0;  // (the scan's n + 1st entry: offs[nchunks] = total)
  __syncthreads();
  constexpr uint32_t NV = CHUNK / 4096;
  const uint64_t chunk0 = (uint64_t)blockIdx.x * CAND_CPW;
  // all of the thread's 16-byte loads of every chunk in flight at once (whole chunks: no
  // per-load test)
  uint4 vv[CAND_CPW][NV];
#pragma unroll
  for (uint32_t ci = 0; ci < CAND_CPW; ++ci) {
    const uint64_t cbase = (chunk0 + ci) * CHUNK;
    if (cbase + CHUNK <= n) {
#pragma unroll
      for (uint32_t i = 0; i < NV; ++i)
        vv[ci][i] = *reinterpret_cast<const uint4 *>(comp + cbase + i * 4096 + threadIdx.x * 16);
    } else {  // ragged end of the shard (or a chunk past it)
#pragma unroll
      for (uint32_t i = 0; i < NV; ++i) {
        const uint64_t p0 = cbase + i * 4096 + threadIdx.x * 16;
        uint32_t w[4] = {0, 0, 0, 0};
        for (uint32_t k = 0; k < 16 && p0 + k < n; ++k) w[k >> 2] |= (uint32_t)comp[p0 + k] << (8 * (k & 3));
        vv[ci][i] = make_uint4(w[0], w[1], w[2], w[3]);
      }
    }
  }
#pragma unroll
  for (uint32_t ci = 0; ci < CAND_CPW; ++ci) {
    const uint64_t cbase = (chunk0 + ci) * CHUNK;
    uint32_t mine = 0, myfirst = ~0u;
#pragma unroll
    for (uint32_t i = 0; i < NV; ++i) {
      const uint32_t o0 = i * 4096 + threadIdx.x * 16;
      const uint64_t p0 = cbase + o0;
      const uint4 v = vv[ci][i];
      // the whole 4-byte magic (31 139 8 4) is tested in registers where the vector holds it,
      // so the header check's dependent loads run only for near-certain headers (and for a
      // 31 in the vector's last 3 bytes), not for every 31 byte (1 in 256 of deflate data)
      const uint32_t m31 = eq16(v, 0x1f1f1f1fu);
      if (m31) {
        const uint32_t mh = m31 & (eq16(v, 0x8b8b8b8bu) >> 1) & (eq16(v, 0x08080808u) >> 2) & (eq16(v, 0x04040404u) >> 3);
        uint32_t mq = (mh & 0x1fffu) | (m31 & 0xe000u);
        while (mq) {
          const uint32_t k = __builtin_ctz(mq);
          mq &= mq - 1;
          if (cand_at(comp, n, from, p0 + k)) {
            ++mine;
            myfirst = min(myfirst, o0 + k);
          }
        }
      }
    }
    if (mine) {
      atomicAdd(&c[ci], mine);
      atomicMin(&f[ci], myfirst);
    }
  }
  __syncthreads();
  if (threadIdx.x < CAND_CPW && chunk0 + threadIdx.x < nchunks) {
    counts[chunk0 + threadIdx.x] = c[threadIdx.x];
    first[chunk0 + threadIdx.x] = f[threadIdx.x];
  }
}

// Pass 2: chunk candidates in position order; only multi-candidate chunks rescan (each
// thread a contiguous CHUNK/256 bytes).
__global__ __launch_bounds__(256) void k_cand_write(const uint8_t *comp, uint64_t n, uint64_t from,
                                                     const uint64_t *counts, const uint32_t *first,
                                                     const uint64_t *offs, uint64_t *cand) {
  const uint64_t cnt = counts[blockIdx.x];
  if (cnt == 0) return;
  const uint64_t cbase = (uint64_t)blockIdx.x * CHUNK;
  if (cnt == 1) {
    if (threadIdx.x == 0) cand[offs[blockIdx.x]] = cbase + first[blockIdx.x];
    return;
  }
  constexpr uint32_t PER = CHUNK / 256;
  __shared__ uint32_t pre[256];
  const uint64_t p0 = cbase + (uint64_t)threadIdx.x * PER;
  uint64_t mask = 0;
  for (uint32_t k = 0; k < PER; ++k)
    if (comp[p0 + k < n ? p0 + k : 0] == 31 && cand_at(comp, n, from, p0 + k)) mask |= 1ull << k;
  const uint32_t mc = (uint32_t)__popcll(mask);
  pre[threadIdx.x] = mc;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    uint32_t x = threadIdx.x >= (unsigned)off ? pre[threadIdx.x - off] : 0;
    __syncthreads();
    pre[threadIdx.x] += x;
    __syncthreads();
  }
  uint64_t o = offs[blockIdx.x] + pre[threadIdx.x] - mc;
  while (mask) {
    cand[o++] = p0 + __builtin_ctzll(mask);
    mask &= mask - 1;
  }
}

constexpr int64_t TERM_END = -2;     // chain reaches the end of the resident bytes exactly
constexpr int64_t TERM_TRUNC = -3;   // block runs past the resident bytes
constexpr int64_t TERM_BROKEN = -4;  // next offset is not a block header

// Link each candidate to the candidate at (pos + csize).  (Thread 0 also zeroes the empty-block
// count k_chain_emit keeps beside the next 18 bytes.)
__global__ void k_cand_link(const uint8_t *comp, uint64_t n, const uint64_t *cand, uint64_t nc,
                            int64_t *next, uint8_t *next18) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) {
    *reinterpret_cast<uint32_t *>(next18 + NEXT18_NEMPTY) = 0;
    next18[NEXT18_NONLIN] = 0;
  }
  if (i >= nc) return;
  const uint64_t p = cand[i];
  const uint64_t cs = u16_at(comp, p + 16) + 1;
  const uint64_t q = p + cs;
  int64_t r;
  if (q > n) r = TERM_TRUNC;
  else if (q == n) r = TERM_END;
  else if (q + 18 > n) r = TERM_TRUNC;  // a partial header: treat like truncation
  else {
    // binary search for q among cand[i+1 ..]
    uint64_t lo = i + 1, hi = nc;
    while (lo < hi) {
      uint64_t m = (lo + hi) >> 1;
      if (cand[m] < q) lo = m + 1; else hi = m;
    }
    r = (lo < nc && cand[lo] == q) ? (int64_t)lo : TERM_BROKEN;
  }
  next[i] = r;
}

// Pointer-jumping marking of the chain from candidate 0: after round k every node at
// distance < 2^(k+1) is marked (marks only ever add true chain nodes).
__global__ void k_jump_mark(const int64_t *J, uint8_t *on, uint64_t nc) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nc) return;
  if (on[i] && J[i] >= 0) on[J[i]] = 1;
}
// One round of both: the mark and the doubling read only J, so they share a launch (a mark
// that another thread of the same round sets early only spreads marks sooner -- still chain
// nodes).  Half the launches of the two-kernel loop (each ~3 us of work behind ~7 us of
// dispatch gap in the bench step's trace).
__global__ void k_jump_round(const int64_t *J, int64_t *J2, uint8_t *on, uint64_t nc) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nc) return;
  const int64_t j = J[i];
  if (j >= 0) {
    if (on[i]) on[j] = 1;
    J2[i] = J[j];
  } else {
    J2[i] = j;
  }
}

// The chain starts at the candidate equal to start_rel (the scan may begin before it, so that
// FindBlockStart from earlier offsets has its candidates): binary search, mark it.
__global__ void k_mark_start(const uint64_t *cand, uint64_t nc, uint64_t start_rel, uint8_t *on) {
  if (threadIdx.x != 0) return;
  uint64_t lo = 0, hi = nc;
  while (lo < hi) {
    const uint64_t m = (lo + hi) >> 1;
    if (cand[m] < start_rel) lo = m + 1;
    else hi = m;
  }
  if (lo < nc && cand[lo] == start_rel) on[lo] = 1;
}

// The common chain: every candidate from the start on is the next one's predecessor (no
// candidate inside a block's bytes, no break).  The start's index by binary search, then each
// candidate's mark / rank directly -- no pointer-jumping rounds -- while every link is checked:
// a candidate whose link is not the next candidate (or a last one that links on) sets
// next18[NEXT18_NONLIN], and the host rebuilds the chain by pointer jumping (build_chain with
// linear = false).  The marks and ranks equal the jumping path's whenever the flag stays clear.
__global__ void k_linear_start(const uint64_t *cand, uint64_t nc, uint64_t start_rel, uint64_t *sidx) {
  if (threadIdx.x != 0) return;
  uint64_t lo = 0, hi = nc;
  while (lo < hi) {
    const uint64_t m = (lo + hi) >> 1;
    if (cand[m] < start_rel) lo = m + 1;
    else hi = m;
  }
  *sidx = lo < nc && cand[lo] == start_rel ? lo : nc;  // nc: the start is not a candidate (empty chain)
}
__global__ void k_linear_chain(const int64_t *J, const uint64_t *sidx, uint8_t *on, uint64_t *v, uint64_t *rank,
                               uint64_t nc, uint8_t *next18) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nc) return;
  const uint64_t s = *sidx;
  const bool m = i >= s;
  on[i] = m ? 1 : 0;
  v[i] = m ? 1 : 0;
  rank[i] = m ? i - s : 0;
  if (m && (i + 1 < nc ? J[i] != (int64_t)(i + 1) : J[i] >= 0)) next18[NEXT18_NONLIN] = 1;
}

__global__ void k_mark_u64(const uint8_t *on, uint64_t *v, uint64_t nc) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nc) return;
  v[i] = on[i] ? 1 : 0;
}

// Emit the chain as the block table (ordered by position).
// (usz is zero beyond the chain, so the flat-offset scan may run over all nc entries; the chain
// length is the last rank plus the last mark, read here rather than by the host; the chain's
// empty blocks are counted at next18 + NEXT18_NEMPTY, so that the host walks the table for its
// segment ends only when there are any)
__global__ void k_chain_emit(const uint8_t *comp, uint64_t n, const uint64_t *cand, const uint8_t *on,
                             const uint64_t *rank, const uint64_t *v, uint64_t nc, DevBlocks bl,
                             uint64_t *usz, uint8_t *next18) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nc || !on[i]) return;
  const uint64_t nchain = rank[nc - 1] + v[nc - 1];
  const uint64_t r = rank[i];
  const uint64_t p = cand[i];
  const uint32_t xlen = u16_at(comp, p + 10);
  const uint32_t hs = 18 + xlen - 6;
  const uint32_t cs = u16_at(comp, p + 16) + 1;
  uint32_t flags = 0, us = 0;
  if (p + cs > n) {
    flags |= BLK_TRUNCATED;
  } else {
    us = u32_at(comp, p + cs - 4);
    if ((int32_t)cs - (int32_t)hs - 8 == 2) {
      flags |= BLK_EMPTY;
      atomicAdd(reinterpret_cast<uint32_t *>(next18 + NEXT18_NEMPTY), 1u);
    }
  }
  bl.cstart[r] = p;
  bl.csize[r] = cs;
  bl.hsize[r] = hs;
  bl.usize[r] = (flags & BLK_EMPTY) ? 0 : us;
  bl.flags[r] = flags;
  bl.status[r] = 0;
  // flat sizes: empty or truncated blocks contribute no bytes; ISIZE > 64 KiB is an
  // inflate error (reported by k_inflate), contributes none
  usz[r] = (flags & (BLK_EMPTY | BLK_TRUNCATED)) || us > 65536u ? 0 : us;
  if (r + 1 == nchain)  // the bytes after the last block: the host checks the next header
    for (uint32_t j = 0; j < 18; ++j) next18[j] = p + cs + j < n ? comp[p + cs + j] : 0;
}

// The block table as the host's sbh_block records (start = file offset, ustart, csize | hsize
// << 32, usize | flags << 32): one device-to-host copy lands it in place.
// (trailer, optional: out[4 n] = the chain length rank[n - 1] + v[n - 1], out[4 n + 1, + 4) = the
// next18 words k_chain_emit left -- so the table, its length and the next header come back in one copy)
__global__ void k_pack_blocks(DevBlocks bl, uint64_t n, uint64_t file_off, uint64_t *out, const uint64_t *rank,
                              const uint64_t *v, const uint64_t *next18) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0 && rank) {
    out[4 * n] = rank[n - 1] + v[n - 1];
    for (int k = 0; k < 3; ++k) out[4 * n + 1 + k] = next18[k];
  }
  if (i >= n) return;
  uint64_t *r = out + 4 * i;
  r[0] = bl.cstart[i] + file_off;
  r[1] = bl.ustart[i];
  r[2] = (uint64_t)bl.csize[i] | (uint64_t)bl.hsize[i] << 32;
  r[3] = (uint64_t)bl.usize[i] | (uint64_t)bl.flags[i] << 32;
}

__global__ void k_copy_u64(const uint64_t *a, uint64_t *b, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = a[i];
}

}  // namespace

// ------------------------------------------------------------------ host launchers
static inline uint32_t nblk(uint64_t n, uint32_t t) { return (uint32_t)((n + t - 1) / t); }

// Exclusive scan of n u64 values (in place allowed for out == in? no: distinct).
// tmp must hold scan_tmp_words(n) u64.  Returns the total via *total (device->host).
uint64_t scan_tmp_words(uint64_t n) {
  uint64_t per = (uint64_t)SCAN_T * SCAN_PER, w = 0;
  while (n > 1) {
    n = (n + per - 1) / per;
    w += 2 * n + 2;
  }
  return w + 4;
}

hipError_t scan_exclusive_u64(const uint64_t *in, uint64_t *out, uint64_t n, uint64_t *tmp,
                              hipStream_t st) {
  if (n == 0) return hipSuccess;
  const uint64_t per = (uint64_t)SCAN_T * SCAN_PER;
  const uint64_t nb = (n + per - 1) / per;
  uint64_t *sums = tmp, *pref = tmp + nb + 1;
  hipLaunchKernelGGL(k_scan_local, dim3((uint32_t)nb), dim3(SCAN_T), 0, st, in, out, sums, n);
  if (nb > 1) {
    hipError_t e = scan_exclusive_u64(sums, pref, nb, tmp + 2 * nb + 2, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_scan_add, dim3((uint32_t)nb), dim3(SCAN_T), 0, st, out, pref, n);
  }
  return hipGetLastError();
}

hipError_t launch_find_block_start(const uint8_t *comp, uint64_t n, uint64_t start, int32_t k,
                                   int at_eof, unsigned long long *best, hipStream_t st) {
  hipLaunchKernelGGL(k_find_block_start, dim3(65536 / 256), dim3(256), 0, st, comp, n, start, k,
                     at_eof, best);
  return hipGetLastError();
}

uint64_t cand_chunks(uint64_t n) { return (n + CHUNK - 1) / CHUNK; }

hipError_t launch_cand_count(const uint8_t *comp, uint64_t n, uint64_t from, uint64_t *counts, uint32_t *first,
                             uint64_t nchunks, hipStream_t st) {
  const uint64_t grid = (nchunks + CAND_CPW - 1) / CAND_CPW;
  if (grid) hipLaunchKernelGGL(k_cand_count, dim3((uint32_t)grid), dim3(256), 0, st, comp, n, from, counts, first, nchunks);
  return hipGetLastError();
}
hipError_t launch_cand_write(const uint8_t *comp, uint64_t n, uint64_t from, const uint64_t *counts,
                             const uint32_t *first, const uint64_t *offs, uint64_t *cand, uint64_t nchunks,
                             hipStream_t st) {
  hipLaunchKernelGGL(k_cand_write, dim3((uint32_t)nchunks), dim3(256), 0, st, comp, n, from, counts, first,
                     offs, cand);
  return hipGetLastError();
}

// Build the chain from the candidate at start_rel over nc candidates.  Scratch: J0, J1 (int64 x
// nc), on (u8 x nc), v/rank (u64 x nc each), tmp (scan).  Writes the block table and usz (u64
// per block, zero past the chain); the block count is rank[nc - 1] + v[nc - 1] (no host round
// trip here: the caller copies those two words back with the block table).
hipError_t launch_pack_blocks(DevBlocks bl, uint64_t n, uint64_t file_off, uint64_t *out, hipStream_t st,
                              const uint64_t *rank, const uint64_t *v, const uint64_t *next18) {
  if (n) hipLaunchKernelGGL(k_pack_blocks, dim3(nblk(n, 256)), dim3(256), 0, st, bl, n, file_off, out, rank, v, next18);
  return hipGetLastError();
}

hipError_t build_chain(const uint8_t *comp, uint64_t n, const uint64_t *cand, uint64_t nc, uint64_t start_rel,
                       int64_t *J0, int64_t *J1, uint8_t *on, uint64_t *v, uint64_t *rank, uint64_t *tmp,
                       DevBlocks bl, uint64_t *usz, uint8_t *next18, uint64_t *sidx, bool linear, hipStream_t st) {
  if (nc == 0) return hipSuccess;
  const uint32_t T = 256;
  hipLaunchKernelGGL(k_cand_link, dim3(nblk(nc, T)), dim3(T), 0, st, comp, n, cand, nc, J0, next18);
  hipError_t e = hipMemsetAsync(usz, 0, nc * sizeof(uint64_t), st);
  if (e != hipSuccess) return e;
  if (linear) {  // (3 launches instead of ~log2(nc) + 6)
    hipLaunchKernelGGL(k_linear_start, dim3(1), dim3(64), 0, st, cand, nc, start_rel, sidx);
    hipLaunchKernelGGL(k_linear_chain, dim3(nblk(nc, T)), dim3(T), 0, st, J0, sidx, on, v, rank, nc, next18);
  } else {
    e = hipMemsetAsync(on, 0, nc, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_mark_start, dim3(1), dim3(64), 0, st, cand, nc, start_rel, on);
    int64_t *a = J0, *b = J1;
    for (uint64_t span = 1; span < nc; span <<= 1) {
      hipLaunchKernelGGL(k_jump_round, dim3(nblk(nc, T)), dim3(T), 0, st, a, b, on, nc);
      int64_t *t = a;
      a = b;
      b = t;
    }
    hipLaunchKernelGGL(k_jump_mark, dim3(nblk(nc, T)), dim3(T), 0, st, a, on, nc);
    // ranks of marked nodes
    hipLaunchKernelGGL(k_mark_u64, dim3(nblk(nc, T)), dim3(T), 0, st, on, v, nc);
    e = scan_exclusive_u64(v, rank, nc, tmp, st);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_chain_emit, dim3(nblk(nc, T)), dim3(T), 0, st, comp, n, cand, on, rank, v, nc, bl, usz,
                     next18);
  return hipGetLastError();
}

}  // namespace sbh
