// deflate.hip -- BGZF writer on CDNA4 (htsjdk-rewrite's block compressor).
//
// The flat uncompressed stream is already resident in HBM (an inflated shard, or bytes the
// caller uploaded).  Members are coded in batches of up to DEFLATE_BATCH 65498-byte pieces,
// one workgroup (4 waves) per member, giving exactly the bytes of deflate_core.h's serial
// definition (tools/deflate_host.cpp):
//  k_prev     the hash chains prev[] of the member: each wave links a quarter of it, 64
//             positions a step (the step's (hash, lane) keys bitonic-sorted across the wave:
//             same-hash neighbours link, the first takes the wave's LDS head table entry),
//             then each quarter's first occurrence of a hash links to the quarters before;
//  k_deflate_parse  the member in LDS; each lane parses one 256-byte segment once into
//             tokens (batch scratch) and the member's histogram (LDS atomics);
//  k_deflate_codes  one 128-thread workgroup per member (small LDS, many per CU, so the
//             serial tree and header work of many members overlaps): symbol ranks over all
//             threads, the two trees on two waves, the header on one lane;
//  k_deflate_emit   the lanes' bit counts from their tokens and a workgroup scan give bit
//             offsets; the bits are written as whole dwords into the member's 64 KiB slot
//             (a lane's first and last dword, shared with its neighbours, through atomicOr);
//  k_footer   CRC32 + ISIZE;  k_gather  packs the slots at the host-computed file offsets.
#define SBH_HD __host__ __device__
#include "deflate_core.h"
#include "sbh_internal.h"

namespace sbh {
namespace {

using namespace sbh_deflate;

constexpr uint32_t QLEN = 16384;  // positions per wave in k_prev (a quarter of a member)
static_assert(4 * QLEN >= PAYLOAD, "four quarters cover a member");
constexpr uint32_t PREV_STRIDE = 65536;  // u16 prev[] entries per member in the batch scratch
constexpr uint32_t TOK_STRIDE = LSEG * NLANE;  // u32 tokens per member in the batch scratch

// prev[] of one member per workgroup.  Each wave links its quarter 64 positions a step: the
// step's (hash, lane) keys are sorted across the wave, so a position's predecessor inside
// the step is its sorted neighbour; the first of a hash in the step takes the wave's head
// table entry, the last one replaces it.  Then the first occurrence of each hash in a
// quarter is linked to the latest one in the quarters before it.
__global__ __launch_bounds__(256) void k_prev(const uint8_t *__restrict__ src, uint64_t n, uint64_t b0,
                                              uint64_t nblocks, uint16_t *__restrict__ prevg) {
  __shared__ uint16_t head[4][HN];   // latest position of each hash in the wave's quarter so far
  __shared__ uint16_t first[4][HN];  // first position of each hash in the quarter
  const uint32_t t = threadIdx.x, w = t / WAVE, lane = t % WAVE;
  const uint64_t b = b0 + blockIdx.x;
  if (b >= nblocks) return;
  const uint64_t s0 = b * PAYLOAD;
  const uint32_t len = (uint32_t)((n - s0) < PAYLOAD ? (n - s0) : PAYLOAD);
  const uint8_t *m = src + s0;
  uint16_t *pv = prevg + (uint64_t)blockIdx.x * PREV_STRIDE;
  for (uint32_t i = t; i < 4 * HN; i += 256) {
    (&head[0][0])[i] = NONE16;
    (&first[0][0])[i] = NONE16;
  }
  __syncthreads();
  const uint32_t hp = len >= 3 ? len - 2 : 0;  // positions with a hash (p + 3 <= len)
  const uint32_t qlo = w * QLEN, qhi = qlo + QLEN < len ? qlo + QLEN : len;
  // the step's three bytes are loaded one step ahead
  uint32_t c0 = 0, c1 = 0, c2 = 0;
  if (qlo + lane < hp) c0 = m[qlo + lane], c1 = m[qlo + lane + 1], c2 = m[qlo + lane + 2];
  for (uint32_t base = qlo; base < qhi; base += WAVE) {
    const uint32_t p = base + lane;
    const bool live = p < hp && p < qhi;
    const uint32_t v = c0 | c1 << 8 | c2 << 16;
    const uint32_t np = p + WAVE;
    if (np < hp && np < qhi) c0 = m[np], c1 = m[np + 1], c2 = m[np + 2];
    // dead lanes get keys past every hash, so they sort last
    const uint32_t h = live ? (v * 2654435761u) >> (32 - HB) : HN + lane;
    const uint32_t k = bitonic64(h << 6 | lane, lane);
    const uint32_t kp = (uint32_t)__shfl_up((int)k, 1), kn = (uint32_t)__shfl_down((int)k, 1);
    const uint32_t hs = k >> 6, ps = base + (k & 63);
    if (hs < HN) {
      uint16_t pr;
      if (lane > 0 && (kp >> 6) == hs) {
        pr = (uint16_t)(base + (kp & 63));
      } else {
        pr = head[w][hs];
        if (pr == NONE16) first[w][hs] = (uint16_t)ps;
      }
      pv[ps] = pr;
      if (lane == WAVE - 1 || (kn >> 6) != hs) head[w][hs] = (uint16_t)ps;
    } else if (ps < qhi) {
      pv[ps] = NONE16;
    }
  }
  __syncthreads();
  // a quarter's first occurrence of h links to the latest h of the quarters before it
  for (uint32_t i = t + HN; i < 4 * HN; i += 256) {
    const uint32_t q = i / HN, h = i % HN;
    const uint16_t f = first[q][h];
    if (f == NONE16) continue;
    for (int32_t r = (int32_t)q - 1; r >= 0; --r) {
      const uint16_t l = head[r][h];
      if (l != NONE16) {
        pv[f] = l;
        break;
      }
    }
  }
}

// Per-member records between the kernels (batch scratch, MEMBER_REC bytes per member):
// the lanes' token counts, the token histogram, then the codes, header bit count and header.
struct MemberRec {
  uint32_t ntok[NLANE];         // tokens of each lane's segment (k_deflate_parse)
  uint32_t fl[286], fd[30];     // histogram, fl[256] = 1 (k_deflate_parse)
  Codes cd;                     // (k_deflate_codes)
  uint32_t hbits;
  uint8_t hdr[HDR_CAP];
};
static_assert(sizeof(MemberRec) <= DEFLATE_REC_BYTES, "member record fits its scratch");

#ifdef SBH_DEFLATE_PROBE
// per-launch phase sums (cycles, thread 0 of each workgroup)
__device__ unsigned long long dp_acc[3][4];
__device__ unsigned int dp_done[3];
#define DP_INIT uint64_t dp_t = __builtin_readcyclecounter()
#define DP_MARK(kern, k)                                                  \
  do {                                                                    \
    if (threadIdx.x == 0) {                                               \
      const uint64_t nw = __builtin_readcyclecounter();                   \
      atomicAdd(&dp_acc[kern][k], (unsigned long long)(nw - dp_t));       \
      dp_t = nw;                                                          \
    }                                                                     \
  } while (0)
#define DP_DONE(kern, what)                                                                       \
  do {                                                                                            \
    if (threadIdx.x == 0) {                                                                       \
      __threadfence();                                                                            \
      if (atomicAdd(&dp_done[kern], 1u) == gridDim.x - 1) {                                       \
        unsigned long long x[4];                                                                  \
        for (int k = 0; k < 4; ++k) x[k] = atomicExch(&dp_acc[kern][k], 0ull);                    \
        dp_done[kern] = 0;                                                                        \
        const double m = (double)gridDim.x;                                                       \
        printf("deflateprobe %s members %u per-member cycles: %.0f %.0f %.0f %.0f\n", what, gridDim.x, \
               x[0] / m, x[1] / m, x[2] / m, x[3] / m);                                           \
      }                                                                                           \
    }                                                                                             \
  } while (0)
#else
#define DP_INIT
#define DP_MARK(kern, k) \
  do {                   \
  } while (0)
#define DP_DONE(kern, what) \
  do {                      \
  } while (0)
#endif

// (1) k_deflate_parse: the member into LDS, each lane's segment parsed once into tokens (batch
// scratch) and the member's histogram (LDS atomics), both written to the member record.
__global__ __launch_bounds__(256) void k_deflate_parse(const uint8_t *__restrict__ src, uint64_t n, uint64_t b0,
                                                       uint64_t nblocks, const uint16_t *__restrict__ prevg,
                                                       uint32_t *__restrict__ toks, uint8_t *__restrict__ recs) {
  __shared__ uint32_t ssrc[(SLOT + 8) / 4];  // the member's bytes, zero padded
  __shared__ uint32_t sfl[286 + 30];
  const uint32_t t = threadIdx.x;
  const uint64_t b = b0 + blockIdx.x;
  if (b >= nblocks) return;
  DP_INIT;
  const uint64_t s0 = b * PAYLOAD;
  const uint32_t len = (uint32_t)((n - s0) < PAYLOAD ? (n - s0) : PAYLOAD);
  const uint16_t *pv = prevg + (uint64_t)blockIdx.x * PREV_STRIDE;
  uint32_t *tk = toks + (uint64_t)blockIdx.x * TOK_STRIDE + t;  // token j of this lane: tk[j * NLANE]
  MemberRec &R = *reinterpret_cast<MemberRec *>(recs + (uint64_t)blockIdx.x * DEFLATE_REC_BYTES);
  // aligned source dwords (never past the buffer's last dword that holds data), realigned
  // with alignbyte, bytes past the member zeroed
  {
    const uint8_t *m = src + s0;
    const uintptr_t a0 = (uintptr_t)m & ~(uintptr_t)3;
    const uint32_t sh = (uint32_t)((uintptr_t)m & 3);
    const uintptr_t end = (uintptr_t)m + len;  // first address past the member
    const uintptr_t lim = (uintptr_t)(src + n);  // first address past the buffer
    for (uint32_t j = t; j < (SLOT + 8) / 4; j += 256) {
      uint32_t v = 0;
      if (4 * j < len) {
        const uintptr_t a = a0 + 4 * (uintptr_t)j;
        const uint32_t lo = *reinterpret_cast<const uint32_t *>(a);
        const uint32_t hi = a + 4 < lim ? *reinterpret_cast<const uint32_t *>(a + 4) : 0u;
        v = __builtin_amdgcn_alignbyte(hi, lo, sh);
        const uintptr_t p = (uintptr_t)m + 4 * (uintptr_t)j;  // first byte of this dword
        if (p + 4 > end) v &= (uint32_t)((1ull << (8 * (end - p))) - 1);
      }
      ssrc[j] = v;
    }
    for (uint32_t i = t; i < 286 + 30; i += 256) sfl[i] = i == 256 ? 1u : 0u;
  }
  __syncthreads();
  DP_MARK(0, 0);
  const auto ld = [&](uint32_t i) -> uint64_t {  // 8 bytes from byte i
    const uint32_t a = i >> 2, r = i & 3;
    const uint32_t x0 = ssrc[a], x1 = ssrc[a + 1], x2 = ssrc[a + 2];
    return (uint64_t)__builtin_amdgcn_alignbyte(x2, x1, r) << 32 | __builtin_amdgcn_alignbyte(x1, x0, r);
  };
  const auto prv = [&](uint32_t i) -> uint32_t { return pv[i]; };
  const uint32_t lo = t * LSEG, hi = lo + LSEG < len ? lo + LSEG : len;
  uint32_t ntok = 0;
  if (lo < len)
    parse_seg(ld, prv, lo, hi, [&](uint32_t tok) {
      tk[(ntok++) * NLANE] = tok;
      uint32_t ls;
      int32_t ds;
      tok_syms(tok, &ls, &ds);
      atomicAdd(&sfl[ls], 1u);
      if (ds >= 0) atomicAdd(&sfl[286 + ds], 1u);
    });
  R.ntok[t] = ntok;
  __syncthreads();
  DP_MARK(0, 1);
  for (uint32_t i = t; i < 286 + 30; i += 256) {
    if (i < 286) R.fl[i] = sfl[i];
    else R.fd[i - 286] = sfl[i];
  }
  DP_DONE(0, "parse (load, parse)");
}

// (2) k_deflate_codes: the member's dynamic Huffman codes and block header from its histogram,
// one 128-thread workgroup per member (symbol ranks over all threads, the two trees on two
// waves, the header on one lane), written to the member record.
struct CodesLds {
  uint32_t fl[286], fd[30];
  Codes cd;
  uint8_t hdr[HDR_CAP];
  HuffWork wl, wd;
  HdrWork H;
  uint32_t hbits;
};
__global__ __launch_bounds__(128) void k_deflate_codes(uint8_t *__restrict__ recs, uint32_t nbatch) {
  __shared__ CodesLds S;
  const uint32_t t = threadIdx.x;
  if (blockIdx.x >= nbatch) return;
  DP_INIT;
  MemberRec &R = *reinterpret_cast<MemberRec *>(recs + (uint64_t)blockIdx.x * DEFLATE_REC_BYTES);
  for (uint32_t i = t; i < 286 + 30; i += 128) {
    if (i < 286) S.fl[i] = R.fl[i];
    else S.fd[i - 286] = R.fd[i - 286];
  }
  __syncthreads();
  for (uint32_t i = t; i < 286 + 30; i += 128) {
    if (i < 286) {
      if (S.fl[i]) S.wl.sym[huff_rank(S.fl, 286, i)] = (uint16_t)i;
    } else if (S.fd[i - 286]) {
      S.wd.sym[huff_rank(S.fd, 30, i - 286)] = (uint16_t)(i - 286);
    }
  }
  __syncthreads();
  DP_MARK(1, 0);
  if (t == 0) huff_tree(S.fl, 286, 15, S.H.ll, S.wl);
  if (t == WAVE) huff_tree(S.fd, 30, 15, S.H.dl, S.wd);
  __syncthreads();
  DP_MARK(1, 1);
  if (t == 0) S.hbits = build_header(S.H, S.wl, S.cd, S.hdr);
  __syncthreads();
  DP_MARK(1, 2);
  for (uint32_t i = t; i < 286 + 30; i += 128) {
    if (i < 286) R.cd.lit[i] = S.cd.lit[i];
    else R.cd.dist[i - 286] = S.cd.dist[i - 286];
  }
  for (uint32_t i = t; i < HDR_CAP / 4; i += 128)
    reinterpret_cast<uint32_t *>(R.hdr)[i] = reinterpret_cast<const uint32_t *>(S.hdr)[i];
  if (t == 0) R.hbits = S.hbits;
  DP_DONE(1, "codes (ranks, trees, header)");
}

// Writes a lane's bit range into the slot as dwords: the first and last dword (shared with
// the neighbouring lanes' ranges) through atomicOr into the zeroed slot, the rest as stores.
struct DwordBits {
  uint32_t *base;
  uint32_t wi, nb;
  uint64_t acc;
  bool first;
  __device__ void put(uint32_t v, uint32_t k) {  // k <= 24
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
    put((uint32_t)v & 0xffffffu, k < 24 ? k : 24);
    if (k > 24) put((uint32_t)(v >> 24), k - 24);
  }
  __device__ void finish() {
    if (nb) atomicOr(base + wi, (uint32_t)acc);
  }
};

// (3) k_deflate_emit: each lane's bit count from its tokens, a workgroup scan for bit offsets,
// the bits written as whole dwords into the member's 64 KiB slot (a lane's first and last
// dword, shared with its neighbours, through atomicOr into the zeroed data dwords); the
// stored form when the coded member would not fit.
__global__ __launch_bounds__(256) void k_deflate_emit(const uint8_t *__restrict__ src, uint64_t n, uint64_t b0,
                                                      uint64_t nblocks, const uint32_t *__restrict__ toks,
                                                      const uint8_t *__restrict__ recs, uint8_t *__restrict__ slots,
                                                      uint32_t *__restrict__ sizes) {
  __shared__ Codes cd;
  __shared__ uint32_t hdr[HDR_CAP / 4];
  __shared__ uint32_t wsum[4];
  const uint32_t t = threadIdx.x, w = t / WAVE, lane = t % WAVE;
  const uint64_t b = b0 + blockIdx.x;
  if (b >= nblocks) return;
  DP_INIT;
  const uint64_t s0 = b * PAYLOAD;
  const uint32_t len = (uint32_t)((n - s0) < PAYLOAD ? (n - s0) : PAYLOAD);
  const uint32_t *tk = toks + (uint64_t)blockIdx.x * TOK_STRIDE + t;
  const MemberRec &R = *reinterpret_cast<const MemberRec *>(recs + (uint64_t)blockIdx.x * DEFLATE_REC_BYTES);
  uint8_t *slot = slots + (uint64_t)blockIdx.x * SLOT;
  for (uint32_t i = t; i < 286 + 30; i += 256) {
    if (i < 286) cd.lit[i] = R.cd.lit[i];
    else cd.dist[i - 286] = R.cd.dist[i - 286];
  }
  for (uint32_t i = t; i < HDR_CAP / 4; i += 256) hdr[i] = reinterpret_cast<const uint32_t *>(R.hdr)[i];
  const uint32_t ntok = R.ntok[t], hbits = R.hbits;
  const uint32_t last_seg = (len - 1) / LSEG;
  __syncthreads();
  uint32_t nbits = 0;
  for (uint32_t j = 0; j < ntok; ++j) {
    uint64_t v;
    nbits += tok_bits(tk[j * NLANE], cd, &v);
  }
  if (t == 0) nbits += hbits;
  if (t == last_seg) nbits += cd.lit[256] >> 16;
  uint32_t x = nbits;
  for (uint32_t d = 1; d < (uint32_t)WAVE; d <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, d);
    if (lane >= d) x += y;
  }
  if (lane == WAVE - 1) wsum[w] = x;
  __syncthreads();
  DP_MARK(2, 0);
  uint32_t off = x - nbits, total = 0;
  for (uint32_t k = 0; k < 4; ++k) {
    off += k < w ? wsum[k] : 0u;
    total += wsum[k];
  }
  uint32_t dsize = (total + 7) / 8;
  uint32_t *words = reinterpret_cast<uint32_t *>(slot);
  if (dsize <= BUDGET) {
    const uint32_t wend = (18 + dsize + 3) / 4;
    for (uint32_t i = 4 + t; i < wend; i += 256) words[i] = 0;
    __syncthreads();
    if (nbits) {
      const uint32_t bit0 = 8 * 18 + off;
      DwordBits o{words, bit0 / 32, bit0 % 32, 0, true};
      if (t == 0)
        for (uint32_t i = 0; i < hbits; i += 8)
          o.put((hdr[i / 32] >> (i % 32)) & 0xffu, hbits - i < 8 ? hbits - i : 8);
      for (uint32_t j = 0; j < ntok; ++j) {
        uint64_t v;
        const uint32_t k = tok_bits(tk[j * NLANE], cd, &v);
        o.put48(v, k);
      }
      if (t == last_seg) o.put(cd.lit[256] & 0xffff, cd.lit[256] >> 16);
      o.finish();
    }
  } else {
    dsize = stored_dsize(len);
    uint8_t *d0 = slot + 18;
    if (t == 0) put_stored_head(d0, len);
    for (uint32_t i = t; i < len; i += 256) d0[5 + i] = src[s0 + i];
  }
  __syncthreads();
  DP_MARK(2, 1);
  if (t == 0) {
    put_header(slot, 18 + dsize + 8);
    sizes[blockIdx.x] = 18 + dsize + 8;
  }
  DP_DONE(2, "emit (count+scan, emit)");
}

// Footer: CRC32 (one wave per member, 1 KiB per lane chained with the GF(2) matrix of 1024
// zero bytes, as in crc.hip) and ISIZE, at the member's end.
constexpr uint32_t CSEG = 1024;
__global__ __launch_bounds__(256) void k_footer(const uint8_t *__restrict__ src, uint64_t n, uint64_t b0,
                                                uint64_t nblocks, uint32_t nbatch, uint8_t *__restrict__ slots,
                                                uint64_t stride, const uint32_t *__restrict__ sizes) {
  __shared__ uint32_t tab[256];
  __shared__ uint32_t T[32];
  const uint32_t t = threadIdx.x, lane = t & (WAVE - 1);
  {
    uint32_t c = t;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    tab[t] = c;
  }
  __syncthreads();
  if (t < 32) {
    uint32_t s = 1u << t;
    for (uint32_t k = 0; k < CSEG; ++k) s = tab[s & 0xff] ^ (s >> 8);
    T[t] = s;
  }
  __syncthreads();
  const uint32_t j = blockIdx.x * (blockDim.x / WAVE) + t / WAVE;  // member within the batch
  const uint64_t b = b0 + j;
  if (j >= nbatch || b >= nblocks) return;
  const uint64_t s0 = b * PAYLOAD;
  const uint32_t len = (uint32_t)((n - s0) < PAYLOAD ? (n - s0) : PAYLOAD);
  const uint8_t *p = src + s0;
  const uint32_t nseg = len / CSEG;
  uint32_t c = 0;
  if (lane < nseg)
    for (uint32_t k = lane * CSEG; k < (lane + 1) * CSEG; ++k) c = tab[(c ^ p[k]) & 0xff] ^ (c >> 8);
  uint32_t s = 0xffffffffu;
  for (uint32_t q = 0; q < nseg; ++q) {
    const uint32_t cq = (uint32_t)__shfl((int)c, (int)q);
    uint32_t r = 0;
    for (uint32_t i = 0; i < 32; ++i)
      if ((s >> i) & 1u) r ^= T[i];
    s = r ^ cq;
  }
  if (lane == 0) {
    for (uint32_t k = nseg * CSEG; k < len; ++k) s = tab[(s ^ p[k]) & 0xff] ^ (s >> 8);
    uint8_t *f = slots + (uint64_t)j * stride + sizes[j] - 8;
    put_le32(f, s ^ 0xffffffffu);
    put_le32(f + 4, len);
  }
}

__global__ __launch_bounds__(256) void k_gather(const uint8_t *__restrict__ slots, uint64_t stride,
                                                const uint32_t *__restrict__ sizes, const uint64_t *__restrict__ offs,
                                                uint64_t nblocks, uint8_t *__restrict__ out) {
  const uint64_t b = blockIdx.x;
  if (b >= nblocks) return;
  const uint8_t *s = slots + b * stride;
  uint8_t *d = out + offs[b];
  const uint32_t m = sizes[b];
  const uint32_t head = (uint32_t)((16 - ((uintptr_t)d & 15)) & 15) < m ? (uint32_t)((16 - ((uintptr_t)d & 15)) & 15) : m;
  for (uint32_t i = threadIdx.x; i < head; i += blockDim.x) d[i] = s[i];
  // destination now 16-byte aligned; the source (slot base + head) is read as bytes packed
  // into 16-byte vectors (the slot stride is a multiple of 16, head < 16)
  const uint32_t nv = (m - head) / 16;
  for (uint32_t v = threadIdx.x; v < nv; v += blockDim.x) {
    const uint8_t *q = s + head + 16 * v;
    uint32_t w[4];
    for (int k = 0; k < 4; ++k)
      w[k] = (uint32_t)q[4 * k] | (uint32_t)q[4 * k + 1] << 8 | (uint32_t)q[4 * k + 2] << 16 |
             (uint32_t)q[4 * k + 3] << 24;
    *reinterpret_cast<uint4 *>(d + head + 16 * v) = make_uint4(w[0], w[1], w[2], w[3]);
  }
  for (uint32_t i = head + 16 * nv + threadIdx.x; i < m; i += blockDim.x) d[i] = s[i];
}

}  // namespace

uint64_t deflate_nblocks(uint64_t n) { return (n + PAYLOAD - 1) / PAYLOAD; }

hipError_t launch_deflate(const uint8_t *src, uint64_t n, uint64_t b0, uint32_t nbatch, uint16_t *prev,
                          uint32_t *toks, uint8_t *recs, uint8_t *slots, uint32_t *sizes, hipStream_t st) {
  const uint64_t nb = deflate_nblocks(n);
  if (!nbatch || b0 >= nb) return hipSuccess;
  if (nbatch > DEFLATE_BATCH || b0 + nbatch > nb) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_prev, dim3(nbatch), dim3(256), 0, st, src, n, b0, nb, prev);
  hipLaunchKernelGGL(k_deflate_parse, dim3(nbatch), dim3(256), 0, st, src, n, b0, nb, prev, toks, recs);
  hipLaunchKernelGGL(k_deflate_codes, dim3(nbatch), dim3(128), 0, st, recs, nbatch);
  hipLaunchKernelGGL(k_deflate_emit, dim3(nbatch), dim3(256), 0, st, src, n, b0, nb, toks, recs, slots, sizes);
  return launch_member_footer(src, n, b0, nb, nbatch, slots, SLOT, sizes, st);
}

hipError_t launch_member_footer(const uint8_t *src, uint64_t n, uint64_t b0, uint64_t nblocks, uint32_t nbatch,
                                uint8_t *slots, uint64_t stride, const uint32_t *sizes, hipStream_t st) {
  hipLaunchKernelGGL(k_footer, dim3((nbatch + 3) / 4), dim3(256), 0, st, src, n, b0, nblocks, nbatch, slots, stride,
                     sizes);
  return hipGetLastError();
}

hipError_t launch_deflate_gather(const uint8_t *slots, uint64_t stride, const uint32_t *sizes, const uint64_t *offs,
                                 uint64_t nblocks, uint8_t *out, hipStream_t st) {
  if (!nblocks) return hipSuccess;
  hipLaunchKernelGGL(k_gather, dim3((uint32_t)nblocks), dim3(256), 0, st, slots, stride, sizes, offs, nblocks, out);
  return hipGetLastError();
}

}  // namespace sbh
