// crc.hip -- BGZF footer CRC32 check of inflated blocks on CDNA4.
//
// The reference never checks the CRC32 of a BGZF block (bgzf/.../block/Stream.scala:47-54
// reads ISIZE only); SURVEY 8d asks for it as the in-run proof that every inflated byte is
// right at full size.  zlib's CRC32 (reflected 0xEDB88320, pre/post inverted) is affine in
// the state: processing L bytes maps state s to T_L(s) ^ c, with T_L linear (the effect of
// L zero bytes) and c the result from state 0.  So one wave per block: lane i folds the
// i-th 1 KiB of the block (lane nseg: the < 1 KiB tail) from state 0, eight bytes per
// dependent step (slicing-by-8 tables in LDS); the segment values combine pairwise in a
// six-level tree over the lanes, the left run shifted past the right one's length by the
// 32x32 GF(2) matrices T_{2^j} of that length's set bits (LDS columns, broadcast reads); lane 0
// applies T_usize to the initial state.
#include "sbh_internal.h"

namespace sbh {
namespace {

constexpr uint32_t CRC_SEG = 1024;  // bytes per lane
constexpr uint32_t CRC_POW = 17;    // T_{2^j}, j < 17 (a block holds at most 65536 bytes)
constexpr uint32_t CRC_T = 256;

// The slicing-by-8 tables (tab[k][b]: the register after byte b, then k zero bytes) and the
// shift matrices P[j] = T_{2^j}, computed at compile time; each workgroup copies them to LDS.
struct CrcTabs {
  uint32_t tab[8][256];
  uint32_t P[CRC_POW][32];
};
constexpr CrcTabs make_crc_tabs() {
  CrcTabs z{};
  for (uint32_t n = 0; n < 256; ++n) {
    uint32_t c = n;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    z.tab[0][n] = c;
  }
  for (uint32_t k = 1; k < 8; ++k)
    for (uint32_t n = 0; n < 256; ++n) z.tab[k][n] = z.tab[0][z.tab[k - 1][n] & 0xff] ^ (z.tab[k - 1][n] >> 8);
  for (uint32_t j = 0; j < 32; ++j) z.P[0][j] = z.tab[0][(1u << j) & 0xff] ^ ((1u << j) >> 8);  // one zero byte
  for (uint32_t l = 1; l < CRC_POW; ++l)  // T_{2L} = T_L o T_L
    for (uint32_t j = 0; j < 32; ++j) {
      uint32_t r = 0;
      for (uint32_t i = 0; i < 32; ++i)
        if ((z.P[l - 1][j] >> i) & 1u) r ^= z.P[l - 1][i];
      z.P[l][j] = r;
    }
  return z;
}
__device__ const CrcTabs kCrcTabs = make_crc_tabs();

// s -> T(s) for the matrix whose column j (the image of state bit j) is M[j]
__device__ __forceinline__ uint32_t gf2_apply(const uint32_t *M, uint32_t s) {
  uint32_t r = 0;
#pragma unroll
  for (uint32_t j = 0; j < 32; ++j) r ^= ((s >> j) & 1u) ? M[j] : 0u;
  return r;
}

// s shifted past n zero bytes: T_n = product of T_{2^j} over n's set bits
__device__ __forceinline__ uint32_t gf2_shift(const uint32_t (*P)[32], uint32_t s, uint32_t n) {
  for (uint32_t j = 0; n; ++j, n >>= 1)
    if (n & 1u) s = gf2_apply(P[j], s);
  return s;
}

__global__ __launch_bounds__(CRC_T) void k_block_crc(const uint8_t *__restrict__ comp, DevBlocks bl, uint64_t nblocks,
                                                     const uint8_t *__restrict__ U, unsigned long long *n_bad,
                                                     unsigned long long *first_bad) {
  __shared__ uint32_t tab[8][256];
  __shared__ uint32_t P[CRC_POW][32];  // P[j] = T_{2^j} (columns)
  const uint32_t t = threadIdx.x, lane = t & (WAVE - 1);
  for (uint32_t i = t; i < 8 * 256; i += CRC_T) (&tab[0][0])[i] = (&kCrcTabs.tab[0][0])[i];
  for (uint32_t i = t; i < CRC_POW * 32; i += CRC_T) (&P[0][0])[i] = (&kCrcTabs.P[0][0])[i];
  __syncthreads();
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x / WAVE);
  for (uint64_t b = (uint64_t)blockIdx.x * (blockDim.x / WAVE) + t / WAVE; b < nblocks; b += nw) {
    if (bl.flags[b] & BLK_TRUNCATED) continue;
    const uint32_t usize = bl.usize[b];
    const uint8_t *src = U + bl.ustart[b];
    const uint32_t nseg = usize / CRC_SEG;  // full segments (<= 64); lane nseg takes the tail
    const uint32_t len = lane < nseg ? CRC_SEG : lane == nseg ? usize - nseg * CRC_SEG : 0u;
    uint32_t c = 0;
    if (len) {
      const uint8_t *q = src + (uint64_t)lane * CRC_SEG;
      const uint32_t *g = reinterpret_cast<const uint32_t *>((uintptr_t)q & ~(uintptr_t)3);
      const uint32_t sh = (uint32_t)((uintptr_t)q & 3);
      const uint32_t n8 = len / 8;
      uint32_t w0 = g[0];
      for (uint32_t i = 0; i < n8; ++i) {
        const uint32_t w1 = g[2 * i + 1], w2 = g[2 * i + 2];
        const uint32_t a = __builtin_amdgcn_alignbyte(w1, w0, sh) ^ c;  // bytes q[8i .. 8i+3]
        const uint32_t d = __builtin_amdgcn_alignbyte(w2, w1, sh);      // bytes q[8i+4 .. 8i+7]
        c = tab[7][a & 0xff] ^ tab[6][(a >> 8) & 0xff] ^ tab[5][(a >> 16) & 0xff] ^ tab[4][a >> 24] ^
            tab[3][d & 0xff] ^ tab[2][(d >> 8) & 0xff] ^ tab[1][(d >> 16) & 0xff] ^ tab[0][d >> 24];
        w0 = w2;
      }
      for (uint32_t k = 8 * n8; k < len; ++k) c = tab[0][(c ^ q[k]) & 0xff] ^ (c >> 8);
    }
    // the runs combine in a tree: at level l, lane 2^(l+1) i absorbs lane 2^(l+1) i + 2^l's
    // run (bytes rr, possibly 0): value = T_rr(left) ^ right
    uint32_t run = len;
#pragma unroll
    for (uint32_t l = 0; l < 6; ++l) {
      const uint32_t o = 1u << l;
      const uint32_t cr = __shfl_down(c, o, WAVE), rr = __shfl_down(run, o, WAVE);
      if ((lane & (2 * o - 1)) == 0 && lane + o < WAVE && rr) {
        c = gf2_shift(P, c, rr) ^ cr;
        run += rr;
      }
    }
    if (lane == 0) {
      const uint32_t s = gf2_shift(P, 0xffffffffu, usize) ^ c;  // from the initial state ~0
      const uint8_t *f = comp + bl.cstart[b] + bl.csize[b] - 8;  // footer: CRC32, ISIZE
      const uint32_t want = (uint32_t)f[0] | (uint32_t)f[1] << 8 | (uint32_t)f[2] << 16 | (uint32_t)f[3] << 24;
      if ((s ^ 0xffffffffu) != want) {
        atomicAdd(n_bad, 1ull);
        atomicMin(first_bad, (unsigned long long)b);
      }
    }
  }
}

}  // namespace

hipError_t launch_block_crc(const uint8_t *comp, DevBlocks bl, uint64_t nblocks, const uint8_t *U,
                            unsigned long long *n_bad, unsigned long long *first_bad, hipStream_t st) {
  if (!nblocks) return hipSuccess;
  const uint32_t g = (uint32_t)((nblocks + 3) / 4 < 16384 ? (nblocks + 3) / 4 : 16384);
  hipLaunchKernelGGL(k_block_crc, dim3(g), dim3(CRC_T), 0, st, comp, bl, nblocks, U, n_bad, first_bad);
  return hipGetLastError();
}

}  // namespace sbh
