// crc.hip -- BGZF footer CRC32 check of inflated blocks on CDNA4.
//
// The reference never checks the CRC32 of a BGZF block (bgzf/.../block/Stream.scala:47-54
// reads ISIZE only); SURVEY 8d asks for it as the in-run proof that every inflated byte is
// right at full size.  zlib's CRC32 (reflected 0xEDB88320, pre/post inverted) is affine in
// the state: processing L bytes maps state s to T_L(s) ^ c, with T_L linear (the effect of
// L zero bytes) and c the result from state 0.  So one wave per block: lane i folds the
// i-th 1 KiB of the block from state 0 (table lookups in LDS), then lane 0 chains the
// segments with the 32x32 GF(2) matrix T_1024 and finishes the < 1 KiB tail serially.
#include "sbh_internal.h"

namespace sbh {
namespace {

constexpr uint32_t CRC_SEG = 1024;  // bytes per lane

__global__ __launch_bounds__(256) void k_block_crc(const uint8_t *__restrict__ comp, DevBlocks bl, uint64_t nblocks,
                                                   const uint8_t *__restrict__ U, unsigned long long *n_bad,
                                                   unsigned long long *first_bad) {
  __shared__ uint32_t tab[256];
  __shared__ uint32_t T[32];  // column j: T_1024 applied to state bit j
  const uint32_t t = threadIdx.x, lane = t & (WAVE - 1);
  {
    uint32_t c = t;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    tab[t] = c;  // blockDim.x == 256
  }
  __syncthreads();
  if (t < 32) {
    uint32_t s = 1u << t;
    for (uint32_t k = 0; k < CRC_SEG; ++k) s = tab[s & 0xff] ^ (s >> 8);
    T[t] = s;
  }
  __syncthreads();
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x / WAVE);
  for (uint64_t b = (uint64_t)blockIdx.x * (blockDim.x / WAVE) + t / WAVE; b < nblocks; b += nw) {
    if (bl.flags[b] & BLK_TRUNCATED) continue;
    const uint32_t usize = bl.usize[b];
    const uint8_t *src = U + bl.ustart[b];
    const uint32_t nseg = usize / CRC_SEG;  // full segments (<= 64)
    uint32_t c = 0;
    if (lane < nseg) {
      const uint8_t *q = src + (uint64_t)lane * CRC_SEG;
      const uint32_t *g = reinterpret_cast<const uint32_t *>((uintptr_t)q & ~(uintptr_t)3);
      const uint32_t sh = (uint32_t)((uintptr_t)q & 3);
      uint32_t lo = g[0];  // (each dword loaded once: the high one of a step is the next step's low one)
#pragma unroll 8
      for (uint32_t k = 0; k < CRC_SEG; k += 4) {
        const uint32_t hi = g[k / 4 + 1];
        const uint32_t w = __builtin_amdgcn_alignbyte(hi, lo, sh);  // bytes q[k .. k+3]
        lo = hi;
        c = tab[(c ^ w) & 0xff] ^ (c >> 8);
        c = tab[(c ^ (w >> 8)) & 0xff] ^ (c >> 8);
        c = tab[(c ^ (w >> 16)) & 0xff] ^ (c >> 8);
        c = tab[(c ^ (w >> 24)) & 0xff] ^ (c >> 8);
      }
    }
    // lane 0: s = ~0; for each segment s = T(s) ^ c_i; then the tail
    uint32_t s = 0xffffffffu;
    for (uint32_t i = 0; i < nseg; ++i) {
      const uint32_t ci = __shfl(c, i);
      uint32_t r = 0;
      for (uint32_t j = 0; j < 32; ++j)
        if ((s >> j) & 1u) r ^= T[j];
      s = r ^ ci;
    }
    if (lane == 0) {
      for (uint32_t k = nseg * CRC_SEG; k < usize; ++k) s = tab[(s ^ src[k]) & 0xff] ^ (s >> 8);
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
  hipLaunchKernelGGL(k_block_crc, dim3(g), dim3(256), 0, st, comp, bl, nblocks, U, n_bad, first_bad);
  return hipGetLastError();
}

}  // namespace sbh
