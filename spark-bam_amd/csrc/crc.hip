// crc.hip -- BGZF footer CRC32 check of inflated blocks on CDNA4.
//
// The reference never checks the CRC32 of a BGZF block (bgzf/.../block/Stream.scala:47-54
// reads ISIZE only); SURVEY 8d asks for it as the in-run proof that every inflated byte is
// right at full size.  zlib's CRC32 (reflected 0xEDB88320, pre/post inverted) is linear in
// the register once the pre-inversion is moved into the message (the register's 4 bytes XORed
// into the first 4 message bytes, then a zero register), and a segment b after a segment a
// combines as crc(a || b) = T_|b|(crc(a)) ^ crc(b), T_L the 32x32 GF(2) matrix of L zero bytes.
//
// One 256-thread workgroup per block: the block is read as 256 segments of 256 bytes ending
// exactly at the block's last byte (the first segment padded in front with zeros, which leave a
// zero register unchanged), lane i folding segment i from a zero register -- 16-byte loads, one
// table lookup per byte in a 32-way replicated table (lane l reads copy l mod 32: no bank
// conflicts) -- then the 256 partial CRCs are combined in a tree (log2 256 levels, matrices
// T_256 .. T_32768 built once per workgroup).
#include "sbh_internal.h"

namespace sbh {
namespace {

constexpr uint32_t CRC_THREADS = 256;
constexpr uint32_t CRC_SEG = 256;       // bytes per lane: CRC_THREADS * CRC_SEG = 65536 >= any ISIZE
constexpr uint32_t CRC_LEVELS = 8;      // log2(CRC_THREADS)

struct CrcSmem {
  uint32_t tab[256 * 32];         // tab[b * 32 + r]: the byte table, replica r
  uint32_t mat[CRC_LEVELS][32];   // mat[l][j]: T_{256 << l} applied to register bit j
  uint32_t part[CRC_THREADS / WAVE];
};

// r <- M(x) for the matrix whose column j is lane j's `col` (lanes 0..31 of the wave)
__device__ __forceinline__ uint32_t mat_apply(uint32_t x, uint32_t col) {
  uint32_t r = 0;
#pragma unroll
  for (uint32_t j = 0; j < 32; ++j) {
    const uint32_t cj = __builtin_amdgcn_readlane(col, j);
    r ^= ((x >> j) & 1u) ? cj : 0u;
  }
  return r;
}

__device__ __forceinline__ uint32_t mat_apply_serial(uint32_t x, const uint32_t *M) {
  uint32_t r = 0;
  for (uint32_t j = 0; j < 32; ++j) r ^= ((x >> j) & 1u) ? M[j] : 0u;
  return r;
}

template <uint32_t M4>
__device__ __forceinline__ uint32_t fold_segment(const uint32_t (&W)[68], uint32_t mb, int32_t o0, const uint32_t *tab,
                                                 uint32_t rep) {
  // dword j of the segment = bytes [4j + 4*M4 + mb, +4) of the loaded window; message offset
  // o0 + 4j (< 0: front padding -> zero bytes; in [0, 4): the register's pre-inversion)
  uint32_t c = 0;
#pragma unroll
  for (uint32_t j = 0; j < 64; ++j) {
    uint32_t w = __builtin_amdgcn_alignbyte(W[j + M4 + 1], W[j + M4], mb);
    const int32_t o = o0 + 4 * (int32_t)j;
    if (o < 4) {  // (only the first segments of a block: a uniform branch per dword)
      // bytes k of this dword sit at message offset o + k: zero where < 0, and the pre-inversion
      // (0xff) on offsets 0..3
      const uint32_t keep = o <= -4 ? 0u : o < 0 ? 0xffffffffu << (8 * -o) : 0xffffffffu;
      const uint32_t inv = o >= 0 ? 0xffffffffu >> (8 * o) : keep;
      w = (w & keep) ^ inv;
    }
    c = tab[(((c ^ w) & 0xffu) << 5) + rep] ^ (c >> 8);
    c = tab[(((c ^ (w >> 8)) & 0xffu) << 5) + rep] ^ (c >> 8);
    c = tab[(((c ^ (w >> 16)) & 0xffu) << 5) + rep] ^ (c >> 8);
    c = tab[(((c ^ (w >> 24)) & 0xffu) << 5) + rep] ^ (c >> 8);
  }
  return c;
}

__global__ __launch_bounds__(CRC_THREADS) void k_block_crc(const uint8_t *__restrict__ comp, DevBlocks bl,
                                                           uint64_t nblocks, const uint8_t *__restrict__ U,
                                                           unsigned long long *n_bad,
                                                           unsigned long long *first_bad) {
  __shared__ CrcSmem sm;
  const uint32_t t = threadIdx.x, lane = t & (WAVE - 1), wv = t / WAVE;
  {  // the byte table, 32 replicas (entry b of replica r at b * 32 + r)
    uint32_t c = t;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    for (uint32_t r = 0; r < 32; ++r) sm.tab[t * 32 + r] = c;
  }
  __syncthreads();
  // T_256 column j (lanes 0..31 of wave 0), then T_512 = T_256 o T_256, ...
  if (t < 32) {
    uint32_t s = 1u << t;
    for (uint32_t k = 0; k < CRC_SEG; ++k) s = sm.tab[((s & 0xffu) << 5) + t] ^ (s >> 8);
    sm.mat[0][t] = s;
  }
  if (wv == 0) {
    for (uint32_t l = 1; l < CRC_LEVELS; ++l) {
      const uint32_t col = sm.mat[l - 1][lane & 31];  // (wave-synchronous: the writes above are this wave's)
      const uint32_t sq = mat_apply(col, col);
      if (lane < 32) sm.mat[l][lane] = sq;
    }
  }
  __syncthreads();
  uint32_t mcol[CRC_LEVELS];
#pragma unroll
  for (uint32_t l = 0; l < CRC_LEVELS; ++l) mcol[l] = sm.mat[l][lane & 31];
  const uint32_t rep = lane & 31;
  for (uint64_t b = blockIdx.x; b < nblocks; b += gridDim.x) {
    const uint32_t usize = bl.usize[b];
    if (bl.flags[b] & BLK_TRUNCATED) continue;  // (uniform)
    const uint64_t a0 = (uint64_t)(uintptr_t)(U + bl.ustart[b]);
    // segment t = message bytes [o0, o0 + 256), o0 = 256 t - (65536 - usize); its first byte's
    // address A = a0 + o0, loaded from aligned16(A) with the uniform shift m = A & 15
    const int32_t o0 = (int32_t)(CRC_SEG * t) - (int32_t)(65536u - usize);
    const uint64_t A = a0 + (uint64_t)(int64_t)o0;
    const uint32_t m = (uint32_t)(A & 15);
    uint32_t c = 0;
    if (usize >= 4 && o0 + (int32_t)CRC_SEG > 0) {
      uint32_t W[68];
      const uint4 *g = reinterpret_cast<const uint4 *>(A - m);
#pragma unroll
      for (uint32_t q = 0; q < 17; ++q) {
        // 16-byte pieces wholly before the block are front padding (never read: they may lie
        // before the buffer); the last piece reaches at most 15 bytes past the block (U's pad)
        const int32_t qo = o0 - (int32_t)m + 16 * (int32_t)q;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (qo + 16 > 0) v = g[q];
        W[4 * q] = v.x, W[4 * q + 1] = v.y, W[4 * q + 2] = v.z, W[4 * q + 3] = v.w;
      }
      const uint32_t mb = m & 3;
      switch (m >> 2) {
        case 0: c = fold_segment<0>(W, mb, o0, sm.tab, rep); break;
        case 1: c = fold_segment<1>(W, mb, o0, sm.tab, rep); break;
        case 2: c = fold_segment<2>(W, mb, o0, sm.tab, rep); break;
        default: c = fold_segment<3>(W, mb, o0, sm.tab, rep); break;
      }
    }
    // combine: at level l, lane pairs (2k, 2k+1) of groups of 2^l segments -> the right group is
    // 256 << l bytes long: crc(left || right) = T_{256 << l}(crc(left)) ^ crc(right)
#pragma unroll
    for (uint32_t l = 0; l < 6; ++l) {
      const uint32_t other = __shfl_xor(c, 1u << l);
      const uint32_t left = (lane >> l) & 1u ? other : c, right = (lane >> l) & 1u ? c : other;
      c = mat_apply(left, mcol[l]) ^ right;
    }
    if (lane == 0) sm.part[wv] = c;
    __syncthreads();
    if (t == 0) {
      uint32_t s = sm.part[0];
      s = mat_apply_serial(s, sm.mat[6]) ^ sm.part[1];
      const uint32_t s2 = mat_apply_serial(sm.part[2], sm.mat[6]) ^ sm.part[3];
      s = mat_apply_serial(s, sm.mat[7]) ^ s2;
      if (usize > 0 && usize < 4) {  // (too short for the folded pre-inversion: bytewise)
        s = 0xffffffffu;
        for (uint32_t k = 0; k < usize; ++k) s = sm.tab[(((s ^ U[bl.ustart[b] + k]) & 0xffu) << 5)] ^ (s >> 8);
        s ^= 0xffffffffu;
      }
      const uint32_t crc = usize >= 4 ? s ^ 0xffffffffu : usize ? s ^ 0u : 0u;
      const uint8_t *f = comp + bl.cstart[b] + bl.csize[b] - 8;  // footer: CRC32, ISIZE
      const uint32_t want = (uint32_t)f[0] | (uint32_t)f[1] << 8 | (uint32_t)f[2] << 16 | (uint32_t)f[3] << 24;
      if (crc != want) {
        atomicAdd(n_bad, 1ull);
        atomicMin(first_bad, (unsigned long long)b);
      }
    }
    __syncthreads();  // (sm.part is reused by the next block)
  }
}

}  // namespace

hipError_t launch_block_crc(const uint8_t *comp, DevBlocks bl, uint64_t nblocks, const uint8_t *U,
                            unsigned long long *n_bad, unsigned long long *first_bad, hipStream_t st) {
  if (!nblocks) return hipSuccess;
  // persistent-ish: each workgroup builds its tables once and takes every g-th block
  const uint32_t g = (uint32_t)(nblocks < 1024 ? nblocks : 1024);
  hipLaunchKernelGGL(k_block_crc, dim3(g), dim3(CRC_THREADS), 0, st, comp, bl, nblocks, U, n_bad, first_bad);
  return hipGetLastError();
}

}  // namespace sbh
