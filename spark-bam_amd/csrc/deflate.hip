// deflate.hip -- BGZF writer on CDNA4 (htsjdk-rewrite's block compressor).
//
// The flat uncompressed stream is already resident in HBM (an inflated shard, or bytes the
// caller uploaded).  k_deflate: four 65498-byte pieces per wave, each runs the
// greedy-LZ77 / fixed-Huffman coder of deflate_core.h, one 4 KiB segment per lane, into
// the member's 64 KiB slot (hash heads and segment streams in HBM scratch) and records the
// member size; k_footer adds CRC32 + ISIZE.  The host turns
// the sizes into file offsets; k_gather then packs the slots into the contiguous BGZF file,
// one workgroup per member with 16-byte stores where the destination allows.
#define SBH_HD __host__ __device__
#include "deflate_core.h"
#include "sbh_internal.h"

namespace sbh {
namespace {

using namespace sbh_deflate;

// Four members per wave, one 4 KiB segment per lane (deflate_core.h seg_encode), the
// segment streams bit-concatenated in the zeroed slot: bytes a lane shares a dword with a
// neighbour (its first and last four) go through atomicOr, the rest are plain stores.
__global__ __launch_bounds__(64) void k_deflate(const uint8_t *__restrict__ src, uint64_t n, uint64_t nblocks,
                                                uint8_t *__restrict__ slots, uint8_t *__restrict__ segbuf,
                                                uint16_t *__restrict__ heads, uint32_t *__restrict__ sizes) {
  const uint32_t lane = threadIdx.x, g = lane / NSEG, i = lane % NSEG;
  const uint64_t b = (uint64_t)blockIdx.x * (64 / NSEG) + g;
  const bool live_blk = b < nblocks;
  const uint64_t s0 = b * PAYLOAD;
  const uint32_t len = live_blk ? (uint32_t)((n - s0) < PAYLOAD ? (n - s0) : PAYLOAD) : 0;
  const uint32_t nseg = (len + SEG - 1) / SEG;
  const uint32_t lo = i * SEG, slen = i < nseg ? ((len - lo) < SEG ? len - lo : SEG) : 0;
  uint8_t *buf = segbuf + (b * NSEG + i) * SEGCAP;
  uint32_t nbits = 0;
  if (slen) nbits = seg_encode(src + s0 + lo, slen, i + 1 == nseg, buf, heads + (b * NSEG + i) * SHSIZE);
  uint32_t off = 0, tot = 0;
  for (uint32_t k = 0; k < NSEG; ++k) {
    const uint32_t v = (uint32_t)__shfl((int)nbits, (int)(g * NSEG + k));
    off += k < i ? v : 0u;
    tot += v;
  }
  if (!live_blk) return;
  uint8_t *slot = slots + b * SLOT;
  uint8_t *d0 = slot + 18;
  uint32_t dsize = (tot + 7) / 8;
  if (dsize <= BUDGET) {
    if (slen) {
      const uint32_t first = off / 8, last = (off + nbits - 1) / 8;
      for (uint32_t j = first; j <= last; ++j) {
        const uint8_t v = seg_byte(buf, nbits, off, j);
        if (j < first + 4 || j + 4 > last) {
          const uintptr_t a = (uintptr_t)(d0 + j);
          if (v) atomicOr(reinterpret_cast<uint32_t *>(a & ~(uintptr_t)3), (uint32_t)v << (8 * (a & 3)));
        } else {
          d0[j] = v;
        }
      }
    }
  } else {
    dsize = stored_dsize(len);
    if (i == 0) put_stored_head(d0, len);
    for (uint32_t k = 0; k < slen; ++k) d0[5 + lo + k] = src[s0 + lo + k];
  }
  if (i == 0) {
    put_header(slot, 18 + dsize + 8);
    sizes[b] = 18 + dsize + 8;
  }
}

// Footer: CRC32 (one wave per member, 1 KiB per lane chained with the GF(2) matrix of 1024
// zero bytes, as in crc.hip) and ISIZE, at the member's end.
constexpr uint32_t CSEG = 1024;
__global__ __launch_bounds__(256) void k_footer(const uint8_t *__restrict__ src, uint64_t n, uint64_t nblocks,
                                                uint8_t *__restrict__ slots, const uint32_t *__restrict__ sizes) {
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
  const uint64_t b = (uint64_t)blockIdx.x * (blockDim.x / WAVE) + t / WAVE;
  if (b >= nblocks) return;
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
    for (uint32_t j = 0; j < 32; ++j)
      if ((s >> j) & 1u) r ^= T[j];
    s = r ^ cq;
  }
  if (lane == 0) {
    for (uint32_t k = nseg * CSEG; k < len; ++k) s = tab[(s ^ p[k]) & 0xff] ^ (s >> 8);
    uint8_t *f = slots + b * SLOT + sizes[b] - 8;
    put_le32(f, s ^ 0xffffffffu);
    put_le32(f + 4, len);
  }
}

__global__ __launch_bounds__(256) void k_gather(const uint8_t *__restrict__ slots, const uint32_t *__restrict__ sizes,
                                                const uint64_t *__restrict__ offs, uint64_t nblocks,
                                                uint8_t *__restrict__ out) {
  const uint64_t b = blockIdx.x;
  if (b >= nblocks) return;
  const uint8_t *s = slots + b * SLOT;
  uint8_t *d = out + offs[b];
  const uint32_t m = sizes[b];
  const uint32_t head = (uint32_t)((16 - ((uintptr_t)d & 15)) & 15) < m ? (uint32_t)((16 - ((uintptr_t)d & 15)) & 15) : m;
  for (uint32_t i = threadIdx.x; i < head; i += blockDim.x) d[i] = s[i];
  // destination now 16-byte aligned; the source (slot base + head) is read as bytes packed
  // into 16-byte vectors (the slot base is 64 KiB aligned, head < 16)
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

hipError_t launch_deflate(const uint8_t *src, uint64_t n, uint8_t *slots, uint8_t *segbuf, uint16_t *heads,
                          uint32_t *sizes, hipStream_t st) {
  const uint64_t nb = deflate_nblocks(n);
  if (!nb) return hipSuccess;
  hipError_t e = hipMemsetAsync(heads, 0, nb * NSEG * SHSIZE * sizeof(uint16_t), st);
  if (e == hipSuccess) e = hipMemsetAsync(slots, 0, nb * SLOT, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_deflate, dim3((uint32_t)((nb + 3) / 4)), dim3(64), 0, st, src, n, nb, slots, segbuf, heads,
                     sizes);
  hipLaunchKernelGGL(k_footer, dim3((uint32_t)((nb + 3) / 4)), dim3(256), 0, st, src, n, nb, slots, sizes);
  return hipGetLastError();
}

hipError_t launch_deflate_gather(const uint8_t *slots, const uint32_t *sizes, const uint64_t *offs, uint64_t nblocks,
                                 uint8_t *out, hipStream_t st) {
  if (!nblocks) return hipSuccess;
  hipLaunchKernelGGL(k_gather, dim3((uint32_t)nblocks), dim3(256), 0, st, slots, sizes, offs, nblocks, out);
  return hipGetLastError();
}

}  // namespace sbh
