// deflate.hip -- BGZF writer on CDNA4 (htsjdk-rewrite's block compressor).
//
// The flat uncompressed stream is already resident in HBM (an inflated shard, or bytes the
// caller uploaded).  k_deflate: one lane per 65498-byte piece, each lane runs the serial
// greedy-LZ77 / fixed-Huffman coder of deflate_core.h into its own 64 KiB slot (hash heads
// in a per-block HBM scratch, CRC table in LDS) and records the member size.  The host turns
// the sizes into file offsets; k_gather then packs the slots into the contiguous BGZF file,
// one workgroup per member with 16-byte stores where the destination allows.
#define SBH_HD __host__ __device__
#include "deflate_core.h"
#include "sbh_internal.h"

namespace sbh {
namespace {

using namespace sbh_deflate;

__global__ __launch_bounds__(64) void k_deflate(const uint8_t *__restrict__ src, uint64_t n, uint64_t nblocks,
                                                uint8_t *__restrict__ slots, uint16_t *__restrict__ heads,
                                                uint32_t *__restrict__ sizes) {
  __shared__ uint32_t tab[256];
  for (uint32_t t = threadIdx.x; t < 256; t += blockDim.x) {
    uint32_t c = t;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    tab[t] = c;
  }
  __syncthreads();
  const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblocks) return;
  const uint64_t s0 = b * PAYLOAD;
  const uint32_t len = (uint32_t)((n - s0) < PAYLOAD ? (n - s0) : PAYLOAD);
  sizes[b] = bgzf_block(src + s0, len, slots + b * SLOT, heads + b * HSIZE, tab);
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

hipError_t launch_deflate(const uint8_t *src, uint64_t n, uint8_t *slots, uint16_t *heads, uint32_t *sizes,
                          hipStream_t st) {
  const uint64_t nb = deflate_nblocks(n);
  if (!nb) return hipSuccess;
  hipError_t e = hipMemsetAsync(heads, 0, nb * HSIZE * sizeof(uint16_t), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_deflate, dim3((uint32_t)((nb + 63) / 64)), dim3(64), 0, st, src, n, nb, slots, heads, sizes);
  return hipGetLastError();
}

hipError_t launch_deflate_gather(const uint8_t *slots, const uint32_t *sizes, const uint64_t *offs, uint64_t nblocks,
                                 uint8_t *out, hipStream_t st) {
  if (!nblocks) return hipSuccess;
  hipLaunchKernelGGL(k_gather, dim3((uint32_t)nblocks), dim3(256), 0, st, slots, sizes, offs, nblocks, out);
  return hipGetLastError();
}

}  // namespace sbh
