// calib_counters.hip -- FETCH_SIZE / WRITE_SIZE calibration for the access widths of the inflate
// pair (MI355X_MICROARCH.md, HBM section: the counters are calibrated only for 16-byte-per-lane
// streaming; "calibrate on a known byte count in your own access pattern before trusting an
// absolute").  Each kernel moves a known number of bytes in one of the path's patterns, over
// 1 GiB buffers (4x the 256 MiB Infinity Cache, so nothing is served on-die):
//
//   k_cal_read16    16 B per lane, coalesced loads                 (the guide's reference read)
//   k_cal_write16   16 B per lane, coalesced stores                (k_lz's image store, k_eager)
//   k_cal_runs4     k_huff's token stores: 256 lanes per 64 KiB region, each lane a run of
//                   4-byte stores through its own 256-byte slice (lane stride 256 B: every wave
//                   instruction touches 64 lines)
//   k_cal_runs2     the same with 2-byte stores (a 16-bit-per-code token format)
//   k_cal_tok12     k_lz's token loads: 512 threads, 3 consecutive dwords per thread per chunk
//                   (12 B per lane, the wave's 768 bytes contiguous)
//   k_cal_tok8      2 consecutive dwords + the next thread's first u16 (a 16-bit format's chunk)
//
// Run each counter in its own pass (tools/calib_counters.sh); tools/calib_report.py divides the
// counter by the known bytes per kernel.  Not part of the library or the product path.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

constexpr uint64_t BYTES = 1ull << 30;
constexpr uint32_t REGION = 65536;  // bytes per workgroup region (a BGZF block's token span)

__global__ __launch_bounds__(256) void k_cal_read16(const uint4 *__restrict__ a, uint32_t *out) {
  const uint64_t n = BYTES / 16;
  uint32_t s = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    s ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (s == 0x12345678u) out[0] = s;  // (keeps the loads)
}

__global__ __launch_bounds__(256) void k_cal_write16(uint4 *__restrict__ a) {
  const uint64_t n = BYTES / 16;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    a[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

// one workgroup per 64 KiB region; lane l stores words [64 l, 64 l + 64) of it in order
__global__ __launch_bounds__(256) void k_cal_runs4(uint32_t *__restrict__ a) {
  uint32_t *r = a + (uint64_t)blockIdx.x * (REGION / 4) + 64u * threadIdx.x;
  for (uint32_t i = 0; i < 64; ++i) r[i] = i ^ threadIdx.x;
}

__global__ __launch_bounds__(256) void k_cal_runs2(uint16_t *__restrict__ a) {
  uint16_t *r = a + (uint64_t)blockIdx.x * (REGION / 2) + 128u * threadIdx.x;
  for (uint32_t i = 0; i < 128; ++i) r[i] = (uint16_t)(i ^ threadIdx.x);
}

// one 512-thread workgroup per 64 KiB region, chunks of 1536 dwords (3 per thread)
__global__ __launch_bounds__(512) void k_cal_tok12(const uint32_t *__restrict__ a, uint32_t *out) {
  const uint32_t *r = a + (uint64_t)blockIdx.x * (REGION / 4);
  uint32_t s = 0;
  for (uint32_t c = 0; c < REGION / 4; c += 1536)
    for (uint32_t k = 0; k < 3; ++k) {
      const uint32_t i = c + 3 * threadIdx.x + k;
      if (i < REGION / 4) s ^= r[i];
    }
  if (s == 0x12345678u) out[blockIdx.x] = s;
}

__global__ __launch_bounds__(512) void k_cal_tok8(const uint16_t *__restrict__ a, uint32_t *out) {
  const uint16_t *r = a + (uint64_t)blockIdx.x * (REGION / 2);
  uint32_t s = 0;
  for (uint32_t c = 0; c < REGION / 2; c += 2048) {
    const uint32_t i = c + 4 * threadIdx.x;
    if (i + 4 <= REGION / 2) {
      const uint2 v = *reinterpret_cast<const uint2 *>(r + i);
      s ^= v.x ^ v.y;
    }
    if (i + 4 < REGION / 2) s ^= r[i + 4];
  }
  if (s == 0x12345678u) out[blockIdx.x] = s;
}

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

int main() {
  void *a = nullptr, *b = nullptr;
  uint32_t *out = nullptr;
  CK(hipMalloc(&a, BYTES));
  CK(hipMalloc(&b, BYTES));
  CK(hipMalloc(reinterpret_cast<void **>(&out), (BYTES / REGION) * 4));
  CK(hipMemset(a, 1, BYTES));
  CK(hipMemset(b, 2, BYTES));
  CK(hipDeviceSynchronize());
  const uint32_t regions = (uint32_t)(BYTES / REGION);
  for (int rep = 0; rep < 3; ++rep) {  // the counters take the median launch
    // (a and b alternate so no kernel reads what the previous one left in the caches)
    hipLaunchKernelGGL(k_cal_read16, dim3(8192), dim3(256), 0, 0, static_cast<const uint4 *>(a), out);
    hipLaunchKernelGGL(k_cal_write16, dim3(8192), dim3(256), 0, 0, static_cast<uint4 *>(b));
    hipLaunchKernelGGL(k_cal_runs4, dim3(regions), dim3(256), 0, 0, static_cast<uint32_t *>(a));
    hipLaunchKernelGGL(k_cal_tok12, dim3(regions), dim3(512), 0, 0, static_cast<const uint32_t *>(b), out);
    hipLaunchKernelGGL(k_cal_runs2, dim3(regions), dim3(256), 0, 0, static_cast<uint16_t *>(b));
    hipLaunchKernelGGL(k_cal_tok8, dim3(regions), dim3(512), 0, 0, static_cast<const uint16_t *>(a), out);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
  }
  // known bytes per launch (k_cal_tok8 reads the next thread's u16 too: one more u16 per thread
  // and chunk, inside the same lines)
  std::printf("{\"bytes\": {\"k_cal_read16\": %llu, \"k_cal_write16\": %llu, \"k_cal_runs4\": %llu, "
              "\"k_cal_runs2\": %llu, \"k_cal_tok12\": %llu, \"k_cal_tok8\": %llu}}\n",
              (unsigned long long)BYTES, (unsigned long long)BYTES, (unsigned long long)BYTES,
              (unsigned long long)BYTES, (unsigned long long)BYTES, (unsigned long long)BYTES);
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipFree(out));
  return 0;
}
