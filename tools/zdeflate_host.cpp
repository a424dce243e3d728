// Host build of spark-bam_amd/csrc/zdeflate_core.h for the CPU test suite only: the serial
// definition of the byte-exact (zlib 1.2.11 level 5) BGZF writer, checked against the
// container's zlib by tests/test_zdeflate_cpu.py.  Not part of the product library.
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../spark-bam_amd/csrc/zdeflate_core.h"

using namespace sbh_zlib;

static ZTreeState g_st;

extern "C" {

// raw deflate of src[0, n) (n <= 65536) as zlib writes it at level 4..9; returns its size
uint32_t sbh_host_zdeflate_raw(const uint8_t *src, uint32_t n, int level, uint8_t *out, uint32_t cap) {
  std::vector<uint16_t> prev(n + 1), head(HASH_MASK + 1);
  std::vector<uint32_t> tok(n + 1);
  std::vector<uint64_t> info(n + 1);
  return z_deflate_serial(src, n, level, out, cap, prev.data(), head.data(), tok.data(), info.data(), g_st);
}

}  // extern "C"
