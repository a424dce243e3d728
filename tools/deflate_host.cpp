// Host build of spark-bam_amd/csrc/deflate_core.h for the CPU test suite only: lets
// tests/test_deflate_cpu.py round-trip the device coder's exact algorithm through zlib
// without a GPU.  Not part of the product library (libsparkbam_hip.so runs it in k_deflate).
#include <stdint.h>
#include <string.h>
#include <vector>

#include "../spark-bam_amd/csrc/deflate_core.h"

using namespace sbh_deflate;

extern "C" uint64_t sbh_host_bgzf_compress(const uint8_t *src, uint64_t n, uint8_t *out) {
  uint32_t tab[256];
  for (uint32_t t = 0; t < 256; ++t) {
    uint32_t c = t;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    tab[t] = c;
  }
  std::vector<uint16_t> head(SHSIZE);
  std::vector<uint8_t> slot(SLOT), segbuf(NSEG * SEGCAP);
  uint64_t o = 0;
  for (uint64_t s = 0; s < n; s += PAYLOAD) {
    const uint32_t len = (uint32_t)(n - s < PAYLOAD ? n - s : PAYLOAD);
    std::fill(slot.begin(), slot.end(), 0);
    const uint32_t m = bgzf_block(src + s, len, slot.data(), segbuf.data(), head.data(), tab);
    memcpy(out + o, slot.data(), m);
    o += m;
  }
  put_eof(out + o);
  return o + EOF_SIZE;
}
