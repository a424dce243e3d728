// Host build of spark-bam_amd/csrc/deflate_core.h for the CPU test suite only: the serial
// definition of the writer's coder (the GPU's k_deflate must give the same bytes), round-tripped
// through zlib by tests/test_deflate_cpu.py without a GPU.  Not part of the product library.
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../spark-bam_amd/csrc/deflate_core.h"

using namespace sbh_deflate;

// One member of n <= PAYLOAD bytes into out (SLOT zeroed bytes); returns its size.  hl / hd
// (optional): add the member's lit/len and distance symbol counts when it is coded (not stored).
static uint32_t member(const uint8_t *src, uint32_t n, uint8_t *out, const uint32_t *crctab, uint64_t *hl = nullptr,
                       uint64_t *hd = nullptr) {
  std::vector<uint8_t> pad(n + 8, 0);  // 8-byte loads run up to 7 bytes past the data
  memcpy(pad.data(), src, n);
  std::vector<uint16_t> prev(n + 1, NONE16), head(HN, NONE16);
  for (uint32_t p = 0; p + 3 <= n; ++p) {
    const uint32_t h = hash3(src + p);
    prev[p] = head[h];
    head[h] = (uint16_t)p;
  }
  auto ld = [&](uint32_t i) {
    uint64_t v;
    memcpy(&v, pad.data() + i, 8);
    return v;
  };
  auto pv = [&](uint32_t i) -> uint32_t { return prev[i]; };
  std::vector<uint32_t> toks;
  for (uint32_t lo = 0; lo < n; lo += LSEG)
    parse_seg(ld, pv, lo, lo + LSEG < n ? lo + LSEG : n, [&](uint32_t t) { toks.push_back(t); });
  uint32_t fl[286] = {0}, fd[30] = {0};
  for (uint32_t t : toks) {
    uint32_t ls;
    int32_t ds;
    tok_syms(t, &ls, &ds);
    fl[ls]++;
    if (ds >= 0) fd[ds]++;
  }
  fl[256]++;
  static Codes cd;
  static HuffWork wl, wd;
  static HdrWork hw;
  uint8_t hdr[HDR_CAP] = {0};
  const uint32_t hbits = build_codes(fl, fd, cd, hdr, wl, wd, hw);
  uint64_t nbits = hbits + (cd.lit[256] >> 16);
  for (uint32_t t : toks) {
    uint64_t v;
    nbits += tok_bits(t, cd, &v);
  }
  uint8_t *d0 = out + 18;
  uint32_t dsize = (uint32_t)((nbits + 7) / 8);
  if (dsize <= BUDGET) {
    if (hl && hd) {
      for (uint32_t i = 0; i < 286; ++i) hl[i] += fl[i];
      for (uint32_t i = 0; i < 30; ++i) hd[i] += fd[i];
    }
    Bits b{d0, 0, 0};
    for (uint32_t i = 0; i < hbits; i += 8) b.put(hdr[i / 8], hbits - i < 8 ? hbits - i : 8);
    for (uint32_t t : toks) {
      uint64_t v;
      uint32_t k = tok_bits(t, cd, &v);
      b.put((uint32_t)v & 0xffffff, k < 24 ? k : 24);
      if (k > 24) b.put((uint32_t)(v >> 24), k - 24);
    }
    b.put(cd.lit[256] & 0xffff, cd.lit[256] >> 16);
    b.flush();
  } else {
    dsize = stored_dsize(n);
    put_stored_head(d0, n);
    memcpy(d0 + 5, src, n);
  }
  const uint32_t total = 18 + dsize + 8;
  put_header(out, total);
  put_le32(d0 + dsize, crc32_bytes(src, n, crctab));
  put_le32(d0 + dsize + 4, n);
  return total;
}

extern "C" uint64_t sbh_host_bgzf_compress(const uint8_t *src, uint64_t n, uint8_t *out) {
  uint32_t tab[256];
  for (uint32_t t = 0; t < 256; ++t) {
    uint32_t c = t;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    tab[t] = c;
  }
  std::vector<uint8_t> slot(SLOT);
  uint64_t o = 0;
  for (uint64_t s = 0; s < n; s += PAYLOAD) {
    const uint32_t len = (uint32_t)(n - s < PAYLOAD ? n - s : PAYLOAD);
    std::fill(slot.begin(), slot.end(), 0);
    const uint32_t m = member(src + s, len, slot.data(), tab);
    memcpy(out + o, slot.data(), m);
    o += m;
  }
  put_eof(out + o);
  return o + EOF_SIZE;
}

// Symbol statistics of the coder over src (tests: which length / distance codes it emits).
extern "C" void sbh_host_bgzf_symstats(const uint8_t *src, uint64_t n, uint64_t *lit_hist, uint64_t *dist_hist) {
  uint32_t tab[256];
  for (uint32_t t = 0; t < 256; ++t) {
    uint32_t c = t;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    tab[t] = c;
  }
  std::vector<uint8_t> slot(SLOT);
  for (uint64_t s = 0; s < n; s += PAYLOAD) {
    const uint32_t len = (uint32_t)(n - s < PAYLOAD ? n - s : PAYLOAD);
    std::fill(slot.begin(), slot.end(), 0);
    member(src + s, len, slot.data(), tab, lit_hist, dist_hist);
  }
}
