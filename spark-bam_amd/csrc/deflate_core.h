// deflate_core.h -- one BGZF block of the writer: greedy LZ77 + fixed-Huffman deflate, the
// BGZF member framing (RFC 1952 + the BC extra subfield) and its CRC32 / ISIZE footer.
//
// Replaces, for HTSJDKRewrite (cli/src/main/scala/org/hammerlab/bam/rewrite/HTSJDKRewrite.scala:62-67),
// the block compressor htsjdk's BAM writer drives (BlockCompressedOutputStream, third-party:
// htsjdk, not in /root/reference): the uncompressed stream is cut every 65498 bytes
// (the payload size visible in every full block of test_bams/.../2.bam.blocks) and each
// piece becomes one member; a piece whose deflate output would not fit the 64 KiB member
// is stored instead.  The deflate bytes are NOT zlib level-5 output (htsjdk's Deflater):
// the member boundaries and uncompressed layout match, the compressed bytes do not.
//
// Written once for both sides: the device kernel (deflate.hip) runs it one lane per block;
// tests/ build the same header for the host (tools/deflate_host.cpp) to round-trip it
// through zlib without a GPU.  SBH_HD is __host__ __device__ under hipcc, empty otherwise.
#pragma once
#include <stdint.h>

#ifndef SBH_HD
#define SBH_HD
#endif

namespace sbh_deflate {

constexpr uint32_t PAYLOAD = 65498;  // htsjdk DEFAULT_UNCOMPRESSED_BLOCK_SIZE (2.bam.blocks)
constexpr uint32_t SLOT = 65536;     // max BGZF member size (BSIZE is u16)
constexpr uint32_t HBITS = 13;       // hash table: 8192 u16 heads per block (position + 1)
constexpr uint32_t HSIZE = 1u << HBITS;
constexpr uint32_t BUDGET = SLOT - 26;  // deflate bytes that fit a member with header + footer
constexpr uint32_t MAXD = 32768;

struct Bits {
  uint8_t *p;
  uint64_t acc;
  uint32_t nb;
  SBH_HD void put(uint32_t v, uint32_t n) {  // n <= 32, LSB first (RFC 1951 3.1.1)
    acc |= (uint64_t)v << nb;
    nb += n;
    while (nb >= 8) {
      *p++ = (uint8_t)acc;
      acc >>= 8;
      nb -= 8;
    }
  }
  SBH_HD void flush() {
    if (nb) *p++ = (uint8_t)acc;
    acc = 0;
    nb = 0;
  }
};

SBH_HD inline uint32_t rev(uint32_t c, uint32_t n) {
  uint32_t r = 0;
  for (uint32_t i = 0; i < n; ++i) r |= ((c >> i) & 1u) << (n - 1 - i);
  return r;
}

SBH_HD inline uint32_t lg2(uint32_t x) { return 31u - (uint32_t)__builtin_clz(x); }

// Fixed literal/length code (RFC 1951 3.2.6), already bit-reversed for the LSB-first writer.
SBH_HD inline void put_sym(Bits &b, uint32_t s) {
  if (s < 144) b.put(rev(0x30 + s, 8), 8);
  else if (s < 256) b.put(rev(0x190 + s - 144, 9), 9);
  else if (s < 280) b.put(rev(s - 256, 7), 7);
  else b.put(rev(0xc0 + s - 280, 8), 8);
}

// Length 3..258 -> code 257..285 + extra bits; distance 1..32768 -> code 0..29 + extra.
SBH_HD inline void put_match(Bits &b, uint32_t len, uint32_t dist) {
  if (len == 258) {
    put_sym(b, 285);
  } else {
    const uint32_t m = len - 3;
    if (m < 8) {
      put_sym(b, 257 + m);
    } else {
      const uint32_t l = lg2(m), x = l - 2;
      put_sym(b, 257 + 4 * (l - 1) + ((m >> x) & 3u));
      b.put(m & ((1u << x) - 1), x);
    }
  }
  const uint32_t d = dist - 1;
  if (d < 4) {
    b.put(rev(d, 5), 5);
  } else {
    const uint32_t l = lg2(d), x = l - 1;
    b.put(rev(2 * l + ((d >> x) & 1u), 5), 5);
    b.put(d & ((1u << x) - 1), x);
  }
}

SBH_HD inline uint32_t hash3(const uint8_t *s) {
  const uint32_t v = (uint32_t)s[0] | (uint32_t)s[1] << 8 | (uint32_t)s[2] << 16;
  return (v * 2654435761u) >> (32 - HBITS);
}

SBH_HD inline void put_le32(uint8_t *o, uint32_t v) {
  o[0] = (uint8_t)v;
  o[1] = (uint8_t)(v >> 8);
  o[2] = (uint8_t)(v >> 16);
  o[3] = (uint8_t)(v >> 24);
}

// A member's payload is coded as NSEG independent fixed-Huffman deflate blocks of SEG
// bytes each (matches stay inside their segment; the last segment's block is BFINAL), so the
// device can give every segment its own lane.  The blocks are bit-concatenated (RFC 1951
// blocks are not byte aligned); a payload whose blocks would not fit the member is stored.
constexpr uint32_t SEG = 4096, NSEG = 16;   // NSEG * SEG >= PAYLOAD
constexpr uint32_t SEGCAP = 4624;           // >= 9 bits per byte + header/EOB, 16-aligned
constexpr uint32_t SHBITS = 12, SHSIZE = 1u << SHBITS;  // per-segment hash heads (pos + 1)

SBH_HD inline uint32_t hash3s(const uint8_t *s) {
  const uint32_t v = (uint32_t)s[0] | (uint32_t)s[1] << 8 | (uint32_t)s[2] << 16;
  return (v * 2654435761u) >> (32 - SHBITS);
}

// Greedy LZ77 over seg[0, n) into buf (SEGCAP bytes): one fixed-Huffman block.  head:
// SHSIZE zeroed u16.  Returns the block's exact bit count.
SBH_HD inline uint32_t seg_encode(const uint8_t *seg, uint32_t n, bool final, uint8_t *buf, uint16_t *head) {
  Bits b{buf, 0, 0};
  b.put(final ? 1u : 0u, 1);
  b.put(1, 2);  // BTYPE = 01
  uint32_t p = 0;
  while (p < n) {
    uint32_t len = 0, dist = 0;
    if (p + 3 <= n) {
      const uint32_t h = hash3s(seg + p);
      const uint32_t c = head[h];
      head[h] = (uint16_t)(p + 1);
      if (c) {
        const uint32_t q = c - 1, lim = (n - p < 258u) ? n - p : 258u;
        while (len < lim && seg[q + len] == seg[p + len]) ++len;
        dist = p - q;
      }
    }
    if (len >= 3) {
      put_match(b, len, dist);
      const uint32_t e = p + len;
      for (++p; p < e; ++p)
        if (p + 3 <= n) head[hash3s(seg + p)] = (uint16_t)(p + 1);
    } else {
      put_sym(b, seg[p]);
      ++p;
    }
  }
  put_sym(b, 256);
  const uint32_t nbits = (uint32_t)(b.p - buf) * 8 + b.nb;
  b.flush();
  return nbits;
}

// Output byte j (relative to the member's deflate data) of a segment stream of nbits bits
// placed at bit offset off: the bits of byte j that come from this stream (others zero).
SBH_HD inline uint8_t seg_byte(const uint8_t *buf, uint32_t nbits, uint32_t off, uint32_t j) {
  const int32_t p = (int32_t)(8 * j) - (int32_t)off;  // stream bit at the byte's bit 0
  const uint32_t nbytes = (nbits + 7) / 8;
  uint32_t v;
  if (p >= 0) {
    const uint32_t q = (uint32_t)p >> 3, r = (uint32_t)p & 7;
    v = (q < nbytes ? (uint32_t)buf[q] >> r : 0u) | (q + 1 < nbytes && r ? (uint32_t)buf[q + 1] << (8 - r) : 0u);
  } else {  // -7 <= p < 0: the stream starts inside this byte
    v = (uint32_t)buf[0] << (uint32_t)(-p);
  }
  // clear stream bits past nbits
  const int32_t valid = (int32_t)nbits - p;  // stream bits available from p on
  if (valid < 8) v &= (1u << (valid > 0 ? valid : 0)) - 1u;
  if (p < 0) v &= 0xffu << (uint32_t)(-p);
  return (uint8_t)v;
}

SBH_HD inline void put_header(uint8_t *out, uint32_t total) {
  const uint8_t hdr[16] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0};
  for (int i = 0; i < 16; ++i) out[i] = hdr[i];
  out[16] = (uint8_t)(total - 1);
  out[17] = (uint8_t)((total - 1) >> 8);
}

SBH_HD inline uint32_t stored_dsize(uint32_t n) { return 5 + n; }
SBH_HD inline void put_stored_head(uint8_t *d0, uint32_t n) {  // BFINAL=1 BTYPE=00, LEN, NLEN
  d0[0] = 1;
  d0[1] = (uint8_t)n;
  d0[2] = (uint8_t)(n >> 8);
  d0[3] = (uint8_t)~n;
  d0[4] = (uint8_t)(~n >> 8);
}

SBH_HD inline uint32_t crc32_bytes(const uint8_t *s, uint32_t n, const uint32_t *crctab) {
  uint32_t crc = 0xffffffffu;
  for (uint32_t i = 0; i < n; ++i) crc = crctab[(crc ^ s[i]) & 0xff] ^ (crc >> 8);
  return crc ^ 0xffffffffu;
}

// Serial restatement of the whole member (host build; the device splits it over lanes and
// must produce the same bytes).  out: SLOT zeroed bytes; segbuf: NSEG * SEGCAP; head: SHSIZE.
SBH_HD inline uint32_t bgzf_block(const uint8_t *src, uint32_t n, uint8_t *out, uint8_t *segbuf, uint16_t *head,
                                  const uint32_t *crctab) {
  const uint32_t nseg = (n + SEG - 1) / SEG;
  uint32_t nbits[NSEG], off[NSEG], tot = 0;
  for (uint32_t i = 0; i < nseg; ++i) {
    for (uint32_t h = 0; h < SHSIZE; ++h) head[h] = 0;
    const uint32_t lo = i * SEG, len = (n - lo < SEG) ? n - lo : SEG;
    nbits[i] = seg_encode(src + lo, len, i + 1 == nseg, segbuf + i * SEGCAP, head);
    off[i] = tot;
    tot += nbits[i];
  }
  uint8_t *const d0 = out + 18;
  uint32_t dsize = (tot + 7) / 8;
  if (dsize <= BUDGET) {
    for (uint32_t i = 0; i < nseg; ++i)
      for (uint32_t j = off[i] / 8; j <= (off[i] + nbits[i] - 1) / 8; ++j)
        d0[j] |= seg_byte(segbuf + i * SEGCAP, nbits[i], off[i], j);
  } else {
    dsize = stored_dsize(n);
    put_stored_head(d0, n);
    for (uint32_t i = 0; i < n; ++i) d0[5 + i] = src[i];
  }
  const uint32_t total = 18 + dsize + 8;
  put_header(out, total);
  put_le32(d0 + dsize, crc32_bytes(src, n, crctab));
  put_le32(d0 + dsize + 4, n);
  return total;
}

// The empty member htsjdk appends at close (BlockCompressedStreamConstants.EMPTY_GZIP_BLOCK).
constexpr uint32_t EOF_SIZE = 28;
SBH_HD inline void put_eof(uint8_t *o) {
  const uint8_t e[28] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0, 27, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 28; ++i) o[i] = e[i];
}

}  // namespace sbh_deflate
