/*
 * sbam_oracle.c -- TEST INFRASTRUCTURE ONLY: CPU restatement of spark-bam's BGZF +
 * record-boundary hot path, used as the parity oracle (see sbam_oracle.h).  Every
 * function cites the reference file:line it restates (paths relative to the reference
 * repository root).  Never linked into or called by the product (spark-bam_amd/).
 */
#include "sbam_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <zlib.h>

#define EXPECTED_HEADER_SIZE 18 /* Header.scala:19 */
#define FOOTER_SIZE 8           /* Block.scala:51  */
#define MAX_BLOCK_SIZE 65536    /* Block.scala:49  */
#define FIXED_FIELDS_SIZE 36    /* check/Checker.scala:19 */
#define MAX_CIGAR_OP 8          /* check/Checker.scala:21 */

static inline int32_t rd_i32(const uint8_t *p) {
  return (int32_t)((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
                   ((uint32_t)p[3] << 24));
}
static inline uint32_t rd_u16(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }

const char *or_zlib_version(void) { return zlibVersion(); }

uint32_t or_crc32(const uint8_t *b, int64_t n) {
  uLong c = crc32(0L, Z_NULL, 0);
  while (n > 0) {
    uInt k = n > (1 << 30) ? (1 << 30) : (uInt)n;
    c = crc32(c, b, k);
    b += k;
    n -= k;
  }
  return (uint32_t)c;
}

/* ------------------------------------------------------------------------- */
/* Header.make -- bgzf/src/main/scala/org/hammerlab/bgzf/block/Header.scala:48-83 */
int or_header_make(const uint8_t *b, int64_t avail, int32_t *hsize, int32_t *csize) {
  if (avail < EXPECTED_HEADER_SIZE) return OR_END; /* readFully -> EOFException */
  /* gzip magic (:61-64) */
  if (b[0] != 31 || b[1] != 139 || b[2] != 8 || b[3] != 4) return OR_HEADER_PARSE;
  int32_t xlen = (int32_t)rd_u16(b + 10); /* :66 */
  /* BAM-specific subfield id 'B','C' and SLEN low byte 2 (:73-75); byte 15 unchecked */
  if (b[12] != 66 || b[13] != 67 || b[14] != 2) return OR_HEADER_PARSE;
  *hsize = EXPECTED_HEADER_SIZE + xlen - 6; /* :69-70 */
  *csize = (int32_t)rd_u16(b + 16) + 1;     /* :77 */
  return OR_OK;
}

/* MetadataStream._advance -- bgzf/.../block/MetadataStream.scala:23-54 */
int or_metadata_next(const uint8_t *file, int64_t fsize, int64_t pos, or_block *out) {
  int32_t hs, cs;
  int64_t avail = pos < fsize ? fsize - pos : 0;
  int rc = or_header_make(file + (pos < fsize ? pos : 0), avail, &hs, &cs);
  if (rc != OR_OK) return rc; /* EOF -> None (:32-33); parse error propagates */
  int32_t remaining = cs - hs;               /* :36 */
  if (remaining - 4 < 0) return OR_TRUNCATED; /* negative skip: malformed      */
  /* ch.skip(hsize-18); ch.skip(remaining-4); getInt (:38-39) */
  if (pos + (int64_t)cs > fsize) return OR_TRUNCATED; /* getInt EOFException */
  int32_t usize = rd_i32(file + pos + cs - 4);
  out->start = pos;
  out->csize = cs;
  out->hsize = hs;
  out->usize = usize;
  out->empty = (remaining - FOOTER_SIZE) == 2; /* :41-45 */
  return out->empty ? OR_END : OR_OK;
}

int64_t or_metadata_stream(const uint8_t *file, int64_t fsize, int64_t start, or_block *out,
                           int64_t cap) {
  int64_t n = 0, pos = start;
  while (n < cap) {
    or_block b;
    int rc = or_metadata_next(file, fsize, pos, &b);
    if (rc == OR_END) break;
    if (rc != OR_OK) return -rc;
    out[n++] = b;
    pos += b.csize;
  }
  return n;
}

/* FindBlockStart.apply -- bgzf/.../block/FindBlockStart.scala:8-36 */
int or_find_block_start(const uint8_t *file, int64_t fsize, int64_t start,
                        int32_t blocks_to_check, int64_t *out) {
  for (int32_t pos = 0; pos < MAX_BLOCK_SIZE; ++pos) {
    int64_t p = start + pos;
    int ok = 1;
    for (int32_t k = 0; k < blocks_to_check; ++k) { /* headerStream.take(n).size */
      or_block b;
      int rc = or_metadata_next(file, fsize, p, &b);
      if (rc == OR_END) break;
      if (rc == OR_HEADER_PARSE) { ok = 0; break; } /* caught: pos += 1 (:26-27) */
      if (rc != OR_OK) return rc;                    /* any other exception escapes */
      p += b.csize;
    }
    if (ok) {
      *out = start + pos;
      return OR_OK;
    }
  }
  return OR_SEARCH_FAILED; /* HeaderSearchFailedException (:31-35) */
}

/* StreamI._advance -- bgzf/.../block/Stream.scala:31-71 */
int or_stream_next(const uint8_t *file, int64_t fsize, int64_t pos, uint8_t *out,
                   or_block *blk) {
  int32_t hs, cs;
  int64_t avail = pos < fsize ? fsize - pos : 0;
  int rc = or_header_make(file + (pos < fsize ? pos : 0), avail, &hs, &cs);
  if (rc != OR_OK) return rc; /* EOFException -> None; HeaderParseException escapes */
  int32_t remaining = cs - hs;
  int32_t data_len = remaining - FOOTER_SIZE; /* :42 */
  if (pos + (int64_t)cs > fsize) return OR_END; /* readFully EOF -> None (:67-69) */
  if (data_len < 0) return OR_INFLATE_DATA;
  int32_t usize = rd_i32(file + pos + cs - 4); /* :47 */
  if (usize < 0 || usize > MAX_BLOCK_SIZE) return OR_BAD_ISIZE;
  /* new Inflater(true); setInput(hsize, dataLength); inflate(decBuf, 0, usize) (:49-51) */
  z_stream zs;
  memset(&zs, 0, sizeof zs);
  if (inflateInit2(&zs, -15) != Z_OK) return OR_NOMEM;
  zs.next_in = (Bytef *)(file + pos + hs);
  zs.avail_in = (uInt)data_len;
  zs.next_out = out;
  zs.avail_out = (uInt)usize;
  int zr = Z_OK;
  zr = inflate(&zs, Z_PARTIAL_FLUSH); /* zlib runs even with avail_out == 0 */
  int32_t produced = usize - (int32_t)zs.avail_out;
  inflateEnd(&zs);
  if (zr == Z_DATA_ERROR || zr == Z_NEED_DICT || zr == Z_MEM_ERROR || zr == Z_STREAM_ERROR)
    return OR_INFLATE_DATA;
  if (produced != usize) return OR_INFLATE_SIZE; /* :52-54 */
  blk->start = pos;
  blk->csize = cs;
  blk->hsize = hs;
  blk->usize = usize;
  blk->empty = data_len == 2;
  return blk->empty ? OR_END : OR_OK; /* :56-58: empty block ends the stream */
}

/* ------------------------------------------------------------------------- */
/* Flat uncompressed view: UncompressedBytes.scala:13-87 + SeekableStream (Stream.scala:80-122) */
struct or_stream {
  const uint8_t *file;
  int64_t fsize;
  int64_t next_pos; /* compressed offset of the next block to inflate */
  uint8_t *data;
  int64_t size, cap;
  or_block *blocks;
  int64_t *ustart;
  int64_t nblocks, bcap;
  int32_t ended, error, owned;
};

or_stream *or_stream_open(const uint8_t *file, int64_t fsize, int64_t start) {
  or_stream *s = (or_stream *)calloc(1, sizeof *s);
  if (!s) return NULL;
  s->file = file;
  s->fsize = fsize;
  s->next_pos = start;
  s->owned = 1;
  return s;
}

static or_stream *wrap_buffer(or_stream *tmp, const uint8_t *U, int64_t total) {
  memset(tmp, 0, sizeof *tmp);
  tmp->data = (uint8_t *)U;
  tmp->size = total;
  tmp->ended = 1;
  return tmp;
}

void or_stream_close(or_stream *s) {
  if (!s) return;
  if (s->owned) {
    free(s->data);
    free(s->blocks);
    free(s->ustart);
  }
  free(s);
}

static int stream_advance(or_stream *s) {
  if (s->ended || s->error) return 0;
  if (s->cap - s->size < MAX_BLOCK_SIZE) {
    int64_t nc = s->cap ? s->cap * 2 : (1 << 20);
    while (nc - s->size < MAX_BLOCK_SIZE) nc *= 2;
    uint8_t *d = (uint8_t *)realloc(s->data, (size_t)nc);
    if (!d) { s->error = OR_NOMEM; return 0; }
    s->data = d;
    s->cap = nc;
  }
  if (s->nblocks == s->bcap) {
    int64_t nb = s->bcap ? s->bcap * 2 : 64;
    or_block *b = (or_block *)realloc(s->blocks, (size_t)nb * sizeof *b);
    int64_t *u = (int64_t *)realloc(s->ustart, (size_t)nb * sizeof *u);
    if (!b || !u) { s->error = OR_NOMEM; return 0; }
    s->blocks = b;
    s->ustart = u;
    s->bcap = nb;
  }
  or_block blk;
  int rc = or_stream_next(s->file, s->fsize, s->next_pos, s->data + s->size, &blk);
  if (rc == OR_END) { s->ended = 1; return 0; }
  if (rc != OR_OK) { s->error = rc; s->ended = 1; return 0; }
  s->blocks[s->nblocks] = blk;
  s->ustart[s->nblocks] = s->size;
  s->nblocks++;
  s->size += blk.usize;
  s->next_pos += blk.csize;
  return 1;
}

/* Make bytes [.., want) available if the stream has them; returns available end. */
static inline int64_t have(or_stream *s, int64_t want) {
  while (s->size < want && !s->ended) stream_advance(s);
  return s->size < want ? s->size : want;
}

int or_stream_load_all(or_stream *s) {
  while (!s->ended) stream_advance(s);
  return s->error;
}
int64_t or_stream_size(or_stream *s) { return s->size; }
int32_t or_stream_ended(or_stream *s) { return s->ended; }
int32_t or_stream_error(or_stream *s) { return s->error; }
const uint8_t *or_stream_data(or_stream *s) { return s->data; }
int64_t or_stream_nblocks(or_stream *s) { return s->nblocks; }
int64_t *or_stream_ustarts(or_stream *s) { return s->ustart; }
int64_t or_stream_blocks(or_stream *s, or_block *out, int64_t cap) {
  int64_t n = s->nblocks < cap ? s->nblocks : cap;
  memcpy(out, s->blocks, (size_t)n * sizeof *out);
  return n;
}

int64_t or_stream_flat_of(or_stream *s, int64_t block_pos, int32_t offset) {
  /* make sure the block is loaded */
  while (!s->ended && (s->nblocks == 0 || s->blocks[s->nblocks - 1].start < block_pos))
    stream_advance(s);
  int64_t lo = 0, hi = s->nblocks;
  while (lo < hi) {
    int64_t m = (lo + hi) / 2;
    if (s->blocks[m].start < block_pos) lo = m + 1; else hi = m;
  }
  if (lo < s->nblocks && s->blocks[lo].start == block_pos) return s->ustart[lo] + offset;
  /* Pos(end-of-stream block, 0) -> end of data */
  if (s->ended && block_pos >= s->next_pos) return s->size + offset;
  return -1;
}

/* curPos semantics: a position at a block's end rolls to Pos(next, 0)
 * (ByteStreamTest.scala:48-53); positions are canonical. */
int or_stream_pos_of(or_stream *s, int64_t flat, int64_t *block_pos, int32_t *offset) {
  have(s, flat + 1);
  if (flat >= s->size) {
    if (!s->ended) return OR_END;
    *block_pos = s->next_pos; /* one past the last block: Pos(next, 0) */
    *offset = (int32_t)(flat - s->size);
    return OR_END;
  }
  int64_t lo = 0, hi = s->nblocks - 1;
  while (lo < hi) { /* last block with ustart <= flat */
    int64_t m = (lo + hi + 1) / 2;
    if (s->ustart[m] <= flat) lo = m; else hi = m - 1;
  }
  /* skip zero-length blocks sharing the same ustart: pick the one containing flat */
  while (lo < s->nblocks && s->ustart[lo] + s->blocks[lo].usize <= flat) lo++;
  *block_pos = s->blocks[lo].start;
  *offset = (int32_t)(flat - s->ustart[lo]);
  return OR_OK;
}

/* ------------------------------------------------------------------------- */
/* PosChecker.getRefPosError -- check/.../bam/check/PosChecker.scala:43-63.
 * Returns bits {0: negativeRefIdx, 1: tooLargeRefIdx, 2: negativeRefPos,
 * 3: tooLargeRefPos} as in full/error/RefPosError.scala. */
static inline uint32_t ref_pos_error(int32_t idx, int32_t pos, const int32_t *len, int32_t n) {
  if (idx < -1) return pos < -1 ? (1u | 4u) : 1u;
  if (idx >= n) return pos < -1 ? (2u | 4u) : 2u;
  if (pos < -1) return 4u;
  if (idx >= 0 && (int64_t)pos > (int64_t)len[idx]) return 8u;
  return 0;
}

/* Checker.allowedReadNameChars: '!'..'?' ++ 'A'..'~' (check/.../Checker.scala:12-17) */
static inline int name_char_ok(uint8_t c) {
  return (c >= 0x21 && c <= 0x3F) || (c >= 0x41 && c <= 0x7E);
}

/* Java int arithmetic: (seqLen + 1) / 2 + seqLen, and 32 + rnl + 4*nc + nsq (wrap). */
static inline int32_t implied_min_remaining(int32_t rnl, int32_t nc, int32_t seq_len) {
  int32_t s1 = (int32_t)((uint32_t)seq_len + 1u);
  int32_t nsq = (int32_t)((uint32_t)(s1 / 2) + (uint32_t)seq_len);
  return (int32_t)(32u + (uint32_t)rnl + 4u * (uint32_t)nc + (uint32_t)nsq);
}

/* eager.Checker.apply -- check/.../check/eager/Checker.scala:24-126 (with
 * PosChecker.apply, PosChecker.scala:32-35).  `cur` is the channel cursor, `start`
 * the nominal record start (startPos / nextOffset). */
static int eager_check(or_stream *s, int64_t p, const int32_t *len, int32_t n_ctg, int32_t rtc) {
  int64_t cur = p, start = p;
  for (int32_t n = 0;; ++n) {
    if (n == rtc) return 1; /* :29-30 */
    if (have(s, cur + FIXED_FIELDS_SIZE) < cur + FIXED_FIELDS_SIZE) {
      /* readFully EOF: partial read consumes to EOF (:33-42) */
      return (s->size == start && n > 0) ? 1 : 0;
    }
    const uint8_t *r = s->data + cur;
    int32_t rem = rd_i32(r);
    int64_t nominal = start + 4 + (int64_t)rem; /* :47 */
    if (ref_pos_error(rd_i32(r + 4), rd_i32(r + 8), len, n_ctg)) return 0; /* :49-50 */
    int32_t rnl = rd_i32(r + 12) & 0xff;                                     /* :52 */
    if (rnl == 0 || rnl == 1) return 0;                                      /* :53-57 */
    uint32_t fnc = (uint32_t)rd_i32(r + 16);
    uint32_t flags = fnc >> 16;
    int32_t nc = (int32_t)(fnc & 0xffff);
    int32_t seq_len = rd_i32(r + 20);
    if ((flags & 4) == 0 && (seq_len == 0 || nc == 0)) return 0; /* :68-69 */
    if (rem < implied_min_remaining(rnl, nc, seq_len)) return 0; /* :71-74 */
    if (ref_pos_error(rd_i32(r + 24), rd_i32(r + 28), len, n_ctg)) return 0; /* :76-77 */
    cur += FIXED_FIELDS_SIZE;
    /* read name (:81-95) */
    if (have(s, cur + rnl) < cur + rnl) return 0;
    r = s->data + cur;
    if (r[rnl - 1] != 0) return 0;
    for (int32_t i = 0; i < rnl - 1; ++i)
      if (!name_char_ok(r[i])) return 0;
    cur += rnl;
    /* cigar ops (:97-109) */
    for (int32_t k = 0; k < nc; ++k) {
      if (have(s, cur + 4) < cur + 4) return 0;
      if ((s->data[cur] & 0xf) > MAX_CIGAR_OP) return 0;
      cur += 4;
    }
    /* skip to the next record (:116-119); skip clamps at EOF */
    if (nominal - cur > 0) {
      int64_t e = have(s, nominal);
      cur = e;
    }
    start = nominal; /* apply(nextOffset)(n + 1) (:121-125) */
  }
}

/* full.Checker.apply / build -- check/.../check/full/Checker.scala:22-184 */
static uint32_t full_check(or_stream *s, int64_t p, const int32_t *len, int32_t n_ctg,
                           int32_t rtc) {
  int64_t cur = p, start = p;
  for (int32_t n = 0;; ++n) {
    if (n == rtc) return OR_FULL_SUCCESS | ((uint32_t)n << OR_FULL_N_SHIFT); /* :27-28 */
    if (have(s, cur + FIXED_FIELDS_SIZE) < cur + FIXED_FIELDS_SIZE) {            /* :30-48 */
      if (s->size == start && n > 0) return OR_FULL_SUCCESS | ((uint32_t)n << OR_FULL_N_SHIFT);
      return 1u | ((uint32_t)n << OR_FULL_N_SHIFT); /* tooFewFixedBlockBytes */
    }
    const uint8_t *r = s->data + cur;
    int32_t rem = rd_i32(r);
    int64_t nominal = start + 4 + (int64_t)rem;
    uint32_t f = ref_pos_error(rd_i32(r + 4), rd_i32(r + 8), len, n_ctg) << 1; /* bits 1-4 */
    int32_t rnl = rd_i32(r + 12) & 0xff;
    uint32_t fnc = (uint32_t)rd_i32(r + 16);
    uint32_t flags = fnc >> 16;
    int32_t nc = (int32_t)(fnc & 0xffff);
    int32_t seq_len = rd_i32(r + 20);
    if (rem < implied_min_remaining(rnl, nc, seq_len)) f |= 1u << 18; /* :70-71 */
    f |= ref_pos_error(rd_i32(r + 24), rd_i32(r + 28), len, n_ctg) << 5; /* bits 5-8 */
    cur += FIXED_FIELDS_SIZE;
    int name_eof = 0;
    if (rnl == 0) f |= 1u << 12;      /* noReadName    */
    else if (rnl == 1) f |= 1u << 13; /* emptyReadName */
    else {
      if (have(s, cur + rnl) < cur + rnl) {
        f |= 1u << 9; /* tooFewBytesForReadName (:140-143); no cigar check */
        name_eof = 1;
      } else {
        r = s->data + cur;
        if (r[rnl - 1] != 0) f |= 1u << 10;
        else {
          for (int32_t i = 0; i < rnl - 1; ++i)
            if (!name_char_ok(r[i])) { f |= 1u << 11; break; }
        }
        cur += rnl;
      }
    }
    if (!name_eof) { /* :111-136 */
      int cig_err = 0;
      for (int32_t k = 0; k < nc; ++k) {
        if (have(s, cur + 4) < cur + 4) { f |= 1u << 14; cig_err = 1; break; }
        if ((s->data[cur] & 0xf) > MAX_CIGAR_OP) { f |= 1u << 15; cig_err = 1; cur += 4; break; }
        cur += 4;
      }
      if (!cig_err && (flags & 4) == 0 && (seq_len == 0 || nc == 0)) {
        /* EmptyMapped(emptySeq, emptyCigar) into (emptyMappedCigar, emptyMappedSeq) */
        if (seq_len == 0) f |= 1u << 16;
        if (nc == 0) f |= 1u << 17;
      }
    }
    if (f) return f | ((uint32_t)n << OR_FULL_N_SHIFT); /* Flags(readsBeforeError = n) */
    if (nominal - cur > 0) cur = have(s, nominal);        /* build: skip (:167-170) */
    start = nominal;
  }
}

int or_eager_check(or_stream *s, int64_t p, const int32_t *contig_len, int32_t n_contigs,
                   int32_t reads_to_check) {
  return eager_check(s, p, contig_len, n_contigs, reads_to_check);
}
uint32_t or_full_check(or_stream *s, int64_t p, const int32_t *contig_len, int32_t n_contigs,
                       int32_t reads_to_check) {
  return full_check(s, p, contig_len, n_contigs, reads_to_check);
}
int or_eager_check_buf(const uint8_t *U, int64_t total, int64_t p, const int32_t *contig_len,
                       int32_t n_contigs, int32_t reads_to_check) {
  or_stream t;
  return eager_check(wrap_buffer(&t, U, total), p, contig_len, n_contigs, reads_to_check);
}
uint32_t or_full_check_buf(const uint8_t *U, int64_t total, int64_t p,
                           const int32_t *contig_len, int32_t n_contigs,
                           int32_t reads_to_check) {
  or_stream t;
  return full_check(wrap_buffer(&t, U, total), p, contig_len, n_contigs, reads_to_check);
}

int64_t or_eager_range(or_stream *s, int64_t begin, int64_t end, const int32_t *contig_len,
                       int32_t n_contigs, int32_t reads_to_check, uint8_t *out_bits) {
  int64_t trues = 0;
  if (out_bits) memset(out_bits, 0, (size_t)((end - begin + 7) / 8));
  for (int64_t p = begin; p < end; ++p) {
    if (eager_check(s, p, contig_len, n_contigs, reads_to_check)) {
      ++trues;
      if (out_bits) out_bits[(p - begin) >> 3] |= (uint8_t)(1u << ((p - begin) & 7));
    }
  }
  return trues;
}

/* FullCheck.scala:142-192: keyBy(numNonZeroFields) -> Counts |+| per key. */
int64_t or_full_range(or_stream *s, int64_t begin, int64_t end, const int32_t *contig_len,
                      int32_t n_contigs, int32_t reads_to_check, uint32_t *out,
                      int64_t *counts, int64_t *rbe_hist) {
  int64_t n_success = 0;
  for (int64_t p = begin; p < end; ++p) {
    uint32_t r = full_check(s, p, contig_len, n_contigs, reads_to_check);
    if (out) out[p - begin] = r;
    if (r & OR_FULL_SUCCESS) { ++n_success; continue; }
    uint32_t f = r & OR_FULL_FLAGS_MASK;
    uint32_t rbe = (r >> OR_FULL_N_SHIFT) & 0x7FF;
    if (f == 1u && rbe == 0) continue; /* flags != TooFewFixedBlockBytes (:145-146) */
    int nnz = __builtin_popcount(f) + (rbe > 0); /* Flags.numNonZeroFields (:118-123) */
    if (counts)
      for (int b = 0; b < 19; ++b)
        if (f & (1u << b)) counts[nnz * 19 + b]++;
    if (rbe_hist && rbe > 0 && rbe < 64) rbe_hist[nnz * 64 + rbe]++;
  }
  return n_success;
}

/* FindRecordStart.withDelta -- check/.../spark/FindRecordStart.scala:30-63 */
int or_find_record_start(or_stream *s, int64_t from_flat, const int32_t *contig_len,
                         int32_t n_contigs, int32_t reads_to_check, int32_t max_read_size,
                         int64_t *out_flat, int32_t *out_delta) {
  for (int32_t idx = 0; idx < max_read_size; ++idx) {
    int64_t p = from_flat + idx;
    if (have(s, p + 1) < p + 1) return OR_NO_READ_FOUND; /* curPos None / !hasNext */
    if (eager_check(s, p, contig_len, n_contigs, reads_to_check)) {
      *out_flat = p;
      *out_delta = idx;
      return OR_OK;
    }
  }
  return OR_NO_READ_FOUND;
}

/* header.Header.apply -- check/.../header/Header.scala:26-60 */
int32_t or_parse_header(or_stream *s, int32_t *contig_len, int32_t cap, int64_t *end_flat) {
  int64_t c = 0;
  if (have(s, 8) < 8) return -OR_TRUNCATED;
  const uint8_t *d = s->data;
  if (d[0] != 'B' || d[1] != 'A' || d[2] != 'M' || d[3] != 1) return -OR_HEADER_PARSE;
  int32_t l_text = rd_i32(d + 4);
  c = 8 + (int64_t)l_text;
  if (have(s, c + 4) < c + 4) return -OR_TRUNCATED;
  int32_t n_ref = rd_i32(s->data + c);
  c += 4;
  for (int32_t i = 0; i < n_ref; ++i) {
    if (have(s, c + 4) < c + 4) return -OR_TRUNCATED;
    int32_t l_name = rd_i32(s->data + c);
    c += 4 + (int64_t)l_name;
    if (have(s, c + 4) < c + 4) return -OR_TRUNCATED;
    if (i < cap) contig_len[i] = rd_i32(s->data + c);
    c += 4;
  }
  *end_flat = c;
  return n_ref;
}

/* PosStream._advance -- check/.../iterator/PosStream.scala:14-22 */
int64_t or_record_chain(or_stream *s, int64_t from, int64_t stop_flat, int64_t *out,
                        int64_t cap) {
  int64_t n = 0, p = from;
  while (p < stop_flat) {
    if (have(s, p + 4) < p + 4) break; /* EOF ends the stream */
    if (out && n < cap) out[n] = p;
    ++n;
    p += 4 + (int64_t)rd_i32(s->data + p);
  }
  return n;
}

/* Hadoop FileInputFormat.getSplits (SPLIT_SLOP = 1.1), as driven by
 * hammerlab FileSplits.asJava(path, splitSize) (CanLoadBam.scala:205,314). */
int64_t or_file_splits(int64_t file_size, int64_t split_size, int64_t *starts, int64_t *ends,
                       int64_t cap) {
  int64_t n = 0, rem = file_size;
  while ((double)rem / (double)split_size > 1.1) {
    if (starts && n < cap) { starts[n] = file_size - rem; ends[n] = file_size - rem + split_size; }
    ++n;
    rem -= split_size;
  }
  if (rem != 0) {
    if (starts && n < cap) { starts[n] = file_size - rem; ends[n] = file_size; }
    ++n;
  }
  return n;
}

/* CanLoadBam.loadReadsAndPositions per split (CanLoadBam.scala:316-356) */
int or_split(const uint8_t *file, int64_t fsize, int64_t start, int64_t end,
             const int32_t *contig_len, int32_t n_contigs, int32_t blocks_to_check,
             int32_t reads_to_check, int32_t max_read_size, uint64_t *first_vpos,
             int64_t *count) {
  int64_t bstart;
  int rc = or_find_block_start(file, fsize, start, blocks_to_check, &bstart);
  if (rc != OR_OK) return rc;
  or_stream *s = or_stream_open(file, fsize, bstart);
  if (!s) return OR_NOMEM;
  int64_t first;
  int32_t delta;
  rc = or_find_record_start(s, 0, contig_len, n_contigs, reads_to_check, max_read_size, &first,
                            &delta);
  if (rc != OR_OK) { or_stream_close(s); return rc; }
  int64_t bp;
  int32_t off;
  or_stream_pos_of(s, first, &bp, &off);
  *first_vpos = ((uint64_t)bp << 16) | (uint32_t)off;
  /* RecordStream.takeWhile(pos < Pos(end, 0)): records whose block starts before end */
  int64_t n = 0, p = first;
  for (;;) {
    if (have(s, p + 4) < p + 4) break;
    if (or_stream_pos_of(s, p, &bp, &off) != OR_OK) break;
    if (bp >= end) break;
    ++n;
    p += 4 + (int64_t)rd_i32(s->data + p);
  }
  *count = n;
  or_stream_close(s);
  return OR_OK;
}

/* ------------------------------------------------------------------------- */
/* CPU baseline: the same work as the GPU step (inflate + eager at every offset). */
typedef struct {
  const uint8_t *file;
  int64_t fsize;
  const or_block *blocks;
  int64_t b0, b1;
  const int64_t *ustart;
  uint8_t *flat;
  int64_t flat_total;
  const int32_t *len;
  int32_t n_ctg, rtc;
  int64_t pos_begin, pos_end, trues;
  int phase, err;
} bench_job;

static void *bench_worker(void *arg) {
  bench_job *j = (bench_job *)arg;
  if (j->phase == 0) {
    for (int64_t b = j->b0; b < j->b1; ++b) {
      or_block blk;
      int rc = or_stream_next(j->file, j->fsize, j->blocks[b].start, j->flat + j->ustart[b], &blk);
      if (rc != OR_OK && rc != OR_END) j->err = rc;
    }
  } else {
    int64_t t = 0;
    for (int64_t p = j->pos_begin; p < j->pos_end; ++p)
      t += or_eager_check_buf(j->flat, j->flat_total, p, j->len, j->n_ctg, j->rtc);
    j->trues = t;
  }
  return NULL;
}

double or_bench_inflate_check(const uint8_t *file, int64_t fsize, const or_block *blocks,
                              int64_t b0, int64_t b1, const int32_t *contig_len,
                              int32_t n_contigs, int32_t reads_to_check, int32_t threads,
                              int64_t *positions, int64_t *trues) {
  int64_t nb = b1 - b0;
  int64_t *ustart = (int64_t *)malloc((size_t)(nb + 1) * sizeof(int64_t));
  int64_t tot = 0;
  for (int64_t i = 0; i < nb; ++i) { ustart[i] = tot; tot += blocks[b0 + i].usize; }
  ustart[nb] = tot;
  uint8_t *flat = (uint8_t *)malloc((size_t)tot + 16);
  if (threads < 1) threads = 1;
  pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof *th);
  bench_job *jobs = (bench_job *)calloc((size_t)threads, sizeof *jobs);
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int phase = 0; phase < 2; ++phase) {
    for (int i = 0; i < threads; ++i) {
      bench_job *j = &jobs[i];
      j->file = file; j->fsize = fsize; j->blocks = blocks + b0; j->ustart = ustart;
      j->flat = flat; j->flat_total = tot; j->len = contig_len; j->n_ctg = n_contigs;
      j->rtc = reads_to_check; j->phase = phase;
      j->b0 = nb * i / threads; j->b1 = nb * (i + 1) / threads;
      j->pos_begin = tot * i / threads; j->pos_end = tot * (i + 1) / threads;
      pthread_create(&th[i], NULL, bench_worker, j);
    }
    for (int i = 0; i < threads; ++i) pthread_join(th[i], NULL);
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  int64_t tr = 0;
  for (int i = 0; i < threads; ++i) tr += jobs[i].trues;
  *positions = tot;
  *trues = tr;
  free(th); free(jobs); free(flat); free(ustart);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
