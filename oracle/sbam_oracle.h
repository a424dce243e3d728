/*
 * sbam_oracle.h -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * Plain-C CPU restatement of spark-bam's BGZF + BAM record-boundary hot path, used by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the oracle the
 * HIP path is compared against.  Nothing under spark-bam_amd/ links or calls this.
 *
 * Pinned against the reference's own fixtures (tests/golden/, copied from the
 * reference's test resources): every .blocks and .records file, the full-check
 * "Total error counts" outputs, the FindBlockStart / FindRecordStart / full-Checker
 * unit-test vectors and the compute-splits / LoadBAMTest split goldens
 * (tests/test_oracle.py).
 *
 * DEFLATE: the reference inflates through java.util.zip.Inflater(nowrap=true), i.e. the
 * JDK-bundled zlib (JDK 8, zlib 1.2.x; call site bgzf/.../block/Stream.scala:49-51).
 * The oracle calls the system zlib (1.2.11) raw-inflate with the same one-shot
 * "fill exactly ISIZE bytes" contract.
 */
#ifndef SBAM_ORACLE_H
#define SBAM_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Result codes shared with the product's status vocabulary (include/sparkbam.h). */
#define OR_OK 0
#define OR_END 1              /* iterator exhausted: EOF or empty block          */
#define OR_HEADER_PARSE 2     /* HeaderParseException  (Header.scala:50-57)     */
#define OR_TRUNCATED 3        /* EOFException escaping MetadataStream / skip     */
#define OR_INFLATE_SIZE 4     /* IOException "Expected N decompressed bytes"     */
#define OR_INFLATE_DATA 5     /* DataFormatException from Inflater               */
#define OR_BAD_ISIZE 6        /* ISIZE outside [0, 65536] (array bounds in JVM)  */
#define OR_SEARCH_FAILED 7    /* HeaderSearchFailedException                     */
#define OR_NO_READ_FOUND 8    /* NoReadFoundException                            */
#define OR_NOMEM 9

/* Full-checker result word (product uses the same encoding):
 *   bit 31     : Success
 *   bits 20-30 : readsParsed (Success) / readsBeforeError (Flags)
 *   bits 0-18  : Flags bits in the serde order of full/error/Flags.scala:203-222 */
#define OR_FULL_SUCCESS 0x80000000u
#define OR_FULL_N_SHIFT 20
#define OR_FULL_FLAGS_MASK 0x7FFFFu

typedef struct {
  int64_t start;   /* compressed offset of the block header              */
  int32_t csize;   /* BSIZE + 1                                           */
  int32_t hsize;   /* 18 + XLEN - 6                                       */
  int32_t usize;   /* ISIZE                                               */
  int32_t empty;   /* dataLength == 2 (the stream ends here)              */
} or_block;

/* Header.make (bgzf/.../block/Header.scala:48-83).  avail = bytes available at b.
 * Returns OR_OK, OR_END (fewer than 18 bytes: readFully EOF) or OR_HEADER_PARSE. */
int or_header_make(const uint8_t *b, int64_t avail, int32_t *hsize, int32_t *csize);

/* One MetadataStream._advance (MetadataStream.scala:23-54) at compressed offset pos. */
int or_metadata_next(const uint8_t *file, int64_t fsize, int64_t pos, or_block *out);

/* MetadataStream from `start`: fills up to cap blocks, returns count (>=0) or -code. */
int64_t or_metadata_stream(const uint8_t *file, int64_t fsize, int64_t start,
                           or_block *out, int64_t cap);

/* FindBlockStart.apply (FindBlockStart.scala:8-36).  Returns OR_OK and *out, or
 * OR_SEARCH_FAILED / OR_TRUNCATED. */
int or_find_block_start(const uint8_t *file, int64_t fsize, int64_t start,
                        int32_t blocks_to_check, int64_t *out);

/* One StreamI._advance (Stream.scala:31-71): inflates the block at pos into out
 * (capacity 65536).  Returns OR_OK (block in *blk), OR_END, or an error code. */
int or_stream_next(const uint8_t *file, int64_t fsize, int64_t pos, uint8_t *out,
                   or_block *blk);

/* ---- flat uncompressed view of a Stream started at a compressed offset ---- */
typedef struct or_stream or_stream;
or_stream *or_stream_open(const uint8_t *file, int64_t fsize, int64_t start);
void or_stream_close(or_stream *s);
/* Inflate the whole stream eagerly; returns OR_OK or an error code. */
int or_stream_load_all(or_stream *s);
int64_t or_stream_size(or_stream *s);          /* flat bytes inflated so far       */
int32_t or_stream_ended(or_stream *s);
int32_t or_stream_error(or_stream *s);
const uint8_t *or_stream_data(or_stream *s);
int64_t or_stream_nblocks(or_stream *s);
int64_t or_stream_blocks(or_stream *s, or_block *out, int64_t cap);
int64_t *or_stream_ustarts(or_stream *s);      /* flat start of each block         */
/* Pos <-> flat.  Pos is canonical (offset < usize of a non-empty block). */
int64_t or_stream_flat_of(or_stream *s, int64_t block_pos, int32_t offset);
int or_stream_pos_of(or_stream *s, int64_t flat, int64_t *block_pos, int32_t *offset);

/* eager.Checker.apply (check/.../eager/Checker.scala:24-126) at flat position p. */
int or_eager_check(or_stream *s, int64_t p, const int32_t *contig_len, int32_t n_contigs,
                   int32_t reads_to_check);
/* full.Checker.apply (check/.../full/Checker.scala:22-184) at flat position p. */
uint32_t or_full_check(or_stream *s, int64_t p, const int32_t *contig_len,
                       int32_t n_contigs, int32_t reads_to_check);

/* Same checks over a caller-provided flat buffer of `total` bytes (stream end = total). */
int or_eager_check_buf(const uint8_t *U, int64_t total, int64_t p, const int32_t *contig_len,
                       int32_t n_contigs, int32_t reads_to_check);
uint32_t or_full_check_buf(const uint8_t *U, int64_t total, int64_t p,
                           const int32_t *contig_len, int32_t n_contigs,
                           int32_t reads_to_check);

/* Eager at every flat position in [begin, end): bit i of out_bits <- eager(begin+i).
 * Returns the number of true positions. */
int64_t or_eager_range(or_stream *s, int64_t begin, int64_t end, const int32_t *contig_len,
                       int32_t n_contigs, int32_t reads_to_check, uint8_t *out_bits);
/* Full check at every flat position in [begin, end) -> out[i] (may be NULL), plus the
 * FullCheck aggregation (FullCheck.scala:142-192):
 *   counts[nnz*19 + f]   for nnz in [0, 21): flag f set at a position with nnz fields
 *   rbe_hist[nnz*64 + r] positions with readsBeforeError r (r < 64) and nnz fields
 *   n_success            positions returning Success
 * Positions equal to Flags.TooFewFixedBlockBytes (bit0 only, rbe 0) are excluded. */
int64_t or_full_range(or_stream *s, int64_t begin, int64_t end, const int32_t *contig_len,
                      int32_t n_contigs, int32_t reads_to_check, uint32_t *out,
                      int64_t *counts, int64_t *rbe_hist);

/* FindRecordStart.withDelta (check/.../spark/FindRecordStart.scala:30-63) from
 * Pos(block_pos, 0): returns OR_OK with flat position/delta, or OR_NO_READ_FOUND. */
int or_find_record_start(or_stream *s, int64_t from_flat, const int32_t *contig_len,
                         int32_t n_contigs, int32_t reads_to_check, int32_t max_read_size,
                         int64_t *out_flat, int32_t *out_delta);

/* BAM header (check/.../header/Header.scala:26-60): contig lengths + end position.
 * Returns n_ref (>= 0) or -code; writes up to cap lengths; *end_flat = flat end. */
int32_t or_parse_header(or_stream *s, int32_t *contig_len, int32_t cap, int64_t *end_flat);

/* PosStream chain (check/.../iterator/PosStream.scala:14-22) from flat `from`:
 * record starts while start < stop_flat; writes up to cap flats; returns count. */
int64_t or_record_chain(or_stream *s, int64_t from, int64_t stop_flat, int64_t *out,
                        int64_t cap);

/* Hadoop FileInputFormat split arithmetic (SPLIT_SLOP 1.1).  Returns the number of
 * splits; writes starts/ends when non-NULL. */
int64_t or_file_splits(int64_t file_size, int64_t split_size, int64_t *starts,
                       int64_t *ends, int64_t cap);

/* loadSplitsAndReads / loadBam per split (CanLoadBam.scala:196-357): for split
 * [start, end): FindBlockStart -> FindRecordStart -> chain records while
 * vpos < Pos(end, 0).  Outputs the first record vpos (htsjdk encoding) and count.
 * Returns OR_OK or an error code (OR_SEARCH_FAILED, OR_NO_READ_FOUND, ...). */
int or_split(const uint8_t *file, int64_t fsize, int64_t start, int64_t end,
             const int32_t *contig_len, int32_t n_contigs, int32_t blocks_to_check,
             int32_t reads_to_check, int32_t max_read_size, uint64_t *first_vpos,
             int64_t *count);

/* CPU baseline: inflate the blocks [b0, b1) of a loaded whole-file stream again into a
 * scratch buffer and run eager at every position of them, on `threads` pthreads.
 * Returns elapsed seconds; *positions / *trues report the work done. */
double or_bench_inflate_check(const uint8_t *file, int64_t fsize, const or_block *blocks,
                              int64_t b0, int64_t b1, const int32_t *contig_len,
                              int32_t n_contigs, int32_t reads_to_check, int32_t threads,
                              int64_t *positions, int64_t *trues);

/* CRC32 of a buffer (zlib), for block footers. */
uint32_t or_crc32(const uint8_t *b, int64_t n);

/* zlib version string of the library the oracle links (stated beside the CPU baseline). */
const char *or_zlib_version(void);

#ifdef __cplusplus
}
#endif
#endif
