/*
 * sparkbam.h -- C-ABI of libsparkbam_hip.so, the MI355X (gfx950) implementation of
 * spark-bam's BGZF-inflate + BAM record-boundary hot path.
 *
 * This is the drop-in boundary: plain pointers and sizes, no framework types.  Each
 * entry point names the reference interface it replaces (paths relative to the
 * reference repository root).  The reference's host side is Scala on the JVM; the
 * JNI binding a maintainer would add is shown in INTEGRATION.md.
 *
 * Conventions:
 *  - Every call returns an int status: SBH_OK or one of SBH_E_*, which map one-to-one
 *    onto the reference's exceptions (see below).  sbh_last_error() gives the message.
 *  - The caller owns every host buffer.  A context owns its device memory.
 *  - Threading.  One context per device per process, shared by every thread (a Spark
 *    executor's concurrent tasks).  Any number of threads may call into one context at once
 *    as long as each SHARD is used by one thread at a time -- the reference's model, where
 *    each task builds its own channel and Checker (load/.../CanLoadBam.scala:316-320,
 *    check/.../PosChecker.scala:19-20 share buffers inside one checker only).  Each shard
 *    enqueues its device work on its own HIP stream, so two tasks' shards run concurrently
 *    and one task's waits cover its own work only; context-level calls (sbh_run_stream2,
 *    sbh_check_stream, sbh_find_blocks, sbh_bgzf_compress*) build their own shards per call
 *    (sbh_run_stream2 takes a window cache from a pool in the context, one per concurrent
 *    caller).  sbh_last_error / sbh_last_error_detail report the calling THREAD's last failed
 *    call on that context, so a task always reads back its own failure.  sbh_ctx_set_stream
 *    and sbh_ctx_destroy are setup/teardown calls: no other call may run on the context then
 *    (shards created after sbh_ctx_set_stream enqueue on the caller's stream instead of their own).
 *  - Offsets: "file offsets" are byte offsets in the compressed BGZF file; "flat"
 *    offsets index the shard's concatenated uncompressed bytes (the reference's
 *    UncompressedBytes view, bgzf/.../block/UncompressedBytes.scala:13-87).  A
 *    virtual position Pos(blockPos, offset) is the htsjdk long blockPos<<16|offset
 *    (bgzf/.../Pos.scala:24).
 */
#ifndef SPARKBAM_H
#define SPARKBAM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---- */
#define SBH_OK 0
#define SBH_E_ARG 1                  /* IllegalArgumentException                     */
#define SBH_E_HIP 2                  /* device/runtime failure                       */
#define SBH_E_NOMEM 3
#define SBH_E_HEADER_PARSE 10        /* HeaderParseException (Header.scala:50-57)    */
#define SBH_E_HEADER_SEARCH_FAILED 11 /* HeaderSearchFailedException (FindBlockStart.scala:31-35) */
#define SBH_E_TRUNCATED 12           /* EOFException escaping MetadataStream         */
#define SBH_E_INFLATE_SIZE 13        /* IOException "Expected N decompressed bytes"  (Stream.scala:52-54) */
#define SBH_E_INFLATE_DATA 14        /* java.util.zip.DataFormatException             */
#define SBH_E_BAD_ISIZE 15           /* ISIZE outside [0, 65536]                      */
#define SBH_E_NO_READ_FOUND 16       /* NoReadFoundException (FindRecordStart.scala:66-71) */
#define SBH_E_NEED_HALO 17           /* result depends on bytes past the resident range */
#define SBH_E_STATE 18               /* call order violated (e.g. check before inflate) */
#define SBH_E_NOT_FOUND 19           /* Pos not in the indexed block chain            */
#define SBH_E_BAD_RECORD 20          /* record does not fit its block / the stream (htsjdk decode throws) */

/* ---- full-checker result word (check/.../full/error/Flags.scala:21-45) ----
 *  bit 31     : Success(readsParsed)
 *  bit 30     : unknown (needs bytes past an open shard end; never in a valid run)
 *  bits 20-29 : readsParsed (Success) or readsBeforeError (Flags)
 *  bits 0-18  : the 19 Flags booleans in the serde order of Flags.scala:203-222:
 *    0 tooFewFixedBlockBytes  1 negativeReadIdx  2 tooLargeReadIdx  3 negativeReadPos
 *    4 tooLargeReadPos  5 negativeNextReadIdx  6 tooLargeNextReadIdx
 *    7 negativeNextReadPos  8 tooLargeNextReadPos  9 tooFewBytesForReadName
 *    10 nonNullTerminatedReadName  11 nonASCIIReadName  12 noReadName  13 emptyReadName
 *    14 tooFewBytesForCigarOps  15 invalidCigarOp  16 emptyMappedCigar
 *    17 emptyMappedSeq  18 tooFewRemainingBytesImplied                              */
#define SBH_FULL_SUCCESS 0x80000000u
#define SBH_FULL_UNKNOWN 0x40000000u
#define SBH_FULL_N_SHIFT 20
#define SBH_FULL_FLAGS_MASK 0x7FFFFu
/* Counts aggregation layout: counts[nnz * 19 + flag], nnz = Flags.numNonZeroFields
 * (Flags.scala:118-123) in [0, 21); rbe_hist[nnz * 64 + readsBeforeError]. */
#define SBH_NNZ_MAX 21
#define SBH_RBE_MAX 64

/* block flags */
#define SBH_BLOCK_EMPTY 1u     /* dataLength == 2: the stream ends at this block (Stream.scala:56-58) */
#define SBH_BLOCK_TRUNCATED 2u /* runs past the resident bytes                     */

typedef struct sbh_ctx sbh_ctx;
typedef struct sbh_shard sbh_shard;

/* bgzf Metadata(start, compressedSize, uncompressedSize) (bgzf/.../block/Metadata.scala:6-8)
 * plus the header size, flat start and inflate status. */
typedef struct {
  uint64_t start;  /* file offset of the block header */
  uint64_t ustart; /* flat offset of its first uncompressed byte */
  uint32_t csize;
  uint32_t hsize;
  uint32_t usize;
  uint32_t flags;  /* SBH_BLOCK_* */
} sbh_block;

/* ---- context ---- */
int sbh_ctx_create(int device, sbh_ctx **out);
int sbh_ctx_destroy(sbh_ctx *ctx);
const char *sbh_last_error(const sbh_ctx *ctx);
/* The last error's status and the fields the reference's exception is constructed from;
 * returns how many fields the error carries (fields[0..min(n, cap)) are written):
 *   SBH_E_HEADER_PARSE         {header file offset, idx, actual, expected}  -> HeaderParseException(idx: Int,
 *                              actual: Byte, expected: Byte) (bgzf/.../block/HeaderParseException.scala:6-11)
 *   SBH_E_HEADER_SEARCH_FAILED {start, positionsAttempted}  -> HeaderSearchFailedException(path, start,
 *                              positionsAttempted) (bgzf/.../block/HeaderSearchFailedException.scala:7-12)
 *   SBH_E_NO_READ_FOUND        {start (file offset of a split, or the flat position searched from),
 *                              maxReadSize} -> NoReadFoundException(path, start, maxReadSize)
 *                              (check/.../spark/FindRecordStart.scala:66-71)
 *   SBH_E_INFLATE_SIZE         {block start, expected bytes}  -> IOException (Stream.scala:52-54)
 *   SBH_E_INFLATE_DATA         {block start}  -> DataFormatException
 *   anything else              no fields */
int32_t sbh_last_error_detail(const sbh_ctx *ctx, int32_t *code, int64_t *fields, int32_t cap);
/* Use a caller-owned hipStream_t (e.g. torch.cuda.current_stream().cuda_stream). */
int sbh_ctx_set_stream(sbh_ctx *ctx, void *hip_stream);
int sbh_ctx_synchronize(sbh_ctx *ctx);
const char *sbh_version(void);

/* Page-locked host memory (hipHostMalloc): compressed bytes handed over in it are copied to
 * HBM asynchronously, overlapping the kernels (sbh_run_stream).  A JNI binding wraps it in a
 * direct ByteBuffer. */
int sbh_host_alloc(uint64_t n, void **out);
int sbh_host_free(void *p);

/* Header.make (bgzf/.../block/Header.scala:48-83): host-side parse of 18 bytes. */
int sbh_header_make(const uint8_t *bytes, uint64_t avail, int32_t *hsize, int32_t *csize);

/* ---- shards: compressed bytes [file_offset, file_offset + n) resident in HBM ----
 * comp may be a host or a device pointer (comp_on_device); the shard keeps a copy
 * (device pointers are copied device-to-device).  file_size locates EOF: when
 * file_offset + n == file_size the resident bytes end at EOF, otherwise the end is
 * "open" and results that would need later bytes report SBH_E_NEED_HALO. */
int sbh_shard_create(sbh_ctx *ctx, const void *comp, uint64_t n, uint64_t file_offset,
                     uint64_t file_size, int comp_on_device, sbh_shard **out);
int sbh_shard_destroy(sbh_shard *sh);
/* Replace a shard's resident bytes with [file_offset, file_offset + n) of the same file (same
 * file_size), keeping its device allocations (grow-only): a window sliding along a file
 * (jni/Native.scala GpuWindow, sbh_check_stream) reuses one shard instead of allocating per
 * window.  Index, inflate and checker state are reset; the contig lengths are kept. */
int sbh_shard_load(sbh_shard *sh, const void *comp, uint64_t n, uint64_t file_offset, int comp_on_device);
/* Device pointer of the resident compressed bytes (padded). */
const void *sbh_shard_comp_device_ptr(sbh_shard *sh);

/* FindBlockStart.apply(path, start, in, bgzfBlocksToCheck) (FindBlockStart.scala:8-36):
 * smallest file offset >= start where bgzf_blocks_to_check consecutive headers parse. */
int sbh_find_block_start(sbh_shard *sh, uint64_t start, int32_t bgzf_blocks_to_check,
                         uint64_t *out);

/* MetadataStream from `start` (MetadataStream.scala:16-58) over the resident bytes:
 * builds the device block table (the chain of blocks from start, empty blocks
 * included and flagged) and the flat layout.  start must be a block start. */
int sbh_index(sbh_shard *sh, uint64_t start, uint64_t *n_blocks, uint64_t *flat_size);
int sbh_get_blocks(sbh_shard *sh, uint64_t first, uint64_t count, sbh_block *out);

/* StreamI._advance's Inflater(nowrap=true).inflate (Stream.scala:31-71) for every
 * indexed block: the shard's flat uncompressed buffer in HBM.  Fails with the first
 * block error in file order (SBH_E_INFLATE_SIZE / _DATA / _BAD_ISIZE, *bad_block). */
int sbh_inflate(sbh_shard *sh, uint64_t *bad_block);

/* CRC32 of every inflated block's bytes against its BGZF footer (the reference reads only
 * ISIZE, Stream.scala:47-54; SURVEY 8d asks for CRC32 as the in-run correctness check).
 * *n_bad = blocks whose CRC differs; *first_bad (optional) = the first one's file offset. */
int sbh_verify_crc(sbh_shard *sh, uint64_t *n_bad, uint64_t *first_bad);
/* Copy flat bytes [flat, flat + n) to host memory. */
int sbh_read_flat(sbh_shard *sh, uint64_t flat, uint64_t n, uint8_t *out);
/* Device pointer of the flat bytes (read-only: the library keeps the zero pad past the flat
 * end between calls and does not re-zero it when the size is unchanged). */
const void *sbh_flat_device_ptr(sbh_shard *sh);

/* Pos <-> flat (canonical positions, Pos.scala; curPos rolls to the next block). */
int sbh_flat_of(sbh_shard *sh, uint64_t block_pos, uint32_t offset, uint64_t *flat);
int sbh_pos_of(sbh_shard *sh, uint64_t flat, uint64_t *block_pos, uint32_t *offset);
/* Flat offset of the first block whose file offset is >= file_off (the flat image
 * of Pos(file_off, 0) as an exclusive bound). */
int sbh_flat_bound(sbh_shard *sh, uint64_t file_off, uint64_t *flat);

/* Contig lengths (BAM header n_ref x l_ref; check/.../header/Header.scala:37-53). */
int sbh_set_contigs(sbh_shard *sh, const int32_t *lens, int32_t n);

/* eager.Checker.apply at every flat position of [begin, end)
 * (check/.../eager/Checker.scala:24-126).  The bitmap stays on the device (used by
 * find_record_start / count_records); out_bits (optional, (end-begin+7)/8 bytes,
 * bit i = position begin+i, LSB first) receives a copy. */
int sbh_check_eager(sbh_shard *sh, uint64_t begin, uint64_t end, int32_t reads_to_check,
                    uint8_t *out_bits, uint64_t *n_true);

/* Copy [begin, end) of the eager bitmap the last sbh_check_eager / sbh_run_shard left on
 * the device (the batch behind Checker.apply(pos) answers).  begin must lie in the
 * bitmap's range at a multiple of 8 positions from its start; SBH_E_STATE if there is
 * no bitmap. */
int sbh_eager_bits(sbh_shard *sh, uint64_t begin, uint64_t end, uint8_t *out_bits);

/* full.Checker.apply at every flat position of [begin, end)
 * (check/.../full/Checker.scala:22-184) with the FullCheck aggregation
 * (cli/.../check/full/FullCheck.scala:142-192).  Optional outputs: out_words
 * (end-begin words), counts (21*19), rbe_hist (21*64), close-call positions
 * (numNonZeroFields <= 2) as (flat, word) pairs up to close_cap. */
int sbh_check_full(sbh_shard *sh, uint64_t begin, uint64_t end, int32_t reads_to_check,
                   uint32_t *out_words, uint64_t *counts, uint64_t *rbe_hist,
                   uint64_t *n_success, uint64_t *close_flat, uint32_t *close_word,
                   uint64_t close_cap, uint64_t *n_close);

/* FindRecordStart.withDelta (check/.../spark/FindRecordStart.scala:30-63) from flat
 * position from_flat: first eager-true position within max_read_size positions of
 * the stream. */
int sbh_find_record_start(sbh_shard *sh, uint64_t from_flat, int32_t reads_to_check,
                          int32_t max_read_size, uint64_t *out_flat, int32_t *out_delta);

/* Record chain from first_flat (PosStream.scala:14-22): number of records whose
 * start is < end_flat (RecordStream.takeWhile(pos < Pos(end, 0)),
 * CanLoadBam.scala:350-355).  Uses the eager bitmap when it covers the range and
 * the chain verifies against it; otherwise an exact sequential walk. */
int sbh_count_records(sbh_shard *sh, uint64_t first_flat, uint64_t end_flat,
                      uint64_t *count);

/* One Hadoop split of loadReadsAndPositions / loadSplitsAndReads
 * (load/.../CanLoadBam.scala:316-356): FindBlockStart(start) -> FindRecordStart ->
 * records while vpos < Pos(end, 0).  first_vpos = htsjdk virtual offset of the
 * first record (valid when *count > 0). */
int sbh_split(sbh_shard *sh, uint64_t start, uint64_t end, int32_t bgzf_blocks_to_check,
              int32_t reads_to_check, int32_t max_read_size, uint64_t *first_vpos,
              uint64_t *count);

/* The record chain from first_flat (PosStream.scala:14-22) as sbh_count_records, plus its
 * exit: the first chain record at/after end_flat (or the stream end).  The multi-GPU stitch
 * re-walks a shard from its upstream neighbour's exit with this. */
int sbh_chain_from(sbh_shard *sh, uint64_t first_flat, uint64_t end_flat, uint64_t *count,
                   uint64_t *exit_flat);

/* Every split of loadSplitsAndReads at once (CanLoadBam.scala:283-297, 316-356): for split
 * i = [starts[i], ends[i]) (file offsets) the same (status[i], first_vpos[i], counts[i]) as
 * sbh_split.  FindBlockStart + FindRecordStart of all splits run in one launch over the
 * eager bitmap, the record chain is proven once over their union, and every count is one
 * more launch; a split off that path (a failed or halo-crossing search, an empty block, a
 * record start outside the bitmap, a start that is a false positive) is decided by
 * sbh_split.  *n_host (optional) = how many were.  Returns SBH_OK unless the batch itself
 * failed; per-split errors are in status[]. */
int sbh_split_starts(sbh_shard *sh, const uint64_t *starts, const uint64_t *ends, uint64_t n,
                     int32_t bgzf_blocks_to_check, int32_t reads_to_check, int32_t max_read_size,
                     uint64_t *first_vpos, uint64_t *counts, int32_t *status, uint64_t *n_host);

/* check-bam -s's comparison of the eager checker with the `.records` truth
 * (cli/.../CheckerApp.scala:65-227, CheckBam.scala) on the device, over the flat ranges
 * [range_begin[r], range_end[r]) (sorted, disjoint): rec_vpos[] are the truth records as
 * htsjdk virtual positions (the `.records` lines, any order).  out[0..3] = true positives,
 * false positives, false negatives, truth records whose block is not in the shard.  fp_flat /
 * fn_flat (optional) receive up to fp_cap / fn_cap mismatching flat positions, sorted (all of
 * them when out[1] <= fp_cap, resp. out[2] <= fn_cap; past the cap an arbitrary subset, not
 * the first ones by position). */
int sbh_check_records(sbh_shard *sh, const uint64_t *range_begin, const uint64_t *range_end,
                      uint64_t n_ranges, int32_t reads_to_check, const uint64_t *rec_vpos,
                      uint64_t n_rec, uint64_t *out, uint64_t *fp_flat, uint64_t fp_cap,
                      uint64_t *fn_flat, uint64_t fn_cap);

/* The whole per-shard hot path as one call (the benchmark step): index from
 * index_start, inflate, eager check at every position of the owned flat range
 * [flat(own_begin_file), flat_bound(own_end_file)), then the owned split:
 * first record >= Pos(own_begin_block, 0) and the record count while
 * vpos < Pos(own_end_file, 0).  All device work is enqueued on the context stream;
 * results are read back at the end. */
typedef struct {
  uint64_t n_blocks;
  uint64_t comp_bytes;   /* compressed bytes of the owned blocks              */
  uint64_t flat_bytes;   /* uncompressed bytes of the owned blocks (positions) */
  uint64_t n_true;       /* eager-true positions in the owned range           */
  uint64_t first_vpos;   /* first record of the owned split (if count > 0)    */
  uint64_t count;        /* records of the owned split                        */
  uint64_t exit_flat;    /* first chain record at/after the owned end         */
  int32_t status;
  int32_t anomalies;     /* chain/bitmap disagreements resolved by the walk   */
} sbh_shard_result;

int sbh_run_shard(sbh_shard *sh, uint64_t index_start, uint64_t own_end_file,
                  int32_t reads_to_check, int32_t max_read_size, sbh_shard_result *res);

/* Device time (ms, HIP events) of the stages of the last sbh_run_shard: [0] index,
 * [1] inflate + eager check (one pipeline over block batches on three streams),
 * [2] k_eager, [3] record split/count, [4] k_huff, [5] k_lz -- [2], [4], [5] summed
 * over the pipeline's launches, each timed on its own stream.  Returns the number of
 * stages written (<= cap, at most 6). */
int sbh_stage_times(sbh_shard *sh, double *ms, int32_t cap);

/* ---- a shard streamed through bounded HBM ----
 * sbh_run_shard over host-resident compressed bytes [file_offset, file_offset + n) (pinned
 * memory lets the copies overlap the kernels), in windows of about `window` compressed bytes:
 * window w owns the blocks starting in [lo_w, hi_w), loads [lo_w, hi_w + halo), and its
 * successor's bytes are copied host -> HBM on a second stream while it runs, so HBM holds two
 * windows' compressed bytes and one window's working set however large the shard
 * (Stream.scala:80-122 / SplitRDD.scala:33-52 bound the reference per split).  index_start is
 * the owned range's first block (UINT64_MAX: FindBlockStart(file_offset, 5)).  Windows stitch
 * like ranks (a mismatch re-walks the later window from the earlier exit); a window
 * that needs bytes past its halo grows the halo x4 and runs again.  out_bits (optional, host,
 * zeroed by the caller, out_bits_cap bytes): the eager bit of every owned flat position. */
typedef struct {
  uint64_t n_windows, n_blocks;
  uint64_t comp_bytes;  /* compressed bytes of the owned blocks                      */
  uint64_t flat_bytes;  /* their uncompressed bytes (checked positions)              */
  uint64_t n_true;      /* eager-true owned positions                                */
  uint64_t count;       /* records of the owned range (the stitched chain)           */
  uint64_t first_vpos;  /* first record (UINT64_MAX if none)                         */
  uint64_t exit_vpos;   /* first chain record at/after the owned end (UINT64_MAX: none) */
  int32_t status, rewalks, host_pinned, pad;
  double ms_wall;       /* wall time of the call (host clock), copies included       */
  double ms_h2d;        /* summed host -> HBM copy time (HIP events on the copy stream) */
  double stage_ms[6];   /* sbh_stage_times summed over the windows                   */
  uint64_t halo_final;
  /* sbh_run_stream2 only (zero otherwise): */
  uint64_t crc_bad_blocks;  /* owned blocks whose BGZF footer CRC32 differs (opts.verify_crc) */
  uint64_t crc_first_bad;   /* file offset of the first such block                   */
  uint64_t splits_host;     /* splits decided by the exact per-split path (sbh_split)  */
  double ms_splits;         /* device + host time of the per-split work, summed       */
  double ms_crc;            /* CRC32 kernel time, summed over the windows              */
} sbh_stream_result;
int sbh_run_stream(sbh_ctx *ctx, const void *host_comp, uint64_t n, uint64_t file_offset,
                   uint64_t file_size, uint64_t index_start, uint64_t own_end_file, uint64_t window,
                   uint64_t halo, const int32_t *contig_len, int32_t n_contigs, int32_t reads_to_check,
                   int32_t max_read_size, uint8_t *out_bits, uint64_t out_bits_cap,
                   sbh_stream_result *res);

/* sbh_run_stream with per-split results and an in-run CRC check: loadSplitsAndReads' per-split
 * answer for a shard larger than HBM (CanLoadBam.scala:283-297,316-356 over SplitRDD.scala:
 * 33-52's partitions).  When n_splits > 0, split i = [split_start[i], split_end[i]) (file
 * offsets, sorted, split_start[i] < split_end[i] <= split_start[i + 1], every start in
 * [file_offset, own_end_file), the last end <= own_end_file): windows are cut at split starts,
 * so every split lies in one window, and each window's splits get sbh_split_starts' (status,
 * first_vpos, count) -- exactly what sbh_split returns for them on the whole file.
 * verify_crc: every owned block's inflated bytes against its footer CRC32 (crc_bad_blocks). */
typedef struct {
  uint64_t window, halo;
  int32_t reads_to_check, max_read_size, bgzf_blocks_to_check, verify_crc;
  const uint64_t *split_start, *split_end; /* n_splits entries, or NULL with n_splits = 0 */
  uint64_t n_splits;
  uint64_t *split_first_vpos, *split_count; /* out, n_splits entries                      */
  int32_t *split_status;                   /* out: SBH_OK or the split's SBH_E_* status */
  uint8_t *out_bits;
  uint64_t out_bits_cap;
} sbh_stream_opts;
int sbh_run_stream2(sbh_ctx *ctx, const void *host_comp, uint64_t n, uint64_t file_offset,
                    uint64_t file_size, uint64_t index_start, uint64_t own_end_file,
                    const int32_t *contig_len, int32_t n_contigs, const sbh_stream_opts *opts,
                    sbh_stream_result *res);

/* ---- the all-positions modes over a file of any size ----
 * Blocks.apply (check/src/main/scala/org/hammerlab/bam/check/Blocks.scala:47-208) picks the
 * BGZF blocks whose every position check-bam / full-check examine; CallPartition
 * (cli/.../CallPartition.scala:23-54) and FullCheck.checkPartition (cli/.../full/FullCheck.scala:
 * 65-86) then call the checkers at every offset of those blocks, reading the chain past them
 * freely.  Both calls below take the whole file in host memory (mapped or pinned) and move it
 * through HBM in windows of about `window` compressed bytes, so HBM use is bounded whatever
 * the file size; a window whose answers need bytes past its halo grows the halo x4 and runs
 * again. */

/* Blocks.apply's branch without a `.blocks` file (Blocks.scala:141-206): for split i =
 * [split_start[i], split_end[i]) (file offsets, ascending), FindBlockStart(split_start[i],
 * bgzf_blocks_to_check) then MetadataStream from there while the block start is < split_end[i]
 * (an empty block ends the stream, MetadataStream.scala:43-45).  Writes (start, csize, usize)
 * of each block into out[] (ustart / hsize / flags zero; ustart = the split index) up to cap
 * entries, in split order; *n_out = how many there are.  A split whose search fails answers
 * SBH_E_HEADER_SEARCH_FAILED (HeaderSearchFailedException) for the whole call. */
int sbh_find_blocks(sbh_ctx *ctx, const void *host_file, uint64_t file_size, const uint64_t *split_start,
                    const uint64_t *split_end, uint64_t n_splits, int32_t bgzf_blocks_to_check, uint64_t window,
                    sbh_block *out, uint64_t cap, uint64_t *n_out);

/* check-bam -s and full-check over the given blocks (file offsets of block starts, ascending --
 * Blocks.apply's partitions concatenated): every uncompressed offset of every listed block is
 * checked.  truth_vpos (optional, ascending htsjdk virtual positions: the `.records` file,
 * CheckerApp.scala:65-227) turns the eager calls into TP / FP / FN with the mismatching
 * positions (first fp_cap / fn_cap of them, as vpos); full != 0 adds full.Checker's FullCheck
 * aggregation (FullCheck.scala:142-192): Counts and readsBeforeError histograms by
 * numNonZeroFields (include/sparkbam.h layout above) and the close calls (<= 2 non-zero
 * fields) as (vpos, word) up to close_cap, ascending. */
typedef struct {
  uint64_t window, halo;
  int32_t reads_to_check, full;
  const uint64_t *blocks;
  uint64_t n_blocks;
  const uint64_t *truth_vpos; /* NULL: no comparison (n_true only) */
  uint64_t n_truth;
  uint64_t *fp_vpos, *fn_vpos;
  uint64_t fp_cap, fn_cap;
  uint64_t *counts;   /* full: 21 * 19 */
  uint64_t *rbe_hist; /* full: 21 * 64 */
  uint64_t *close_vpos;
  uint32_t *close_word;
  uint64_t close_cap;
} sbh_check_opts;
typedef struct {
  uint64_t n_windows, positions, comp_bytes; /* checked positions and their blocks' compressed bytes */
  uint64_t n_true;                           /* eager-true checked positions                      */
  uint64_t tp, fp, fn, unknown;              /* vs truth_vpos (unknown: truth records off the chain) */
  uint64_t n_success, n_close;               /* full                                             */
  uint64_t halo_final;
  double ms_wall, ms_h2d;
} sbh_check_result;
int sbh_check_stream(sbh_ctx *ctx, const void *host_file, uint64_t file_size, const int32_t *contig_len,
                     int32_t n_contigs, const sbh_check_opts *opts, sbh_check_result *res);

/* ---- record field extraction ----
 * RecordStream from first_flat while the record start is < end_flat, decoded like
 * htsjdk BAMRecordCodec.decode (check/.../iterator/RecordStream.scala:16-41,
 * load/.../CanLoadBam.scala:244-264), into columns.  Record starts follow the chain
 * (next = start + 4 + block_size; the verified eager bitmap when it covers the range).
 * sbh_records_scan decodes on the device and reports the sizes; sbh_records_fetch copies
 * the columns of the last scan into caller buffers (any pointer may be NULL). */
typedef struct {
  uint64_t n;           /* records                                              */
  uint64_t name_bytes;  /* read names, each l_read_name bytes with its NUL      */
  uint64_t cigar_ops;   /* CIGAR ops                                            */
  uint64_t bases;       /* sequence letters (= quality bytes)                   */
  uint64_t aux_bytes;   /* raw tag bytes                                        */
} sbh_records_sizes;
typedef struct {
  uint64_t *flat;                                          /* [n] record start (flat) */
  int32_t *ref_id, *pos, *next_ref_id, *next_pos, *tlen;   /* [n] as stored (pos 0-based, -1 unset) */
  uint16_t *flag, *bin;                                    /* [n] */
  uint8_t *mapq;                                           /* [n] */
  uint64_t *name_off, *cigar_off, *seq_off, *aux_off;      /* [n + 1] exclusive prefix offsets */
  char *names;                                             /* [name_bytes] */
  uint32_t *cigar;                                         /* [cigar_ops] op_len << 4 | op */
  char *seq;                                               /* [bases] "=ACMGRSVTWYHKDBN" letters */
  uint8_t *qual;                                           /* [bases] phred (0xff: absent) */
  uint8_t *aux;                                            /* [aux_bytes] tags as stored */
  uint64_t *vpos;                                          /* [n] record start as an htsjdk virtual
                                                              position (canonical Pos, Pos.scala:12-43);
                                                              available after sbh_split_records too */
} sbh_records_out;
int sbh_records_scan(sbh_shard *sh, uint64_t first_flat, uint64_t end_flat, sbh_records_sizes *out);
int sbh_records_fetch(sbh_shard *sh, const sbh_records_out *out);

/* One Hadoop FileSplit [start, end) of loadReadsAndPositions in ONE call (load/.../CanLoadBam.scala:
 * 316-356, the body of its fileSplitsRDD.flatMap): FindBlockStart(start, bgzf_blocks_to_check)
 * (FindBlockStart.scala:8-36), MetadataStream + inflate from that block, the eager check at every
 * position of [Pos(blockStart, 0), Pos(end, 0)), FindRecordStart from Pos(blockStart, 0)
 * (FindRecordStart.scala:11-30), and the records from it while pos < Pos(end, 0) (RecordStream.
 * takeWhile): their starts, and with decode != 0 BAMRecordCodec.decode's columns, for
 * sbh_records_fetch (decode == 0: only its `flat` column may be asked for).  The shard must hold
 * the split's bytes from `start` plus a halo (sbh_shard_load reuses one shard for every split a
 * thread runs).  Errors: SBH_E_HEADER_SEARCH_FAILED {start, positionsAttempted};
 * SBH_E_NO_READ_FOUND {blockStart, maxReadSize} (NoReadFoundException(path, blockStart,
 * maxReadSize)); SBH_E_NEED_HALO when an answer needs bytes past the resident range (reload with
 * a larger halo) -- a last record running past the halo included. */
typedef struct {
  uint64_t block_start;     /* FindBlockStart(start)                                        */
  uint64_t n_blocks;        /* blocks indexed from it (sbh_get_blocks), halo included        */
  uint64_t flat_size;       /* their uncompressed bytes                                      */
  uint64_t owned_flat;      /* flat image of Pos(end, 0): the split's positions [0, owned)   */
  uint64_t first_flat;      /* FindRecordStart(Pos(blockStart, 0)) (may be >= owned_flat)    */
  uint64_t first_vpos;      /* its htsjdk virtual position (when sizes.n > 0)                */
  uint64_t n_true;          /* eager-true positions of [0, owned_flat)                       */
  sbh_records_sizes sizes;  /* sizes.n = the split's records; column sizes when decoded      */
} sbh_split_records_result;
int sbh_split_records(sbh_shard *sh, uint64_t start, uint64_t end, int32_t bgzf_blocks_to_check,
                      int32_t reads_to_check, int32_t max_read_size, int32_t decode,
                      sbh_split_records_result *out);

/* ---- loadBamIntervals ----
 * CanLoadBam.loadBamIntervals (load/.../CanLoadBam.scala:78-154) after the host has turned
 * the intervals into BAI chunks (getIntevalChunks, :410-444; Index.scala:11-93): for each
 * chunk [chunk_begin[c], chunk_end[c]) (flat positions of the chunk's start/end Pos), the
 * records from the chunk start while the start is < the chunk end, in chunk order, kept
 * when region(record) (:446-454) overlaps one of the intervals: (iv_ref[k], [iv_begin[k],
 * iv_end[k])) 0-based half-open, sorted by (ref, begin) and disjoint (a merged LociSet).
 * Leaves the kept records' columns for sbh_records_fetch, like sbh_records_scan. */
int sbh_records_scan_regions(sbh_shard *sh, const uint64_t *chunk_begin, const uint64_t *chunk_end,
                             uint64_t n_chunks, const int32_t *iv_ref, const int64_t *iv_begin,
                             const int64_t *iv_end, uint32_t n_iv, sbh_records_sizes *out);

/* ---- BGZF writer -------------------------------------------------
 * The block compressor behind HTSJDKRewrite (cli/src/main/scala/org/hammerlab/bam/rewrite/
 * HTSJDKRewrite.scala:62-67: SAMFileWriterFactory.makeBAMWriter -> htsjdk
 * BlockCompressedOutputStream): the uncompressed stream src[0, n) is cut every 65498 bytes and
 * each piece becomes one BGZF member, CRC32 + ISIZE footer, then the 28-byte empty EOF member.
 * sbh_bgzf_compress writes exactly htsjdk's bytes: each member is what java.util.zip.Deflater
 * (level 5, nowrap) = zlib 1.2.11 deflate_slow produces, and a member whose deflate stream does
 * not finish within htsjdk's 65518-byte buffer is re-deflated at level 0 (one stored block).
 * sbh_bgzf_compress_level: level 5 (SBH_LEVEL_HTSJDK) as above; 4 and 6..9 the same zlib at
 * that level (6 is samtools' default); 0 stored members; SBH_LEVEL_FAST this library's own
 * faster coder (hash-chain LZ77 with lazy matching, one dynamic-Huffman block per member, not
 * zlib's bytes).  src is a host or device pointer (src_on_device); out is host memory of at
 * least sbh_bgzf_compress_bound(n) bytes.  Device scratch is bounded by a batch of members,
 * whatever n: about 1.04 MB per member at levels 4..9 (prev 128 KiB, match records 512 KiB,
 * tokens 256 KiB, block record 16 KiB, two 65.6 KB slots), batches of up to 8192 members
 * (~8.5 GB; SBH_ZDEFLATE_BATCH overrides) and never more than half of the free HBM at the call
 * (at least 256 members); SBH_LEVEL_FAST batches up to 2048 members of ~0.4 MB.  The uncompressed
 * input (n bytes, when src is host memory) is staged in HBM as well.  *deflate_ms (optional): the
 * compress kernels' device time, summed over the batches (HIP events on the context's stream). */
#define SBH_LEVEL_HTSJDK 5
#define SBH_LEVEL_FAST (-1)
uint64_t sbh_bgzf_compress_bound(uint64_t n);
int sbh_bgzf_compress(sbh_ctx *ctx, const void *src, uint64_t n, int src_on_device, uint8_t *out,
                      uint64_t out_cap, uint64_t *out_size, uint64_t *n_blocks, float *deflate_ms);
int sbh_bgzf_compress_level(sbh_ctx *ctx, const void *src, uint64_t n, int src_on_device, int level,
                            uint8_t *out, uint64_t out_cap, uint64_t *out_size, uint64_t *n_blocks,
                            float *deflate_ms);

#ifdef __cplusplus
}
#endif
#endif /* SPARKBAM_H */
