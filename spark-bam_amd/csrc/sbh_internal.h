// sbh_internal.h -- device-side layouts shared by the HIP kernels and the C-ABI layer.
// CDNA4 (gfx950) only: 64-lane waves, 160 KiB LDS per CU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/sparkbam.h"

namespace sbh {

constexpr int WAVE = 64;

// Inclusive prefix sum over the 64 lanes of a wave in DPP steps (no LDS round trips):
// row_shr 1/2/4/8 within each 16-lane row, then row_bcast:15 and row_bcast:31 carry
// the row totals across rows (gfx9 DPP).  Inactive lanes must contribute 0.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return x;
}

// v from lane ^ M: quad DPP for 1 and 2, ds_swizzle (bit mode, within 32 lanes) for 4..16,
// ds_bpermute for 32.
template <uint32_t M>
__device__ __forceinline__ uint32_t xor_lane(uint32_t v) {
  if constexpr (M == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, false);
  else if constexpr (M == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, false);
  else if constexpr (M < 32) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, (int)((M << 10) | 0x1f));
  else return (uint32_t)__shfl_xor((int)v, (int)M);
}
template <uint32_t SIZE, uint32_t STRIDE>
__device__ __forceinline__ uint32_t bitonic_step(uint32_t k, uint32_t lane) {
  const uint32_t o = xor_lane<STRIDE>(k);
  const bool up = (lane & SIZE) == 0, lower = (lane & STRIDE) == 0;
  return (lower == up) ? (k < o ? k : o) : (k > o ? k : o);
}
// ascending sort of one key per lane across the wave
__device__ __forceinline__ uint32_t bitonic64(uint32_t k, uint32_t lane) {
  k = bitonic_step<2, 1>(k, lane);
  k = bitonic_step<4, 2>(k, lane), k = bitonic_step<4, 1>(k, lane);
  k = bitonic_step<8, 4>(k, lane), k = bitonic_step<8, 2>(k, lane), k = bitonic_step<8, 1>(k, lane);
  k = bitonic_step<16, 8>(k, lane), k = bitonic_step<16, 4>(k, lane), k = bitonic_step<16, 2>(k, lane);
  k = bitonic_step<16, 1>(k, lane);
  k = bitonic_step<32, 16>(k, lane), k = bitonic_step<32, 8>(k, lane), k = bitonic_step<32, 4>(k, lane);
  k = bitonic_step<32, 2>(k, lane), k = bitonic_step<32, 1>(k, lane);
  k = bitonic_step<64, 32>(k, lane), k = bitonic_step<64, 16>(k, lane), k = bitonic_step<64, 8>(k, lane);
  k = bitonic_step<64, 4>(k, lane), k = bitonic_step<64, 2>(k, lane), k = bitonic_step<64, 1>(k, lane);
  return k;
}

// Block table (struct of arrays, one entry per BGZF block of the chain, in file
// order).  Mirrors bgzf Metadata(start, compressedSize, uncompressedSize)
// (bgzf/.../block/Metadata.scala:6-8) plus the header size and flat start.
struct DevBlocks {
  uint64_t *cstart;  // compressed offset relative to the shard's first byte
  uint32_t *csize;   // BSIZE + 1
  uint32_t *hsize;   // 18 + XLEN - 6
  uint32_t *usize;   // ISIZE (0 for an empty block)
  uint64_t *ustart;  // flat offset of the block's first uncompressed byte
  uint32_t *flags;   // BLK_* bits
  uint32_t *status;  // inflate status per block (INF_*)
  uint32_t *ntok;    // LZ77 tokens k_huff emitted for the block (k_lz input)
};

constexpr uint32_t BLK_EMPTY = 1u;     // dataLength == 2: the stream ends here
constexpr uint32_t BLK_TRUNCATED = 2u;  // block runs past the resident bytes

// Inflate status codes per block (written by k_huff).
constexpr uint32_t INF_OK = 0;
constexpr uint32_t INF_SIZE = 1;      // fewer than ISIZE bytes produced
constexpr uint32_t INF_DATA = 2;      // DataFormatException (zlib Z_DATA_ERROR)
constexpr uint32_t INF_BAD_ISIZE = 3; // ISIZE outside [0, 65536]
constexpr uint32_t INF_SERIAL = 0xffu; // (inside inflate only) left to the serial decoder

// Eager tile geometry (check.hip): a workgroup decides ETILE positions and stages those
// plus a look-ahead; EAGER_REACH bounds the flat bytes past a tile's first position
// that its staged window touches (the pipelined run launches a tile only once they are
// inflated; reads beyond, by the exact path, defer the position instead).
#ifndef SBH_ETILE
#define SBH_ETILE 16384
#endif
constexpr uint64_t EAGER_TILE = SBH_ETILE;
constexpr uint64_t EAGER_REACH = SBH_ETILE + 4096 + 512 + 64;
constexpr uint64_t EAGER_SUB = EAGER_TILE / 4;  // one k_eager wave's share of a tile (4 waves)
#ifndef SBH_TSUM_CODE
// 1: compile the per-quarter-tile chain summaries (k_eager writes them, k_verify_chain_w reads
// them; SBH_TSUM=1 at run time turns them on).  0 (default): measured net slower (proof 0.46 ->
// 0.36 ms, k_eager 3.00 -> 3.24 ms per config-B step), and their branches alone cost the proof
// 0.34 -> 0.42 ms with the summaries off (r04q kernel trace).
#define SBH_TSUM_CODE 0
#endif
// Per quarter of an eager tile (EAGER_SUB positions, one k_eager wave's result words; written on
// k_eager's fast path; the chain proof, k_verify_chain_w, reads it instead of every true
// position's record length): the record step of the quarter's last true position, and the true
// positions whose step misses the next true position of the same quarter.
struct TileSum {
  uint64_t step_last;   // TS_NONE: none, or the record ends the stream; TS_DIRTY: no summary
  uint32_t n_anom;      // true positions whose step is not the tile's next true position
  uint32_t first_anom;  // offset of the first of them in the quarter (~0u: none)
};
constexpr uint64_t TS_NONE = ~0ull;
constexpr uint64_t TS_DIRTY = ~1ull;  // bits settled after k_eager (long-record queue, deferred,
                                      // unknown positions) or by its fallback path
// Bitmap set-bit prefix (launch_rec_positions_bits): one u64 per group of WPRE_GROUP
// consecutive words of [first, E) -- the set bits before the group; a lookup adds the
// popcounts of the group's earlier words (one 64-byte read).
constexpr uint32_t WPRE_GROUP = 16;

// Launchers (defined in the .hip files, called from sbh_api.hip).
// Inflate = k_huff (Huffman decode -> LZ77 tokens, block status) then k_lz (tokens ->
// flat bytes; a block that is one stored deflate block is copied from comp).  tok_buf: >= 4 B
// of token scratch per flat byte of the launched blocks, tok_buf[0] standing for flat offset
// tok_base (block b's tokens at tok_buf[ustart_b - tok_base ...]), so a shard can be inflated
// in batches of blocks that reuse one bounded token buffer.
hipError_t launch_huff(const uint8_t *comp, DevBlocks blocks, uint64_t nblocks, uint32_t *tok_buf, uint64_t tok_base,
                       hipStream_t stream);
// sieve (optional): bit p of the flat bitmap = position p may pass eager.Checker's refID / next
// refID range and pos / next pos sign tests (k_eager's first filter, evaluated by k_lz on the bytes
// still in its LDS ring; 1 wherever the block's WG cannot decide: seams, stored blocks).  nref1 =
// contigs + 1.
hipError_t launch_lz(const uint8_t *comp, DevBlocks blocks, uint64_t nblocks, const uint32_t *tok_buf,
                     uint64_t tok_base, uint8_t *U, hipStream_t stream, uint32_t *sieve = nullptr,
                     uint32_t nref1 = 0);
// *first = the first block of [0, n) whose status is not INF_OK (~0 if none).
// (init: set *first to ~0 first; false when the caller already did)
hipError_t launch_first_bad(const uint32_t *status, uint64_t n, unsigned long long *first, hipStream_t stream,
                            bool init = true);

// Record field extraction (records.hip): device columns of a decoded batch (the host
// view is sbh_records_out in sparkbam.h).
struct RecCols {
  int32_t *ref_id, *pos, *next_ref_id, *next_pos, *tlen;
  uint16_t *flag, *bin;
  uint8_t *mapq;
  char *names;
  uint32_t *cigar;
  char *seq;
  uint8_t *qual, *aux;
};
hipError_t launch_rec_positions_bits(const uint32_t *bits, uint64_t begin, uint64_t first, uint64_t E, uint64_t *cnt,
                                     uint64_t *wpre, uint64_t *tmp, uint64_t *pos, hipStream_t st);
hipError_t launch_rec_positions_chain(const uint8_t *U, uint64_t first, uint64_t E, uint64_t total, uint64_t cap,
                                      uint64_t *pos, hipStream_t st);
hipError_t launch_rec_sizes(const uint8_t *U, const uint64_t *pos, uint64_t n, uint64_t total, uint64_t *nm,
                            uint64_t *cg, uint64_t *sq, uint64_t *ax, unsigned long long *bad, hipStream_t st);
hipError_t launch_rec_fields(const uint8_t *U, const uint64_t *pos, uint64_t n, const uint64_t *nm_off,
                             const uint64_t *cg_off, const uint64_t *sq_off, const uint64_t *ax_off, const RecCols &c,
                             hipStream_t st);
hipError_t launch_region_keep(const uint8_t *U, const uint64_t *pos, uint64_t n, uint64_t total, const int32_t *iv_ref,
                              const int64_t *iv_begin, const int64_t *iv_end, uint32_t n_iv, uint64_t *keep,
                              hipStream_t st);
hipError_t launch_compact_u64(const uint64_t *in, const uint64_t *keep, const uint64_t *kpre, uint64_t n,
                              uint64_t *out, hipStream_t st);
// the chain proof's chunk of bitmap words (k_verify_chain_w: one wave, 4 words per lane)
constexpr uint64_t VC_CHUNK = 256;
// split counts from the proof's per-chunk set-bit counts (splits.hip): counts[i] += set bits of
// [first[i], E[i]) for the SPLIT_OK splits, the bitmap read only in each range's end chunks
// (chain_E != 0: counts are written, not added, and a range outside [chain_first, chain_E) gets
// SPLIT_NOCOUNT)
hipError_t launch_split_count_cc(const uint32_t *bits, uint64_t begin, const uint32_t *chunk_cnt, const uint64_t *first,
                                 const uint64_t *E, const uint32_t *code, uint64_t nsplit, unsigned long long *counts,
                                 hipStream_t st, uint64_t chain_first = 0, uint64_t chain_E = 0);
// record starts (flat) -> htsjdk virtual positions over the device block table
hipError_t launch_rec_vpos(const uint64_t *pos, uint64_t n, DevBlocks bl, uint64_t nblocks, uint64_t file_off,
                           uint64_t *vpos, hipStream_t st);
// BGZF footer CRC32 of every inflated, non-truncated block (crc.hip).
hipError_t launch_block_crc(const uint8_t *comp, DevBlocks bl, uint64_t nblocks, const uint8_t *U,
                            unsigned long long *n_bad, unsigned long long *first_bad, hipStream_t st);

// BGZF writer (deflate.hip): members are coded in batches of at most DEFLATE_BATCH 65498-byte
// pieces: k_prev (hash chains into prev), k_deflate (tokens into toks, one 64 KiB slot per
// member and its size), k_footer; k_gather packs the slots at host-computed offsets.
constexpr uint32_t DEFLATE_BATCH = 2048;
constexpr uint64_t DEFLATE_PREV_BYTES = 65536ull * 2;  // prev scratch per member
constexpr uint64_t DEFLATE_TOK_BYTES = 65536ull * 4;   // token scratch per member (256 lanes x 256)
constexpr uint64_t DEFLATE_REC_BYTES = 4096;           // per-member record: token counts, histogram, codes
uint64_t deflate_nblocks(uint64_t n);
hipError_t launch_deflate(const uint8_t *src, uint64_t n, uint64_t b0, uint32_t nbatch, uint16_t *prev,
                          uint32_t *toks, uint8_t *recs, uint8_t *slots, uint32_t *sizes, hipStream_t st);
hipError_t launch_deflate_gather(const uint8_t *slots, uint64_t stride, const uint32_t *sizes, const uint64_t *offs,
                                 uint64_t nblocks, uint8_t *out, hipStream_t st);

// Byte-exact BGZF writer (zdeflate.hip; zlib 1.2.11 deflate_slow at level 4..9, htsjdk's 5 by
// default): members in batches of at most ZDEFLATE_BATCH (env SBH_ZDEFLATE_BATCH overrides),
// per member prev[] (u16), match records (u64), tokens (u32), a record of blocks / trees /
// headers, and an output slot: ~1 MB of scratch per member, 8 GB at 8192 members.  The batch
// is large because k_zparse runs one serial wave per member: 8192 members keep 8 of them per
// SIMD in flight.
constexpr uint32_t ZDEFLATE_BATCH = 8192;
constexpr uint64_t ZDEFLATE_PREV_ENTRIES = 65536;
constexpr uint64_t ZDEFLATE_INFO_ENTRIES = 65536;
constexpr uint64_t ZDEFLATE_TOK_ENTRIES = 65536;
constexpr uint64_t ZDEFLATE_REC_BYTES = 16384;
constexpr uint32_t ZDEFLATE_HDR_BYTES = 640;  // a dynamic block header (<= ~4500 bits)
constexpr uint64_t ZDEFLATE_SLOT = 65536 + 64;  // 18 + (< 65518) + 8 bytes, a multiple of 16
hipError_t launch_zdeflate(const uint8_t *src, uint64_t n, uint64_t b0, uint32_t nbatch, int level, uint16_t *prev,
                           uint64_t *info, uint32_t *toks, uint8_t *recs, uint8_t *slots, uint32_t *sizes,
                           hipStream_t st);
hipError_t launch_member_footer(const uint8_t *src, uint64_t n, uint64_t b0, uint64_t nblocks, uint32_t nbatch,
                                uint8_t *slots, uint64_t stride, const uint32_t *sizes, hipStream_t st);

// Batched splits and check-bam truth comparison (splits.hip).
// The shard's counter buffer (sbh_shard::ctr, device, CTR_WORDS u64, zeroed by
// sbh_shard_create) and its pinned host mirror h_ctr.  Entry points run one at a time on the
// shard's stream and copy their results out before returning, so the per-call regions
// below may overlap each other; the persistent regions may not overlap anything.
//   per call  [0, CTR_CALL_END)   k_eager (n_true, deferred, xq) / k_full (n_success,
//                                 n_unknown, min_unknown, close_n, Counts [4, 403),
//                                 rbe [403, 1747)); FindRecordStart best [8]; chain walk
//                                 [16, 20); chain marks [20, 26); block CRCs [32, 34);
//                                 check-records [40, 46); first bad block [100]
//   persistent [CTR_TRUE_SPREAD, +CTR_TRUE_WORDS)  k_eager's per-wave true counts: must be
//                                 zero before every k_eager launch; k_fold_true folds them
//                                 into n_true and zeroes them again
//   per call  [CTR_NEXT18, +4)    the 18 bytes after an index's last chained block, at byte
//                                 NEXT18_NONLIN the linear chain's "not linear" flag (u8), at
//                                 byte NEXT18_NEMPTY the chain's empty-block count (u32), then
//                                 the linear chain's start index (u64, device only)
constexpr uint32_t CTR_WORDS = 4096;
constexpr uint32_t NEXT18_NONLIN = 18, NEXT18_NEMPTY = 20;
constexpr uint32_t CTR_CALL_END = 4 + 21 * 19 + 21 * 64;
constexpr uint32_t CTR_TRUE_SPREAD = 2048, CTR_TRUE_WORDS = 64 * 16;
constexpr uint32_t CTR_NEXT18 = CTR_TRUE_SPREAD + CTR_TRUE_WORDS;
static_assert(CTR_CALL_END <= CTR_TRUE_SPREAD && CTR_NEXT18 + 4 <= CTR_WORDS, "counter buffer layout");

constexpr uint32_t SPLIT_OK = 0;    // first record and flat end decided on the device
constexpr uint32_t SPLIT_HOST = 1;  // off the common path: the exact per-split host path decides
constexpr uint32_t SPLIT_NOREAD = 2;  // FindBlockStart lands on an empty block: NoReadFoundException (no records)
constexpr unsigned long long SPLIT_NOCOUNT = ~0ull;  // (sbh_split_starts fast path) the count is the host's to decide
struct SplitArgs {
  const uint8_t *comp;
  uint64_t n;
  int at_eof;
  const uint64_t *cand;
  uint64_t ncand, cand_from;
  int32_t k_check;
  const uint64_t *cstart, *ustart;
  const uint32_t *flags;
  uint64_t nblocks, utotal, last_start;
  const uint64_t *seg_end;
  uint32_t nseg;
  const uint32_t *bits;
  uint64_t bits_begin, bits_end;
  int64_t mrs;
};
// n host words to dst on st: up to 128 as a kernel's arguments (no DMA), more by a copy
hipError_t set_words(uint64_t *dst, const uint64_t *src, uint64_t n, hipStream_t st);
hipError_t launch_split_prologue(const SplitArgs &a, const uint64_t *starts, const uint64_t *ends, uint64_t nsplit,
                                 uint64_t *first, uint64_t *E, uint32_t *code, hipStream_t st);
hipError_t launch_split_popcount(const uint32_t *bits, uint64_t begin, const uint64_t *first, const uint64_t *E,
                                 const uint32_t *code, uint64_t nsplit, uint64_t max_span,
                                 unsigned long long *counts, hipStream_t st);
hipError_t launch_split_cm_count(const uint64_t *pos, const uint64_t *mark, const uint64_t *mpre, uint64_t n,
                                 const uint64_t *first, const uint64_t *E, uint32_t *code, uint64_t nsplit,
                                 unsigned long long *counts, hipStream_t st);
hipError_t launch_truth_scatter(const uint64_t *vpos, uint64_t n, const uint64_t *cstart, const uint64_t *ustart,
                                uint64_t nblocks, uint64_t file_off, uint64_t begin, uint64_t end, uint32_t *tbits,
                                unsigned long long *bad, hipStream_t st);
hipError_t launch_truth_compare(const uint32_t *ebits, uint64_t ebegin, const uint32_t *tbits, uint64_t begin,
                                uint64_t end, const uint64_t *rb, const uint64_t *re, uint64_t nr,
                                unsigned long long *acc, uint64_t *fp_pos, uint64_t fp_cap, uint64_t *fn_pos,
                                uint64_t fn_cap, hipStream_t st);

// Host-side streaming over a shard (sbh_check_stream, check_stream.hip): the next window's
// compressed bytes -- and optionally a host array of u64 riding with it (check-bam's truth
// slice) -- copied into the shard's spare device buffers by a host thread while the current
// window's kernels run.  shard_prefetch starts the copy; shard_prefetch_finish waits for it and,
// with `use`, makes it the shard's bytes exactly as sbh_shard_load(src, n, file_offset) would
// (the u64 array becomes the resident truth of check_records_resident); without, drops it.
int shard_prefetch(sbh_shard *sh, const void *src, uint64_t n, uint64_t file_offset, const uint64_t *aux,
                   uint64_t n_aux);
int shard_prefetch_finish(sbh_shard *sh, bool use, double *copy_ms = nullptr);
bool shard_prefetch_pending(const sbh_shard *sh, uint64_t *file_offset, uint64_t *n);
// sbh_check_records with the truth already on the device (the prefetched u64 array, n_rec of it)
int check_records_resident(sbh_shard *sh, const uint64_t *range_begin, const uint64_t *range_end, uint64_t n_ranges,
                           int32_t rtc, uint64_t n_rec, uint64_t *out, uint64_t *fp_flat, uint64_t fp_cap,
                           uint64_t *fn_flat, uint64_t fn_cap);

}  // namespace sbh
