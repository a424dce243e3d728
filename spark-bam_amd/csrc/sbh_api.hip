// sbh_api.hip -- the C-ABI (include/sparkbam.h): context/shard lifetime, device
// buffers, and the orchestration of the HIP kernels (bgzf_index.hip, inflate.hip,
// check.hip) that replace spark-bam's per-split Scala/JDK-zlib work.
#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <initializer_list>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "sbh_internal.h"

namespace sbh {
// Pinned host storage for the host copy of the block table: the device writes it in the
// sbh_block layout and one DMA lands it in place (no staging copy, no per-block host loop);
// elements are default-initialised (resize() does not zero what the copy overwrites).
template <class T>
struct PinnedAlloc {
  using value_type = T;
  PinnedAlloc() = default;
  template <class U>
  PinnedAlloc(const PinnedAlloc<U> &) {}
  T *allocate(size_t n) {
    void *p = nullptr;
    if (hipHostMalloc(&p, n * sizeof(T), hipHostMallocDefault) != hipSuccess) {
      std::fprintf(stderr, "sparkbam: pinned host allocation of %zu bytes failed\n", n * sizeof(T));
      std::abort();
    }
    return static_cast<T *>(p);
  }
  void deallocate(T *p, size_t) { (void)hipHostFree(p); }
  template <class U>
  void construct(U *p) { ::new (static_cast<void *>(p)) U; }
  template <class U, class... A>
  void construct(U *p, A &&...a) { ::new (static_cast<void *>(p)) U(static_cast<A &&>(a)...); }
  bool operator==(const PinnedAlloc &) const { return true; }
  bool operator!=(const PinnedAlloc &) const { return false; }
};
uint64_t scan_tmp_words(uint64_t n);
hipError_t scan_exclusive_u64(const uint64_t *in, uint64_t *out, uint64_t n, uint64_t *tmp, hipStream_t st);
hipError_t launch_chain_mark(const uint8_t *U, const uint32_t *bits, uint64_t begin, uint64_t from, uint64_t E,
                             uint64_t total, const uint64_t *pos, const uint64_t *wpre, uint64_t n, uint32_t *J,
                             uint32_t *J2, uint32_t *J0, uint64_t *mark, unsigned long long *exit_pos,
                             uint32_t *final_code, hipStream_t st);
hipError_t launch_find_block_start(const uint8_t *comp, uint64_t n, uint64_t start, int32_t k, int at_eof,
                                   unsigned long long *best, hipStream_t st);
uint64_t cand_chunks(uint64_t n);
hipError_t launch_cand_count(const uint8_t *comp, uint64_t n, uint64_t from, uint64_t *counts, uint32_t *first,
                             uint64_t nchunks, hipStream_t st);
hipError_t launch_cand_write(const uint8_t *comp, uint64_t n, uint64_t from, const uint64_t *counts,
                             const uint32_t *first, const uint64_t *offs, uint64_t *cand, uint64_t nchunks,
                             hipStream_t st);
hipError_t launch_pack_blocks(DevBlocks bl, uint64_t n, uint64_t file_off, uint64_t *out, hipStream_t st,
                              const uint64_t *rank = nullptr, const uint64_t *v = nullptr,
                              const uint64_t *next18 = nullptr);
hipError_t build_chain(const uint8_t *comp, uint64_t n, const uint64_t *cand, uint64_t nc, uint64_t start_rel,
                       int64_t *J0, int64_t *J1, uint8_t *on, uint64_t *v, uint64_t *rank, uint64_t *tmp,
                       DevBlocks bl, uint64_t *usz, uint8_t *next18, uint64_t *sidx, bool linear, hipStream_t st);
hipError_t launch_eager(const uint8_t *U, uint64_t u_pad, uint64_t begin, uint64_t end, const uint64_t *seg_end,
                        uint32_t nseg, uint32_t open_last, const int32_t *ctg, int32_t nctg, int32_t rtc,
                        uint32_t *bits, unsigned long long *counters, hipStream_t st, uint64_t front,
                        uint64_t *defer_pos, uint64_t defer_cap, uint64_t *xq_pos, uint64_t xq_cap, TileSum *tsum,
                        const uint32_t *sieve = nullptr);
hipError_t launch_eager_xq(const uint8_t *U, uint64_t begin, const uint64_t *seg_end, uint32_t nseg,
                           uint32_t open_last, const int32_t *ctg, int32_t nctg, int32_t rtc, uint32_t *bits,
                           unsigned long long *counters, uint64_t *xq_pos, uint64_t cap, hipStream_t st);
hipError_t launch_eager_defer(const uint8_t *U, uint64_t begin, const uint64_t *seg_end, uint32_t nseg,
                              uint32_t open_last, const int32_t *ctg, int32_t nctg, int32_t rtc, uint32_t *bits,
                              unsigned long long *counters, const uint64_t *defer_pos, uint64_t cap,
                              hipStream_t st);
hipError_t launch_full(const uint8_t *U, uint64_t u_pad, uint64_t begin, uint64_t end, const uint64_t *seg_end,
                       uint32_t nseg, uint32_t open_last, const int32_t *ctg, int32_t nctg, int32_t rtc,
                       uint32_t *words, unsigned long long *counters, uint64_t *close_pos, uint32_t *close_word,
                       uint64_t close_cap, uint32_t *op_words, uint64_t op_cap_words, hipStream_t st);
hipError_t launch_first_set(const uint32_t *bits, uint64_t begin, uint64_t from, uint64_t to,
                            unsigned long long *best, hipStream_t st);
hipError_t launch_verify_chain_count(const uint8_t *U, const uint32_t *bits, uint64_t begin, uint64_t bits_end,
                                     uint64_t from, uint64_t E, uint64_t total, unsigned long long *n_anom,
                                     unsigned long long *first_anom, unsigned long long *exit_pos,
                                     unsigned long long *n_set, const TileSum *tsum, hipStream_t st,
                                     const unsigned long long *from_dev = nullptr, uint32_t *chunk_cnt = nullptr);
hipError_t launch_chain_walk(const uint8_t *U, uint64_t first, uint64_t E, uint64_t total,
                             unsigned long long *count, unsigned long long *last, hipStream_t st);
}  // namespace sbh

using namespace sbh;

struct StreamCache;  // sbh_run_stream's window shard, buffers and copy stream (kept between calls)
static void stream_cache_free(StreamCache *sc);

// Threading (include/sparkbam.h): one context serves every thread of its process on its device
// -- a Spark executor's concurrent tasks share it (jni/Native.scala Device).  What a context holds
// is therefore either immutable after creation (device, the context stream used by context-level
// calls) or guarded by `mu` (the pool of streaming-window caches).  Each shard has its own HIP
// stream (sbh_shard_create), so two tasks' shards run concurrently on the device and a task's
// hipStreamSynchronize waits for its own work only; a shard itself belongs to one thread at a time.
// The last error (message, status, the reference exception's fields) is kept per thread and per
// context (t_err below), so one task's failure never overwrites what another task reads back.
struct sbh_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  std::mutex mu;                       // guards sc_free
  std::vector<StreamCache *> sc_free;  // idle sbh_run_stream2 window caches (one per concurrent caller)
};

namespace {
// the calling thread's last failed call: which context it was on, the message, the status and the
// fields the reference's exception is constructed from (e.g. HeaderParseException(idx, actual,
// expected)); sbh_last_error / sbh_last_error_detail read it back on the same thread
struct ErrRec {
  const sbh_ctx *ctx = nullptr;
  std::string msg;
  int32_t code = 0, n = 0;
  int64_t fields[4] = {0, 0, 0, 0};
};
thread_local ErrRec t_err;
}  // namespace

namespace {

template <typename T>
struct DBuf {  // grow-only device buffer
  T *p = nullptr;
  uint64_t cap = 0;
  hipError_t ensure(uint64_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(reinterpret_cast<void **>(&p), std::max<uint64_t>(n, 1) * sizeof(T));
    if (e == hipSuccess) cap = n;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

}  // namespace

struct sbh_shard {
  sbh_ctx *ctx = nullptr;
  // the shard's own stream (every device call on the shard is enqueued here), or the caller's
  // stream when the context was given one (sbh_ctx_set_stream)
  hipStream_t st = nullptr;
  bool own_st = false;
  uint64_t file_off = 0, n = 0, file_size = 0;
  bool at_eof = false;
  DBuf<uint8_t> comp;
  // index
  bool indexed = false;
  uint64_t index_start = 0, nblocks = 0, utotal = 0;
  DBuf<uint64_t> b_cstart, b_ustart, usz;
  DBuf<uint32_t> b_csize, b_hsize, b_usize, b_flags, b_status, b_ntok;
  DBuf<uint64_t> counts, offs, cand, v, rank, tmp, blkpack;
  DBuf<uint32_t> cfirst;  // per scan chunk: offset of its first candidate
  uint64_t ncand = 0, cand_from = 0;  // header candidates in cand[] (shard-relative, >= cand_from)
  // sbh_index scans for header candidates from this file offset when it lies in
  // [file_off, start] (~0: from the shard's first byte), so that every split starting in the
  // resident bytes -- a rank's or a streamed window's first one included -- has its
  // FindBlockStart candidates on the device; the block chain still starts at `start`
  uint64_t scan_from = ~0ull;
  DBuf<int64_t> J0, J1;
  DBuf<uint8_t> on;
  std::vector<sbh_block, PinnedAlloc<sbh_block>> hb;
  std::vector<uint64_t> seg_end;
  bool open_last = false, broken_end = false;
  DBuf<uint64_t> d_seg;
  // inflate
  bool inflated = false;
  DBuf<uint8_t> U;
  // U's pad [utotal, + pad) is zero for this utotal and allocation (only k_lz writes U, and only
  // below utotal): a step over the same shard skips the memset (an unaligned one is 3 fills)
  uint64_t u_pad_clean = ~0ull, u_pad_cap = 0;
  DBuf<uint32_t> tok;  // LZ77 tokens between k_huff and k_lz (4 B per flat byte)
  // checker
  DBuf<int32_t> ctg;
  int32_t nctg = -1;
  DBuf<uint32_t> bits;
  DBuf<TileSum> tsum;
  // k_lz's first-filter bitmap for k_eager (launch_lz's sieve), valid for the inflated bytes and
  // the contig count it was computed with (sieve_nref1 = contigs + 1; 0: none)
  DBuf<uint32_t> sieve;
  uint32_t sieve_nref1 = 0;
  bool pipe_fallback = false;  // run_pipelined redid the eager pass (a deferral overflow)  // per quarter eager tile of bits (from bits_begin): the chain proof's summaries
  // chain marking (pointer doubling) over the set bits of [cm_first, cm_E) when the bitmap
  // is not the chain: node positions, per-word prefix counts, jumps, marks and their prefix
  DBuf<uint64_t> cm_pos, cm_wcnt, cm_wpre, cm_mark, cm_mpre;
  DBuf<uint32_t> cm_j, cm_j2, cm_j0;
  uint64_t cm_first = 0, cm_E = 0, cm_n = 0;
  bool cm_valid = false;
  // the bitmap verified equal to the record chain over [chain_first, chain_E) (k_verify_chain)
  bool chain_ok = false;
  uint64_t chain_first = 0, chain_E = 0;
  // that proof's set bits per VC_CHUNK bitmap words (chunk k = words [VC_CHUNK k, ...) from
  // bits_begin), valid with chain_ok for the same range (cc_ok): the split counts' inner chunks
  DBuf<uint32_t> cc;
  bool cc_ok = false;
  bool bits_valid = false;
  uint64_t bits_begin = 0, bits_end = 0;
  uint64_t run_first = ~0ull;  // sbh_run_shard's first record (flat), ~0: none found
  int32_t bits_rtc = 0;
  DBuf<uint32_t> words;
  DBuf<uint32_t> opix;  // the full checker's bad-CIGAR-op index (launch_full)
  DBuf<uint64_t> close_pos;
  DBuf<uint32_t> close_word;
  DBuf<unsigned long long> ctr;  // scratch counters
  unsigned long long *h_ctr = nullptr;  // pinned mirror
  uint64_t pad = 4096;
  // pipelined run (run_pipelined): extra streams, per-batch events, deferred positions
  hipStream_t s_lz = nullptr, s_eg = nullptr;
  hipStream_t cs = nullptr;  // sbh_shard_load's copy stream (created on first use)
  std::vector<hipEvent_t> pev;
  DBuf<uint64_t> defer;
  DBuf<uint64_t> xq;  // long-record eager candidates for the wave-cooperative exact pass
  // record field extraction (sbh_records_scan / fetch): positions, sizes -> offsets, columns
  struct Recs {
    DBuf<uint64_t> pos, wcnt, wpre, nm, cg, sq, ax, nmo, cgo, sqo, axo, keep, kpre, pos2, vpos;
    DBuf<int64_t> iv_b, iv_e;
    DBuf<int32_t> iv_ref;
    DBuf<int32_t> ref_id, p0, nref, npos, tlen;
    DBuf<uint16_t> flag, bin;
    DBuf<uint8_t> mapq, qual, aux;
    DBuf<char> names, seq;
    DBuf<uint32_t> cigar;
    sbh_records_sizes sz{};
    bool valid = false;
    bool decoded = false;  // the columns were decoded (else only the starts, sbh_split_records decode = 0)
    void release() {
      for (auto *b : {&pos, &wcnt, &wpre, &nm, &cg, &sq, &ax, &nmo, &cgo, &sqo, &axo, &keep, &kpre, &pos2, &vpos})
        b->release();
      iv_b.release(); iv_e.release(); iv_ref.release();
      for (auto *b : {&ref_id, &p0, &nref, &npos, &tlen}) b->release();
      flag.release(); bin.release(); mapq.release(); qual.release(); aux.release();
      names.release(); seq.release(); cigar.release();
      valid = false;
    }
  } rec;
  // batched splits (sbh_split_starts) and check-bam truth (sbh_check_records)
  DBuf<uint64_t> sp_start, sp_end, sp_first, sp_E, sp_vpos;
  DBuf<uint32_t> sp_code;
  DBuf<unsigned long long> sp_count;
  // sbh_split_starts' fast path: [start, end, first, E, count] x n + code x n in one device
  // buffer and its page-locked mirror (one copy each way)
  DBuf<uint64_t> sp_pack;
  uint64_t *sp_pin = nullptr;
  uint64_t sp_pin_cap = 0;
  DBuf<uint32_t> tbits;
  DBuf<uint64_t> t_rb, t_re, t_fp, t_fn;
  // the next window prefetched by a host thread (shard_prefetch): spare compressed bytes and
  // a u64 array riding with them (check-bam's truth slice; sp_vpos once used)
  DBuf<uint8_t> comp2;
  DBuf<uint64_t> aux2;
  std::vector<std::thread> pf;
  std::vector<hipStream_t> pf_stream;
  std::vector<hipError_t> pf_err;
  bool pf_active = false;
  uint64_t pf_off = 0, pf_n = 0, pf_naux = 0;
  std::vector<double> pf_ms;  // each copy thread's wall time
  std::vector<uint8_t *> pf_pin;  // page-locked staging, PF_SLOTS chunks per copy thread
  std::vector<hipEvent_t> pf_ev;  // (one per staging chunk: its DMA is done)
  hipEvent_t ev[9] = {};
  bool ev_ok = false, timing = false;
  double stage_ms[6] = {0, 0, 0, 0, 0, 0};
  double pipe_ms[3] = {0, 0, 0};  // k_huff, k_lz, k_eager summed over the pipelined launches

  DevBlocks dev_blocks() {
    return DevBlocks{b_cstart.p, b_csize.p, b_hsize.p, b_usize.p, b_ustart.p, b_flags.p, b_status.p, b_ntok.p};
  }
};

struct StreamCache {
  sbh_shard *sh = nullptr;
  DBuf<uint8_t> buf[2];
  hipStream_t cs = nullptr;
  hipEvent_t done[2] = {nullptr, nullptr}, c0[2] = {nullptr, nullptr};
};

static void stream_cache_free(StreamCache *sc) {
  if (sc->cs) (void)hipStreamSynchronize(sc->cs);
  if (sc->sh) {
    sc->sh->comp.p = nullptr;
    sc->sh->comp.cap = 0;
    sbh_shard_destroy(sc->sh);
  }
  sc->buf[0].release();
  sc->buf[1].release();
  for (int i = 0; i < 2; ++i) {
    if (sc->done[i]) (void)hipEventDestroy(sc->done[i]);
    if (sc->c0[i]) (void)hipEventDestroy(sc->c0[i]);
  }
  if (sc->cs) (void)hipStreamDestroy(sc->cs);
  delete sc;
}

static int vfail(sbh_ctx *ctx, int code, std::initializer_list<int64_t> fields, const char *fmt, va_list ap) {
  if (ctx) {
    char buf[512];
    vsnprintf(buf, sizeof buf, fmt, ap);
    ErrRec &E = t_err;
    E.ctx = ctx;
    E.msg = buf;
    E.code = code;
    E.n = 0;
    for (int64_t f : fields)
      if (E.n < 4) E.fields[E.n++] = f;
  }
  return code;
}

static int fail(sbh_ctx *ctx, int code, const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfail(ctx, code, {}, fmt, ap);
  va_end(ap);
  return code;
}

// fail() with the fields the reference's exception takes (sbh_last_error_detail)
static int fail_with(sbh_ctx *ctx, int code, std::initializer_list<int64_t> fields, const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfail(ctx, code, fields, fmt, ap);
  va_end(ap);
  return code;
}

#define HIPCHK(ctx, x)                                                                              \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) return fail((ctx), SBH_E_HIP, "%s: %s", #x, hipGetErrorString(e_));       \
  } while (0)

static void mark(sbh_shard *sh, int i) {
  if (!sh->timing) return;
  if (!sh->ev_ok) {
    sh->ev_ok = true;
    for (hipEvent_t &e : sh->ev)
      if (hipEventCreate(&e) != hipSuccess) sh->ev_ok = false;
  }
  if (sh->ev_ok) (void)hipEventRecord(sh->ev[i], sh->st);
}

static int set_device(sbh_ctx *ctx) {
  HIPCHK(ctx, hipSetDevice(ctx->device));
  return SBH_OK;
}

extern "C" {

static int records_positions(sbh_shard *sh, uint64_t first, uint64_t E, uint64_t total, uint64_t n, int32_t anomalies,
                             uint64_t *pos);
static int records_finish(sbh_shard *sh, uint64_t n, uint64_t total, sbh_records_sizes *out);

const char *sbh_version(void) { return "sparkbam-hip 0.1 (gfx950)"; }

int sbh_ctx_create(int device, sbh_ctx **out) {
  if (!out) return SBH_E_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return SBH_E_HIP;
  sbh_ctx *c = new sbh_ctx();
  c->device = device;
  if (hipSetDevice(device) != hipSuccess) {
    delete c;
    return SBH_E_HIP;
  }
  // SBH_SCHED=spin|yield|block: how a host thread waits in hipStreamSynchronize (the path's
  // host round trips -- index sizes, block table, statuses -- each leave the GPU idle until the
  // host thread wakes); unset: the runtime's default
  if (const char *e = std::getenv("SBH_SCHED")) {
    const unsigned f = !std::strcmp(e, "spin")    ? hipDeviceScheduleSpin
                       : !std::strcmp(e, "yield") ? hipDeviceScheduleYield
                       : !std::strcmp(e, "block") ? hipDeviceScheduleBlockingSync
                                                  : hipDeviceScheduleAuto;
    // the flag only takes before the device's primary context is active; a refusal is reported
    // (stderr) rather than silently ignored, so an A/B of wait modes shows whether it applied
    const hipError_t fe = hipSetDeviceFlags(f);
    std::fprintf(stderr, "sparkbam-hip: SBH_SCHED=%s %s (%s)\n", e, fe == hipSuccess ? "applied" : "NOT applied",
                 hipGetErrorString(fe));
  }
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return SBH_E_HIP;
  }
  c->own_stream = true;
  *out = c;
  return SBH_OK;
}

int sbh_ctx_destroy(sbh_ctx *ctx) {
  if (!ctx) return SBH_OK;
  if (!ctx->sc_free.empty()) {
    (void)hipSetDevice(ctx->device);
    for (StreamCache *sc : ctx->sc_free) stream_cache_free(sc);
    ctx->sc_free.clear();
  }
  if (ctx->own_stream && ctx->stream) {
    (void)hipSetDevice(ctx->device);
    (void)hipStreamDestroy(ctx->stream);
  }
  delete ctx;
  return SBH_OK;
}

const char *sbh_last_error(const sbh_ctx *ctx) {
  if (!ctx) return "no context";
  return t_err.ctx == ctx ? t_err.msg.c_str() : "";
}

int32_t sbh_last_error_detail(const sbh_ctx *ctx, int32_t *code, int64_t *fields, int32_t cap) {
  if (!ctx) return 0;
  const ErrRec &E = t_err;
  const bool mine = E.ctx == ctx;
  if (code) *code = mine ? E.code : 0;
  if (!mine) return 0;
  const int32_t n = fields ? std::min(E.n, std::max(cap, 0)) : 0;
  for (int32_t i = 0; i < n; ++i) fields[i] = E.fields[i];
  return E.n;
}

int sbh_host_alloc(uint64_t n, void **out) {
  if (!out) return SBH_E_ARG;
  *out = nullptr;
  return hipHostMalloc(out, std::max<uint64_t>(n, 1), hipHostMallocDefault) == hipSuccess ? SBH_OK : SBH_E_NOMEM;
}

int sbh_host_free(void *p) { return p && hipHostFree(p) != hipSuccess ? SBH_E_HIP : SBH_OK; }

int sbh_ctx_set_stream(sbh_ctx *ctx, void *hip_stream) {
  if (!ctx) return SBH_E_ARG;
  if (ctx->own_stream && ctx->stream) (void)hipStreamDestroy(ctx->stream);
  ctx->stream = reinterpret_cast<hipStream_t>(hip_stream);
  ctx->own_stream = false;
  return SBH_OK;
}

int sbh_ctx_synchronize(sbh_ctx *ctx) {
  if (!ctx) return SBH_E_ARG;
  int rc = set_device(ctx);
  if (rc) return rc;
  // the context's work is on its own stream and on its shards' streams: wait for the device
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  HIPCHK(ctx, hipDeviceSynchronize());
  return SBH_OK;
}

// Header.make (bgzf/.../block/Header.scala:48-83)
int sbh_header_make(const uint8_t *b, uint64_t avail, int32_t *hsize, int32_t *csize) {
  if (!b || avail < 18) return SBH_E_TRUNCATED;
  if (b[0] != 31 || b[1] != 139 || b[2] != 8 || b[3] != 4) return SBH_E_HEADER_PARSE;
  if (b[12] != 66 || b[13] != 67 || b[14] != 2) return SBH_E_HEADER_PARSE;
  const int32_t xlen = (int32_t)b[10] | ((int32_t)b[11] << 8);
  if (hsize) *hsize = 18 + xlen - 6;
  if (csize) *csize = ((int32_t)b[16] | ((int32_t)b[17] << 8)) + 1;
  return SBH_OK;
}

int sbh_shard_create(sbh_ctx *ctx, const void *src, uint64_t n, uint64_t file_offset, uint64_t file_size,
                     int comp_on_device, sbh_shard **out) {
  if (!ctx || !out || (!src && n) || file_offset + n > file_size) return SBH_E_ARG;
  int rc = set_device(ctx);
  if (rc) return rc;
  sbh_shard *sh = new sbh_shard();
  sh->ctx = ctx;
  if (ctx->own_stream) {
    if (hipStreamCreateWithFlags(&sh->st, hipStreamNonBlocking) != hipSuccess) {
      delete sh;
      return fail(ctx, SBH_E_HIP, "shard create: no stream");
    }
    sh->own_st = true;
  } else {
    sh->st = sh->st;
  }
  sh->file_off = file_offset;
  sh->n = n;
  sh->file_size = file_size;
  sh->at_eof = file_offset + n == file_size;
  hipError_t e = sh->comp.ensure(n + sh->pad);
  if (e == hipSuccess && n)
    e = hipMemcpyAsync(sh->comp.p, src, n, comp_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                       sh->st);
  if (e == hipSuccess) e = hipMemsetAsync(sh->comp.p + n, 0, sh->pad, sh->st);
  if (e == hipSuccess) e = sh->ctr.ensure(CTR_WORDS);
  // (layout: sbh_internal.h; k_eager's true-count slots must start zero, k_fold_true keeps them so)
  if (e == hipSuccess) e = hipMemsetAsync(sh->ctr.p, 0, CTR_WORDS * sizeof(unsigned long long), sh->st);
  if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void **>(&sh->h_ctr), CTR_WORDS * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipStreamSynchronize(sh->st);
  if (e != hipSuccess) {
    sbh_shard_destroy(sh);
    return fail(ctx, SBH_E_HIP, "shard create: %s", hipGetErrorString(e));
  }
  *out = sh;
  return SBH_OK;
}

int sbh_shard_destroy(sbh_shard *sh) {
  if (!sh) return SBH_OK;
  if (sh->pf_active) (void)shard_prefetch_finish(sh, false);
  (void)hipSetDevice(sh->ctx->device);
  (void)hipStreamSynchronize(sh->st);
  sh->comp.release();
  sh->b_cstart.release(); sh->b_ustart.release(); sh->usz.release(); sh->blkpack.release();
  sh->b_csize.release(); sh->b_hsize.release(); sh->b_usize.release(); sh->b_flags.release();
  sh->b_status.release();
  sh->b_ntok.release();
  sh->tok.release();
  sh->counts.release(); sh->cfirst.release(); sh->offs.release(); sh->cand.release(); sh->v.release(); sh->rank.release();
  sh->tmp.release(); sh->J0.release(); sh->J1.release(); sh->on.release(); sh->d_seg.release();
  sh->U.release(); sh->u_pad_clean = ~0ull; sh->ctg.release(); sh->bits.release(); sh->words.release(); sh->close_pos.release();
  sh->close_word.release(); sh->ctr.release(); sh->opix.release(); sh->tsum.release(); sh->sieve.release();
  sh->cc.release();
  sh->comp2.release(); sh->aux2.release();
  for (hipStream_t st : sh->pf_stream) (void)hipStreamDestroy(st);
  for (uint8_t *p : sh->pf_pin) (void)hipHostFree(p);
  for (hipEvent_t e : sh->pf_ev) (void)hipEventDestroy(e);
  for (hipEvent_t &e : sh->ev)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t &e : sh->pev)
    if (e) (void)hipEventDestroy(e);
  if (sh->s_lz) (void)hipStreamDestroy(sh->s_lz);
  if (sh->s_eg) (void)hipStreamDestroy(sh->s_eg);
  if (sh->cs) (void)hipStreamDestroy(sh->cs);
  sh->defer.release();
  sh->xq.release();
  sh->rec.release();
  for (auto *b : {&sh->sp_start, &sh->sp_end, &sh->sp_first, &sh->sp_E, &sh->sp_vpos, &sh->t_rb, &sh->t_re,
                  &sh->t_fp, &sh->t_fn})
    b->release();
  sh->sp_code.release();
  sh->sp_count.release();
  sh->sp_pack.release();
  if (sh->sp_pin) (void)hipHostFree(sh->sp_pin);
  sh->tbits.release();
  sh->cm_pos.release(); sh->cm_wcnt.release(); sh->cm_wpre.release(); sh->cm_mark.release(); sh->cm_mpre.release();
  sh->cm_j.release(); sh->cm_j2.release(); sh->cm_j0.release();
  if (sh->h_ctr) (void)hipHostFree(sh->h_ctr);
  if (sh->own_st && sh->st) (void)hipStreamDestroy(sh->st);
  delete sh;
  return SBH_OK;
}

int sbh_shard_load(sbh_shard *sh, const void *src, uint64_t n, uint64_t file_offset, int comp_on_device) {
  if (!sh || (!src && n) || file_offset + n > sh->file_size) return SBH_E_ARG;
  sbh_ctx *ctx = sh->ctx;
  int rc = set_device(ctx);
  if (rc) return rc;
  HIPCHK(ctx, hipStreamSynchronize(sh->st));  // (no kernel may still read the old bytes)
  HIPCHK(ctx, sh->comp.ensure(n + sh->pad));
  // the copy on the shard's copy stream, at another priority than every compute stream: its
  // hardware queue is then never one another task's kernels wait behind (see sbh_run_stream2)
  hipStream_t cs = sh->st;
  if (!std::getenv("SBH_LOAD_ON_SHARD_STREAM")) {
    if (!sh->cs) {
      int least = 0, greatest = 0;
      if (hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess && greatest != least)
        HIPCHK(ctx, hipStreamCreateWithPriority(&sh->cs, hipStreamNonBlocking, greatest));
    }
    if (sh->cs) cs = sh->cs;
  }
  if (n)
    HIPCHK(ctx, hipMemcpyAsync(sh->comp.p, src, n, comp_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                               cs));
  if (cs != sh->st) HIPCHK(ctx, hipStreamSynchronize(cs));
  HIPCHK(ctx, hipMemsetAsync(sh->comp.p + n, 0, sh->pad, sh->st));
  HIPCHK(ctx, hipStreamSynchronize(sh->st));
  sh->file_off = file_offset;
  sh->n = n;
  sh->at_eof = file_offset + n == sh->file_size;
  sh->sieve_nref1 = 0;
  sh->indexed = sh->inflated = sh->bits_valid = sh->chain_ok = sh->cm_valid = false;
  sh->rec.valid = false;
  sh->ncand = 0;
  sh->scan_from = ~0ull;
  sh->hb.clear();
  sh->nblocks = sh->utotal = 0;
  return SBH_OK;
}

}  // extern "C"

namespace sbh {

// copy threads per prefetch (SBH_PREFETCH_THREADS, default 4), each hipMemcpyAsync-ing its
// part on its own stream.  SBH_PREFETCH_STAGE=1: host memory that is not page-locked (a mapped
// file, a numpy array) goes through page-locked staging chunks instead -- each thread memcpys a
// chunk into its slot and DMAs it while it fills the next (2 slots of 8 MiB per thread).  Measured
// on configs[2]'s 100.9 GiB file (pageable numpy): direct 2.34 s of copies (r05f, ~46 GB/s, the
// same with 1 or 4 threads), staged 2.32 s (r05h) and slower on a 5 GiB file (136 vs 118 ms):
// the host's memory bandwidth share, not the runtime's staging, is the limit, so staging is off
// by default.  Page-locked host memory is DMAed directly (~56 GB/s).
static uint32_t prefetch_threads() {
  const char *e = std::getenv("SBH_PREFETCH_THREADS");
  const long v = e ? std::atol(e) : 4;
  return (uint32_t)std::min<long>(std::max<long>(v, 1), 16);
}
static bool prefetch_stage() {
  const char *e = std::getenv("SBH_PREFETCH_STAGE");
  return e && std::atol(e) == 1;
}
static constexpr uint32_t PF_SLOTS = 2;
static constexpr uint64_t PF_CHUNK = 8ull << 20;

int shard_prefetch(sbh_shard *sh, const void *src, uint64_t n, uint64_t file_offset, const uint64_t *aux,
                   uint64_t n_aux) {
  if (!sh || (!src && n) || (!aux && n_aux) || file_offset + n > sh->file_size || sh->pf_active) return SBH_E_ARG;
  sbh_ctx *ctx = sh->ctx;
  int rc = set_device(ctx);
  if (rc) return rc;
  // buffers are sized here, on the calling thread (the copy threads only copy)
  HIPCHK(ctx, sh->comp2.ensure(n + sh->pad));
  HIPCHK(ctx, sh->aux2.ensure(n_aux + 1));
  const uint32_t nt = prefetch_threads();
  while (sh->pf_stream.size() < nt) {
    hipStream_t st = nullptr;
    HIPCHK(ctx, hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    sh->pf_stream.push_back(st);
  }
  hipPointerAttribute_t pa{};
  const bool pinned = n && hipPointerGetAttributes(&pa, src) == hipSuccess && pa.type == hipMemoryTypeHost;
  (void)hipGetLastError();
  const bool stage = !pinned && prefetch_stage();
  if (stage) {
    while (sh->pf_pin.size() < (size_t)nt * PF_SLOTS) {
      void *p = nullptr;
      HIPCHK(ctx, hipHostMalloc(&p, PF_CHUNK, hipHostMallocDefault));
      sh->pf_pin.push_back(static_cast<uint8_t *>(p));
      hipEvent_t ev = nullptr;
      HIPCHK(ctx, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      sh->pf_ev.push_back(ev);
    }
  }
  sh->pf_active = true;
  sh->pf_off = file_offset, sh->pf_n = n, sh->pf_naux = n_aux;
  sh->pf_err.assign(nt, hipSuccess);
  sh->pf_ms.assign(nt, 0.0);
  sh->pf.clear();
  const int dev = ctx->device;
  uint8_t *dst = sh->comp2.p;
  uint64_t *adst = sh->aux2.p;
  const uint64_t pad = sh->pad, part = (n / nt + 4095) & ~4095ull;
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t k = 0; k < nt; ++k) {
    const uint64_t lo = std::min(n, k * part), hi = k + 1 == nt ? n : std::min(n, (k + 1) * part);
    hipStream_t cs = sh->pf_stream[k];
    hipError_t *err = &sh->pf_err[k];
    double *ms = &sh->pf_ms[k];
    uint8_t *const *pin = stage ? sh->pf_pin.data() + (size_t)k * PF_SLOTS : nullptr;
    hipEvent_t *ev = stage ? sh->pf_ev.data() + (size_t)k * PF_SLOTS : nullptr;
    sh->pf.emplace_back([=]() {
      uint32_t used = 0;  // staging chunks issued by this thread
      // [from, from + len) of host memory to device memory at to
      auto copy = [&](uint8_t *to, const uint8_t *from, uint64_t len) -> hipError_t {
        if (!stage) return len ? hipMemcpyAsync(to, from, len, hipMemcpyHostToDevice, cs) : hipSuccess;
        for (uint64_t o = 0; o < len; o += PF_CHUNK, ++used) {
          const uint32_t slot = used % PF_SLOTS;
          const uint64_t m = std::min(PF_CHUNK, len - o);
          if (used >= PF_SLOTS) {  // the slot's previous DMA must be done before it is refilled
            const hipError_t e = hipEventSynchronize(ev[slot]);
            if (e != hipSuccess) return e;
          }
          std::memcpy(pin[slot], from + o, m);
          hipError_t e = hipMemcpyAsync(to + o, pin[slot], m, hipMemcpyHostToDevice, cs);
          if (e == hipSuccess) e = hipEventRecord(ev[slot], cs);
          if (e != hipSuccess) return e;
        }
        return hipSuccess;
      };
      hipError_t e = hipSetDevice(dev);
      if (e == hipSuccess) e = copy(dst + lo, static_cast<const uint8_t *>(src) + lo, hi - lo);
      if (e == hipSuccess && k == 0) e = hipMemsetAsync(dst + n, 0, pad, cs);
      if (e == hipSuccess && k == 0 && n_aux)
        e = copy(reinterpret_cast<uint8_t *>(adst), reinterpret_cast<const uint8_t *>(aux), 8 * n_aux);
      if (e == hipSuccess) e = hipStreamSynchronize(cs);
      *err = e;
      *ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    });
  }
  return SBH_OK;
}

bool shard_prefetch_pending(const sbh_shard *sh, uint64_t *file_offset, uint64_t *n) {
  if (!sh || !sh->pf_active) return false;
  if (file_offset) *file_offset = sh->pf_off;
  if (n) *n = sh->pf_n;
  return true;
}

int shard_prefetch_finish(sbh_shard *sh, bool use, double *copy_ms) {
  if (!sh || !sh->pf_active) return SBH_E_STATE;
  sbh_ctx *ctx = sh->ctx;
  for (std::thread &th : sh->pf)
    if (th.joinable()) th.join();
  sh->pf.clear();
  sh->pf_active = false;
  if (copy_ms) *copy_ms = sh->pf_ms.empty() ? 0.0 : *std::max_element(sh->pf_ms.begin(), sh->pf_ms.end());
  for (hipError_t e : sh->pf_err)
    if (e != hipSuccess) return fail(ctx, SBH_E_HIP, "window prefetch: %s", hipGetErrorString(e));
  if (!use) return SBH_OK;
  int rc = set_device(ctx);
  if (rc) return rc;
  HIPCHK(ctx, hipStreamSynchronize(sh->st));  // (no kernel may still read the old bytes)
  std::swap(sh->comp, sh->comp2);
  std::swap(sh->sp_vpos, sh->aux2);
  sh->file_off = sh->pf_off;
  sh->n = sh->pf_n;
  sh->at_eof = sh->file_off + sh->n == sh->file_size;
  sh->sieve_nref1 = 0;
  sh->indexed = sh->inflated = sh->bits_valid = sh->chain_ok = sh->cm_valid = false;
  sh->rec.valid = false;
  sh->ncand = 0;
  sh->scan_from = ~0ull;
  sh->hb.clear();
  sh->nblocks = sh->utotal = 0;
  return SBH_OK;
}

}  // namespace sbh

extern "C" {

const void *sbh_shard_comp_device_ptr(sbh_shard *sh) { return sh ? sh->comp.p : nullptr; }

// FindBlockStart.apply (bgzf/.../block/FindBlockStart.scala:8-36)
int sbh_find_block_start(sbh_shard *sh, uint64_t start, int32_t k, uint64_t *out) {
  if (!sh || !out || k < 0 || start < sh->file_off) return SBH_E_ARG;
  sbh_ctx *ctx = sh->ctx;
  int rc = set_device(ctx);
  if (rc) return rc;
  const uint64_t rel = start - sh->file_off;
  unsigned long long *best = sh->ctr.p;
  HIPCHK(ctx, hipMemsetAsync(best, 0xff, 8, sh->st));
  HIPCHK(ctx, launch_find_block_start(sh->comp.p, sh->n, rel, k, sh->at_eof ? 1 : 0, best, sh->st));
  HIPCHK(ctx, hipMemcpyAsync(sh->h_ctr, best, 8, hipMemcpyDeviceToHost, sh->st));
  HIPCHK(ctx, hipStreamSynchronize(sh->st));
  const unsigned long long b = sh->h_ctr[0];
  // HeaderSearchFailedException(path, start, positionsAttempted): the search tried every
  // pos < MAX_BLOCK_SIZE (FindBlockStart.scala:18-35)
  if (b == ~0ull)
    return fail_with(ctx, SBH_E_HEADER_SEARCH_FAILED, {(int64_t)start, 65536}, "no BGZF block start in [%llu, %llu)",
                     (unsigned long long)start, (unsigned long long)(start + 65536));
  const uint32_t outcome = (uint32_t)(b & 0xff);
  const uint64_t pos = b >> 8;
  if (outcome == 2) return fail(ctx, SBH_E_TRUNCATED, "truncated BGZF block near %llu", (unsigned long long)(start + pos));
  if (outcome == 3) return fail(ctx, SBH_E_NEED_HALO, "FindBlockStart(%llu) needs bytes past the shard", (unsigned long long)start);
  *out = start + pos;
  return SBH_OK;
}

// SBH_CHAIN_JUMP=1: the index always builds the block chain by pointer jumping (the path a
// chain with false-positive candidates takes), for tests and A/B.
static bool chain_jump_only() {
  const char *e = std::getenv("SBH_CHAIN_JUMP");
  return e && e[0] == '1';
}

// MetadataStream from `start` (bgzf/.../block/MetadataStream.scala:16-58)
int sbh_index(sbh_shard *sh, uint64_t start, uint64_t *n_blocks, uint64_t *flat_size) {
  if (!sh || start < sh->file_off || start > sh->file_off + sh->n) return SBH_E_ARG;
  sbh_ctx *ctx = sh->ctx;
  hipStream_t st = sh->st;
  int rc = set_device(ctx);
  if (rc) return rc;
  sh->sieve_nref1 = 0;
  sh->indexed = sh->inflated = sh->bits_valid = sh->chain_ok = sh->cm_valid = false;
  sh->ncand = 0;
  const uint64_t rel = start - sh->file_off;
  const uint64_t n = sh->n;
  const uint64_t srel = sh->scan_from >= sh->file_off && sh->scan_from <= start ? sh->scan_from - sh->file_off : 0;
  // the start must itself be a header (its 18 bytes come back with the candidate count)
  uint8_t *h18 = reinterpret_cast<uint8_t *>(sh->h_ctr + 512);  // pinned
  auto start_is_header = [&]() -> int {
    if (sbh_header_make(h18, 18, nullptr, nullptr) != SBH_OK) {
      // HeaderParseException(idx, actual, expected): the first byte Header.make's checks
      // reject, in its order (Header.scala:48-71)
      static const uint8_t idx[7] = {0, 1, 2, 3, 12, 13, 14}, want[7] = {31, 139, 8, 4, 66, 67, 2};
      int k = 0;
      while (k < 6 && h18[idx[k]] == want[k]) ++k;
      return fail_with(ctx, SBH_E_HEADER_PARSE, {(int64_t)start, idx[k], (int8_t)h18[idx[k]], (int8_t)want[k]},
                       "Position %d: %d != %d (BGZF header at %llu)", idx[k], (int8_t)h18[idx[k]], (int8_t)want[k],
                       (unsigned long long)start);
    }
    return SBH_OK;
  };
  if (rel + 18 <= n) HIPCHK(ctx, hipMemcpyAsync(h18, sh->comp.p + rel, 18, hipMemcpyDeviceToHost, st));
  const uint64_t nchunks = cand_chunks(n);
  uint64_t nc = 0;
  if (rel + 18 <= n && !nchunks) {
    HIPCHK(ctx, hipStreamSynchronize(st));
    if ((rc = start_is_header()) != SBH_OK) return rc;
  }
  if (nchunks && rel + 18 <= n) {
    // (counts[nchunks] = 0, written by k_cand_count: the scan over nchunks + 1 entries leaves the
    // candidate total in offs[nchunks], one word back)
    HIPCHK(ctx, sh->counts.ensure(nchunks + 1));
    HIPCHK(ctx, sh->cfirst.ensure(nchunks));
    HIPCHK(ctx, sh->offs.ensure(nchunks + 1));
    HIPCHK(ctx, sh->tmp.ensure(scan_tmp_words(nchunks + 1) + scan_tmp_words(1 << 24)));
    HIPCHK(ctx, launch_cand_count(sh->comp.p, n, srel, sh->counts.p, sh->cfirst.p, nchunks, st));
    HIPCHK(ctx, scan_exclusive_u64(sh->counts.p, sh->offs.p, nchunks + 1, sh->tmp.p, st));
    HIPCHK(ctx, hipMemcpyAsync(&sh->h_ctr[0], sh->offs.p + nchunks, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipStreamSynchronize(st));
    if ((rc = start_is_header()) != SBH_OK) return rc;
    nc = sh->h_ctr[0];
  }
  uint64_t nchain = 0;
  // the 18 bytes after the last chain block (the next header, checked below), written by
  // k_chain_emit and copied back with the block table
  uint8_t *next18_dev = reinterpret_cast<uint8_t *>(sh->ctr.p + CTR_NEXT18);
  uint8_t *nx = reinterpret_cast<uint8_t *>(sh->h_ctr + 516);  // pinned
  if (nc) {
    HIPCHK(ctx, sh->cand.ensure(nc));
    HIPCHK(ctx, sh->J0.ensure(nc));
    HIPCHK(ctx, sh->J1.ensure(nc));
    HIPCHK(ctx, sh->on.ensure(nc));
    HIPCHK(ctx, sh->v.ensure(nc));
    HIPCHK(ctx, sh->rank.ensure(nc));
    HIPCHK(ctx, sh->tmp.ensure(scan_tmp_words(nc) + scan_tmp_words(nchunks + 1)));
    HIPCHK(ctx, launch_cand_write(sh->comp.p, n, srel, sh->counts.p, sh->cfirst.p, sh->offs.p, sh->cand.p, nchunks, st));
    HIPCHK(ctx, sh->b_cstart.ensure(nc));
    HIPCHK(ctx, sh->b_ustart.ensure(nc));
    HIPCHK(ctx, sh->usz.ensure(nc));
    HIPCHK(ctx, sh->b_csize.ensure(nc));
    HIPCHK(ctx, sh->b_hsize.ensure(nc));
    HIPCHK(ctx, sh->b_usize.ensure(nc));
    HIPCHK(ctx, sh->b_flags.ensure(nc));
    HIPCHK(ctx, sh->b_status.ensure(nc));
    HIPCHK(ctx, sh->b_ntok.ensure(nc));
  }
  sh->ncand = nc;
  sh->cand_from = srel;
  // host copy of the block table (Pos mapping, segments)
  static_assert(sizeof(sbh_block) == 32, "k_pack_blocks writes 32-byte sbh_block records");
  sh->hb.resize(nc + 1);  // (+ the trailer k_pack_blocks leaves after the table)
  if (nc) {
    HIPCHK(ctx, sh->blkpack.ensure(4 * nc + 4));
    // the linear chain first (every candidate from the start on is chained: no pointer jumping);
    // its flag comes back with the table, and a chain that is not linear is rebuilt by jumping
    for (int pass = chain_jump_only() ? 1 : 0; pass < 2; ++pass) {
      HIPCHK(ctx, build_chain(sh->comp.p, n, sh->cand.p, nc, rel, sh->J0.p, sh->J1.p, sh->on.p, sh->v.p, sh->rank.p,
                              sh->tmp.p, sh->dev_blocks(), sh->usz.p, next18_dev,
                              reinterpret_cast<uint64_t *>(sh->ctr.p + CTR_NEXT18 + 3),
                              pass == 0, st));
      // flat offsets over all nc entries (usz is zero past the chain); the chain length comes
      // back with the block table, so the table is packed and copied for all nc candidates and
      // cut after
      HIPCHK(ctx, scan_exclusive_u64(sh->usz.p, sh->b_ustart.p, nc, sh->tmp.p, st));
      // the table with a 32-byte trailer (hb[nc]): the chain length, then the next18 words (+ the
      // not-linear flag and the empty-block count) -- one copy into hb's page-locked storage
      HIPCHK(ctx, launch_pack_blocks(sh->dev_blocks(), nc, sh->file_off, sh->blkpack.p, st, sh->rank.p, sh->v.p,
                                     reinterpret_cast<const uint64_t *>(next18_dev)));
      HIPCHK(ctx, hipMemcpyAsync(sh->hb.data(), sh->blkpack.p, (nc + 1) * 32, hipMemcpyDeviceToHost, st));
      HIPCHK(ctx, hipStreamSynchronize(st));
      std::memcpy(nx, reinterpret_cast<const uint64_t *>(sh->hb.data() + nc) + 1, 24);
      if (pass == 1 || !nx[NEXT18_NONLIN]) break;
    }
    nchain = *reinterpret_cast<const uint64_t *>(sh->hb.data() + nc);
  }
  sh->hb.resize(nchain);
  // stream end: a truncated last block is not part of the resident stream
  sh->open_last = !sh->at_eof;
  sh->broken_end = false;
  if (!sh->hb.empty() && (sh->hb.back().flags & SBH_BLOCK_TRUNCATED)) {
    sh->hb.pop_back();
    --nchain;
  } else if (!sh->hb.empty()) {
    const sbh_block &l = sh->hb.back();
    const uint64_t q = l.start - sh->file_off + l.csize;
    if (q + 18 <= n) {  // the next header does not parse: HeaderParseException if read
      if (sbh_header_make(nx, 18, nullptr, nullptr) != SBH_OK) {
        sh->broken_end = true;
        sh->open_last = false;
      }
    }
  }
  // segments: each empty block ends one (the table is walked only when the chain has any: a
  // walk over a 1 GB shard's 46 k blocks took ~85 us of host time per step); the flat end is
  // that of the last block with bytes
  uint64_t total = 0;
  sh->seg_end.clear();
  const uint32_t nempty = nc ? *reinterpret_cast<const uint32_t *>(nx + NEXT18_NEMPTY) : 0u;
  if (nempty)
    for (const sbh_block &b : sh->hb)
      if (b.flags & SBH_BLOCK_EMPTY) sh->seg_end.push_back(b.ustart);
  for (size_t i = sh->hb.size(); i-- > 0;) {
    const sbh_block &b = sh->hb[i];
    if (!(b.flags & SBH_BLOCK_EMPTY) && b.usize <= 65536) {
      total = b.ustart + b.usize;
      break;
    }
  }
  sh->seg_end.push_back(total);
  HIPCHK(ctx, sh->d_seg.ensure(sh->seg_end.size()));
  HIPCHK(ctx, set_words(sh->d_seg.p, sh->seg_end.data(), sh->seg_end.size(), st));
  sh->nblocks = nchain;
  sh->utotal = total;
  sh->index_start = start;
  sh->indexed = true;
  if (n_blocks) *n_blocks = nchain;
  if (flat_size) *flat_size = total;
  return SBH_OK;
}

int sbh_get_blocks(sbh_shard *sh, uint64_t first, uint64_t count, sbh_block *out) {
  if (!sh || !out) return SBH_E_ARG;
  if (!sh->indexed) return fail(sh->ctx, SBH_E_STATE, "not indexed");
  if (first + count > sh->hb.size()) return SBH_E_ARG;
  std::memcpy(out, sh->hb.data() + first, count * sizeof(sbh_block));
  return SBH_OK;
}

// After the inflate kernels on `st`: the first block whose status is not INF_OK decides the
// error (the reference's exception for that block); 8 bytes come back, not every status.
// `extra`/`extra_dst`/`extra_n` ride along in the same round trip.
// whole_ctr: the caller set ctr[0, CTR_RUN_WORDS) from ctr_run_template (fb = ~0 included), and
// those words all come back to h_ctr in one copy (the eager counters, the step tail's answers)
constexpr uint32_t CTR_RUN_WORDS = 101;
static int inflate_status(sbh_shard *sh, hipStream_t st, uint64_t *bad_block, const void *extra = nullptr,
                          void *extra_dst = nullptr, size_t extra_n = 0, bool whole_ctr = false) {
  sbh_ctx *ctx = sh->ctx;
  unsigned long long *fb = sh->ctr.p + 100;
  HIPCHK(ctx, launch_first_bad(sh->b_status.p, sh->nblocks, fb, st, !whole_ctr));
  if (whole_ctr) {
    HIPCHK(ctx, hipMemcpyAsync(sh->h_ctr, sh->ctr.p, CTR_RUN_WORDS * 8, hipMemcpyDeviceToHost, st));
  } else {
    HIPCHK(ctx, hipMemcpyAsync(sh->h_ctr + 100, fb, 8, hipMemcpyDeviceToHost, st));
    if (extra_n) HIPCHK(ctx, hipMemcpyAsync(extra_dst, extra, extra_n, hipMemcpyDeviceToHost, st));
  }
  HIPCHK(ctx, hipStreamSynchronize(st));
  const uint64_t i = sh->h_ctr[100];
  if (i == ~0ull) return SBH_OK;
  uint32_t *hs = reinterpret_cast<uint32_t *>(sh->h_ctr + 101);
  HIPCHK(ctx, hipMemcpyAsync(hs, sh->b_status.p + i, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipStreamSynchronize(st));
  if (bad_block) *bad_block = i;
  const sbh_block &b = sh->hb[i];
  if (*hs == INF_SIZE)
    return fail_with(ctx, SBH_E_INFLATE_SIZE, {(int64_t)b.start, b.usize},
                     "Expected %u decompressed bytes (block %llu)", b.usize, (unsigned long long)b.start);
  if (*hs == INF_BAD_ISIZE) return fail(ctx, SBH_E_BAD_ISIZE, "block %llu: ISIZE %u", (unsigned long long)b.start, b.usize);
  return fail_with(ctx, SBH_E_INFLATE_DATA, {(int64_t)b.start}, "block %llu: invalid deflate data",
                   (unsigned long long)b.start);
}

// SBH_SPLIT_CC=0: split counts by a popcount of each split's whole bitmap range (A/B)
static bool split_cc_on() {
  const char *e = std::getenv("SBH_SPLIT_CC");
  return !(e && e[0] == '0');
}

// SBH_SIEVE=1 (with k_lz built -DSBH_LZ_SIEVE=1): k_lz leaves k_eager's first filter as a bitmap
// (measured slower, DESIGN.md §10: off by default; k_eager sweeps refIDs itself)
static bool sieve_on() {
  const char *e = std::getenv("SBH_SIEVE");
  return e && e[0] == '1';
}
// The sieve k_lz fills for k_eager (launch_lz): one bit per flat position of the shard, plus the
// look-ahead an eager window past the last tile reads (masked there); nullptr when off or when the
// contig count is not known yet.
static uint32_t *sieve_for(sbh_shard *sh) {
  if (!sieve_on() || sh->nctg < 0) return nullptr;
  if (sh->sieve.ensure((sh->utotal + sh->pad + 65536) / 32 + 2) != hipSuccess) return nullptr;
  return sh->sieve.p;
}

static hipError_t zero_u_pad(sbh_shard *sh, hipStream_t st) {
  if (sh->u_pad_clean == sh->utotal && sh->u_pad_cap == sh->U.cap) return hipSuccess;
  const hipError_t e = hipMemsetAsync(sh->U.p + sh->utotal, 0, sh->pad, st);
  if (e == hipSuccess) {
    sh->u_pad_clean = sh->utotal;
    sh->u_pad_cap = sh->U.cap;
  }
  return e;
}

static DevBlocks blocks_from(DevBlocks d, uint64_t b) {
  return DevBlocks{d.cstart + b, d.csize + b, d.hsize + b, d.usize + b, d.ustart + b, d.flags + b, d.status + b, d.ntok + b};
}

// Token buffer between k_huff and k_lz: 4 B per flat byte of the blocks inflated at once.  A
// shard whose flat bytes exceed the budget (SBH_TOK_BUDGET bytes, default 16 GiB) is inflated in
// consecutive batches of blocks that reuse one buffer, so HBM holds the compressed and flat
// bytes plus a bounded token buffer whatever the shard size.
static uint64_t tok_cap_flat() {
  const char *e = std::getenv("SBH_TOK_BUDGET");
  const long long v = e ? std::atoll(e) : 0;
  return (v > 0 ? (uint64_t)v : (16ull << 30)) / 4;
}

struct TokPlan {
  std::vector<std::pair<uint64_t, uint64_t>> batches;  // blocks [b0, b1)
  bool reuse = false;                                  // batches share tok (base = ustart of b0)
  uint64_t tok_len = 0;                                // tok entries to allocate
};

// Blocks [0, nblocks) in batches of at most max_blocks blocks and (when the whole shard does
// not fit the token budget) at most the budget's flat bytes each (one block at least).
static TokPlan tok_plan(const sbh_shard *sh, uint64_t max_blocks) {
  TokPlan P;
  const uint64_t nb = sh->nblocks, cap = tok_cap_flat();
  P.reuse = sh->utotal + 64 > cap;
  uint64_t b0 = 0;
  while (b0 < nb) {
    const uint64_t u0 = sh->hb[b0].ustart;
    // (no block walk unless the budget binds; max_blocks may be ~0)
    uint64_t b1 = max_blocks >= nb - b0 ? nb : b0 + std::max<uint64_t>(max_blocks, 1);
    if (P.reuse) {
      b1 = b0 + 1;
      while (b1 < nb && b1 - b0 < max_blocks && sh->hb[b1].ustart + sh->hb[b1].usize - u0 <= cap) ++b1;
    }
    P.batches.emplace_back(b0, b1);
    const uint64_t ext = sh->hb[b1 - 1].ustart + sh->hb[b1 - 1].usize - u0;
    P.tok_len = std::max(P.tok_len, ext);
    b0 = b1;
  }
  if (P.batches.empty()) P.batches.emplace_back(0, 0);  // (an empty shard: one empty batch)
  if (!P.reuse) P.tok_len = sh->utotal;
  P.tok_len += 64;
  return P;
}

int sbh_inflate(sbh_shard *sh, uint64_t *bad_block) {
  if (!sh) return SBH_E_ARG;
  sbh_ctx *ctx = sh->ctx;
  if (!sh->indexed) return fail(ctx, SBH_E_STATE, "inflate before index");
  int rc = set_device(ctx);
  if (rc) return rc;
  hipStream_t st = sh->st;
  HIPCHK(ctx, sh->U.ensure(sh->utotal + sh->pad));
  const TokPlan P = tok_plan(sh, ~0ull);
  HIPCHK(ctx, sh->tok.ensure(P.tok_len));
  HIPCHK(ctx, zero_u_pad(sh, st));
  uint32_t *sv = sieve_for(sh);
  const uint32_t nref1 = (uint32_t)sh->nctg + 1;
  mark(sh, 2);
  for (const auto &bt : P.batches) {  // (one stream: a batch's k_lz finishes before the next k_huff)
    const DevBlocks d = blocks_from(sh->dev_blocks(), bt.first);
    const uint64_t base = P.reuse ? sh->hb[bt.first].ustart : 0;
    HIPCHK(ctx, launch_huff(sh->comp.p, d, bt.second - bt.first, sh->tok.p, base, st));
    HIPCHK(ctx, launch_lz(sh->comp.p, d, bt.second - bt.first, sh->tok.p, base, sh->U.p, st, sv, nref1));
  }
  mark(sh, 3);
  rc = inflate_status(sh, st, bad_block);
  if (rc) return rc;
  sh->inflated = true;
  sh->sieve_nref1 = sv ? nref1 : 0;
  sh->bits_valid = sh->chain_ok = sh->cm_valid = false;
  return SBH_OK;
}

// BGZF footer CRC32 of every inflated block vs its bytes in U (crc.hip): the full-size
// bit-exactness check of the inflate (the reference itself never checks CRC32).
int sbh_verify_crc(sbh_shard *sh, uint64_t *n_bad, uint64_t *first_bad) {
  if (!sh || !n_bad) return SBH_E_ARG;
  sbh_ctx *ctx = sh->ctx;
  if (!sh->inflated) return fail(ctx, SBH_E_STATE, "verify_crc before inflate");
  int rc = set_device(ctx);
  if (rc) return rc;
  hipStream_t st = sh->st;
  unsigned long long *c = sh->ctr.p + 32;
  HIPCHK(ctx, hipMemsetAsync(c, 0, 8, st));
  HIPCHK(ctx, hipMemsetAsync(c + 1, 0xff, 8, st));
  HIPCHK(ctx, launch_block_crc(sh->comp.p, sh->dev_blocks(), sh->nblocks, sh->U.p, c, c + 1, st));
  HIPCHK(ctx, hipMemcpyAsync(sh->h_ctr + 32, c, 16, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipStreamSynchronize(st));
  *n_bad = sh->h_ctr[32];
  if (first_bad) *first_bad = sh->h_ctr[32] ? sh->hb[sh->h_ctr[33]].start : 0;
  return SBH_OK;
}

int sbh_read_flat(sbh_shard *sh, uint64_t flat, uint64_t n, uint8_t *out) {
  if (!sh || (!out && n)) return SBH_E_ARG;
  if (!sh->inflated) return fail(sh->ctx, SBH_E_STATE, "not inflated");
  if (flat + n > sh->utotal) return SBH_E_ARG;
  int rc = set_device(sh->ctx);
  if (rc) return rc;
  HIPCHK(sh->ctx, hipMemcpyAsync(out, sh->U.p + flat, n, hipMemcpyDeviceToHost, sh->st));
  HIPCHK(sh->ctx, hipStreamSynchronize(sh->st));
  return SBH_OK;
}

const void *sbh_flat_device_ptr(sbh_shard *sh) { return sh ? sh->U.p : nullptr; }

static int64_t block_index_of(const sbh_shard *sh, uint64_t file_pos) {
  auto it = std::lower_bound(sh->hb.begin(), sh->hb.end(), file_pos,
                             [](const sbh_block &b, uint64_t v) { return b.start < v; });
  if (it == sh->hb.end() || it->start != file_pos) return -1;
  return it - sh->hb.begin();
}

int sbh_flat_of(sbh_shard *sh, uint64_t block_pos, uint32_t offset, uint64_t *flat) {
  if (!sh || !flat) return SBH_E_ARG;
  if (!sh->indexed) return fail(sh->ctx, SBH_E_STATE, "not indexed");
  const int64_t i = block_index_of(sh, block_pos);
  if (i < 0) return fail(sh->ctx, SBH_E_NOT_FOUND, "%llu is not an indexed block start", (unsigned long long)block_pos);
  *flat = sh->hb[i].ustart + offset;
  return SBH_OK;
}

int sbh_pos_of(sbh_shard *sh, uint64_t flat, uint64_t *block_pos, uint32_t *offset) {
  if (!sh || !block_pos || !offset) return SBH_E_ARG;
  if (!sh->indexed) return fail(sh->ctx, SBH_E_STATE, "not indexed");
  // last block with ustart <= flat and flat < ustart + usize (skips empty blocks)
  auto it = std::upper_bound(sh->hb.begin(), sh->hb.end(), flat,
                             [](uint64_t v, const sbh_block &b) { return v < b.ustart; });
  int64_t i = (it - sh->hb.begin()) - 1;
  while (i >= 0 && (uint64_t)i < sh->hb.size() && sh->hb[i].ustart + sh->hb[i].usize <= flat) ++i;
  if (i < 0 || (uint64_t)i >= sh->hb.size()) {
    // one past the last byte: Pos(next block, 0)
    if (!sh->hb.empty() && flat == sh->utotal) {
      const sbh_block &l = sh->hb.back();
      *block_pos = l.start + l.csize;
      *offset = 0;
      return SBH_OK;
    }
    return fail(sh->ctx, SBH_E_NOT_FOUND, "flat %llu outside the indexed stream", (unsigned long long)flat);
  }
  // skip zero-size blocks sharing this ustart
  while ((uint64_t)i < sh->hb.size() && (sh->hb[i].usize == 0 || (sh->hb[i].flags & SBH_BLOCK_EMPTY))) ++i;
  if ((uint64_t)i >= sh->hb.size()) return SBH_E_NOT_FOUND;
  *block_pos = sh->hb[i].start;
  *offset = (uint32_t)(flat - sh->hb[i].ustart);
  return SBH_OK;
}

int sbh_flat_bound(sbh_shard *sh, uint64_t file_off, uint64_t *flat) {
  if (!sh || !flat) return SBH_E_ARG;
  if (!sh->indexed) return fail(sh->ctx, SBH_E_STATE, "not indexed");
  auto it = std::lower_bound(sh->hb.begin(), sh->hb.end(), file_off,
                             [](const sbh_block &b, uint64_t v) { return b.start < v; });
  *flat = it == sh->hb.end() ? sh->utotal : it->ustart;
  return SBH_OK;
}

int sbh_set_contigs(sbh_shard *sh, const int32_t *lens, int32_t n) {
  if (!sh || n < 0 || (n && !lens)) return SBH_E_ARG;
  int rc = set_device(sh->ctx);
  if (rc) return rc;
  HIPCHK(sh->ctx, sh->ctg.ensure(n + 1));
  if (n) HIPCHK(sh->ctx, hipMemcpyAsync(sh->ctg.p, lens, (uint64_t)n * 4, hipMemcpyHostToDevice, sh->st));
  HIPCHK(sh->ctx, hipStreamSynchronize(sh->st));
  sh->nctg = n;
  sh->bits_valid = sh->chain_ok = sh->cm_valid = false;
  return SBH_OK;
}

static int need_checkable(sbh_shard *sh, uint64_t begin, uint64_t end, int32_t rtc) {
  if (!sh->inflated) return fail(sh->ctx, SBH_E_STATE, "check before inflate");
  if (sh->nctg < 0) return fail(sh->ctx, SBH_E_STATE, "contig lengths not set");
  if (begin > end || end > sh->utotal) return fail(sh->ctx, SBH_E_ARG, "range [%llu,%llu) outside [0,%llu)",
                                                  (unsigned long long)begin, (unsigned long long)end,
                                                  (unsigned long long)sh->utotal);
  if (rtc < 0 || rtc > 1023) return fail(sh->ctx, SBH_E_ARG, "readsToCheck must be in [0, 1023]");
  return SBH_OK;
}

static constexpr uint64_t XQ_CAP_MAX = 1 << 22;  // queued long-record eager candidates (2 x 32 MiB)
// SBH_XQ=0 turns the long-record queue off (every exact check inline; for A/B timing)
static uint64_t xq_cap() {
  const char *e = std::getenv("SBH_XQ");
  return e && e[0] == '0' ? 0 : XQ_CAP_MAX;
}
// SBH_TSUM=1: k_eager writes per-quarter-tile chain summaries and the chain proof reads them
// instead of every true position's record length from U (its 4.8x line over-read).  Off by
// default: measured (r04g, config B) the proof 0.46 -> 0.36 ms per step but k_eager 3.00 -> 3.24 ms.
static bool tsum_on() {
  const char *e = std::getenv("SBH_TSUM");
  return SBH_TSUM_CODE && e && e[0] == '1';
}

static int eager_range(sbh_shard *sh, uint64_t begin, uint64_t end, int32_t rtc, uint64_t *n_true) {
  sbh_ctx *ctx = sh->ctx;
  hipStream_t st = sh->st;
  const uint64_t nwords = (end - begin + 31) / 32;
  sh->chain_ok = sh->cm_valid = false;
  HIPCHK(ctx, sh->bits.ensure(nwords + 1));
  if (tsum_on()) HIPCHK(ctx, sh->tsum.ensure((end - begin + EAGER_TILE - 1) / EAGER_TILE * 4 + 4));
  HIPCHK(ctx, sh->xq.ensure(2 * XQ_CAP_MAX));
  unsigned long long *c = sh->ctr.p;
  HIPCHK(ctx, hipMemsetAsync(c, 0, 48, st));
  HIPCHK(ctx, hipMemsetAsync(c + 2, 0xff, 8, st));
  mark(sh, 4);
  HIPCHK(ctx, launch_eager(sh->U.p, sh->utotal + sh->pad, begin, end, sh->d_seg.p, (uint32_t)sh->seg_end.size(),
                           sh->open_last ? 1 : 0, sh->ctg.p, sh->nctg, rtc, sh->bits.p, c, st, ~0ull, nullptr, 0,
                           sh->xq.p, xq_cap(), tsum_on() ? sh->tsum.p : nullptr,
                           sh->sieve_nref1 && sh->sieve_nref1 == (uint32_t)sh->nctg + 1 ? sh->sieve.p : nullptr));
  HIPCHK(ctx, launch_eager_xq(sh->U.p, begin, sh->d_seg.p, (uint32_t)sh->seg_end.size(), sh->open_last ? 1 : 0,
                              sh->ctg.p, sh->nctg, rtc, sh->bits.p, c, sh->xq.p, xq_cap(), st));
  mark(sh, 5);
  HIPCHK(ctx, hipMemcpyAsync(sh->h_ctr, c, 24, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipStreamSynchronize(st));
  sh->bits_valid = true;
  sh->bits_begin = begin;
  sh->bits_end = end;
  sh->bits_rtc = rtc;
  if (n_true) *n_true = sh->h_ctr[0];
  if (sh->h_ctr[1]) {
    sh->bits_valid = false;
    return fail(ctx, SBH_E_NEED_HALO, "%llu positions (first %llu) need bytes past the shard",
                sh->h_ctr[1], sh->h_ctr[2]);
  }
  return SBH_OK;
}

int sbh_check_eager(sbh_shard *sh, uint64_t begin, uint64_t end, int32_t rtc, uint8_t *out_bits, uint64_t *n_true) {
  if (!sh) return SBH_E_ARG;
  int rc = need_checkable(sh, begin, end, rtc);
  if (rc) return rc;
  rc = set_device(sh->ctx);
  if (rc) return rc;
  rc = eager_range(sh, begin, end, rtc, n_true);
  if (rc) return rc;
  if (out_bits && end > begin) {
    HIPCHK(sh->ctx, hipMemcpyAsync(out_bits, sh->bits.p, (end - begin + 7) / 8, hipMemcpyDeviceToHost, sh->st));
    HIPCHK(sh->ctx, hipStreamSynchronize(sh->st));
  }
  return SBH_OK;
}

int sbh_eager_bits(sbh_shard *sh, uint64_t begin, uint64_t end, uint8_t *out_bits) {
  if (!sh || (!out_bits && end > begin)) return SBH_E_ARG;
  if (!sh->bits_valid) return fail(sh->ctx, SBH_E_STATE, "no eager bitmap");
  if (begin > end || begin < sh->bits_begin || end > sh->bits_end || (begin - sh->bits_begin) % 8)
    return fail(sh->ctx, SBH_E_ARG, "range [%llu,%llu) outside the bitmap [%llu,%llu) or unaligned",
                (unsigned long long)begin, (unsigned long long)end, (unsigned long long)sh->bits_begin,
                (unsigned long long)sh->bits_end);
  if (end == begin) return SBH_OK;
  int rc = set_device(sh->ctx);
  if (rc) return rc;
  const uint8_t *src = reinterpret_cast<const uint8_t *>(sh->bits.p) + (begin - sh->bits_begin) / 8;
  HIPCHK(sh->ctx, hipMemcpyAsync(out_bits, src, (end - begin + 7) / 8, hipMemcpyDeviceToHost, sh->st));
  HIPCHK(sh->ctx, hipStreamSynchronize(sh->st));
  return SBH_OK;
}

int sbh_check_full(sbh_shard *sh, uint64_t begin, uint64_t end, int32_t rtc, uint32_t *out_words, uint64_t *counts,
                   uint64_t *rbe_hist, uint64_t *n_success, uint64_t *close_flat, uint32_t *close_word,
                   uint64_t close_cap, uint64_t *n_close) {
  if (!sh) return SBH_E_ARG;
  int rc = need_checkable(sh, begin, end, rtc);
  if (rc) return rc;
  rc = set_device(sh->ctx);
  if (rc) return rc;
  sbh_ctx *ctx = sh->ctx;
  hipStream_t st = sh->st;
  const uint64_t nctr = 4 + 21 * 19 + 21 * 64;
  unsigned long long *c = sh->ctr.p;
  HIPCHK(ctx, hipMemsetAsync(c, 0, nctr * 8, st));
  HIPCHK(ctx, hipMemsetAsync(c + 2, 0xff, 8, st));
  uint32_t *words = nullptr;
  if (out_words) {
    HIPCHK(ctx, sh->words.ensure(end - begin + 1));
    words = sh->words.p;
  }
  const uint64_t cap = close_cap;
  HIPCHK(ctx, sh->close_pos.ensure(cap + 1));
  HIPCHK(ctx, sh->close_word.ensure(cap + 1));
  // the op index launch_full builds: one bit per byte from begin (1 KiB-aligned) to the
  // farthest CIGAR byte a position before `end` can name, plus four residue summaries
  const uint64_t u_pad = sh->utotal + sh->pad, ob0 = begin & ~1023ull;
  const uint64_t ob_top = std::min<uint64_t>(end + 36 + 255 + 4ull * 65535 + 4, u_pad);
  const uint64_t ob_nw = (((ob_top - ob0 + 31) / 32) + 63) & ~63ull;
  HIPCHK(ctx, sh->opix.ensure(ob_nw + ob_nw / 8));
  HIPCHK(ctx, launch_full(sh->U.p, u_pad, begin, end, sh->d_seg.p, (uint32_t)sh->seg_end.size(),
                          sh->open_last ? 1 : 0, sh->ctg.p, sh->nctg, rtc, words, c, sh->close_pos.p,
                          sh->close_word.p, cap, sh->opix.p, sh->opix.cap, st));
  HIPCHK(ctx, hipMemcpyAsync(sh->h_ctr, c, nctr * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipStreamSynchronize(st));
  if (sh->h_ctr[1])
    return fail(ctx, SBH_E_NEED_HALO, "%llu positions (first %llu) need bytes past the shard", sh->h_ctr[1],
                sh->h_ctr[2]);
  if (n_success) *n_success = sh->h_ctr[0];
  const uint64_t nclose = sh->h_ctr[3];
  if (n_close) *n_close = nclose;
  if (counts) for (int i = 0; i < 21 * 19; ++i) counts[i] = sh->h_ctr[4 + i];
  if (rbe_hist) for (int i = 0; i < 21 * 64; ++i) rbe_hist[i] = sh->h_ctr[4 + 21 * 19 + i];
  const uint64_t ncopy = std::min<uint64_t>(nclose, cap);
  if (ncopy && (close_flat || close_word)) {
    // positions arrive in atomic order: sort them on the host
    std::vector<uint64_t> p(ncopy);
    std::vector<uint32_t> w(ncopy);
    HIPCHK(ctx, hipMemcpyAsync(p.data(), sh->close_pos.p, ncopy * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipMemcpyAsync(w.data(), sh->close_word.p, ncopy * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipStreamSynchronize(st));
    std::vector<uint64_t> idx(ncopy);
    for (uint64_t i = 0; i < ncopy; ++i) idx[i] = i;
    std::sort(idx.begin(), idx.end(), [&](uint64_t a, uint64_t b) { return p[a] < p[b]; });
    for (uint64_t i = 0; i < ncopy; ++i) {
      if (close_flat) close_flat[i] = p[idx[i]];
      if (close_word) close_word[i] = w[idx[i]];
    }
  }
  if (out_words && end > begin) {
    HIPCHK(ctx, hipMemcpyAsync(out_words, sh->words.p, (end - begin) * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipStreamSynchronize(st));
  }
  return SBH_OK;
}

static uint64_t seg_end_of(const sbh_shard *sh, uint64_t p) {
  for (uint64_t e : sh->seg_end)
    if (e > p) return e;
  return sh->seg_end.back();
}
static bool seg_is_open(const sbh_shard *sh, uint64_t p) {
  return sh->open_last && seg_end_of(sh, p) == sh->seg_end.back();
}

// FindRecordStart.withDelta (check/.../spark/FindRecordStart.scala:30-63)
int sbh_find_record_start(sbh_shard *sh, uint64_t from, int32_t rtc, int32_t max_read_size, uint64_t *out_flat,
                          int32_t *out_delta) {
  if (!sh || !out_flat) return SBH_E_ARG;
  sbh_ctx *ctx = sh->ctx;
  int rc = need_checkable(sh, from, from, rtc);
  if (rc) return rc;
  rc = set_device(ctx);
  if (rc) return rc;
  hipStream_t st = sh->st;
  const uint64_t seg = seg_end_of(sh, from);
  const uint64_t limit = std::min<uint64_t>(seg, from + (uint64_t)std::max(max_read_size, 0));
  uint64_t lo = from;
  uint64_t window = 1 << 20;
  while (lo < limit) {
    uint64_t hi;
    bool covered = sh->bits_valid && sh->bits_rtc == rtc && sh->bits_begin <= lo && lo < sh->bits_end;
    if (covered) {
      hi = std::min(limit, sh->bits_end);
    } else {
      hi = std::min(limit, lo + window);
      window = std::min<uint64_t>(window * 4, 1ull << 28);
      rc = eager_range(sh, lo, hi, rtc, nullptr);
      if (rc == SBH_E_NEED_HALO) {
        // unknowns are fine only if a true position precedes the first unknown
        const uint64_t first_unknown = sh->h_ctr[2];
        unsigned long long *best = sh->ctr.p + 8;
        HIPCHK(ctx, hipMemsetAsync(best, 0xff, 8, st));
        sh->bits_valid = true;
        HIPCHK(ctx, launch_first_set(sh->bits.p, lo, lo, first_unknown, best, st));
        HIPCHK(ctx, hipMemcpyAsync(sh->h_ctr + 8, best, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(ctx, hipStreamSynchronize(st));
        sh->bits_valid = false;
        if (sh->h_ctr[8] != ~0ull) {
          *out_flat = sh->h_ctr[8];
          if (out_delta) *out_delta = (int32_t)(sh->h_ctr[8] - from);
          return SBH_OK;
        }
        return rc;
      }
      if (rc) return rc;
    }
    unsigned long long *best = sh->ctr.p + 8;
    HIPCHK(ctx, hipMemsetAsync(best, 0xff, 8, st));
    HIPCHK(ctx, launch_first_set(sh->bits.p, sh->bits_begin, lo, hi, best, st));
    HIPCHK(ctx, hipMemcpyAsync(sh->h_ctr + 8, best, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipStreamSynchronize(st));
    if (sh->h_ctr[8] != ~0ull) {
      *out_flat = sh->h_ctr[8];
      if (out_delta) *out_delta = (int32_t)(sh->h_ctr[8] - from);
      return SBH_OK;
    }
    lo = hi;
  }
  if (lo >= seg && seg_is_open(sh, from) && (uint64_t)max_read_size > seg - from)
    return fail(ctx, SBH_E_NEED_HALO, "record search from %llu runs past the shard", (unsigned long long)from);
  return fail_with(ctx, SBH_E_NO_READ_FOUND, {(int64_t)from, max_read_size},
                   "no read start within %d positions of flat %llu", max_read_size, (unsigned long long)from);
}

// Records of the chain from `first` whose start is < E; *exit_flat (optional) = the
// first chain record at/after E (the successor of the last counted record, clamped to
// the stream end) -- what the next shard's first record must equal when stitching.

// `known`: the four chain-proof counters (anomalies, first anomaly, set bits, exit) that a
// k_verify_chain_w launch over this same [first, E) and bitmap already left in h_ctr[16..19]
// (sbh_run_shard's tail): the proof is not run again.
static int count_records_impl(sbh_shard *sh, uint64_t first, uint64_t E, uint64_t *count, int32_t *anomalies,
                              uint64_t *exit_flat = nullptr, bool known = false) {
  sbh_ctx *ctx = sh->ctx;
  hipStream_t st = sh->st;
  const uint64_t total = seg_end_of(sh, first);
  E = std::min(E, total);
  if (anomalies) *anomalies = 0;
  sh->cm_valid = false;
  sh->chain_ok = false;
  if (first >= E) {
    *count = 0;
    if (exit_flat) *exit_flat = first;
    return SBH_OK;
  }
  unsigned long long *c = sh->ctr.p + 16;
  const bool covered = sh->bits_valid && sh->bits_begin <= first && E <= sh->bits_end;
  if (covered) {
    // counters c[0..3]: anomalies, first anomaly, set bits in [first, E), chain exit
    unsigned long long *init = sh->h_ctr + 600;  // pinned
    init[0] = 0;
    init[1] = ~0ull;
    init[2] = 0;
    init[3] = ~0ull;
    if (!known) {
      HIPCHK(ctx, hipMemcpyAsync(c, init, 32, hipMemcpyHostToDevice, st));
      HIPCHK(ctx, sh->cc.ensure((sh->bits_end - sh->bits_begin + 31) / 32 / VC_CHUNK + 2));
      // verify bitmap == chain and count the set bits in one pass (k_verify_chain_w: wave-
      // cooperative successors, so sparse bitmaps of long records cost no word-by-word scans)
      HIPCHK(ctx, launch_verify_chain_count(sh->U.p, sh->bits.p, sh->bits_begin, sh->bits_end, first, E, total, c,
                                            c + 1, c + 3, c + 2, tsum_on() ? sh->tsum.p : nullptr, st, nullptr,
                                            sh->cc.p));
      HIPCHK(ctx, hipMemcpyAsync(sh->h_ctr + 16, c, 32, hipMemcpyDeviceToHost, st));
      HIPCHK(ctx, hipStreamSynchronize(st));
    }
    const uint64_t n = sh->h_ctr[18];
    if (sh->h_ctr[16] == 0 && sh->h_ctr[19] != ~0ull) {
      sh->chain_ok = true;
      sh->cc_ok = true;  // (this proof's chunk counts, or the run's tail proof's over the same range)
      sh->chain_first = first;
      sh->chain_E = E;
      *count = n;
      if (exit_flat) *exit_flat = sh->h_ctr[19];
      return SBH_OK;
    }
    if (anomalies) *anomalies = (int32_t)std::min<uint64_t>(sh->h_ctr[16], INT32_MAX);
    // the bitmap is not exactly the chain (false positives / rejected chain records): mark
    // the chain through the set bits by pointer doubling; the exact walk only when the
    // chain leaves the set bits
    if (n > 0 && n < 0xfffffff0ull) {
      const uint64_t nw = (E - sh->bits_begin + 31) / 32 - (first - sh->bits_begin) / 32;
      HIPCHK(ctx, sh->cm_wcnt.ensure(nw + 2));  // (chunk sums + prefix: 2 per 4096 words)
      HIPCHK(ctx, sh->cm_wpre.ensure(nw));
      HIPCHK(ctx, sh->cm_pos.ensure(n));
      HIPCHK(ctx, sh->cm_mark.ensure(n + 1));
      HIPCHK(ctx, sh->cm_mpre.ensure(n + 1));
      HIPCHK(ctx, sh->cm_j.ensure(n + 1));
      HIPCHK(ctx, sh->cm_j2.ensure(n + 1));
      HIPCHK(ctx, sh->cm_j0.ensure(n + 1));
      HIPCHK(ctx, sh->tmp.ensure(std::max(scan_tmp_words(nw), scan_tmp_words(n + 1))));
      HIPCHK(ctx, launch_rec_positions_bits(sh->bits.p, sh->bits_begin, first, E, sh->cm_wcnt.p, sh->cm_wpre.p,
                                            sh->tmp.p, sh->cm_pos.p, st));
      HIPCHK(ctx, hipMemsetAsync(c + 6, 0xff, 8, st));
      uint32_t *code = reinterpret_cast<uint32_t *>(sh->h_ctr + 22);
      HIPCHK(ctx, launch_chain_mark(sh->U.p, sh->bits.p, sh->bits_begin, first, E, total, sh->cm_pos.p,
                                    sh->cm_wpre.p, n, sh->cm_j.p, sh->cm_j2.p, sh->cm_j0.p, sh->cm_mark.p, c + 6,
                                    code, st));
      HIPCHK(ctx, hipMemsetAsync(sh->cm_mark.p + n, 0, 8, st));
      HIPCHK(ctx, scan_exclusive_u64(sh->cm_mark.p, sh->cm_mpre.p, n + 1, sh->tmp.p, st));
      HIPCHK(ctx, hipMemcpyAsync(sh->h_ctr + 23, sh->cm_mpre.p + n, 8, hipMemcpyDeviceToHost, st));
      HIPCHK(ctx, hipMemcpyAsync(sh->h_ctr + 24, sh->cm_pos.p, 8, hipMemcpyDeviceToHost, st));
      HIPCHK(ctx, hipMemcpyAsync(sh->h_ctr + 25, c + 6, 8, hipMemcpyDeviceToHost, st));
      HIPCHK(ctx, hipStreamSynchronize(st));
      if (*code == (uint32_t)n && sh->h_ctr[24] == first) {
        sh->cm_valid = true;
        sh->cm_first = first;
        sh->cm_E = E;
        sh->cm_n = n;
        *count = sh->h_ctr[23];
        if (exit_flat) *exit_flat = sh->h_ctr[25];
        // set bits off the chain (false positives); 0 means the bitmap is the chain
        if (anomalies) *anomalies = (int32_t)std::min<uint64_t>(n - *count, INT32_MAX);
        return SBH_OK;
      }
    }
  }
  HIPCHK(ctx, launch_chain_walk(sh->U.p, first, E, total, c + 4, c + 5, st));
  HIPCHK(ctx, hipMemcpyAsync(sh->h_ctr + 20, c + 4, 16, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipStreamSynchronize(st));
  *count = sh->h_ctr[20];
  if (exit_flat) *exit_flat = sh->h_ctr[21];
  return SBH_OK;
}

int sbh_count_records(sbh_shard *sh, uint64_t first, uint64_t end_flat, uint64_t *count) {
  if (!sh || !count) return SBH_E_ARG;
  if (!sh->inflated) return fail(sh->ctx, SBH_E_STATE, "count before inflate");
  if (first > sh->utotal) return SBH_E_ARG;
  int rc = set_device(sh->ctx);
  if (rc) return rc;
  return count_records_impl(sh, first, std::min(end_flat, sh->utotal), count, nullptr);
}

// CanLoadBam.loadReadsAndPositions, one split (load/.../CanLoadBam.scala:316-356)
int sbh_split(sbh_shard *sh, uint64_t start, uint64_t end, int32_t k, int32_t rtc, int32_t mrs, uint64_t *first_vpos,
              uint64_t *count) {
  if (!sh || !first_vpos || !count) return SBH_E_ARG;
  sbh_ctx *ctx = sh->ctx;
  if (!sh->inflated) return fail(ctx, SBH_E_STATE, "split before inflate");
  uint64_t b = 0;
  int rc = sbh_find_block_start(sh, start, k, &b);
  if (rc) return rc;
  const int64_t bi = block_index_of(sh, b);
  if (bi < 0) {
    if (b >= sh->file_size || (sh->at_eof && b >= sh->file_off + sh->n))
      return fail_with(ctx, SBH_E_NO_READ_FOUND, {(int64_t)start, mrs}, "split at %llu: no blocks left",
                       (unsigned long long)start);
    return fail(ctx, SBH_E_NOT_FOUND, "block start %llu is not on the indexed chain", (unsigned long long)b);
  }
  if (sh->hb[bi].flags & SBH_BLOCK_EMPTY)  // the stream from an empty block ends at once
    return fail_with(ctx, SBH_E_NO_READ_FOUND, {(int64_t)start, mrs}, "split at %llu starts at an empty block",
                     (unsigned long long)start);
  uint64_t first = 0;
  int32_t delta = 0;
  rc = sbh_find_record_start(sh, sh->hb[bi].ustart, rtc, mrs, &first, &delta);
  if (rc) return rc;
  uint64_t E = 0;
  (void)sbh_flat_bound(sh, end, &E);
  if (!sh->at_eof && end > sh->hb.back().start && E == sh->utotal)
    return fail(ctx, SBH_E_NEED_HALO, "split end %llu past the resident blocks", (unsigned long long)end);
  rc = count_records_impl(sh, first, E, count, nullptr);
  if (rc) return rc;
  uint64_t bp = 0;
  uint32_t off = 0;
  rc = sbh_pos_of(sh, first, &bp, &off);
  if (rc) return rc;
  *first_vpos = (bp << 16) | off;
  return SBH_OK;
}

// The record chain from first_flat (PosStream.scala:14-22): records whose start is < end_flat,
// and the chain's exit (its first record at/after end_flat, or where the stream ends).
int sbh_chain_from(sbh_shard *sh, uint64_t first_flat, uint64_t end_flat, uint64_t *count, uint64_t *exit_flat) {
  if (!sh || !count) return SBH_E_ARG;
  if (!sh->inflated) return fail(sh->ctx, SBH_E_STATE, "chain before inflate");
  if (first_flat > sh->utotal) return SBH_E_ARG;
  int rc = set_device(sh->ctx);
  if (rc) return rc;
  uint64_t ex = first_flat;
  rc = count_records_impl(sh, first_flat, std::min(end_flat, sh->utotal), count, nullptr, &ex);
  if (!rc && exit_flat) *exit_flat = ex;
  return rc;
}

// Every split of loadReadsAndPositions / loadSplitsAndReads at once (CanLoadBam.scala:283-297,
// 316-356; SURVEY 8b sbh_split_starts): one launch runs FindBlockStart + FindRecordStart for
// all splits (splits.hip), one proves the record chain over their union, one counts every
// split.  Splits off the common path take the exact per-split path (sbh_split), so each
// split's (status, first_vpos, count) equals sbh_split's.
int sbh_split_starts(sbh_shard *sh, const uint64_t *starts, const uint64_t *ends, uint64_t n, int32_t k, int32_t rtc,
                     int32_t mrs, uint64_t *first_vpos, uint64_t *counts, int32_t *status, uint64_t *n_host) {
  if (!sh || (n && (!starts || !ends || !first_vpos || !counts || !status)) || k < 0) return SBH_E_ARG;
  sbh_ctx *ctx = sh->ctx;
  if (!sh->inflated) return fail(ctx, SBH_E_STATE, "splits before inflate");
  int rc = need_checkable(sh, 0, 0, rtc);
  if (rc) return rc;
  rc = set_device(ctx);
  if (rc) return rc;
  if (n_host) *n_host = 0;
  if (!n) return SBH_OK;
  hipStream_t st = sh->st;
  const uint64_t end_res = sh->file_off + sh->n;
  // the eager bitmap from the stream start (reused when one is resident, e.g. sbh_run_shard's
  // over the owned range; a record start past its end takes the host path)
  if (!(sh->bits_valid && sh->bits_rtc == rtc && sh->bits_begin == 0)) {
    rc = eager_range(sh, 0, sh->utotal, rtc, nullptr);
    if (rc && rc != SBH_E_NEED_HALO) return rc;
    sh->bits_valid = true;  // positions needing the halo are clear; record starts past them go to the host path
    sh->bits_begin = 0;
    sh->bits_end = sh->utotal;
    sh->bits_rtc = rtc;
    if (rc == SBH_E_NEED_HALO) sh->bits_end = std::min<uint64_t>(sh->utotal, sh->h_ctr[2]);
  }
  auto rel_start = [&](uint64_t i) -> uint64_t {  // (a start off the shard: host path, flagged below)
    return starts[i] < sh->file_off || starts[i] >= end_res ? 0 : starts[i] - sh->file_off;
  };
  auto rel_end = [&](uint64_t i) -> uint64_t { return ends[i] >= sh->file_off ? ends[i] - sh->file_off : 0; };
  const SplitArgs a{sh->comp.p, sh->n, sh->at_eof ? 1 : 0, sh->cand.p, sh->ncand, sh->cand_from, k,
                    sh->b_cstart.p, sh->b_ustart.p, sh->b_flags.p, sh->nblocks, sh->utotal,
                    sh->hb.empty() ? 0 : sh->hb.back().start - sh->file_off, sh->d_seg.p,
                    (uint32_t)sh->seg_end.size(), sh->bits.p, sh->bits_begin, sh->bits_end,
                    (int64_t)std::max(mrs, 0)};
  // Fast path (the step's case): the chain proof covers the splits and left its chunk counts.
  // The ranges go over in one copy, the prologue and the counts run back to back, and
  // [first, E, count, code] come back in one copy: one round trip.  A split whose range leaves
  // the proven chain (SPLIT_NOCOUNT) sends the call down the general path below.
  if (sh->chain_ok && sh->cc_ok && sh->chain_E > 0 && split_cc_on()) {
    const uint64_t words = 5 * n + (n + 1) / 2;
    if (sh->sp_pin_cap < words) {
      if (sh->sp_pin) (void)hipHostFree(sh->sp_pin);
      sh->sp_pin = nullptr;
      sh->sp_pin_cap = 0;
      HIPCHK(ctx, hipHostMalloc(reinterpret_cast<void **>(&sh->sp_pin), words * 8));
      sh->sp_pin_cap = words;
    }
    HIPCHK(ctx, sh->sp_pack.ensure(words));
    uint64_t *hp = sh->sp_pin, *dp = sh->sp_pack.p;
    for (uint64_t i = 0; i < n; ++i) {
      hp[i] = rel_start(i);
      hp[n + i] = rel_end(i);
    }
    uint32_t *dcode = reinterpret_cast<uint32_t *>(dp + 5 * n);
    HIPCHK(ctx, set_words(dp, hp, 2 * n, st));
    HIPCHK(ctx, launch_split_prologue(a, dp, dp + n, n, dp + 2 * n, dp + 3 * n, dcode, st));
    HIPCHK(ctx, launch_split_count_cc(sh->bits.p, sh->bits_begin, sh->cc.p, dp + 2 * n, dp + 3 * n, dcode, n,
                                      reinterpret_cast<unsigned long long *>(dp + 4 * n), st, sh->chain_first,
                                      sh->chain_E));
    // (the same page-locked words: the stream runs the copy in after the copy out has read them)
    HIPCHK(ctx, hipMemcpyAsync(hp + 2 * n, dp + 2 * n, (words - 2 * n) * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipStreamSynchronize(st));
    const uint64_t *first = hp + 2 * n, *E = hp + 3 * n, *cnt = hp + 4 * n;
    const uint32_t *code = reinterpret_cast<const uint32_t *>(hp + 5 * n);
    bool all = true;
    for (uint64_t i = 0; i < n && all; ++i)
      all = !(code[i] == SPLIT_OK && starts[i] >= sh->file_off && starts[i] < end_res && first[i] < E[i] &&
              cnt[i] == SPLIT_NOCOUNT);
    if (all) {
      uint64_t nh = 0;
      for (uint64_t i = 0; i < n; ++i) {
        const uint32_t ci = starts[i] < sh->file_off || starts[i] >= end_res ? SPLIT_HOST : code[i];
        if (ci == SPLIT_OK) {
          uint64_t bp = 0;
          uint32_t off = 0;
          rc = sbh_pos_of(sh, first[i], &bp, &off);
          if (rc) return rc;
          first_vpos[i] = (bp << 16) | off;
          counts[i] = first[i] < E[i] ? cnt[i] : 0;
          status[i] = SBH_OK;
        } else if (ci == SPLIT_NOREAD) {
          first_vpos[i] = counts[i] = 0;
          status[i] = SBH_E_NO_READ_FOUND;
        } else {
          ++nh;
          first_vpos[i] = counts[i] = 0;
          // (sbh_split leaves sp_pin alone: first / E / cnt stay valid)
          status[i] = sbh_split(sh, starts[i], ends[i], k, rtc, mrs, &first_vpos[i], &counts[i]);
        }
      }
      if (n_host) *n_host = nh;
      return SBH_OK;
    }
  }
  std::vector<uint64_t> rs(n), re(n);
  for (uint64_t i = 0; i < n; ++i) {
    rs[i] = rel_start(i);
    re[i] = rel_end(i);
  }
  HIPCHK(ctx, sh->sp_start.ensure(n));
  HIPCHK(ctx, sh->sp_end.ensure(n));
  HIPCHK(ctx, sh->sp_first.ensure(n));
  HIPCHK(ctx, sh->sp_E.ensure(n));
  HIPCHK(ctx, sh->sp_code.ensure(n));
  HIPCHK(ctx, sh->sp_count.ensure(n));
  HIPCHK(ctx, hipMemcpyAsync(sh->sp_start.p, rs.data(), 8 * n, hipMemcpyHostToDevice, st));
  HIPCHK(ctx, hipMemcpyAsync(sh->sp_end.p, re.data(), 8 * n, hipMemcpyHostToDevice, st));
  HIPCHK(ctx, launch_split_prologue(a, sh->sp_start.p, sh->sp_end.p, n, sh->sp_first.p, sh->sp_E.p, sh->sp_code.p, st));
  std::vector<uint64_t> first(n), E(n);
  std::vector<uint32_t> code(n);
  HIPCHK(ctx, hipMemcpyAsync(first.data(), sh->sp_first.p, 8 * n, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipMemcpyAsync(E.data(), sh->sp_E.p, 8 * n, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipMemcpyAsync(code.data(), sh->sp_code.p, 4 * n, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipStreamSynchronize(st));
  uint64_t fmin = ~0ull, Emax = 0, span = 0;
  for (uint64_t i = 0; i < n; ++i) {
    if (starts[i] < sh->file_off || starts[i] >= end_res) code[i] = SPLIT_HOST;
    if (code[i] != SPLIT_OK || first[i] >= E[i]) continue;
    fmin = std::min(fmin, first[i]);
    Emax = std::max(Emax, E[i]);
    span = std::max(span, E[i] - first[i]);
  }
  bool dense = false, marked = false;
  if (fmin < Emax) {
    // the chain proof over the union of the splits: the bitmap verified equal to the chain
    // (then a split's count is a popcount), or the chain marked through the set bits
    dense = sh->chain_ok && sh->chain_first <= fmin && Emax <= sh->chain_E;
    marked = sh->cm_valid && sh->cm_first <= fmin && Emax <= sh->cm_E;
    if (!dense && !marked) {
      uint64_t cnt = 0;
      rc = count_records_impl(sh, fmin, Emax, &cnt, nullptr);
      if (rc) return rc;
      dense = sh->chain_ok && sh->chain_first <= fmin && Emax <= sh->chain_E;
      marked = sh->cm_valid && sh->cm_first <= fmin && Emax <= sh->cm_E;
    }
  }
  HIPCHK(ctx, hipMemsetAsync(sh->sp_count.p, 0, 8 * n, st));
  if (dense) {
    HIPCHK(ctx, hipMemcpyAsync(sh->sp_code.p, code.data(), 4 * n, hipMemcpyHostToDevice, st));
    if (sh->cc_ok && split_cc_on())  // the proof's chunk counts: the bitmap read only at the ranges' ends
      HIPCHK(ctx, launch_split_count_cc(sh->bits.p, sh->bits_begin, sh->cc.p, sh->sp_first.p, sh->sp_E.p,
                                        sh->sp_code.p, n, sh->sp_count.p, st));
    else
      HIPCHK(ctx, launch_split_popcount(sh->bits.p, sh->bits_begin, sh->sp_first.p, sh->sp_E.p, sh->sp_code.p, n,
                                        span, sh->sp_count.p, st));
  } else if (marked) {
    HIPCHK(ctx, hipMemcpyAsync(sh->sp_code.p, code.data(), 4 * n, hipMemcpyHostToDevice, st));
    HIPCHK(ctx, launch_split_cm_count(sh->cm_pos.p, sh->cm_mark.p, sh->cm_mpre.p, sh->cm_n, sh->sp_first.p,
                                      sh->sp_E.p, sh->sp_code.p, n, sh->sp_count.p, st));
    HIPCHK(ctx, hipMemcpyAsync(code.data(), sh->sp_code.p, 4 * n, hipMemcpyDeviceToHost, st));
  } else {
    for (uint64_t i = 0; i < n; ++i)
      if (code[i] == SPLIT_OK && first[i] < E[i]) code[i] = SPLIT_HOST;
  }
  std::vector<unsigned long long> cnt(n);
  HIPCHK(ctx, hipMemcpyAsync(cnt.data(), sh->sp_count.p, 8 * n, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipStreamSynchronize(st));
  uint64_t nh = 0;
  for (uint64_t i = 0; i < n; ++i) {
    if (code[i] == SPLIT_OK) {
      uint64_t bp = 0;
      uint32_t off = 0;
      rc = sbh_pos_of(sh, first[i], &bp, &off);
      if (rc) return rc;
      first_vpos[i] = (bp << 16) | off;
      counts[i] = first[i] < E[i] ? cnt[i] : 0;
      status[i] = SBH_OK;
      continue;
    }
    if (code[i] == SPLIT_NOREAD) {  // as sbh_split: the split starts at an empty block
      first_vpos[i] = counts[i] = 0;
      status[i] = SBH_E_NO_READ_FOUND;
      continue;
    }
    ++nh;
    if (std::getenv("SBH_SPLIT_DEBUG"))
      fprintf(stderr, "[sbh] split %llu [%llu, %llu) host path: shard [%llu, +%llu) first %llu E %llu dense %d marked %d code %#x\n",
              (unsigned long long)i, (unsigned long long)starts[i], (unsigned long long)ends[i],
              (unsigned long long)sh->file_off, (unsigned long long)sh->n, (unsigned long long)first[i],
              (unsigned long long)E[i], (int)dense, (int)marked, code[i]);
    first_vpos[i] = counts[i] = 0;
    status[i] = sbh_split(sh, starts[i], ends[i], k, rtc, mrs, &first_vpos[i], &counts[i]);
  }
  if (n_host) *n_host = nh;
  return SBH_OK;
}

// check-bam's comparison with the `.records` truth (CheckerApp.scala:65-227) on the device:
// the eager bitmap over the hull of the selected flat ranges, the truth (htsjdk vpos of every
// record) scattered into a second bitmap, and one word-parallel compare.  fp_flat / fn_flat
// (optional) receive up to fp_cap / fn_cap mismatching flat positions, sorted: all of them
// when there are at most that many, otherwise an arbitrary subset (the compaction is in
// atomic order), not the first ones by position.
static int check_records_impl(sbh_shard *sh, const uint64_t *range_begin, const uint64_t *range_end,
                              uint64_t n_ranges, int32_t rtc, const uint64_t *rec_vpos, uint64_t n_rec,
                              bool resident, uint64_t *out, uint64_t *fp_flat, uint64_t fp_cap, uint64_t *fn_flat,
                              uint64_t fn_cap);

int sbh_check_records(sbh_shard *sh, const uint64_t *range_begin, const uint64_t *range_end, uint64_t n_ranges,
                      int32_t rtc, const uint64_t *rec_vpos, uint64_t n_rec, uint64_t *out /*tp, fp, fn, unknown*/,
                      uint64_t *fp_flat, uint64_t fp_cap, uint64_t *fn_flat, uint64_t fn_cap) {
  if (!sh || !out || (n_ranges && (!range_begin || !range_end)) || (n_rec && !rec_vpos)) return SBH_E_ARG;
  return check_records_impl(sh, range_begin, range_end, n_ranges, rtc, rec_vpos, n_rec, false, out, fp_flat, fp_cap,
                            fn_flat, fn_cap);
}

}  // extern "C"

int sbh::check_records_resident(sbh_shard *sh, const uint64_t *range_begin, const uint64_t *range_end,
                                uint64_t n_ranges, int32_t rtc, uint64_t n_rec, uint64_t *out, uint64_t *fp_flat,
                                uint64_t fp_cap, uint64_t *fn_flat, uint64_t fn_cap) {
  if (!sh || !out || (n_ranges && (!range_begin || !range_end)) || (n_rec && sh->sp_vpos.cap < n_rec))
    return SBH_E_ARG;
  return check_records_impl(sh, range_begin, range_end, n_ranges, rtc, nullptr, n_rec, true, out, fp_flat, fp_cap,
                            fn_flat, fn_cap);
}

extern "C" {

static int check_records_impl(sbh_shard *sh, const uint64_t *range_begin, const uint64_t *range_end,
                              uint64_t n_ranges, int32_t rtc, const uint64_t *rec_vpos, uint64_t n_rec,
                              bool resident, uint64_t *out, uint64_t *fp_flat, uint64_t fp_cap, uint64_t *fn_flat,
                              uint64_t fn_cap) {
  sbh_ctx *ctx = sh->ctx;
  for (uint64_t r = 0; r < n_ranges; ++r)
    if (range_begin[r] > range_end[r] || (r && range_begin[r] < range_end[r - 1]))
      return fail(ctx, SBH_E_ARG, "ranges must be sorted and disjoint");
  out[0] = out[1] = out[2] = out[3] = 0;
  if (!n_ranges) return SBH_OK;
  const uint64_t begin = range_begin[0], end = range_end[n_ranges - 1];
  int rc = need_checkable(sh, begin, end, rtc);
  if (rc) return rc;
  rc = set_device(ctx);
  if (rc) return rc;
  hipStream_t st = sh->st;
  // the eager bitmap over the hull, aligned so its words line up with the truth words
  const uint64_t hb0 = begin & ~31ull;
  if (!(sh->bits_valid && sh->bits_rtc == rtc && sh->bits_begin <= hb0 && end <= sh->bits_end &&
        sh->bits_begin % 32 == 0)) {
    rc = eager_range(sh, hb0, end, rtc, nullptr);
    if (rc) return rc;
  }
  const uint64_t nw = (end - hb0 + 31) / 32;
  HIPCHK(ctx, sh->tbits.ensure(nw + 1));
  HIPCHK(ctx, hipMemsetAsync(sh->tbits.p, 0, 4 * (nw + 1), st));
  if (!resident) {
    HIPCHK(ctx, sh->sp_vpos.ensure(n_rec + 1));
    if (n_rec) HIPCHK(ctx, hipMemcpyAsync(sh->sp_vpos.p, rec_vpos, 8 * n_rec, hipMemcpyHostToDevice, st));
  }
  HIPCHK(ctx, sh->t_rb.ensure(n_ranges));
  HIPCHK(ctx, sh->t_re.ensure(n_ranges));
  HIPCHK(ctx, hipMemcpyAsync(sh->t_rb.p, range_begin, 8 * n_ranges, hipMemcpyHostToDevice, st));
  HIPCHK(ctx, hipMemcpyAsync(sh->t_re.p, range_end, 8 * n_ranges, hipMemcpyHostToDevice, st));
  const uint64_t cap_fp = fp_flat ? fp_cap : 0, cap_fn = fn_flat ? fn_cap : 0;
  HIPCHK(ctx, sh->t_fp.ensure(cap_fp + 1));
  HIPCHK(ctx, sh->t_fn.ensure(cap_fn + 1));
  unsigned long long *acc = sh->ctr.p + 40;  // tp, fp, fn, fp slots, fn slots, unknown
  HIPCHK(ctx, hipMemsetAsync(acc, 0, 6 * 8, st));
  HIPCHK(ctx, launch_truth_scatter(sh->sp_vpos.p, n_rec, sh->b_cstart.p, sh->b_ustart.p, sh->nblocks, sh->file_off,
                                   hb0, end, sh->tbits.p, acc + 5, st));
  HIPCHK(ctx, launch_truth_compare(sh->bits.p, sh->bits_begin, sh->tbits.p, hb0, end, sh->t_rb.p, sh->t_re.p,
                                   n_ranges, acc, sh->t_fp.p, cap_fp, sh->t_fn.p, cap_fn, st));
  HIPCHK(ctx, hipMemcpyAsync(sh->h_ctr + 40, acc, 6 * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipStreamSynchronize(st));
  out[0] = sh->h_ctr[40];
  out[1] = sh->h_ctr[41];
  out[2] = sh->h_ctr[42];
  out[3] = sh->h_ctr[45];
  // the mismatch lists arrive in atomic order and are sorted here; when there are more
  // mismatches than the cap, the listed ones are a (sorted) subset
  auto fetch = [&](uint64_t *dst, const uint64_t *src, uint64_t cap, uint64_t total) -> int {
    const uint64_t k = std::min(cap, total);
    if (!dst || !k) return SBH_OK;
    HIPCHK(ctx, hipMemcpyAsync(dst, src, 8 * k, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipStreamSynchronize(st));
    std::sort(dst, dst + k);
    return SBH_OK;
  };
  rc = fetch(fp_flat, sh->t_fp.p, cap_fp, out[1]);
  if (!rc) rc = fetch(fn_flat, sh->t_fn.p, cap_fn, out[2]);
  return rc;
}

// Inflate + eager check of flat [0, E) as one pipeline over batches of blocks, on three
// streams: k_huff of batch i+1 runs beside k_lz of batch i and beside the eager tiles
// whose staged windows batch i completed (k_huff is latency-bound on LDS and VALU, k_lz on
// barriers, k_eager on its chain walks: side by side they fill each other's idle issue
// slots).  An eager position whose exact check needs bytes past the inflated frontier is
// deferred and re-checked at the end.  Same results as sbh_inflate + sbh_check_eager.
static constexpr uint64_t PIPE_MAX_BATCHES = 16;
static constexpr uint64_t DEFER_CAP = 1 << 20;

// Batches of at least SBH_PIPE_MIN_BLOCKS blocks (tests: small batches exercise many
// frontiers on small inputs).  Default: one batch.  Measured on MI355X (1 GiB shard,
// this design): 1 batch 34.7 ms/step, 3 batches 35.2, 16 batches 38.2 -- side by side
// the three kernels contend for the same LDS and issue slots, and k_lz (two 80 KiB
// workgroups per CU) loses the most; the pipeline stays for inputs where it pays.
static uint64_t pipe_min_blocks() {
  const char *e = std::getenv("SBH_PIPE_MIN_BLOCKS");
  const long long v = e ? std::atoll(e) : 0;
  return v > 0 ? (uint64_t)v : ~0ull;
}

static hipEvent_t pev(sbh_shard *sh, size_t i) {
  while (sh->pev.size() <= i) {
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    sh->pev.push_back(e);
  }
  return sh->pev[i];
}

// pre_sync (optional): more work enqueued on the main stream after the eager kernels and before
// the one host round trip that brings back the inflate status and the eager counters (its
// results are only meaningful when this returns SBH_OK without a fallback)
static int run_pipelined(sbh_shard *sh, uint64_t E, int32_t rtc, uint64_t *n_true,
                         const std::function<hipError_t(hipStream_t)> &pre_sync = nullptr) {
  sbh_ctx *ctx = sh->ctx;
  if (!sh->indexed) return fail(ctx, SBH_E_STATE, "inflate before index");
  if (sh->nctg < 0) return fail(ctx, SBH_E_STATE, "contig lengths not set");
  if (rtc < 0 || rtc > 1023) return fail(ctx, SBH_E_ARG, "readsToCheck must be in [0, 1023]");
  hipStream_t sa = sh->st;
  HIPCHK(ctx, sh->U.ensure(sh->utotal + sh->pad));
  const uint64_t nb = sh->nblocks;
  const uint64_t npipe = std::max<uint64_t>(1, std::min<uint64_t>(PIPE_MAX_BATCHES, nb / pipe_min_blocks()));
  const TokPlan P = tok_plan(sh, (nb + npipe - 1) / std::max<uint64_t>(npipe, 1));
  // one batch (the default) of a resident shard: every launch on the shard's stream, no
  // cross-stream event waits (each cost the step ~15 us of idle device between the stages)
  hipStream_t sl = sa, se = sa;
  static const char *ps = std::getenv("SBH_PIPE_STREAMS");  // (A/B: 3 = three streams for every shard)
  static const bool three = ps && std::atoi(ps) == 3;
  if (P.batches.size() > 1 || three) {
    if (!sh->s_lz) HIPCHK(ctx, hipStreamCreateWithFlags(&sh->s_lz, hipStreamNonBlocking));
    if (!sh->s_eg) HIPCHK(ctx, hipStreamCreateWithFlags(&sh->s_eg, hipStreamNonBlocking));
    sl = sh->s_lz;
    se = sh->s_eg;
  }
  // s waits for e, recorded on `on` (nothing to wait for on the same stream)
  auto wait = [](hipStream_t s, hipEvent_t e, hipStream_t on) { return s == on ? hipSuccess : hipStreamWaitEvent(s, e, 0); };
  HIPCHK(ctx, sh->tok.ensure(P.tok_len));
  HIPCHK(ctx, sh->bits.ensure((E + 31) / 32 + 1));
  if (tsum_on()) HIPCHK(ctx, sh->tsum.ensure((E + EAGER_TILE - 1) / EAGER_TILE * 4 + 4));
  HIPCHK(ctx, sh->defer.ensure(DEFER_CAP));
  HIPCHK(ctx, sh->xq.ensure(2 * XQ_CAP_MAX));
  HIPCHK(ctx, zero_u_pad(sh, sa));
  unsigned long long *c = sh->ctr.p;
  {
    // ctr[0, CTR_RUN_WORDS) in one copy: k_eager's counters [0, 6) (first-unknown [2] = ~0), the
    // step tail's FindRecordStart best [8] = ~0 and chain-proof counters [16, 20) = {0, ~0, 0, ~0},
    // k_first_bad's [100] = ~0; the rest (per-call regions) zero
    unsigned long long *tpl = sh->h_ctr + 1024;  // pinned
    std::memset(tpl, 0, CTR_RUN_WORDS * 8);
    tpl[2] = tpl[8] = tpl[17] = tpl[19] = tpl[100] = ~0ull;
    HIPCHK(ctx, set_words(reinterpret_cast<uint64_t *>(c), reinterpret_cast<const uint64_t *>(tpl), CTR_RUN_WORDS, sa));
  }
  sh->inflated = sh->bits_valid = sh->chain_ok = sh->cm_valid = false;
  sh->sieve_nref1 = 0;
  uint32_t *sv = sieve_for(sh);
  const uint32_t nref1 = (uint32_t)sh->nctg + 1;
  sh->pipe_fallback = false;
  const uint64_t nbat = P.batches.size();
  // events: per batch [huff start, huff end, lz start, lz end, eager start, eager end]
  for (size_t i = 0; i < 6 * nbat + 4; ++i)
    if (!pev(sh, i)) return fail(ctx, SBH_E_HIP, "hipEventCreate failed");
  hipEvent_t *ev = sh->pev.data();
  HIPCHK(ctx, hipEventRecord(ev[6 * nbat], sa));  // setup done: the other streams start after it
  HIPCHK(ctx, wait(sl, ev[6 * nbat], sa));
  HIPCHK(ctx, wait(se, ev[6 * nbat], sa));
  const DevBlocks all = sh->dev_blocks();
  uint64_t e_done = 0;
  std::vector<int> eager_launched(nbat, 0);
  for (uint64_t i = 0; i < nbat; ++i) {
    const uint64_t b0 = P.batches[i].first, b1 = P.batches[i].second;
    hipEvent_t *e = ev + 6 * i;
    const DevBlocks d = blocks_from(all, b0);
    const uint64_t base = P.reuse ? sh->hb[b0].ustart : 0;
    // a reused token buffer: this batch's k_huff overwrites what the previous k_lz reads
    if (P.reuse && i) HIPCHK(ctx, wait(sa, ev[6 * (i - 1) + 3], sl));
    HIPCHK(ctx, hipEventRecord(e[0], sa));
    HIPCHK(ctx, launch_huff(sh->comp.p, d, b1 - b0, sh->tok.p, base, sa));
    HIPCHK(ctx, hipEventRecord(e[1], sa));
    HIPCHK(ctx, wait(sl, e[1], sa));
    HIPCHK(ctx, hipEventRecord(e[2], sl));
    HIPCHK(ctx, launch_lz(sh->comp.p, d, b1 - b0, sh->tok.p, base, sh->U.p, sl, sv, nref1));
    HIPCHK(ctx, hipEventRecord(e[3], sl));
    // eager tiles whose staged windows lie below the inflated frontier
    const bool last = i + 1 == nbat;
    const uint64_t front = last ? ~0ull : sh->hb[b1].ustart;
    uint64_t hi = E;
    if (!last) {
      hi = front + EAGER_TILE >= EAGER_REACH ? (front + EAGER_TILE - EAGER_REACH) / EAGER_TILE * EAGER_TILE : 0;
      hi = std::min(hi, E);
    }
    if (hi > e_done) {
      HIPCHK(ctx, wait(se, e[3], sl));
      HIPCHK(ctx, hipEventRecord(e[4], se));
      HIPCHK(ctx, launch_eager(sh->U.p, sh->utotal + sh->pad, e_done, hi, sh->d_seg.p, (uint32_t)sh->seg_end.size(),
                               sh->open_last ? 1 : 0, sh->ctg.p, sh->nctg, rtc, sh->bits.p + e_done / 32, c, se,
                               front, sh->defer.p, DEFER_CAP, sh->xq.p, xq_cap(),
                               tsum_on() ? sh->tsum.p + e_done / EAGER_SUB : nullptr, sv));
      HIPCHK(ctx, hipEventRecord(e[5], se));
      eager_launched[i] = 1;
      e_done = hi;
    }
  }
  HIPCHK(ctx, wait(se, ev[6 * (nbat - 1) + 3], sl));
  HIPCHK(ctx, launch_eager_defer(sh->U.p, 0, sh->d_seg.p, (uint32_t)sh->seg_end.size(), sh->open_last ? 1 : 0,
                                 sh->ctg.p, sh->nctg, rtc, sh->bits.p, c, sh->defer.p, DEFER_CAP, se));
  HIPCHK(ctx, hipEventRecord(ev[6 * nbat + 2], se));
  HIPCHK(ctx, launch_eager_xq(sh->U.p, 0, sh->d_seg.p, (uint32_t)sh->seg_end.size(), sh->open_last ? 1 : 0,
                              sh->ctg.p, sh->nctg, rtc, sh->bits.p, c, sh->xq.p, xq_cap(), se));
  HIPCHK(ctx, hipEventRecord(ev[6 * nbat + 3], se));
  HIPCHK(ctx, hipEventRecord(ev[6 * nbat + 1], se));
  HIPCHK(ctx, wait(sa, ev[6 * nbat + 1], se));
  if (pre_sync) HIPCHK(ctx, pre_sync(sa));
  {
    const int rs = inflate_status(sh, sa, nullptr, nullptr, nullptr, 0, true);
    if (rs) return rs;
  }
  sh->inflated = true;
  sh->sieve_nref1 = sv ? nref1 : 0;
  if (sh->timing) {
    double hs = 0, ls = 0, es = 0;
    for (uint64_t i = 0; i < nbat; ++i) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, ev[6 * i], ev[6 * i + 1]) == hipSuccess) hs += ms;
      if (hipEventElapsedTime(&ms, ev[6 * i + 2], ev[6 * i + 3]) == hipSuccess) ls += ms;
      if (eager_launched[i] && hipEventElapsedTime(&ms, ev[6 * i + 4], ev[6 * i + 5]) == hipSuccess) es += ms;
    }
    sh->pipe_ms[0] = hs;
    sh->pipe_ms[1] = ls;
    float xs = 0;
    if (hipEventElapsedTime(&xs, ev[6 * nbat + 2], ev[6 * nbat + 3]) == hipSuccess) es += xs;  // k_eager_xq
    sh->pipe_ms[2] = es;
  }
  if (std::getenv("SBH_XQ_DEBUG"))
    fprintf(stderr, "[sbh] eager: deferred %llu, long-record queue %llu (%llu past the pre-test)\n", sh->h_ctr[3],
            sh->h_ctr[4], sh->h_ctr[5]);
  if (sh->h_ctr[3] > DEFER_CAP) {  // deferral overflow: plain pass
    sh->pipe_fallback = true;
    return eager_range(sh, 0, E, rtc, n_true);
  }
  sh->bits_valid = true;
  sh->bits_begin = 0;
  sh->bits_end = E;
  sh->bits_rtc = rtc;
  if (n_true) *n_true = sh->h_ctr[0];
  if (sh->h_ctr[1]) {
    sh->bits_valid = false;
    return fail(ctx, SBH_E_NEED_HALO, "%llu positions (first %llu) need bytes past the shard", sh->h_ctr[1],
                sh->h_ctr[2]);
  }
  return SBH_OK;
}

int sbh_run_shard(sbh_shard *sh, uint64_t index_start, uint64_t own_end_file, int32_t rtc, int32_t mrs,
                  sbh_shard_result *res) {
  if (!sh || !res) return SBH_E_ARG;
  std::memset(res, 0, sizeof *res);
  sbh_ctx *ctx = sh->ctx;
  (void)hipGetLastError();
  sh->timing = true;
  mark(sh, 0);
  int rc = sbh_index(sh, index_start, &res->n_blocks, nullptr);
  mark(sh, 1);
  if (rc) { sh->timing = false; return res->status = rc; }
  uint64_t E = 0;
  (void)sbh_flat_bound(sh, own_end_file, &E);
  if (!sh->at_eof && E == sh->utotal) {
    sh->timing = false;
    return res->status = fail(ctx, SBH_E_NEED_HALO, "no halo past %llu", (unsigned long long)own_end_file);
  }
  // the blocks starting before own_end_file (the chain is contiguous: each block starts where
  // the one before it ends, so their bytes are one span)
  const uint64_t owned_blocks = (uint64_t)(std::lower_bound(sh->hb.begin(), sh->hb.end(), own_end_file,
                                                           [](const sbh_block &b, uint64_t v) { return b.start < v; }) -
                                           sh->hb.begin());
  const uint64_t cbytes =
      owned_blocks ? sh->hb[owned_blocks - 1].start + sh->hb[owned_blocks - 1].csize - sh->hb[0].start : 0;
  res->n_blocks = owned_blocks;
  res->comp_bytes = cbytes;
  res->flat_bytes = E;
  mark(sh, 2);
  // The step's tail rides in the inflate-status round trip: FindRecordStart from flat 0 (the
  // first set bit of the verified bitmap below min(segment end, maxReadSize, E)) and the chain
  // proof from that record, which k_verify_chain_w reads from the device.  The answers are taken
  // when the record lies in the first segment and the bitmap is exactly the chain; anything else
  // (no bit found, an anomaly, a fallback inside run_pipelined) goes the long way below, as
  // sbh_find_record_start and count_records_impl would on their own.
  const uint64_t total0 = sh->seg_end.empty() ? 0 : sh->seg_end[0];
  const uint64_t hi0 = std::min(std::min<uint64_t>(total0, (uint64_t)std::max(mrs, 0)), E);
  const uint64_t E0 = std::min(E, total0);
  unsigned long long *tbest = sh->ctr.p + 8, *tc = sh->ctr.p + 16;
  bool tail = rtc >= 0 && hi0 > 0;
  if (tail && sh->cc.ensure((E + 31) / 32 / VC_CHUNK + 2) != hipSuccess) tail = false;
  // (tbest and tc start as run_pipelined's counter template sets them, and come back to h_ctr[8]
  // and h_ctr[16, 20) with its one status copy)
  auto tail_launch = [&](hipStream_t s) -> hipError_t {
    hipError_t e = launch_first_set(sh->bits.p, 0, 0, hi0, tbest, s);
    if (e == hipSuccess)
      e = launch_verify_chain_count(sh->U.p, sh->bits.p, 0, E, 0, E0, total0, tc, tc + 1, tc + 3, tc + 2, nullptr, s,
                                    tbest, sh->cc.p);
    return e;
  };
  rc = tail ? run_pipelined(sh, E, rtc, &res->n_true, tail_launch) : run_pipelined(sh, E, rtc, &res->n_true);
  mark(sh, 5);
  if (rc) { sh->timing = false; return res->status = rc; }
  // (a deferral overflow re-ran the eager pass inside run_pipelined: the bitmap is new)
  tail = tail && sh->bits_valid && sh->bits_begin == 0 && sh->bits_end == E && sh->bits_rtc == rtc &&
         !sh->pipe_fallback;
  uint64_t first = 0;
  int32_t delta = 0;
  sh->run_first = ~0ull;
  if (tail && sh->h_ctr[8] != ~0ull) {
    first = sh->h_ctr[8];
    sh->run_first = first;
    rc = SBH_OK;
    if (first < E0 && sh->h_ctr[16] == 0 && sh->h_ctr[19] != ~0ull) {  // count_records_impl's proof, done
      sh->cm_valid = false;
      sh->chain_ok = true;
      sh->cc_ok = true;
      sh->chain_first = first;
      sh->chain_E = E0;
      res->count = sh->h_ctr[18];
      res->anomalies = 0;
      res->exit_flat = sh->h_ctr[19];
    } else {
      // (the tail's proof covered [first, E0) of this bitmap: its counters are reused when first
      // lies in the first segment, which is the range count_records_impl proves)
      rc = count_records_impl(sh, first, E, &res->count, &res->anomalies, &res->exit_flat, first < E0);
    }
    uint64_t bp = 0;
    uint32_t off = 0;
    if (!rc && sbh_pos_of(sh, first, &bp, &off) == SBH_OK) res->first_vpos = (bp << 16) | off;
  } else {
    rc = sbh_find_record_start(sh, 0, rtc, mrs, &first, &delta);
    if (rc == SBH_E_NO_READ_FOUND) {
      res->count = 0;
      rc = SBH_OK;
    } else if (rc == SBH_OK) {
      sh->run_first = first;
      rc = count_records_impl(sh, first, E, &res->count, &res->anomalies, &res->exit_flat);
      uint64_t bp = 0;
      uint32_t off = 0;
      if (!rc && sbh_pos_of(sh, first, &bp, &off) == SBH_OK) res->first_vpos = (bp << 16) | off;
    }
  }
  if (res->count == 0) res->exit_flat = E;
  mark(sh, 6);
  sh->timing = false;
  if (sh->ev_ok) {
    (void)hipEventSynchronize(sh->ev[6]);
    // [index, inflate + eager pipeline, eager (sum of launches), split/count, k_huff, k_lz]
    const int from[2] = {0, 5}, to[2] = {1, 6};
    for (int i = 0; i < 2; ++i) {
      float ms = 0;
      (void)hipEventElapsedTime(&ms, sh->ev[from[i]], sh->ev[to[i]]);
      sh->stage_ms[i == 0 ? 0 : 3] = ms;
    }
    float ms = 0;
    (void)hipEventElapsedTime(&ms, sh->ev[2], sh->ev[5]);
    sh->stage_ms[1] = ms;
    sh->stage_ms[2] = sh->pipe_ms[2];
    sh->stage_ms[4] = sh->pipe_ms[0];
    sh->stage_ms[5] = sh->pipe_ms[1];
  }
  return res->status = rc;
}

int sbh_stage_times(sbh_shard *sh, double *ms, int32_t cap) {
  if (!sh || !ms || cap < 0) return 0;
  int n = cap < 6 ? cap : 6;
  for (int i = 0; i < n; ++i) ms[i] = sh->stage_ms[i];
  return n;
}

// A shard larger than the HBM budget, streamed through it (Stream.scala:80-122 and
// SplitRDD.scala:33-52 bound the reference's memory the same way: per split, a bounded
// block cache).  The owned range [index_start, own_end_file) is cut into windows of about
// `window` compressed bytes; window w owns the blocks starting in [lo_w, hi_w) and loads
// [lo_w, hi_w + halo).  While window w runs the whole per-shard path (sbh_run_shard), the
// bytes of window w+1 move host -> HBM on a copy stream into the other of two buffers, so
// HBM holds two windows of compressed bytes and one window's flat bytes, tokens and bitmap,
// whatever the shard size.  Window w+1 indexes from the first block at/after hi_w (known
// from window w's block table).  Consecutive non-empty windows stitch like ranks (SURVEY
// 8e): the chain leaving window w must enter window w+1 at its first record, else window
// w+1 is re-walked from that exit.  A result that needs bytes past a window's halo grows
// the halo x4 and redoes the window.
int sbh_run_stream(sbh_ctx *ctx, const void *host, uint64_t n, uint64_t file_offset, uint64_t file_size,
                   uint64_t index_start, uint64_t own_end_file, uint64_t window, uint64_t halo, const int32_t *contigs,
                   int32_t n_contigs, int32_t rtc, int32_t mrs, uint8_t *out_bits, uint64_t out_bits_cap,
                   sbh_stream_result *res) {
  sbh_stream_opts o{};
  o.window = window;
  o.halo = halo;
  o.reads_to_check = rtc;
  o.max_read_size = mrs;
  o.bgzf_blocks_to_check = 5;
  o.out_bits = out_bits;
  o.out_bits_cap = out_bits_cap;
  return sbh_run_stream2(ctx, host, n, file_offset, file_size, index_start, own_end_file, contigs, n_contigs, &o, res);
}

// CRC32 of the first nb blocks of the table (a window's owned blocks) against their footers.
static int verify_crc_prefix(sbh_shard *sh, uint64_t nb, uint64_t *n_bad, uint64_t *first_bad, float *ms) {
  sbh_ctx *ctx = sh->ctx;
  hipStream_t st = sh->st;
  unsigned long long *c = sh->ctr.p + 32;
  HIPCHK(ctx, hipMemsetAsync(c, 0, 8, st));
  HIPCHK(ctx, hipMemsetAsync(c + 1, 0xff, 8, st));
  mark(sh, 7);
  HIPCHK(ctx, launch_block_crc(sh->comp.p, sh->dev_blocks(), nb, sh->U.p, c, c + 1, st));
  mark(sh, 8);
  HIPCHK(ctx, hipMemcpyAsync(sh->h_ctr + 32, c, 16, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipStreamSynchronize(st));
  *n_bad = sh->h_ctr[32];
  *first_bad = sh->h_ctr[32] ? sh->hb[sh->h_ctr[33]].start : 0;
  *ms = 0.f;
  if (sh->ev_ok) (void)hipEventElapsedTime(ms, sh->ev[7], sh->ev[8]);
  return SBH_OK;
}

int sbh_run_stream2(sbh_ctx *ctx, const void *host, uint64_t n, uint64_t file_offset, uint64_t file_size,
                    uint64_t index_start, uint64_t own_end_file, const int32_t *contigs, int32_t n_contigs,
                    const sbh_stream_opts *opts, sbh_stream_result *res) {
  if (!ctx || !res || !opts || (!host && n) || !opts->window || file_offset + n > file_size ||
      own_end_file > file_offset + n || own_end_file <= file_offset || n_contigs < 0 || (n_contigs && !contigs))
    return SBH_E_ARG;
  const sbh_stream_opts &O = *opts;
  const uint64_t window = O.window;
  uint64_t halo = O.halo;
  const int32_t rtc = O.reads_to_check, mrs = O.max_read_size, kcheck = O.bgzf_blocks_to_check;
  uint8_t *out_bits = O.out_bits;
  const uint64_t out_bits_cap = O.out_bits_cap, ns = O.n_splits;
  std::memset(res, 0, sizeof *res);
  res->first_vpos = res->exit_vpos = ~0ull;
  if (ns) {  // splits: sorted, disjoint, inside the owned range, with their outputs
    if (!O.split_start || !O.split_end || !O.split_first_vpos || !O.split_count || !O.split_status)
      return fail(ctx, SBH_E_ARG, "run_stream2: split arrays missing");
    for (uint64_t i = 0; i < ns; ++i) {
      const uint64_t a = O.split_start[i], e = O.split_end[i];
      if (a < file_offset || a >= own_end_file || e <= a || e > own_end_file || (i + 1 < ns && e > O.split_start[i + 1]))
        return fail(ctx, SBH_E_ARG, "run_stream2: split %llu [%llu, %llu) out of order or outside [%llu, %llu)",
                    (unsigned long long)i, (unsigned long long)a, (unsigned long long)e,
                    (unsigned long long)file_offset, (unsigned long long)own_end_file);
      O.split_first_vpos[i] = O.split_count[i] = 0;
      O.split_status[i] = SBH_OK;
    }
  }
  const auto t_start = std::chrono::steady_clock::now();
  int rc = set_device(ctx);
  if (rc) return res->status = rc;
  const uint8_t *src = static_cast<const uint8_t *>(host);
  hipPointerAttribute_t pa{};
  res->host_pinned = hipPointerGetAttributes(&pa, host) == hipSuccess && pa.type == hipMemoryTypeHost ? 1 : 0;
  (void)hipGetLastError();
  // the window shard, the two window buffers and the copy stream persist in the context (grow-only),
  // so repeated calls allocate nothing; concurrent callers each take their own cache from the pool
  StreamCache *scp = nullptr;
  {
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (!ctx->sc_free.empty()) {
      scp = ctx->sc_free.back();
      ctx->sc_free.pop_back();
    }
  }
  if (!scp) {
    scp = new StreamCache();
    rc = sbh_shard_create(ctx, nullptr, 0, file_offset, file_size, 0, &scp->sh);
    if (rc) {
      delete scp;
      return res->status = rc;
    }
    scp->sh->comp.release();
    // the copy stream at another priority than the compute streams: its hardware queue then comes
    // from another pool, so no compute stream shares it (a copy in flight on a shared queue held
    // the next window's kernels behind it: e2e 130 -> 84 GB/s depending on stream creation order)
    int least = 0, greatest = 0;
    hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
    if (e == hipSuccess)
      e = greatest != least && !std::getenv("SBH_CS_SAME_PRIORITY")
              ? hipStreamCreateWithPriority(&scp->cs, hipStreamNonBlocking, greatest)
              : hipStreamCreateWithFlags(&scp->cs, hipStreamNonBlocking);
    for (int i = 0; i < 2 && e == hipSuccess; ++i) {
      e = hipEventCreate(&scp->done[i]);
      if (e == hipSuccess) e = hipEventCreate(&scp->c0[i]);
    }
    if (e != hipSuccess) {
      stream_cache_free(scp);
      return res->status = fail(ctx, SBH_E_HIP, "run_stream2: %s", hipGetErrorString(e));
    }
  }
  struct Return {  // the cache goes back to the pool on every return path
    sbh_ctx *ctx;
    StreamCache *sc;
    ~Return() {
      std::lock_guard<std::mutex> lk(ctx->mu);
      ctx->sc_free.push_back(sc);
    }
  } give_back{ctx, scp};
  StreamCache &R = *scp;
  struct Detach {  // the window buffers are never the shard's own: detach on every return path
    StreamCache &R;
    ~Detach() {
      if (R.cs) (void)hipStreamSynchronize(R.cs);
      R.sh->comp.p = nullptr;
      R.sh->comp.cap = 0;
    }
  } detach{R};
  sbh_shard *sh = R.sh;
  sh->file_size = file_size;
  rc = sbh_set_contigs(sh, contigs, n_contigs);
  if (rc) return res->status = rc;
  const uint64_t data_end = file_offset + n, pad = sh->pad;
  // the first window is short: its copy is the only one no kernel overlaps
  const uint64_t first_window = std::max<uint64_t>(std::min<uint64_t>(window, 64ull << 20), window / 8);
  // window ends: the last split start in (lo, lo + window] when splits are given, so a split
  // lies in one window unless it is longer than a window; such a split is cut at lo + window and
  // its chain followed window by window (the straddling split below), so HBM stays bounded
  // whatever the split size (one split per rank included)
  auto win_end = [&](uint64_t lo) {
    const uint64_t want = lo + (lo == file_offset ? first_window : window);
    uint64_t hi = std::min(want, own_end_file);
    if (own_end_file - hi < window / 4) hi = own_end_file;  // no sliver of a last window
    if (ns && hi < own_end_file) {
      const uint64_t *S = O.split_start;
      const uint64_t k = (uint64_t)(std::upper_bound(S, S + ns, hi) - S);  // starts <= hi: [0, k)
      if (k > 0 && S[k - 1] > lo) hi = S[k - 1];
    }
    return hi;
  };
  // the split that runs past its first window: its index, and the htsjdk vpos of the next record
  // of its own chain (from its first record, CanLoadBam.scala:338-355) not yet counted
  int64_t strad = -1;
  uint64_t strad_cur = 0;
  auto load_end = [&](uint64_t hi) { return std::min(hi + halo, data_end); };
  auto size_bufs = [&]() -> hipError_t {  // (enqueue grows a buffer for a longer split-aligned window)
    const uint64_t cap = window + window / 4 + halo + pad;
    for (auto &b : R.buf) {
      hipError_t e = b.ensure(cap);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  };
  auto fit_buf = [&](int b, uint64_t need) -> hipError_t {  // grow buffer b (not in use) to `need` bytes
    hipError_t e = hipStreamSynchronize(R.cs);
    if (e == hipSuccess) e = hipStreamSynchronize(sh->st);
    if (e == hipSuccess) e = R.buf[b].ensure(need);
    return e;
  };
  double h2d_ms = 0;
  bool timed[2] = {false, false};
  auto account = [&](int b) {  // copy time of the last copy into buffer b
    if (!timed[b]) return;
    float ms = 0;
    if (hipEventElapsedTime(&ms, R.c0[b], R.done[b]) == hipSuccess) h2d_ms += ms;
    timed[b] = false;
  };
  uint64_t win_len[2] = {0, 0};  // bytes copied into each window buffer
  auto enqueue = [&](int b, uint64_t lo, uint64_t ld) -> hipError_t {
    hipError_t e = hipSuccess;
    if (R.buf[b].cap < ld - lo + pad) {  // an oversized (split-aligned) window
      e = fit_buf(b, ld - lo + pad);
      if (e != hipSuccess) return e;
    }
    // (the copy stream carries the copy alone: the window's zero pad is set on the shard's stream
    // after it waits for the copy -- a fill queued behind the copy on the copy stream would be a
    // kernel waiting on the DMA, and a hardware queue the copy stream shares with a compute
    // stream would hold that stream's kernels behind it)
    e = hipEventRecord(R.c0[b], R.cs);
    if (e == hipSuccess) e = hipMemcpyAsync(R.buf[b].p, src + (lo - file_offset), ld - lo, hipMemcpyHostToDevice, R.cs);
    if (e == hipSuccess) e = hipEventRecord(R.done[b], R.cs);
    win_len[b] = ld - lo;
    timed[b] = e == hipSuccess;
    return e;
  };
  HIPCHK(ctx, size_bufs());
  uint64_t lo = file_offset, hi = win_end(lo), start = index_start;
  int cur = 0;
  HIPCHK(ctx, enqueue(cur, lo, load_end(hi)));
  bool prefetch = true, have_prev = false;
  uint64_t prev_exit = ~0ull, flat_base = 0;
  std::vector<uint32_t> wbits;
  for (;;) {
    const bool more = hi < own_end_file;
    const uint64_t lo2 = hi, hi2 = more ? win_end(lo2) : 0;
    if (prefetch && more) HIPCHK(ctx, enqueue(1 - cur, lo2, load_end(hi2)));
    const uint64_t ld = load_end(hi);
    HIPCHK(ctx, hipStreamWaitEvent(sh->st, R.done[cur], 0));
    HIPCHK(ctx, hipMemsetAsync(R.buf[cur].p + win_len[cur], 0, pad, sh->st));
    sh->comp.p = R.buf[cur].p;
    sh->comp.cap = R.buf[cur].cap;
    sh->file_off = lo;
    sh->n = ld - lo;
    sh->at_eof = ld == file_size;
    if (start == ~0ull) {
      rc = sbh_find_block_start(sh, lo, kcheck, &start);  // BGZFBlocksToCheck (bgzf/.../block/package.scala:20)
      if (rc) return res->status = rc;
    }
    sbh_shard_result r{};
    sh->scan_from = lo;  // header candidates from the window's first byte (its first split's FindBlockStart)
    rc = sbh_run_shard(sh, start, hi, rtc, mrs, &r);
    // this window's splits (every one starting in [lo, hi)): the batched per-split path for the
    // ones that end by hi; the last one may run past hi (a split longer than the window)
    uint64_t k0 = 0, k1 = 0, nh = 0;
    double split_ms = 0;
    // the straddling split's progress in this window, committed once the window holds
    int64_t s_idx = strad;
    uint64_t s_cur = strad_cur, s_add = 0, s_first = 0;
    int32_t s_status = SBH_OK;
    bool s_new = false, s_done = false;
    if (!rc && ns) {
      const auto ts0 = std::chrono::steady_clock::now();
      k0 = (uint64_t)(std::lower_bound(O.split_start, O.split_start + ns, lo) - O.split_start);
      k1 = (uint64_t)(std::lower_bound(O.split_start, O.split_start + ns, hi) - O.split_start);
      const bool straddles = k1 > k0 && O.split_end[k1 - 1] > hi;
      const uint64_t kb = straddles ? k1 - 1 : k1;
      if (kb > k0) {
        rc = sbh_split_starts(sh, O.split_start + k0, O.split_end + k0, kb - k0, kcheck, rtc, mrs,
                              O.split_first_vpos + k0, O.split_count + k0, O.split_status + k0, &nh);
        if (!rc)
          for (uint64_t i = k0; i < kb; ++i)
            if (O.split_status[i] == SBH_E_NEED_HALO) rc = SBH_E_NEED_HALO;
      }
      uint64_t E_hi = 0;
      if (!rc) rc = sbh_flat_bound(sh, hi, &E_hi);
      // follow a chain from flat f while its records start before min(Pos(split end, 0), Pos(hi, 0))
      auto follow = [&](uint64_t f, uint64_t split_end) -> int {
        uint64_t E_end = 0, n = 0, x = 0, bp = 0;
        uint32_t off = 0;
        int r = sbh_flat_bound(sh, split_end, &E_end);
        if (!r) r = sbh_chain_from(sh, f, std::min(E_end, E_hi), &n, &x);
        if (!r && x >= sh->utotal && !sh->at_eof) r = SBH_E_NEED_HALO;  // its next record is past the halo
        if (!r) r = sbh_pos_of(sh, x, &bp, &off);
        if (r) return r;
        s_add += n;
        s_cur = bp << 16 | off;
        s_done = E_end <= E_hi || s_cur >= (split_end << 16);
        return SBH_OK;
      };
      if (!rc && s_idx >= 0 && (s_cur >> 16) < hi) {  // a split from an earlier window goes on here
        uint64_t f = 0;
        rc = sbh_flat_of(sh, s_cur >> 16, (uint32_t)(s_cur & 0xffff), &f);
        if (!rc) rc = follow(f, O.split_end[s_idx]);
      }
      if (!rc && straddles) {  // FindBlockStart + FindRecordStart here, then its chain to hi
        const uint64_t a = O.split_start[k1 - 1], e = O.split_end[k1 - 1];
        uint64_t fbs = 0, f0 = 0, first = 0, bp = 0;
        uint32_t off = 0;
        int32_t delta = 0;
        s_idx = (int64_t)(k1 - 1), s_new = true, s_add = 0;
        rc = sbh_find_block_start(sh, a, kcheck, &fbs);
        if (!rc) rc = sbh_flat_of(sh, fbs, 0, &f0);
        if (!rc) rc = sbh_find_record_start(sh, f0, rtc, mrs, &first, &delta);
        if (!rc) rc = sbh_pos_of(sh, first, &bp, &off);
        if (rc == SBH_E_NO_READ_FOUND || rc == SBH_E_HEADER_SEARCH_FAILED) {
          s_status = rc, s_done = true, rc = SBH_OK;
        } else if (!rc) {
          s_first = bp << 16 | off;
          s_cur = s_first;
          if (s_first >= (e << 16)) s_done = true;
          else rc = follow(first, e);
        }
      }
      split_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ts0).count();
    }
    if (rc == SBH_E_NEED_HALO && ld < data_end) {  // grow the halo and redo this window
      HIPCHK(ctx, hipStreamSynchronize(R.cs));
      HIPCHK(ctx, hipStreamSynchronize(sh->st));
      account(0);
      account(1);
      halo *= 4;
      for (auto &b : R.buf) b.release();
      sh->comp.p = nullptr;
      sh->comp.cap = 0;
      HIPCHK(ctx, size_bufs());
      HIPCHK(ctx, enqueue(cur, lo, load_end(hi)));
      prefetch = true;
      continue;
    }
    if (rc) return res->status = rc;
    if (s_idx >= 0) {  // commit the straddling split's progress
      if (s_new) {
        O.split_status[s_idx] = s_status;
        O.split_first_vpos[s_idx] = s_first;
        O.split_count[s_idx] = 0;
      }
      O.split_count[s_idx] += s_add;
      strad = s_done ? -1 : s_idx;
      strad_cur = s_cur;
    }
    res->ms_splits += split_ms;
    res->splits_host += nh;  // (a window redone with a larger halo counts its final attempt only)
    account(cur);
    if (O.verify_crc && r.n_blocks) {  // the owned blocks are the block table's prefix
      uint64_t nbad = 0, fbad = 0;
      float cms = 0.f;
      const bool was = sh->timing;
      sh->timing = true;
      rc = verify_crc_prefix(sh, std::min<uint64_t>(r.n_blocks, sh->nblocks), &nbad, &fbad, &cms);
      sh->timing = was;
      if (rc) return res->status = rc;
      if (nbad && !res->crc_bad_blocks) res->crc_first_bad = fbad;
      res->crc_bad_blocks += nbad;
      res->ms_crc += cms;
    }
    // this window's chain exit, and the stitch with the previous non-empty window
    uint64_t count = r.count, exit_vpos = ~0ull;
    auto vpos_of = [&](uint64_t flat, uint64_t *v) {
      uint64_t bp = 0;
      uint32_t off = 0;
      if (sbh_pos_of(sh, flat, &bp, &off) != SBH_OK) return false;
      *v = (bp << 16) | off;
      return true;
    };
    if (count) {
      uint64_t first_v = r.first_vpos;
      if (have_prev && prev_exit != ~0ull && first_v != prev_exit) {
        uint64_t f = 0, x = 0, E = 0;
        rc = sbh_flat_of(sh, prev_exit >> 16, (uint32_t)(prev_exit & 0xffff), &f);
        if (!rc) rc = sbh_flat_bound(sh, hi, &E);
        if (!rc) rc = sbh_chain_from(sh, f, E, &count, &x);
        if (rc) return res->status = rc;
        r.exit_flat = x;
        first_v = prev_exit;
        ++res->rewalks;
      }
      if (!vpos_of(r.exit_flat, &exit_vpos)) exit_vpos = ~0ull;
      if (res->first_vpos == ~0ull) res->first_vpos = first_v;
      if (count) {
        prev_exit = exit_vpos;
        have_prev = true;
      }
    }
    if (out_bits && r.flat_bytes) {  // this window's owned bits at global flat offset flat_base
      const uint64_t nb = (flat_base + r.flat_bytes + 7) / 8;
      if (nb > out_bits_cap) return res->status = fail(ctx, SBH_E_ARG, "out_bits_cap too small");
      wbits.assign((r.flat_bytes + 31) / 32 + 1, 0);
      HIPCHK(ctx, hipMemcpyAsync(wbits.data(), sh->bits.p, (r.flat_bytes + 7) / 8, hipMemcpyDeviceToHost, sh->st));
      HIPCHK(ctx, hipStreamSynchronize(sh->st));
      for (uint64_t i = 0; i < r.flat_bytes; ++i)
        if ((wbits[i >> 5] >> (i & 31)) & 1u) out_bits[(flat_base + i) >> 3] |= (uint8_t)(1u << ((flat_base + i) & 7));
    }
    ++res->n_windows;
    res->n_blocks += r.n_blocks;
    res->comp_bytes += r.comp_bytes;
    res->flat_bytes += r.flat_bytes;
    res->n_true += r.n_true;
    res->count += count;
    if (count) res->exit_vpos = exit_vpos;
    for (int i = 0; i < 6; ++i) res->stage_ms[i] += sh->stage_ms[i];
    flat_base += r.flat_bytes;
    if (!more) break;
    // the next window indexes from its first block: the first block at/after hi
    auto it = std::lower_bound(sh->hb.begin(), sh->hb.end(), hi,
                               [](const sbh_block &b, uint64_t v) { return b.start < v; });
    if (it == sh->hb.end()) return res->status = fail(ctx, SBH_E_NEED_HALO, "halo %llu holds no block past %llu",
                                                     (unsigned long long)halo, (unsigned long long)hi);
    start = it->start;
    sh->comp.p = nullptr;
    sh->comp.cap = 0;
    lo = lo2;
    hi = hi2;
    cur = 1 - cur;
    prefetch = true;
  }
  HIPCHK(ctx, hipStreamSynchronize(R.cs));
  account(0);
  account(1);
  res->ms_h2d = h2d_ms;
  res->halo_final = halo;
  res->ms_wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
  return res->status = SBH_OK;
}

// RecordStream + BAMRecordCodec.decode over [first, end) (check/.../iterator/RecordStream.scala:16-41,
// load/.../CanLoadBam.scala:244-264): record starts by the chain, sizes -> prefix offsets,
// then one wave per record decodes into the columns.
int sbh_records_scan(sbh_shard *sh, uint64_t first, uint64_t end_flat, sbh_records_sizes *out) {
  if (!sh || !out) return SBH_E_ARG;
  sbh_ctx *ctx = sh->ctx;
  if (!sh->inflated) return fail(ctx, SBH_E_STATE, "records before inflate");
  if (first > sh->utotal) return SBH_E_ARG;
  int rc = set_device(ctx);
  if (rc) return rc;
  auto &R = sh->rec;
  R.valid = false;
  const uint64_t total = seg_end_of(sh, first);
  const uint64_t E = std::min(std::min(end_flat, sh->utotal), total);
  uint64_t n = 0;
  int32_t anomalies = 0;
  rc = count_records_impl(sh, first, E, &n, &anomalies);
  if (rc) return rc;
  HIPCHK(ctx, R.pos.ensure(n));
  rc = records_positions(sh, first, E, total, n, anomalies, R.pos.p);
  if (rc) return rc;
  return records_finish(sh, n, total, out);
}

// One FileSplit of loadReadsAndPositions (load/.../CanLoadBam.scala:316-356) in one call:
// FindBlockStart(start) (FindBlockStart.scala:8-36), then sbh_run_shard's step from that block --
// MetadataStream + inflate + the eager check at every position of [Pos(blockStart, 0), Pos(end, 0))
// + FindRecordStart from Pos(blockStart, 0) (FindRecordStart.scala:11-30) + the chain proof of the
// records while pos < Pos(end, 0) (RecordStream.takeWhile, :338-355) -- then the record starts (and
// with decode, BAMRecordCodec.decode's columns) for sbh_records_fetch.  The per-split facade
// (jni/Native.scala GpuSplitPartition) made seven calls with a host round trip each.
int sbh_split_records(sbh_shard *sh, uint64_t start, uint64_t end, int32_t k, int32_t rtc, int32_t mrs, int32_t decode,
                      sbh_split_records_result *out) {
  if (!sh || !out || end <= start) return SBH_E_ARG;
  sbh_ctx *ctx = sh->ctx;
  std::memset(out, 0, sizeof *out);
  int rc = set_device(ctx);
  if (rc) return rc;
  auto &R = sh->rec;
  R.valid = R.decoded = false;
  uint64_t b = 0;
  rc = sbh_find_block_start(sh, start, k, &b);
  if (rc) return rc;
  out->block_start = b;
  sbh_shard_result r{};
  rc = sbh_run_shard(sh, b, end, rtc, mrs, &r);
  if (rc) return rc;
  out->n_blocks = sh->nblocks;
  out->flat_size = sh->utotal;
  out->owned_flat = r.flat_bytes;
  out->n_true = r.n_true;
  uint64_t first = sh->run_first;
  if (r.count == 0) {
    // no record of the chain below Pos(end, 0): FindRecordStart's own answer decides between an
    // empty split and NoReadFoundException(path, blockStart, maxReadSize)
    int32_t delta = 0;
    rc = sbh_find_record_start(sh, 0, rtc, mrs, &first, &delta);
    if (rc == SBH_E_NO_READ_FOUND)
      return fail_with(ctx, SBH_E_NO_READ_FOUND, {(int64_t)b, mrs},
                       "Failed to find a valid read-start in %d attempts from %llu", mrs, (unsigned long long)b);
    if (rc) return rc;
    out->first_flat = first;
    R.sz = sbh_records_sizes{0, 0, 0, 0, 0};
    R.valid = true;
    R.decoded = decode != 0;
    return SBH_OK;
  }
  out->first_flat = first;
  out->first_vpos = r.first_vpos;
  const uint64_t total = seg_end_of(sh, first);
  const uint64_t E = std::min(std::min(r.flat_bytes, sh->utotal), total);
  HIPCHK(ctx, R.pos.ensure(r.count));
  rc = records_positions(sh, first, E, total, r.count, r.anomalies, R.pos.p);
  if (rc) return rc;
  if (!decode) {
    HIPCHK(ctx, hipStreamSynchronize(sh->st));
    R.sz = sbh_records_sizes{r.count, 0, 0, 0, 0};
    R.valid = true;
    out->sizes = R.sz;
    return SBH_OK;
  }
  rc = records_finish(sh, r.count, total, &out->sizes);
  // the split's last record runs past the resident bytes: more halo, not a malformed record
  if (rc == SBH_E_BAD_RECORD && !sh->at_eof)
    return fail(ctx, SBH_E_NEED_HALO, "a record of the split runs past the shard");
  return rc;
}

// Record starts of the chain from first while the start is < E, written at pos (cap n).
static int records_positions(sbh_shard *sh, uint64_t first, uint64_t E, uint64_t total, uint64_t n, int32_t anomalies,
                             uint64_t *pos) {
  sbh_ctx *ctx = sh->ctx;
  hipStream_t st = sh->st;
  auto &R = sh->rec;
  const bool covered = sh->bits_valid && sh->bits_begin <= first && E <= sh->bits_end && anomalies == 0;
  if (n && covered) {
    const uint64_t nw = (E - sh->bits_begin + 31) / 32 - (first - sh->bits_begin) / 32;
    HIPCHK(ctx, R.wcnt.ensure(nw + 2));  // (chunk sums + prefix: 2 per 4096 words)
    HIPCHK(ctx, R.wpre.ensure(nw));
    HIPCHK(ctx, sh->tmp.ensure(scan_tmp_words(nw)));
    HIPCHK(ctx, launch_rec_positions_bits(sh->bits.p, sh->bits_begin, first, E, R.wcnt.p, R.wpre.p, sh->tmp.p, pos, st));
  } else if (n && sh->cm_valid && sh->cm_first == first && sh->cm_E == E) {
    // the chain marked by count_records_impl's pointer doubling: compact its nodes
    HIPCHK(ctx, launch_compact_u64(sh->cm_pos.p, sh->cm_mark.p, sh->cm_mpre.p, sh->cm_n, pos, st));
  } else if (n) {
    HIPCHK(ctx, launch_rec_positions_chain(sh->U.p, first, E, total, n, pos, st));
  }
  return SBH_OK;
}

// Sizes -> prefix offsets -> columns for the n record starts in R.pos.
static int records_finish(sbh_shard *sh, uint64_t n, uint64_t total, sbh_records_sizes *out) {
  sbh_ctx *ctx = sh->ctx;
  hipStream_t st = sh->st;
  auto &R = sh->rec;
  // per-record sizes (a trailing zero makes the exclusive scan's last entry the total)
  DBuf<uint64_t> *sz[4] = {&R.nm, &R.cg, &R.sq, &R.ax}, *of[4] = {&R.nmo, &R.cgo, &R.sqo, &R.axo};
  for (int k = 0; k < 4; ++k) {
    HIPCHK(ctx, sz[k]->ensure(n + 1));
    HIPCHK(ctx, of[k]->ensure(n + 1));
    HIPCHK(ctx, hipMemsetAsync(sz[k]->p + n, 0, 8, st));
  }
  unsigned long long *bad = sh->ctr.p + 24;
  HIPCHK(ctx, hipMemsetAsync(bad, 0xff, 8, st));
  HIPCHK(ctx, launch_rec_sizes(sh->U.p, R.pos.p, n, total, R.nm.p, R.cg.p, R.sq.p, R.ax.p, bad, st));
  HIPCHK(ctx, sh->tmp.ensure(scan_tmp_words(n + 1)));
  for (int k = 0; k < 4; ++k) HIPCHK(ctx, scan_exclusive_u64(sz[k]->p, of[k]->p, n + 1, sh->tmp.p, st));
  uint64_t tot[4] = {0, 0, 0, 0};
  for (int k = 0; k < 4; ++k) HIPCHK(ctx, hipMemcpyAsync(&tot[k], of[k]->p + n, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipMemcpyAsync(sh->h_ctr + 24, bad, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipStreamSynchronize(st));
  if (sh->h_ctr[24] != ~0ull) return fail(ctx, SBH_E_BAD_RECORD, "record %llu of the range is malformed",
                                          (unsigned long long)sh->h_ctr[24]);
  HIPCHK(ctx, R.ref_id.ensure(n)); HIPCHK(ctx, R.p0.ensure(n)); HIPCHK(ctx, R.nref.ensure(n));
  HIPCHK(ctx, R.npos.ensure(n)); HIPCHK(ctx, R.tlen.ensure(n)); HIPCHK(ctx, R.flag.ensure(n));
  HIPCHK(ctx, R.bin.ensure(n)); HIPCHK(ctx, R.mapq.ensure(n));
  HIPCHK(ctx, R.names.ensure(tot[0])); HIPCHK(ctx, R.cigar.ensure(tot[1]));
  HIPCHK(ctx, R.seq.ensure(tot[2])); HIPCHK(ctx, R.qual.ensure(tot[2])); HIPCHK(ctx, R.aux.ensure(tot[3]));
  const RecCols cols{R.ref_id.p, R.p0.p, R.nref.p, R.npos.p, R.tlen.p, R.flag.p, R.bin.p, R.mapq.p,
                     R.names.p, R.cigar.p, R.seq.p, R.qual.p, R.aux.p};
  HIPCHK(ctx, launch_rec_fields(sh->U.p, R.pos.p, n, R.nmo.p, R.cgo.p, R.sqo.p, R.axo.p, cols, st));
  HIPCHK(ctx, hipStreamSynchronize(st));
  R.sz = sbh_records_sizes{n, tot[0], tot[1], tot[2], tot[3]};
  R.valid = true;
  R.decoded = true;
  *out = R.sz;
  return SBH_OK;
}

// loadBamIntervals (load/.../CanLoadBam.scala:78-154): for each BAI chunk, the records from
// chunk.start while the start is < chunk.end (records.seek(chunk.start) + takeWhile), then the
// region filter on the device, then the same column decode as sbh_records_scan.
int sbh_records_scan_regions(sbh_shard *sh, const uint64_t *chunk_begin, const uint64_t *chunk_end, uint64_t n_chunks,
                             const int32_t *iv_ref, const int64_t *iv_begin, const int64_t *iv_end, uint32_t n_iv,
                             sbh_records_sizes *out) {
  if (!sh || !out || (n_chunks && (!chunk_begin || !chunk_end)) || (n_iv && (!iv_ref || !iv_begin || !iv_end)))
    return SBH_E_ARG;
  sbh_ctx *ctx = sh->ctx;
  if (!sh->inflated) return fail(ctx, SBH_E_STATE, "records before inflate");
  for (uint32_t k = 0; k < n_iv; ++k) {
    if (iv_begin[k] >= iv_end[k]) return fail(ctx, SBH_E_ARG, "interval %u is empty", k);
    if (k && (iv_ref[k] < iv_ref[k - 1] || (iv_ref[k] == iv_ref[k - 1] && iv_begin[k] < iv_end[k - 1])))
      return fail(ctx, SBH_E_ARG, "intervals must be sorted by (ref, begin) and disjoint");
  }
  int rc = set_device(ctx);
  if (rc) return rc;
  hipStream_t st = sh->st;
  auto &R = sh->rec;
  R.valid = false;
  std::vector<uint64_t> cn(n_chunks, 0), cfirst(n_chunks, 0), cE(n_chunks, 0), ctot(n_chunks, 0);
  std::vector<int32_t> can(n_chunks, 0);
  uint64_t n = 0;
  for (uint64_t c = 0; c < n_chunks; ++c) {
    const uint64_t first = chunk_begin[c];
    if (first > sh->utotal) return fail(ctx, SBH_E_ARG, "chunk %llu starts past the stream", (unsigned long long)c);
    ctot[c] = seg_end_of(sh, first);
    cE[c] = std::min(std::min(chunk_end[c], sh->utotal), ctot[c]);
    cfirst[c] = first;
    if (first < cE[c]) {
      rc = count_records_impl(sh, first, cE[c], &cn[c], &can[c]);
      if (rc) return rc;
    }
    n += cn[c];
  }
  HIPCHK(ctx, R.pos2.ensure(n + 1));
  uint64_t o = 0;
  for (uint64_t c = 0; c < n_chunks; ++c) {
    rc = records_positions(sh, cfirst[c], cE[c], ctot[c], cn[c], can[c], R.pos2.p + o);
    if (rc) return rc;
    o += cn[c];
  }
  HIPCHK(ctx, R.keep.ensure(n + 1));
  HIPCHK(ctx, R.kpre.ensure(n + 1));
  HIPCHK(ctx, R.iv_ref.ensure(n_iv + 1));
  HIPCHK(ctx, R.iv_b.ensure(n_iv + 1));
  HIPCHK(ctx, R.iv_e.ensure(n_iv + 1));
  if (n_iv) {
    HIPCHK(ctx, hipMemcpyAsync(R.iv_ref.p, iv_ref, 4ull * n_iv, hipMemcpyHostToDevice, st));
    HIPCHK(ctx, hipMemcpyAsync(R.iv_b.p, iv_begin, 8ull * n_iv, hipMemcpyHostToDevice, st));
    HIPCHK(ctx, hipMemcpyAsync(R.iv_e.p, iv_end, 8ull * n_iv, hipMemcpyHostToDevice, st));
  }
  HIPCHK(ctx, hipMemsetAsync(R.keep.p + n, 0, 8, st));
  HIPCHK(ctx, launch_region_keep(sh->U.p, R.pos2.p, n, sh->utotal, R.iv_ref.p, R.iv_b.p, R.iv_e.p, n_iv, R.keep.p, st));
  HIPCHK(ctx, sh->tmp.ensure(scan_tmp_words(n + 1)));
  HIPCHK(ctx, scan_exclusive_u64(R.keep.p, R.kpre.p, n + 1, sh->tmp.p, st));
  uint64_t kept = 0;
  HIPCHK(ctx, hipMemcpyAsync(&kept, R.kpre.p + n, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipStreamSynchronize(st));
  HIPCHK(ctx, R.pos.ensure(kept + 1));
  HIPCHK(ctx, launch_compact_u64(R.pos2.p, R.keep.p, R.kpre.p, n, R.pos.p, st));
  return records_finish(sh, kept, sh->utotal, out);
}

int sbh_records_fetch(sbh_shard *sh, const sbh_records_out *o) {
  if (!sh || !o) return SBH_E_ARG;
  sbh_ctx *ctx = sh->ctx;
  auto &R = sh->rec;
  if (!R.valid) return fail(ctx, SBH_E_STATE, "records_fetch without a records_scan");
  if (!R.decoded && (o->ref_id || o->pos || o->next_ref_id || o->next_pos || o->tlen || o->flag || o->bin || o->mapq ||
                     o->name_off || o->cigar_off || o->seq_off || o->aux_off || o->names || o->cigar || o->seq ||
                     o->qual || o->aux))
    return fail(ctx, SBH_E_STATE, "records_fetch: only the starts were scanned (sbh_split_records, decode = 0)");
  int rc = set_device(ctx);
  if (rc) return rc;
  const uint64_t n = R.sz.n;
  if (o->vpos && n) {  // the starts' virtual positions, computed on the device from the block table
    HIPCHK(ctx, R.vpos.ensure(n));
    HIPCHK(ctx, launch_rec_vpos(R.pos.p, n, sh->dev_blocks(), sh->nblocks, sh->file_off, R.vpos.p, sh->st));
    HIPCHK(ctx, hipMemcpyAsync(o->vpos, R.vpos.p, 8 * n, hipMemcpyDeviceToHost, sh->st));
  }
  // (every column is copied on the shard's stream, then one wait)
  auto cp = [&](void *dst, const void *src, uint64_t bytes) -> hipError_t {
    return dst && bytes ? hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, sh->st) : hipSuccess;
  };
  HIPCHK(ctx, cp(o->flat, R.pos.p, 8 * n));
  HIPCHK(ctx, cp(o->ref_id, R.ref_id.p, 4 * n));
  HIPCHK(ctx, cp(o->pos, R.p0.p, 4 * n));
  HIPCHK(ctx, cp(o->next_ref_id, R.nref.p, 4 * n));
  HIPCHK(ctx, cp(o->next_pos, R.npos.p, 4 * n));
  HIPCHK(ctx, cp(o->tlen, R.tlen.p, 4 * n));
  HIPCHK(ctx, cp(o->flag, R.flag.p, 2 * n));
  HIPCHK(ctx, cp(o->bin, R.bin.p, 2 * n));
  HIPCHK(ctx, cp(o->mapq, R.mapq.p, n));
  HIPCHK(ctx, cp(o->name_off, R.nmo.p, 8 * (n + 1)));
  HIPCHK(ctx, cp(o->cigar_off, R.cgo.p, 8 * (n + 1)));
  HIPCHK(ctx, cp(o->seq_off, R.sqo.p, 8 * (n + 1)));
  HIPCHK(ctx, cp(o->aux_off, R.axo.p, 8 * (n + 1)));
  HIPCHK(ctx, cp(o->names, R.names.p, R.sz.name_bytes));
  HIPCHK(ctx, cp(o->cigar, R.cigar.p, 4 * R.sz.cigar_ops));
  HIPCHK(ctx, cp(o->seq, R.seq.p, R.sz.bases));
  HIPCHK(ctx, cp(o->qual, R.qual.p, R.sz.bases));
  HIPCHK(ctx, cp(o->aux, R.aux.p, R.sz.aux_bytes));
  HIPCHK(ctx, hipStreamSynchronize(sh->st));
  return SBH_OK;
}

// ---- BGZF writer (zdeflate.hip / deflate.hip; HTSJDKRewrite.scala:62-67) ------------------
uint64_t sbh_bgzf_compress_bound(uint64_t n) { return deflate_nblocks(n) * ZDEFLATE_SLOT + 28; }

int sbh_bgzf_compress(sbh_ctx *ctx, const void *src, uint64_t n, int src_on_device, uint8_t *out,
                      uint64_t out_cap, uint64_t *out_size, uint64_t *n_blocks, float *deflate_ms) {
  return sbh_bgzf_compress_level(ctx, src, n, src_on_device, SBH_LEVEL_HTSJDK, out, out_cap, out_size, n_blocks,
                                 deflate_ms);
}

int sbh_bgzf_compress_level(sbh_ctx *ctx, const void *src, uint64_t n, int src_on_device, int level, uint8_t *out,
                            uint64_t out_cap, uint64_t *out_size, uint64_t *n_blocks, float *deflate_ms) {
  if (!ctx || !out_size || (!src && n) || !out) return SBH_E_ARG;
  const bool fast = level == SBH_LEVEL_FAST;
  if (!fast && (level < 0 || (level > 0 && level < 4) || level > 9))
    return fail(ctx, SBH_E_ARG, "bgzf_compress: level %d (0, 4..9 or SBH_LEVEL_FAST)", level);
  const uint64_t nb = deflate_nblocks(n);
  if (out_cap < sbh_bgzf_compress_bound(n)) return fail(ctx, SBH_E_ARG, "bgzf_compress: out_cap < bound");
  int rc = set_device(ctx);
  if (rc) return rc;
  struct Bufs {  // per-call scratch (and stream), freed on every return path
    DBuf<uint8_t> in, slots, packed, recs;
    DBuf<uint16_t> prev;
    DBuf<uint32_t> toks, sizes;
    DBuf<uint64_t> offs, info;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    hipStream_t own = nullptr;
    ~Bufs() {
      if (own) (void)hipStreamSynchronize(own);
      in.release(), slots.release(), packed.release(), recs.release(), prev.release(), toks.release(), sizes.release(),
          offs.release(), info.release();
      if (e0) (void)hipEventDestroy(e0);
      if (e1) (void)hipEventDestroy(e1);
      if (own) (void)hipStreamDestroy(own);
    }
  } B;
  // a stream of the call's own unless the caller gave the context one: concurrent callers of one
  // context (include/sparkbam.h, threading) neither wait for nor time each other's kernels
  if (ctx->own_stream) HIPCHK(ctx, hipStreamCreateWithFlags(&B.own, hipStreamNonBlocking));
  hipStream_t st = B.own ? B.own : ctx->stream;
  const uint8_t *d_src = static_cast<const uint8_t *>(src);
  if (!src_on_device && n) {
    HIPCHK(ctx, B.in.ensure(n));
    HIPCHK(ctx, hipMemcpyAsync(B.in.p, src, n, hipMemcpyHostToDevice, st));
    d_src = B.in.p;
  }
  uint64_t total = 0;
  float kms = 0.f;
  if (nb) {
    // members in batches: scratch bounded by the batch, not the input
    uint64_t bmax = fast ? DEFLATE_BATCH : ZDEFLATE_BATCH;
    if (const char *e = std::getenv("SBH_ZDEFLATE_BATCH"))
      if (!fast && std::strtoull(e, nullptr, 10) > 0) bmax = std::strtoull(e, nullptr, 10);
    const uint64_t stride = fast ? 65536ull : ZDEFLATE_SLOT;
    // scratch per member; the batch shrinks to half of the free HBM (a resident shard may hold
    // the rest), never below 256 members
    const uint64_t per_member =
        2 * stride + (fast ? DEFLATE_PREV_BYTES + DEFLATE_TOK_BYTES + DEFLATE_REC_BYTES
                           : level > 0 ? ZDEFLATE_PREV_ENTRIES * 2 + ZDEFLATE_INFO_ENTRIES * 8 +
                                             ZDEFLATE_TOK_ENTRIES * 4 + ZDEFLATE_REC_BYTES
                                       : 0) + 16;
    size_t hbm_free = 0, hbm_total = 0;
    if (hipMemGetInfo(&hbm_free, &hbm_total) == hipSuccess && hbm_free / 2 / per_member < bmax)
      bmax = std::max<uint64_t>(256, hbm_free / 2 / per_member);
    const uint64_t cap = nb < bmax ? nb : bmax;
    HIPCHK(ctx, B.slots.ensure(cap * stride));
    HIPCHK(ctx, B.packed.ensure(cap * stride));
    if (fast) {
      HIPCHK(ctx, B.prev.ensure(cap * (DEFLATE_PREV_BYTES / 2)));
      HIPCHK(ctx, B.toks.ensure(cap * (DEFLATE_TOK_BYTES / 4)));
      HIPCHK(ctx, B.recs.ensure(cap * DEFLATE_REC_BYTES));
    } else if (level > 0) {
      HIPCHK(ctx, B.prev.ensure(cap * ZDEFLATE_PREV_ENTRIES));
      HIPCHK(ctx, B.info.ensure(cap * ZDEFLATE_INFO_ENTRIES));
      HIPCHK(ctx, B.toks.ensure(cap * ZDEFLATE_TOK_ENTRIES));
      HIPCHK(ctx, B.recs.ensure(cap * ZDEFLATE_REC_BYTES));
    }
    HIPCHK(ctx, B.sizes.ensure(cap));
    HIPCHK(ctx, B.offs.ensure(cap));
    HIPCHK(ctx, hipEventCreate(&B.e0));
    HIPCHK(ctx, hipEventCreate(&B.e1));
    std::vector<uint32_t> hs(cap);
    std::vector<uint64_t> ho(cap);
    for (uint64_t b0 = 0; b0 < nb; b0 += cap) {
      const uint32_t k = (uint32_t)(nb - b0 < cap ? nb - b0 : cap);
      HIPCHK(ctx, hipEventRecord(B.e0, st));
      if (fast)
        HIPCHK(ctx, launch_deflate(d_src, n, b0, k, B.prev.p, B.toks.p, B.recs.p, B.slots.p, B.sizes.p, st));
      else
        HIPCHK(ctx, launch_zdeflate(d_src, n, b0, k, level, B.prev.p, B.info.p, B.toks.p, B.recs.p, B.slots.p,
                                    B.sizes.p, st));
      HIPCHK(ctx, hipEventRecord(B.e1, st));
      HIPCHK(ctx, hipMemcpyAsync(hs.data(), B.sizes.p, 4ull * k, hipMemcpyDeviceToHost, st));
      HIPCHK(ctx, hipStreamSynchronize(st));
      float ms = 0.f;
      HIPCHK(ctx, hipEventElapsedTime(&ms, B.e0, B.e1));
      kms += ms;
      uint64_t bt = 0;
      for (uint32_t j = 0; j < k; ++j) {
        if (hs[j] < 26 || hs[j] > stride)
          return fail(ctx, SBH_E_HIP, "bgzf_compress: block %llu size %u", (unsigned long long)(b0 + j), hs[j]);
        ho[j] = bt;
        bt += hs[j];
      }
      if (total + bt + 28 > out_cap) return fail(ctx, SBH_E_ARG, "bgzf_compress: out_cap exceeded");
      HIPCHK(ctx, hipMemcpyAsync(B.offs.p, ho.data(), 8ull * k, hipMemcpyHostToDevice, st));
      HIPCHK(ctx, launch_deflate_gather(B.slots.p, stride, B.sizes.p, B.offs.p, k, B.packed.p, st));
      HIPCHK(ctx, hipMemcpyAsync(out + total, B.packed.p, bt, hipMemcpyDeviceToHost, st));
      HIPCHK(ctx, hipStreamSynchronize(st));
      total += bt;
    }
  }
  if (deflate_ms) *deflate_ms = kms;
  static const uint8_t eof[28] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0,
                                  27, 0,   3, 0, 0, 0, 0, 0, 0, 0,   0, 0};
  memcpy(out + total, eof, 28);
  *out_size = total + 28;
  if (n_blocks) *n_blocks = nb;
  return SBH_OK;
}

}  // extern "C"

