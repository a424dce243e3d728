// check_stream.hip -- the all-positions modes over a file of any size (include/sparkbam.h:
// sbh_find_blocks, sbh_check_stream).  Host orchestration only: one shard slides along the
// file (sbh_shard_load keeps its device buffers), each window is indexed, inflated and checked
// by the same kernels as a resident shard, and only small results come back.
//
//   Blocks.apply without `.blocks`      check/src/main/scala/org/hammerlab/bam/check/Blocks.scala:141-206
//   CallPartition / CheckerApp (-s)     cli/.../check/CallPartition.scala:23-54, CheckerApp.scala:65-227
//   FullCheck.checkPartition + Counts   cli/.../check/full/FullCheck.scala:65-86, 142-192
#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <vector>

#include <hip/hip_runtime.h>

#include "sbh_internal.h"

namespace {

using Clock = std::chrono::steady_clock;

// The window shard: created empty, re-loaded per window, destroyed on every return path.
struct WinShard {
  sbh_shard *sh = nullptr;
  ~WinShard() { sbh_shard_destroy(sh); }
};

std::vector<sbh_block> table(sbh_shard *sh, uint64_t nb, int *rc) {
  std::vector<sbh_block> t(nb);
  *rc = nb ? sbh_get_blocks(sh, 0, nb, t.data()) : SBH_OK;
  return t;
}

// index of the block starting at `start` in t, or -1
int64_t find_block(const std::vector<sbh_block> &t, uint64_t start) {
  auto it = std::lower_bound(t.begin(), t.end(), start, [](const sbh_block &b, uint64_t v) { return b.start < v; });
  return it != t.end() && it->start == start ? it - t.begin() : -1;
}

double ms_since(Clock::time_point t) { return std::chrono::duration<double, std::milli>(Clock::now() - t).count(); }

}  // namespace

extern "C" {

// Blocks.apply's unindexed branch (Blocks.scala:141-206) over windows of splits.  Per split:
// FindBlockStart on the device, then the device block chain from there (MetadataStream: next
// block = start + csize) while the start is < the split end, stopping at an empty block.  One
// index per window serves every split whose FindBlockStart lands on its chain; a split whose
// search lands off it (a header-shaped byte run) re-indexes from there, as its own
// MetadataStream would.
int sbh_find_blocks(sbh_ctx *ctx, const void *host_file, uint64_t file_size, const uint64_t *S, const uint64_t *E,
                    uint64_t ns, int32_t k, uint64_t window, sbh_block *out, uint64_t cap, uint64_t *n_out) {
  if (!ctx || !n_out || (!host_file && file_size) || (ns && (!S || !E)) || (cap && !out) || k < 0) return SBH_E_ARG;
  *n_out = 0;
  for (uint64_t i = 0; i < ns; ++i)
    if (E[i] <= S[i] || E[i] > file_size || (i && S[i] < E[i - 1])) return SBH_E_ARG;
  if (!window) window = 1ull << 30;
  const uint8_t *src = static_cast<const uint8_t *>(host_file);
  WinShard W;
  int rc = sbh_shard_create(ctx, nullptr, 0, 0, file_size, 0, &W.sh);
  if (rc) return rc;
  uint64_t halo = 1ull << 20, count = 0;
  std::vector<sbh_block> got;
  for (uint64_t i = 0; i < ns;) {
    uint64_t j = i + 1;
    while (j < ns && S[j] < S[i] + window) ++j;
    for (;;) {
      const uint64_t lo = S[i], ld = std::min(file_size, E[j - 1] + halo);
      const bool at_eof = ld == file_size;
      got.clear();
      rc = sbh_shard_load(W.sh, src + lo, ld - lo, lo, 0);
      std::vector<sbh_block> t;
      for (uint64_t s = i; !rc && s < j; ++s) {
        uint64_t fbs = 0;
        rc = sbh_find_block_start(W.sh, S[s], k, &fbs);
        if (rc) break;
        int64_t q = find_block(t, fbs);
        if (q < 0) {  // (the first split of the window, or a search off the current chain)
          uint64_t nb = 0;
          rc = sbh_index(W.sh, fbs, &nb, nullptr);
          if (!rc) t = table(W.sh, nb, &rc);
          if (rc) break;
          q = 0;
        }
        for (;; ++q) {
          if ((uint64_t)q == t.size()) {  // ran off the resident chain
            if (!at_eof) rc = SBH_E_NEED_HALO;
            break;
          }
          const sbh_block &b = t[q];
          if (b.start >= E[s] || (b.flags & SBH_BLOCK_EMPTY)) break;
          sbh_block m{};
          m.start = b.start;
          m.csize = b.csize;
          m.usize = b.usize;
          m.ustart = s;
          got.push_back(m);
        }
      }
      if (rc == SBH_E_NEED_HALO && !at_eof) {
        halo *= 4;
        continue;
      }
      if (rc) return rc;
      break;
    }
    for (const sbh_block &m : got) {
      if (count < cap) out[count] = m;
      ++count;
    }
    i = j;
  }
  *n_out = count;
  return SBH_OK;
}

int sbh_check_stream(sbh_ctx *ctx, const void *host_file, uint64_t file_size, const int32_t *contigs,
                     int32_t n_contigs, const sbh_check_opts *o, sbh_check_result *res) {
  if (!ctx || !o || !res || (!host_file && file_size) || (o->n_blocks && !o->blocks) ||
      (o->n_truth && !o->truth_vpos) || (o->full && (!o->counts || !o->rbe_hist)) || n_contigs < 0)
    return SBH_E_ARG;
  const uint64_t *B = o->blocks, nb = o->n_blocks;
  for (uint64_t i = 1; i < nb; ++i)
    if (B[i] <= B[i - 1]) return SBH_E_ARG;
  for (uint64_t i = 1; i < o->n_truth; ++i)
    if (o->truth_vpos[i] < o->truth_vpos[i - 1]) return SBH_E_ARG;
  if (nb && B[nb - 1] >= file_size) return SBH_E_ARG;
  std::memset(res, 0, sizeof *res);
  const auto t0 = Clock::now();
  const uint64_t window = o->window ? o->window : 1ull << 30;
  uint64_t halo = o->halo ? o->halo : 4ull << 20;
  const int32_t rtc = o->reads_to_check;
  const bool truth = o->truth_vpos != nullptr;
  if (o->full) {
    std::memset(o->counts, 0, sizeof(uint64_t) * SBH_NNZ_MAX * 19);
    std::memset(o->rbe_hist, 0, sizeof(uint64_t) * SBH_NNZ_MAX * SBH_RBE_MAX);
  }
  const uint8_t *src = static_cast<const uint8_t *>(host_file);
  WinShard W;
  int rc = sbh_shard_create(ctx, nullptr, 0, 0, file_size, 0, &W.sh);
  if (!rc) rc = sbh_set_contigs(W.sh, contigs, n_contigs);
  if (rc) return rc;
  sbh_shard *sh = W.sh;
  // per-window scratch (a window redone with a larger halo starts them over)
  struct Acc {
    uint64_t positions = 0, comp = 0, n_true = 0, tp = 0, fp = 0, fn = 0, unk = 0, ns = 0, nclose = 0;
    std::vector<uint64_t> fpv, fnv, closev;
    std::vector<uint32_t> closew;
    std::vector<uint64_t> counts, rbe;
  } A;
  std::vector<uint64_t> rb, re, fl, fl2, cf;
  std::vector<uint32_t> cw;
  std::vector<uint64_t> wc(SBH_NNZ_MAX * 19), wr(SBH_NNZ_MAX * SBH_RBE_MAX);
  auto vpos_of = [&](uint64_t flat, uint64_t *v) {
    uint64_t bp = 0;
    uint32_t off = 0;
    const int r = sbh_pos_of(sh, flat, &bp, &off);
    *v = bp << 16 | off;
    return r;
  };
  // window k: the listed blocks [i, j) starting in [B[i], B[i] + window), loaded with a halo
  // past the last one, and its truth slice (the `.records` of those blocks)
  auto window_end = [&](uint64_t i) {
    uint64_t j = i + 1;
    while (j < nb && B[j] < B[i] + window) ++j;
    return j;
  };
  auto truth_slice = [&](uint64_t lo, uint64_t last, uint64_t *t0, uint64_t *t1) {
    const uint64_t *T = o->truth_vpos;
    *t0 = truth ? (uint64_t)(std::lower_bound(T, T + o->n_truth, lo << 16) - T) : 0;
    *t1 = truth ? (uint64_t)(std::lower_bound(T, T + o->n_truth, (last + 1) << 16) - T) : 0;
  };
  // The next window's bytes (and truth slice) are copied by a host thread while this window's
  // kernels run (sbh::shard_prefetch); a window redone with a larger halo loads synchronously.
  struct PrefetchGuard {  // no copy thread outlives the call
    sbh_shard *sh;
    ~PrefetchGuard() {
      if (sbh::shard_prefetch_pending(sh, nullptr, nullptr)) (void)sbh::shard_prefetch_finish(sh, false);
    }
  } pf_guard{sh};
  for (uint64_t i = 0; i < nb;) {
    const uint64_t lo = B[i];
    const uint64_t j = window_end(i);
    const uint64_t last = B[j - 1];
    uint64_t t0i = 0, t1i = 0;
    truth_slice(lo, last, &t0i, &t1i);
    for (;;) {  // this window, grown until its answers fit the halo
      const uint64_t ld = std::min(file_size, last + halo);
      const bool at_eof = ld == file_size;
      A = Acc{};
      A.counts.assign(SBH_NNZ_MAX * 19, 0);
      A.rbe.assign(SBH_NNZ_MAX * SBH_RBE_MAX, 0);
      // this window's bytes: the prefetch started during the previous window when it matches
      // (a window redone with a larger halo does not), else a copy of its own (the same copy
      // threads, waited for at once)
      uint64_t poff = 0, pn = 0;
      rc = SBH_OK;
      if (sbh::shard_prefetch_pending(sh, &poff, &pn) && !(poff == lo && pn == ld - lo))
        rc = sbh::shard_prefetch_finish(sh, false);
      if (!rc && !sbh::shard_prefetch_pending(sh, nullptr, nullptr))
        rc = sbh::shard_prefetch(sh, src + lo, ld - lo, lo, truth ? o->truth_vpos + t0i : nullptr, t1i - t0i);
      double cms = 0;
      if (!rc) rc = sbh::shard_prefetch_finish(sh, true, &cms);
      res->ms_h2d += cms;
      const bool truth_resident = truth;
      if (!rc && j < nb) {  // the next window starts copying now
        const uint64_t lo2 = B[j], last2 = B[window_end(j) - 1];
        const uint64_t ld2 = std::min(file_size, last2 + halo);
        uint64_t u0 = 0, u1 = 0;
        truth_slice(lo2, last2, &u0, &u1);
        rc = sbh::shard_prefetch(sh, src + lo2, ld2 - lo2, lo2, truth ? o->truth_vpos + u0 : nullptr, u1 - u0);
      }
      uint64_t nblk = 0;
      if (!rc) rc = sbh_index(sh, lo, &nblk, nullptr);
      std::vector<sbh_block> t;
      if (!rc) t = table(sh, nblk, &rc);
      if (!rc) rc = sbh_inflate(sh, nullptr);
      // the listed blocks' flat ranges (adjacent blocks merged)
      rb.clear();
      re.clear();
      for (uint64_t q = i; !rc && q < j; ++q) {
        const int64_t x = find_block(t, B[q]);
        if (x < 0) {
          rc = (!at_eof && (t.empty() || t.back().start < B[q])) ? SBH_E_NEED_HALO : SBH_E_NOT_FOUND;
          break;
        }
        const sbh_block &b = t[x];
        A.comp += b.csize;
        if ((b.flags & SBH_BLOCK_EMPTY) || !b.usize) continue;
        A.positions += b.usize;
        if (!re.empty() && re.back() == b.ustart) re.back() = b.ustart + b.usize;
        else rb.push_back(b.ustart), re.push_back(b.ustart + b.usize);
      }
      // eager calls, against the truth when given
      if (!rc && truth) {
        const uint64_t *T = o->truth_vpos;
        fl.assign(o->fp_cap + 1, 0);
        fl2.assign(o->fn_cap + 1, 0);
        uint64_t r4[4] = {0, 0, 0, 0};
        rc = truth_resident ? sbh::check_records_resident(sh, rb.data(), re.data(), rb.size(), rtc, t1i - t0i, r4,
                                                          fl.data(), o->fp_cap, fl2.data(), o->fn_cap)
                            : sbh_check_records(sh, rb.data(), re.data(), rb.size(), rtc, T + t0i, t1i - t0i, r4,
                                                fl.data(), o->fp_cap, fl2.data(), o->fn_cap);
        if (!rc) {
          A.tp = r4[0], A.fp = r4[1], A.fn = r4[2], A.unk = r4[3];
          A.n_true = A.tp + A.fp;
          for (uint64_t q = 0; !rc && q < std::min(A.fp, o->fp_cap); ++q) {
            uint64_t v = 0;
            rc = vpos_of(fl[q], &v);
            A.fpv.push_back(v);
          }
          for (uint64_t q = 0; !rc && q < std::min(A.fn, o->fn_cap); ++q) {
            uint64_t v = 0;
            rc = vpos_of(fl2[q], &v);
            A.fnv.push_back(v);
          }
        }
      } else if (!rc) {
        for (size_t r = 0; !rc && r < rb.size(); ++r) {
          uint64_t nt = 0;
          rc = sbh_check_eager(sh, rb[r], re[r], rtc, nullptr, &nt);
          A.n_true += nt;
        }
      }
      // the full checker's aggregation
      if (!rc && o->full) {
        const uint64_t ccap = o->close_cap;
        cf.assign(ccap + 1, 0);
        cw.assign(ccap + 1, 0);
        for (size_t r = 0; !rc && r < rb.size(); ++r) {
          uint64_t ns = 0, nclose = 0;
          rc = sbh_check_full(sh, rb[r], re[r], rtc, nullptr, wc.data(), wr.data(), &ns, cf.data(), cw.data(), ccap,
                              &nclose);
          if (rc) break;
          for (size_t q = 0; q < wc.size(); ++q) A.counts[q] += wc[q];
          for (size_t q = 0; q < wr.size(); ++q) A.rbe[q] += wr[q];
          A.ns += ns;
          A.nclose += nclose;
          for (uint64_t q = 0; !rc && q < std::min(nclose, ccap); ++q) {
            uint64_t v = 0;
            rc = vpos_of(cf[q], &v);
            A.closev.push_back(v);
            A.closew.push_back(cw[q]);
          }
        }
      }
      if (rc == SBH_E_NEED_HALO && !at_eof) {
        halo *= 4;
        continue;
      }
      if (rc) return rc;
      break;
    }
    // commit the window (lists in ascending vpos: windows ascend and each list is sorted)
    ++res->n_windows;
    res->positions += A.positions;
    res->comp_bytes += A.comp;
    res->n_true += A.n_true;
    res->tp += A.tp, res->fp += A.fp, res->fn += A.fn, res->unknown += A.unk;
    {
      const uint64_t before_fp = res->fp - A.fp, before_fn = res->fn - A.fn;
      for (size_t q = 0; q < A.fpv.size() && before_fp + q < o->fp_cap; ++q)
        if (o->fp_vpos) o->fp_vpos[before_fp + q] = A.fpv[q];
      for (size_t q = 0; q < A.fnv.size() && before_fn + q < o->fn_cap; ++q)
        if (o->fn_vpos) o->fn_vpos[before_fn + q] = A.fnv[q];
    }
    if (o->full) {
      for (size_t q = 0; q < A.counts.size(); ++q) o->counts[q] += A.counts[q];
      for (size_t q = 0; q < A.rbe.size(); ++q) o->rbe_hist[q] += A.rbe[q];
      res->n_success += A.ns;
      const uint64_t before = res->n_close;
      res->n_close += A.nclose;
      // close calls of several ranges of one window: sort this window's list
      std::vector<size_t> idx(A.closev.size());
      for (size_t q = 0; q < idx.size(); ++q) idx[q] = q;
      std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return A.closev[a] < A.closev[b]; });
      for (size_t q = 0; q < idx.size() && before + q < o->close_cap; ++q) {
        if (o->close_vpos) o->close_vpos[before + q] = A.closev[idx[q]];
        if (o->close_word) o->close_word[before + q] = A.closew[idx[q]];
      }
    }
    i = j;
  }
  res->halo_final = halo;
  res->ms_wall = ms_since(t0);
  return SBH_OK;
}

}  // extern "C"
