"""Byte-range sharding of one BAM file across ranks, one process per GPU.

The reference's own decomposition is Hadoop file splits (`FileSplits.asJava(path,
splitSize)`, load/.../CanLoadBam.scala:205,314; SplitRDD.scala:33-52): every split is
self-contained given a halo of following bytes.  Rank r owns a contiguous run of those
splits, loads compressed bytes [lo_r, hi_r + halo) into its device, and runs the whole
hot path there (index -> inflate -> eager check at every owned position -> per-split
FindBlockStart / FindRecordStart / record count).  Nothing crosses ranks on the data
path.  The one exchange is an allgather of each rank's small result
({per-split first vpos, count}, plus the rank's chain exit), after which every rank holds
the reference's answer:

  splits = sliding2 over the first records of the non-empty splits, closed by
           Pos(fileSize, 0)                          (CanLoadBam.scala:283-297)
  counts = per-split record counts, in split order   (loadBam(...).count = their sum)

The stitch check is the §8e invariant: the record chain that leaves rank r's owned range
must enter rank r+1 exactly at rank r+1's first record (`exit_r == first_{r+1}` for
non-empty neighbours).  A mismatch means one side found a false-positive boundary; the
reference's outputs are per split either way, so they are returned unchanged and the
mismatch is reported in `stitch`.

The allgather goes through torch.distributed (RCCL over xGMI with backend "nccl", gloo
for the CPU tests); it carries a few hundred bytes per rank.
"""
import os
from collections import namedtuple

import numpy as np

from ._lib import SBH_E_NEED_HALO, SparkBamError
from .api import (DEFAULT_BGZF_BLOCKS_TO_CHECK, DEFAULT_MAX_READ_SIZE, DEFAULT_READS_TO_CHECK,
                  Pos, Split, file_splits, parse_bam_header)
from .device import Context

DEFAULT_HALO = 1 << 20  # compressed bytes past the owned range; grown x4 on SBH_E_NEED_HALO
# A rank whose compressed shard exceeds this many bytes streams it through HBM in windows
# (sbh_run_stream2) instead of holding it resident: ~5 B of HBM per compressed byte resident
# (compressed + flat + bitmap, token buffer bounded), so 24 GiB keeps a resident shard well
# inside 288 GB; configs[2]'s 100 GB file at N <= 4 streams.  SBH_RESIDENT_MAX overrides.
RESIDENT_MAX = int(os.environ.get("SBH_RESIDENT_MAX", str(24 << 30)))
STREAM_WINDOW = int(os.environ.get("SBH_STREAM_WINDOW", str(1 << 30)))

# One rank's contribution to the exchange.  firsts[i] is the htsjdk vpos of split i's
# first record (None when the split is empty); exit_vpos is the first record of the
# rank's chain at/after its owned end (None when the chain ran into the stream end).
RankPart = namedtuple("RankPart", "rank split_index firsts counts first_vpos count exit_vpos")


def rank_splits(file_size, split_size, world, rank):
    """Hadoop splits of the file dealt to ranks as contiguous runs balanced by count:
    (index of the rank's first split, [(start, end), ...])."""
    splits = file_splits(file_size, split_size)
    a = rank * len(splits) // world
    b = (rank + 1) * len(splits) // world
    return a, splits[a:b]


def file_reader(path):
    """read(lo, hi) -> the compressed bytes [lo, hi) of `path`, memory-mapped, so a rank
    never holds more of the file than its shard + halo."""
    mm = np.memmap(path, dtype=np.uint8, mode="r")

    def read(lo, hi):
        return np.ascontiguousarray(mm[lo:hi])

    read.size = int(mm.size)
    return read


def bytes_reader(data):
    arr = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data

    def read(lo, hi):
        return np.ascontiguousarray(arr[lo:hi])

    read.size = int(arr.size)
    return read


def read_header(ctx, read, file_size, first=DEFAULT_HALO):
    """Header(path) (check/.../header/Header.scala:26-60) from the file's leading blocks,
    inflated on the device: (contig names, contig lengths, flat end of the header)."""
    n = min(file_size, first)
    while True:
        sh = ctx.shard(read(0, n), file_offset=0, file_size=file_size)
        try:
            sh.index(0)
            sh.inflate()
            try:
                return parse_bam_header(sh.read_flat(0, sh.flat_size))
            except (IndexError, ValueError):
                if n >= file_size:
                    raise
        finally:
            sh.close()
        n = min(file_size, n * 4)


class RankRun:
    """One rank's share of the hot path over its splits [lo, hi).  A shard up to
    RESIDENT_MAX compressed bytes stays resident after the run, so the stitch can re-walk its
    chain later; a larger one (or stream=True) is streamed through HBM in windows cut at split
    starts (sbh_run_stream2, Stream.scala:80-122's bounded memory) and re-walks window by
    window."""

    def __init__(self, ctx, read, file_size, split_index, splits, contig_len, rank=0, halo=DEFAULT_HALO,
                 bgzf_blocks_to_check=DEFAULT_BGZF_BLOCKS_TO_CHECK,
                 reads_to_check=DEFAULT_READS_TO_CHECK, max_read_size=DEFAULT_MAX_READ_SIZE,
                 stream=None, window=None):
        self.sh = None
        self.rank = rank
        self.ctx, self.read, self.file_size, self.contig_len = ctx, read, file_size, contig_len
        self.rtc, self.mrs = reads_to_check, max_read_size
        if not splits:
            self.part = RankPart(rank, split_index, [], [], None, 0, None)
            return
        lo, hi = splits[0][0], splits[-1][1]
        self.lo, self.hi = lo, hi
        self.halo = halo
        self.streamed = (hi - lo > RESIDENT_MAX) if stream is None else bool(stream)
        if self.streamed:
            self._run_streamed(split_index, splits, halo, window or STREAM_WINDOW, bgzf_blocks_to_check)
            return
        while True:
            end = min(file_size, hi + halo)
            sh = ctx.shard(read(lo, end), file_offset=lo, file_size=file_size)
            try:
                sh.set_contigs(contig_len)
                start = sh.find_block_start(lo, bgzf_blocks_to_check)
                r = sh.run(start, hi, reads_to_check, max_read_size)
                # every split of the rank in one batch (FindBlockStart + FindRecordStart +
                # counts on the device; CanLoadBam.scala:283-297, 316-356)
                status, v, n, _ = sh.split_starts(splits, bgzf_blocks_to_check, reads_to_check, max_read_size)
                self.part = self._part(split_index, splits, status, v, n, r["first_vpos"] if r["count"] else None,
                                       r["count"], sh.exit_vpos(r))
                self.sh = sh
                self.halo = halo
                return
            except SparkBamError as err:
                sh.close()
                if err.code != SBH_E_NEED_HALO or end >= file_size:
                    raise
                halo *= 4
            except BaseException:
                sh.close()
                raise

    def _part(self, split_index, splits, status, v, n, first, count, exit_vpos):
        # one policy on every path (resident, streamed, CLI): a split's error is the job's error,
        # NoReadFoundException included, as FindRecordStart throws it (FindRecordStart.scala:66-71)
        for k in np.flatnonzero(status != 0):
            raise SparkBamError(int(status[k]), f"split {splits[k][0]}-{splits[k][1]}")
        counts = [int(c) for c in n]
        firsts = [int(x) if c else None for x, c in zip(v, counts)]
        return RankPart(self.rank, split_index, firsts, counts, first, count, exit_vpos)

    def _run_streamed(self, split_index, splits, halo, window, kcheck):
        lo, hi = self.lo, self.hi
        while True:
            end = min(self.file_size, hi + halo)
            comp = self.read(lo, end)
            try:
                r, _ = self.ctx.run_stream(comp, self.contig_len, file_offset=lo, file_size=self.file_size,
                                           own_end=hi, window=window, halo=min(halo, 4 << 20),
                                           reads_to_check=self.rtc, max_read_size=self.mrs, splits=splits,
                                           bgzf_blocks_to_check=kcheck)
            except SparkBamError as err:
                if err.code != SBH_E_NEED_HALO or end >= self.file_size:
                    raise
                halo *= 4
                continue
            self.stream_result = r
            self.halo = halo
            self.part = self._part(split_index, splits, r["split_status"], r["split_first_vpos"], r["split_count"],
                                   r["first_vpos"] if r["count"] else None, r["count"], r["exit_vpos"])
            return

    def rewalk_reload(self, from_vpos):
        """rewalk() from the file bytes again (the shard need not be kept): what a Spark task that
        re-walks a finished task's range does (jni/Native.scala GpuLoadBam.rewalk)."""
        return self._rewalk_streamed(from_vpos)

    def rewalk(self, from_vpos):
        """The chain from the upstream rank's exit (SURVEY 8e stitch fix-up): (records from
        from_vpos that start before the owned end, the chain's exit vpos or None)."""
        if self.streamed:
            return self._rewalk_streamed(from_vpos)
        sh = self.sh
        f = sh.flat_of(from_vpos >> 16, from_vpos & 0xFFFF)
        n, x = sh.chain_from(f, sh.flat_bound(self.hi))
        return n, sh.exit_vpos({"count": n, "exit_flat": x})

    def _rewalk_streamed(self, from_vpos, window=None):
        """The re-walk through bounded HBM: window by window from the entry record's block, the
        eager bitmap of the window first (so the chain is proven against it, not walked one
        record at a time), then the chain to the window's end; its exit enters the next."""
        window = window or STREAM_WINDOW
        total, v = 0, from_vpos
        while True:
            blo = v >> 16
            if blo >= self.hi:
                return total, v
            whi = min(self.hi, blo + window)
            halo = max(self.halo, 1 << 20)
            while True:
                end = min(self.file_size, whi + halo)
                sh = self.ctx.shard(self.read(blo, end), file_offset=blo, file_size=self.file_size)
                try:
                    sh.set_contigs(self.contig_len)
                    sh.index(blo)
                    sh.inflate()
                    f = sh.flat_of(blo, v & 0xFFFF)
                    E = sh.flat_bound(whi)
                    sh.check_eager(f, E, self.rtc, want_bits=False)
                    n, x = sh.chain_from(f, E)
                    ex = sh.exit_vpos({"count": n, "exit_flat": x}) if n else v
                    # (no record started in this window: the walk goes on from its next block)
                    nxt = next((b[0] for b in sh.blocks() if b[0] >= whi), None)
                    break
                except SparkBamError as err:
                    if err.code != SBH_E_NEED_HALO or end >= self.file_size:
                        raise
                    halo *= 4
                finally:
                    sh.close()
            total += n
            if ex is None or whi >= self.hi:
                return total, ex
            if ex == v:  # no record started in this window: continue at the first block after it
                if nxt is None:
                    raise SparkBamError(SBH_E_NEED_HALO, f"re-walk: no block past {whi} in the halo")
                ex = nxt << 16
            v = ex

    def close(self):
        if self.sh is not None:
            self.sh.close()
            self.sh = None


def run_rank(ctx, read, file_size, split_index, splits, contig_len, rank=0, halo=DEFAULT_HALO, **kw):
    """One rank's RankPart (RankRun without keeping the shard)."""
    run = RankRun(ctx, read, file_size, split_index, splits, contig_len, rank, halo, **kw)
    run.close()
    return run.part


def stitch(parts, file_size, rewalks=None):
    """Every rank's RankPart (any order) -> (splits, counts, stitch report).

    The splits and counts are the reference's per-split answer.  The report checks the
    record chain across ranks: `exit_r == first_{r+1}` for non-empty neighbours (`ok`,
    `mismatches`).  `rewalks` ({rank: (from_vpos, count, exit_vpos)}) replaces a rank's
    chain by its re-walk from the upstream exit; `chain_ok` / `chain_mismatches` /
    `chain_count` describe the chain after those re-walks (SURVEY 8e fix-up)."""
    parts = sorted(parts, key=lambda p: p.split_index)
    firsts, counts = [], []
    for p in parts:
        firsts += p.firsts
        counts += p.counts
    starts = [Pos.from_htsjdk(v) for v, n in zip(firsts, counts) if n > 0 and v is not None]
    ends = starts[1:] + [Pos(file_size, 0)]
    splits = [Split(a, b) for a, b in zip(starts, ends)]

    def mism(chain):
        nonempty = [c for c in chain if c[2] > 0]
        return [{"rank": a[0], "exit": a[3], "next_rank": b[0], "next_first": b[1]}
                for a, b in zip(nonempty, nonempty[1:]) if a[3] != b[1]]

    orig = [(p.rank, p.first_vpos, p.count, p.exit_vpos) for p in parts]
    rewalks = rewalks or {}
    eff = [(r, *rewalks[r]) if r in rewalks else (r, f, n, x) for r, f, n, x in orig]
    mismatches, chain_mismatches = mism(orig), mism(eff)
    return splits, counts, {"ok": not mismatches, "mismatches": mismatches,
                            "rank_counts": [p.count for p in parts],
                            "rewalk": {r: {"from": f, "count": n, "exit": x} for r, (f, n, x) in rewalks.items()},
                            "chain_ok": not chain_mismatches, "chain_mismatches": chain_mismatches,
                            "chain_count": sum(c[2] for c in eff)}


def _allgather(obj, group=None):
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return [obj]
    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, obj, group=group)
    return out


def _wire(x):
    """An exception as what the other ranks receive."""
    return ("error", x.code if isinstance(x, SparkBamError) else -1, repr(x) if not isinstance(x, SparkBamError)
            else str(x))


def exchange(part, group=None):
    """Allgather of the ranks' RankParts (torch.distributed; RCCL under "nccl").  A rank
    that failed contributes its exception instead, and every rank then raises it, so no
    rank is left waiting in a later collective."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        if isinstance(part, BaseException):
            raise part
        return [part]
    out = _allgather(_wire(part) if isinstance(part, BaseException) else tuple(part), group)
    for i, p in enumerate(out):
        if p[0] == "error":
            if isinstance(part, BaseException):
                raise part
            raise SparkBamError(p[1], f"rank {i}: {p[2]}")
    return [RankPart(*p) for p in out]


def reconcile(parts, file_size, rank, rewalk, group=None, max_rounds=None):
    """The stitch with the SURVEY 8e fix-up: while the chain leaving a rank does not enter
    its next non-empty rank at that rank's first record (a false-positive record start on
    one side), the next rank re-walks its chain from the upstream exit (`rewalk(vpos) ->
    (count, exit_vpos)`, run on the rank that holds those bytes), and every rank learns the
    re-walk through one more allgather.  A re-walk can move a rank's exit, so this repeats
    until the chain holds (at most world rounds).  The per-split answer is unchanged."""
    world = len(parts)
    rewalks = {}
    for _ in range(max_rounds or world):
        splits, counts, st = stitch(parts, file_size, rewalks)
        if st["chain_ok"]:
            break
        mine = None
        # (an upstream chain that ran into its stream end has no exit to re-walk from)
        todo = [m for m in st["chain_mismatches"] if m["next_rank"] == rank and m["exit"] is not None]
        if todo:
            try:
                n, ex = rewalk(todo[0]["exit"])
                mine = (rank, todo[0]["exit"], n, ex)
            except Exception as err:  # every rank must reach the allgather
                mine = err
        got = _allgather(_wire(mine) if isinstance(mine, BaseException) else mine, group)
        for i, g in enumerate(got):
            if g and g[0] == "error":
                if isinstance(mine, BaseException):
                    raise mine
                raise SparkBamError(g[1], f"rank {i}: {g[2]}")
        new = {g[0]: (g[1], g[2], g[3]) for g in got if g}
        if not new:
            break
        rewalks.update(new)
    return stitch(parts, file_size, rewalks)


def reconcile_local(parts, file_size, rewalk_of, max_rounds=None):
    """reconcile() with every rank's part in one process (a Spark driver after collect): the
    re-walk of rank r is rewalk_of[r](vpos) -> (count, exit_vpos)."""
    rewalks = {}
    for _ in range(max_rounds or len(parts)):
        _, _, st = stitch(parts, file_size, rewalks)
        if st["chain_ok"]:
            break
        new = {}
        for m in st["chain_mismatches"]:
            if m["exit"] is not None and m["next_rank"] not in new:
                n, ex = rewalk_of[m["next_rank"]](m["exit"])
                new[m["next_rank"]] = (m["exit"], n, ex)
        if not new:
            break
        rewalks.update(new)
    return stitch(parts, file_size, rewalks)


def load_splits_and_reads_tasks(path_or_bytes, split_size, tasks, ctx=None, halo=DEFAULT_HALO, **kw):
    """loadSplitsAndReads the way jni/Native.scala's GpuLoadBam runs it on Spark, call for call:
    the Hadoop splits dealt to `tasks` tasks as contiguous runs (rank_splits), each task a RankRun
    on its own bytes (sbh_shard_create over [lo, hi + halo), sbh_find_block_start, sbh_run_shard,
    sbh_split_starts, the exit's sbh_pos_of) whose shard is closed when the task ends; the
    driver's collect, the sliding2 stitch (CanLoadBam.scala:283-297), and a chain re-walk from the
    upstream exit, re-reading the task's bytes, wherever the chain does not enter a task at its
    first record.  Returns (splits, counts, stitch report)."""
    read = file_reader(path_or_bytes) if isinstance(path_or_bytes, (str, os.PathLike)) else bytes_reader(path_or_bytes)
    own_ctx = ctx is None
    ctx = ctx or Context(int(os.environ.get("LOCAL_RANK", "0")))
    try:
        _, contig_len, _ = read_header(ctx, read, read.size)
        runs = []
        for t in range(tasks):
            a, mine = rank_splits(read.size, split_size, tasks, t)
            run = RankRun(ctx, read, read.size, a, mine, contig_len, t, halo, stream=False, **kw)
            run.close()  # (the task ends; a re-walk reads its bytes again)
            runs.append(run)
        return reconcile_local([r.part for r in runs], read.size, {r.rank: r.rewalk_reload for r in runs})
    finally:
        if own_ctx:
            ctx.close()


def load_splits_and_reads(path_or_bytes, split_size=None, ctx=None, rank=None, world=None,
                          group=None, halo=DEFAULT_HALO, **kw):
    """CanLoadBam.loadSplitsAndReads (load/.../CanLoadBam.scala:268-302) over the ranks of
    the default (or given) process group, each on its own device.  `split_size` defaults to
    ceil(fileSize / world): one byte-range shard per rank.  Returns (splits, counts, stitch),
    identical on every rank.  Any failure on a rank (not only a SparkBamError) is exchanged,
    so every rank raises it instead of waiting in a collective."""
    import torch.distributed as dist

    on = dist.is_available() and dist.is_initialized()
    rank = rank if rank is not None else (dist.get_rank(group) if on else 0)
    world = world if world is not None else (dist.get_world_size(group) if on else 1)
    own_ctx = ctx is None
    run = None
    try:
        try:
            read = file_reader(path_or_bytes) if isinstance(path_or_bytes, (str, os.PathLike)) \
                else bytes_reader(path_or_bytes)
            file_size = read.size
            if split_size is None:
                split_size = max(1, -(-file_size // world))
            ctx = ctx or Context(int(os.environ.get("LOCAL_RANK", "0")))
            _, contig_len, _ = read_header(ctx, read, file_size)
            a, mine = rank_splits(file_size, split_size, world, rank)
            run = RankRun(ctx, read, file_size, a, mine, contig_len, rank, halo, **kw)
            part = run.part
        except Exception as err:  # exchanged: the peers must not block in the allgather
            if world == 1:
                raise
            part = err
        if world == 1:  # one rank owns every split: nothing to exchange, whatever process group exists
            return stitch([part], file_size)
        parts = exchange(part, group)
        return reconcile(parts, file_size, rank, run.rewalk, group)
    finally:
        if run is not None:
            run.close()
        if own_ctx and ctx is not None:
            ctx.close()
