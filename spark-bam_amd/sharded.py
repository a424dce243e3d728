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

from ._lib import SBH_E_NEED_HALO, SBH_E_NO_READ_FOUND, SparkBamError
from .api import (DEFAULT_BGZF_BLOCKS_TO_CHECK, DEFAULT_MAX_READ_SIZE, DEFAULT_READS_TO_CHECK,
                  Pos, Split, file_splits, parse_bam_header)
from .device import Context

DEFAULT_HALO = 1 << 20  # compressed bytes past the owned range; grown x4 on SBH_E_NEED_HALO

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


def run_rank(ctx, read, file_size, split_index, splits, contig_len, rank=0, halo=DEFAULT_HALO,
             bgzf_blocks_to_check=DEFAULT_BGZF_BLOCKS_TO_CHECK,
             reads_to_check=DEFAULT_READS_TO_CHECK, max_read_size=DEFAULT_MAX_READ_SIZE):
    """One rank's share of the hot path over its splits [lo, hi): the shard is loaded with
    a halo that grows until no result depends on bytes past it (SBH_E_NEED_HALO)."""
    if not splits:
        return RankPart(rank, split_index, [], [], None, 0, None)
    lo, hi = splits[0][0], splits[-1][1]
    while True:
        end = min(file_size, hi + halo)
        sh = ctx.shard(read(lo, end), file_offset=lo, file_size=file_size)
        try:
            sh.set_contigs(contig_len)
            start = sh.find_block_start(lo, bgzf_blocks_to_check)
            r = sh.run(start, hi, reads_to_check, max_read_size)
            firsts, counts = [], []
            for s, e in splits:
                try:
                    v, n = sh.split(s, e, bgzf_blocks_to_check, reads_to_check, max_read_size)
                except SparkBamError as err:
                    if err.code != SBH_E_NO_READ_FOUND:  # an empty split
                        raise
                    v, n = 0, 0
                firsts.append(v if n else None)
                counts.append(n)
            exit_vpos = sh.exit_vpos(r)
            return RankPart(rank, split_index, firsts, counts,
                            r["first_vpos"] if r["count"] else None, r["count"], exit_vpos)
        except SparkBamError as err:
            if err.code != SBH_E_NEED_HALO or end >= file_size:
                raise
            halo *= 4
        finally:
            sh.close()


def stitch(parts, file_size):
    """Every rank's RankPart (any order) -> (splits, counts, stitch report)."""
    parts = sorted(parts, key=lambda p: p.split_index)
    firsts, counts = [], []
    for p in parts:
        firsts += p.firsts
        counts += p.counts
    starts = [Pos.from_htsjdk(v) for v, n in zip(firsts, counts) if n > 0 and v is not None]
    ends = starts[1:] + [Pos(file_size, 0)]
    splits = [Split(a, b) for a, b in zip(starts, ends)]
    nonempty = [p for p in parts if p.count > 0]
    mismatches = []
    for a, b in zip(nonempty, nonempty[1:]):
        if a.exit_vpos != b.first_vpos:
            mismatches.append({"rank": a.rank, "exit": a.exit_vpos, "next_rank": b.rank,
                               "next_first": b.first_vpos})
    return splits, counts, {"ok": not mismatches, "mismatches": mismatches,
                            "rank_counts": [p.count for p in parts]}


def exchange(part, group=None):
    """Allgather of the ranks' RankParts (torch.distributed; RCCL under "nccl").  A rank
    that failed contributes its exception instead, and every rank then raises it, so no
    rank is left waiting in a later collective."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        if isinstance(part, BaseException):
            raise part
        return [part]
    mine = ("error", part.code if isinstance(part, SparkBamError) else -1, str(part)) \
        if isinstance(part, BaseException) else tuple(part)
    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, mine, group=group)
    for i, p in enumerate(out):
        if p[0] == "error":
            if isinstance(part, BaseException):
                raise part
            raise SparkBamError(p[1], f"rank {i}: {p[2]}")
    return [RankPart(*p) for p in out]


def load_splits_and_reads(path_or_bytes, split_size=None, ctx=None, rank=None, world=None,
                          group=None, halo=DEFAULT_HALO, **kw):
    """CanLoadBam.loadSplitsAndReads (load/.../CanLoadBam.scala:268-302) over the ranks of
    the default (or given) process group, each on its own device.  `split_size` defaults to
    ceil(fileSize / world): one byte-range shard per rank.  Returns (splits, counts, stitch),
    identical on every rank."""
    import torch.distributed as dist

    on = dist.is_available() and dist.is_initialized()
    rank = rank if rank is not None else (dist.get_rank(group) if on else 0)
    world = world if world is not None else (dist.get_world_size(group) if on else 1)
    read = file_reader(path_or_bytes) if isinstance(path_or_bytes, (str, os.PathLike)) \
        else bytes_reader(path_or_bytes)
    file_size = read.size
    if split_size is None:
        split_size = max(1, -(-file_size // world))
    own_ctx = ctx is None
    ctx = ctx or Context(int(os.environ.get("LOCAL_RANK", "0")))
    try:
        _, contig_len, _ = read_header(ctx, read, file_size)
        a, mine = rank_splits(file_size, split_size, world, rank)
        part = run_rank(ctx, read, file_size, a, mine, contig_len, rank, halo, **kw)
    except SparkBamError as err:
        part = err
    finally:
        if own_ctx:
            ctx.close()
    return stitch(exchange(part, group), file_size)
