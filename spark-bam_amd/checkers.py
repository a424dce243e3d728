"""The reference's per-position Checker plugins, answered from GPU windows.

spark-bam's callers ask a checker one position at a time, in file order within a partition:
`Checker.apply(pos)` (check/src/main/scala/org/hammerlab/bam/check/Checker.scala:7-9),
driven by CallPartition (cli/.../CallPartition.scala:35-52), FullCheck.checkPartition
(cli/.../full/FullCheck.scala:65-86) and CheckBlocks, and
`ReadStartFinder.nextReadStart(start)` (check/.../ReadStartFinder.scala:5-11) from
FindRecordStart (check/.../spark/FindRecordStart.scala:40-46).  A device launch per position
would be absurd, so a checker here owns a WINDOW of the file: the compressed bytes of the
blocks starting in [lo, lo + window) plus a halo, indexed, inflated and checked at every owned
position in ONE batch call; apply(pos) is then a host lookup in that batch.

These classes are the Python twin of jni/Native.scala's GpuWindow / GpuEagerChecker /
GpuFullChecker: the same C-ABI calls in the same order (sbh_shard_create, sbh_set_contigs,
sbh_find_block_start, sbh_index, sbh_inflate, sbh_flat_bound, sbh_get_blocks, then sbh_check_eager /
sbh_check_full over the OWNED flat range [0, flat_bound(lo + window)) only, and
sbh_find_record_start / sbh_pos_of for nextReadStart), so tests/test_checkers_gpu.py proves the
Scala façade's call sequence on the GPU.  A window whose results need bytes past its halo
(SBH_E_NEED_HALO, or no block past the owned range in the halo) is reloaded with 4x the halo;
the grown halo is kept for later windows.
"""
import numpy as np

from ._lib import (FULL_FLAGS_MASK, FULL_N_SHIFT, FULL_SUCCESS, SBH_E_NEED_HALO, SBH_E_NO_READ_FOUND,
                   SparkBamError)
from .device import Context


def _reader(path_or_bytes):
    """read(lo, hi) over a path (memory-mapped) or in-memory bytes; read.size = file size."""
    if isinstance(path_or_bytes, (bytes, bytearray, memoryview, np.ndarray)):
        arr = path_or_bytes if isinstance(path_or_bytes, np.ndarray) else np.frombuffer(path_or_bytes, np.uint8)
    else:
        arr = np.memmap(path_or_bytes, dtype=np.uint8, mode="r")

    def read(lo, hi):
        return np.ascontiguousarray(arr[lo:hi])

    read.size = int(arr.size)
    return read


class GpuWindow:
    """Compressed bytes [lo, min(size, lo + window + halo)) resident on the device, indexed from
    FindBlockStart(lo) (bgzf/.../block/FindBlockStart.scala:8-36) and inflated.  It owns the
    blocks whose start lies in [lo, hi = lo + window): flat positions [0, owned) with
    owned = flat_bound(hi).  Raises SBH_E_NEED_HALO when the halo holds no block past hi (the
    owned range's last block, or what follows it, is cut off) -- Native.scala GpuWindow.load."""

    def __init__(self, ctx, read, lo, window, halo, contig_len, bgzf_blocks_to_check=5):
        size = read.size
        self.lo, self.hi = lo, lo + window
        self.end = min(size, lo + window + halo)
        self.at_eof = self.end == size
        self.shard = ctx.shard(read(lo, self.end), file_offset=lo, file_size=size)
        try:
            sh = self.shard
            sh.set_contigs(contig_len)
            start = sh.find_block_start(lo, bgzf_blocks_to_check)
            sh.index(start)
            sh.inflate()
            self.owned = sh.flat_bound(self.hi)
            if not self.at_eof and self.owned == sh.flat_size:
                raise SparkBamError(SBH_E_NEED_HALO, f"halo {halo} holds no block past {self.hi}")
            # the host block table: flatOf(pos) without a library call per position
            self.ustart = {b[0]: b[3] for b in sh.blocks()}
        except BaseException:
            self.shard.close()
            raise

    def owns(self, block_pos):
        return self.lo <= block_pos < self.hi

    def flat_of(self, pos):
        u = self.ustart.get(pos.block_pos)
        if u is None:
            raise SparkBamError(19, f"{pos.block_pos} is not a block start of this window")
        return u + pos.offset

    def pos_of(self, flat):
        from .api import Pos
        return Pos(*self.shard.pos_of(flat))

    def close(self):
        self.shard.close()


class _WindowedChecker:
    """The window cache both checkers share (Native.scala WindowedChecker)."""

    def __init__(self, path_or_bytes, contig_len, reads_to_check=10, window=256 << 20, halo=4 << 20, ctx=None,
                 bgzf_blocks_to_check=5):
        self.read = _reader(path_or_bytes)
        self.contig_len = np.asarray(contig_len, dtype=np.int32)
        self.rtc = reads_to_check
        self.window, self.halo = int(window), int(halo)
        self.kcheck = bgzf_blocks_to_check
        self.own_ctx = ctx is None
        self.ctx = ctx or Context(0)
        self.w = None
        self.loads = 0  # windows loaded (halo growth included)

    def _fill(self, w):  # the window's batch (eager bits / full words)
        raise NotImplementedError

    def _load(self, lo):
        """GpuWindow at lo plus its batch, growing the halo x4 while either needs more bytes."""
        while True:
            self.loads += 1
            w = None
            try:
                w = GpuWindow(self.ctx, self.read, lo, self.window, self.halo, self.contig_len, self.kcheck)
                self._fill(w)
                return w
            except SparkBamError as err:
                if w is not None:
                    w.close()
                if err.code != SBH_E_NEED_HALO or lo + self.window + self.halo >= self.read.size:
                    raise
                self.halo *= 4

    def window_for(self, block_pos, reload=False):
        if reload or self.w is None or not self.w.owns(block_pos):
            if self.w is not None:
                self.w.close()
                self.w = None
            self.w = self._load(block_pos)
        return self.w

    def close(self):
        if self.w is not None:
            self.w.close()
            self.w = None
        if self.own_ctx and self.ctx is not None:
            self.ctx.close()
            self.ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class WindowedEagerChecker(_WindowedChecker):
    """eager.Checker (check/.../eager/Checker.scala:24-162) as Checker[Boolean] with
    ReadStartFinder: apply(pos) from the window's eager bitmap over its owned positions;
    next_read_start(start) = FindRecordStart.withDelta's search on the device."""

    def _fill(self, w):
        _, bits = w.shard.check_eager(0, w.owned, self.rtc)
        w.bits = bits.tobytes()

    def apply(self, pos):
        w = self.window_for(pos.block_pos)
        f = w.flat_of(pos)
        return (w.bits[f >> 3] >> (f & 7)) & 1 == 1

    __call__ = apply

    def next_read_start(self, start, max_read_size=100000000):
        """nextReadStart (eager/Checker.scala:134-147): the first eager-true position at or after
        `start` within max_read_size positions of the stream, or None."""
        r = self.next_read_start_with_delta(start, max_read_size)
        return None if r is None else r[0]

    def next_read_start_with_delta(self, start, max_read_size=100000000):
        reload = False
        while True:
            w = self.window_for(start.block_pos, reload)
            try:
                f, d = w.shard.find_record_start(w.flat_of(start), self.rtc, max_read_size)
                return w.pos_of(f), d
            except SparkBamError as err:
                if err.code == SBH_E_NO_READ_FOUND:
                    return None
                if err.code != SBH_E_NEED_HALO or w.at_eof:
                    raise
                self.halo *= 4
                reload = True


class WindowedFullChecker(_WindowedChecker):
    """full.Checker (check/.../full/Checker.scala:22-184) as Checker[Result]: apply(pos) is the
    window's full-checker word (include/sparkbam.h layout) at pos; result(word) turns it into
    the reference's Success(readsParsed) / Flags(..., readsBeforeError)."""

    def __init__(self, *a, window=32 << 20, **kw):
        super().__init__(*a, window=window, **kw)

    def _fill(self, w):
        r = w.shard.check_full(0, w.owned, self.rtc, want_words=True, close_cap=0)
        w.words = r["words"]

    def apply(self, pos):
        w = self.window_for(pos.block_pos)
        return int(w.words[w.flat_of(pos)])

    __call__ = apply

    @staticmethod
    def result(word):
        """("success", readsParsed) or ("flags", [flag names], readsBeforeError)
        (full/error/Flags.scala:21-45, Success: full/error/Result.scala)."""
        from .api import FLAG_NAMES
        n = (word >> FULL_N_SHIFT) & 0x3FF
        if word & FULL_SUCCESS:
            return ("success", n)
        return ("flags", [FLAG_NAMES[i] for i in range(19) if word & FULL_FLAGS_MASK & (1 << i)], n)
