"""Reference-shaped host API over the C-ABI.

Each function names the spark-bam entry point it mirrors (paths relative to the
reference repository root).  All byte work runs in libsparkbam_hip.so on the GPU;
this module only moves small results around (splits, counts, histograms).
"""
import ctypes as C
import os
from collections import namedtuple

import numpy as np

from ._lib import FULL_FLAGS_MASK, FULL_N_SHIFT, SBH_E_NEED_HALO, SBH_OK, SparkBamError, lib
from .device import Context
from .records import Reads

FLAG_NAMES = [  # check/.../full/error/Flags.scala:203-222 (serde order)
    "tooFewFixedBlockBytes", "negativeReadIdx", "tooLargeReadIdx", "negativeReadPos",
    "tooLargeReadPos", "negativeNextReadIdx", "tooLargeNextReadIdx", "negativeNextReadPos",
    "tooLargeNextReadPos", "tooFewBytesForReadName", "nonNullTerminatedReadName",
    "nonASCIIReadName", "noReadName", "emptyReadName", "tooFewBytesForCigarOps",
    "invalidCigarOp", "emptyMappedCigar", "emptyMappedSeq", "tooFewRemainingBytesImplied",
]

DEFAULT_BGZF_BLOCKS_TO_CHECK = 5      # bgzf/.../block/package.scala:20
DEFAULT_READS_TO_CHECK = 10          # check/.../check/package.scala:17-18
DEFAULT_MAX_READ_SIZE = 100000000    # check/.../check/package.scala:28-29
DEFAULT_SPLIT_SIZE = 32 * 1024 * 1024  # Hadoop local-FS block size (MaxSplitSize default)


class Pos(namedtuple("Pos", "block_pos offset")):
    """bgzf Pos(blockPos, offset) (bgzf/.../Pos.scala:12-43)."""

    def to_htsjdk(self):
        return (self.block_pos << 16) | self.offset

    @classmethod
    def from_htsjdk(cls, v):
        return cls(v >> 16, v & 0xFFFF)

    def __str__(self):
        return f"{self.block_pos}:{self.offset}"

    def minus(self, other, ratio=3.0):  # Pos.- with EstimatedCompressionRatio (Pos.scala:17-22)
        return float(max(0, self.block_pos - other.block_pos + int((self.offset - other.offset) / ratio)))


Split = namedtuple("Split", "start end")  # check/.../spark/Split.scala:9-13
Metadata = namedtuple("Metadata", "start compressed_size uncompressed_size")  # Metadata.scala:6-8


class Header:
    @staticmethod
    def make(b):
        """Header.make (bgzf/.../block/Header.scala:48-83) -> (size, compressedSize)."""
        arr = np.frombuffer(bytes(b), dtype=np.uint8)
        hs, cs = C.c_int32(), C.c_int32()
        rc = lib().sbh_header_make(arr.ctypes.data_as(C.c_void_p), arr.size, C.byref(hs), C.byref(cs))
        if rc != SBH_OK:
            raise SparkBamError(rc, "bad BGZF header")
        return hs.value, cs.value


def file_splits(file_size, split_size):
    """Hadoop FileInputFormat.getSplits arithmetic (SPLIT_SLOP 1.1), as driven by
    FileSplits.asJava(path, splitSize) (load/.../CanLoadBam.scala:205,314)."""
    out, rem = [], file_size
    while rem / split_size > 1.1:
        out.append((file_size - rem, file_size - rem + split_size))
        rem -= split_size
    if rem != 0:
        out.append((file_size - rem, file_size))
    return out


def parse_bam_header(flat):
    """check/.../header/Header.scala:26-60: contig lengths + flat end of the header."""
    b = bytes(flat)
    if b[:4] != b"BAM\1":
        raise SparkBamError(1, "not a BAM file (missing BAM\\1 magic)")
    l_text = int.from_bytes(b[4:8], "little", signed=True)
    c = 8 + l_text
    n_ref = int.from_bytes(b[c:c + 4], "little", signed=True)
    c += 4
    names, lens = [], []
    for _ in range(n_ref):
        l_name = int.from_bytes(b[c:c + 4], "little", signed=True)
        names.append(b[c + 4:c + 4 + l_name].rstrip(b"\0").decode())
        c += 4 + l_name
        lens.append(int.from_bytes(b[c:c + 4], "little", signed=True))
        c += 4
    return names, np.asarray(lens, dtype=np.int32), c


def bam_header(shard):
    """Header(path) over an indexed + inflated shard starting at file offset 0."""
    n = min(shard.flat_size, 1 << 16)
    while True:
        try:
            return parse_bam_header(shard.read_flat(0, n))
        except (IndexError, ValueError):
            if n >= shard.flat_size:
                raise
            n = min(shard.flat_size, n * 4)


def _read(path_or_bytes):
    if isinstance(path_or_bytes, (bytes, bytearray, memoryview, np.ndarray)):
        return np.frombuffer(bytes(path_or_bytes), dtype=np.uint8) if not isinstance(
            path_or_bytes, np.ndarray) else path_or_bytes
    with open(path_or_bytes, "rb") as f:
        return np.frombuffer(f.read(), dtype=np.uint8)


class _Loaded:
    """A whole BGZF file resident on one device: indexed, inflated, header parsed."""

    def __init__(self, path_or_bytes, ctx=None, reads_to_check=DEFAULT_READS_TO_CHECK):
        self.data = _read(path_or_bytes)
        self.own_ctx = ctx is None
        self.ctx = ctx or Context(0)
        self.shard = self.ctx.shard(self.data)
        self.shard.index(0)
        self.shard.inflate()
        self.names, self.contig_len, self.header_end = bam_header(self.shard)
        self.shard.set_contigs(self.contig_len)
        self.reads_to_check = reads_to_check

    def close(self):
        self.shard.close()
        if self.own_ctx:
            self.ctx.close()


def load_splits_and_reads(path_or_bytes, split_size=DEFAULT_SPLIT_SIZE, ctx=None,
                          bgzf_blocks_to_check=DEFAULT_BGZF_BLOCKS_TO_CHECK,
                          reads_to_check=DEFAULT_READS_TO_CHECK, max_read_size=DEFAULT_MAX_READ_SIZE):
    """CanLoadBam.loadSplitsAndReads (load/.../CanLoadBam.scala:268-302): the splits
    (first record of every non-empty partition, sliding2 with Pos(fileSize, 0)) and
    the per-partition record counts.  A file larger than sharded.RESIDENT_MAX compressed bytes
    is memory-mapped and streamed through HBM (windows cut at split starts, each split decided
    in its window) instead of being held resident."""
    from . import sharded  # (sharded builds on this module)
    size = os.path.getsize(path_or_bytes) if isinstance(path_or_bytes, (str, os.PathLike)) else len(path_or_bytes)
    if size > sharded.RESIDENT_MAX:
        splits, counts, _ = sharded.load_splits_and_reads(
            path_or_bytes, split_size, ctx=ctx, rank=0, world=1, bgzf_blocks_to_check=bgzf_blocks_to_check,
            reads_to_check=reads_to_check, max_read_size=max_read_size)
        return splits, counts
    L = _Loaded(path_or_bytes, ctx, reads_to_check)
    try:
        sh = L.shard
        # every split in one batch (FindBlockStart + FindRecordStart + counts on the device)
        status, v, n, _ = sh.split_starts(file_splits(L.data.size, split_size), bgzf_blocks_to_check,
                                          reads_to_check, max_read_size)
        bad = np.flatnonzero(status)
        if bad.size:
            raise SparkBamError(int(status[bad[0]]), f"split {int(bad[0])}")
        counts = [int(x) for x in n]
        firsts = [Pos.from_htsjdk(int(x)) for x, c in zip(v, n) if c > 0]
        ends = firsts[1:] + [Pos(L.data.size, 0)]
        return [Split(a, b) for a, b in zip(firsts, ends)], counts
    finally:
        L.close()


def load_reads(path_or_bytes, ctx=None, reads_to_check=DEFAULT_READS_TO_CHECK, window=None):
    """CanLoadBam.loadReads (load/.../CanLoadBam.scala:244-264) on one device: every
    record of the file's BAM stream, in file order, decoded on the GPU into a columnar
    `Reads` batch (RecordStream.scala:16-41 semantics: records from the first one after
    the header while they start before the stream's end).  The eager bitmap of the
    record range is computed first, so record starts come from it in parallel (verified
    against the chain) rather than from a sequential chain walk.  A file larger than
    sharded.RESIDENT_MAX (or with `window` given) is decoded a window at a time (iter_reads)
    and the batches joined."""
    from . import sharded
    size = os.path.getsize(path_or_bytes) if isinstance(path_or_bytes, (str, os.PathLike)) else len(path_or_bytes)
    if window is not None or size > sharded.RESIDENT_MAX:
        own_ctx = ctx is None
        ctx = ctx or Context(0)
        try:
            batches = list(iter_reads(path_or_bytes, window=window or sharded.STREAM_WINDOW, ctx=ctx,
                                      reads_to_check=reads_to_check))
            names = file_header(ctx, _file_array(path_or_bytes))[0]
        finally:
            if own_ctx:
                ctx.close()
        return Reads.concat(batches, names)
    L = _Loaded(path_or_bytes, ctx, reads_to_check)
    try:
        sh = L.shard
        end = sh.flat_size
        for b in sh.blocks():
            if b[5] & 1:  # BLOCK_EMPTY: the stream ends at its flat start
                end = b[3]
                break
        sh.check_eager(L.header_end, end, reads_to_check, want_bits=False)
        cols = sh.records(L.header_end, end)
        return Reads(cols, L.names)
    finally:
        L.close()


def _vpos_of(flat, blocks):
    """htsjdk vpos of flat positions (numpy) from a shard's block table (Pos.scala's canonical
    form: a record at a block's end is Pos(next block, 0); empty blocks never hold one)."""
    blk = np.asarray([(b[0], b[3], b[2]) for b in blocks if b[2] > 0], dtype=np.int64).reshape(-1, 3)
    if flat.size == 0 or blk.size == 0:
        return np.zeros(flat.size, dtype=np.uint64)
    f = flat.astype(np.int64)
    i = np.searchsorted(blk[:, 1], f, side="right") - 1
    return (blk[i, 0].astype(np.uint64) << np.uint64(16)) | (f - blk[i, 1]).astype(np.uint64)


def iter_reads(path_or_bytes, window=None, halo=4 << 20, ctx=None, reads_to_check=DEFAULT_READS_TO_CHECK):
    """CanLoadBam.loadReads (load/.../CanLoadBam.scala:244-264) over a file of any size: the
    records from the first one after the header while they start before the stream's end
    (RecordStream.scala:16-41), decoded on the GPU a window of `window` compressed bytes at a
    time; yields one columnar `Reads` batch per window, in file order, each with a `vpos` column
    (htsjdk virtual offsets; `flat` is window-relative).  A window starts at the block of the
    previous window's chain exit, so batches never overlap."""
    window = int(window or STREAM_WINDOW)
    data = _file_array(path_or_bytes)
    size = int(data.size)
    own_ctx = ctx is None
    ctx = ctx or Context(0)
    try:
        names, contig_len, header_end = file_header(ctx, data)
        lo, start = 0, None  # window start (a block) and the record to start from (vpos; None: after the header)
        while lo < size:
            hi = lo + window
            while True:
                end = min(size, hi + halo)
                sh = ctx.shard(np.ascontiguousarray(data[lo:end]), file_offset=lo, file_size=size)
                try:
                    sh.set_contigs(contig_len)
                    sh.index(lo)
                    sh.inflate()
                    blocks = sh.blocks()
                    E = sh.flat_bound(hi)
                    if end < size and E == sh.flat_size:
                        raise SparkBamError(SBH_E_NEED_HALO, "no block past the window in the halo")
                    f = header_end if start is None else sh.flat_of(start >> 16, start & 0xFFFF)
                    seg = next((b[3] for b in blocks if b[5] & 1 and b[3] >= f), None)  # an empty block ends the stream
                    last = seg is not None and seg <= E or end == size and E == sh.flat_size
                    if seg is not None:
                        E = min(E, seg)
                    sh.check_eager(f, E, reads_to_check, want_bits=False)
                    cols = sh.records(f, E) if E > f else None
                    n, x = sh.chain_from(f, E) if E > f else (0, f)
                    if not last and x >= sh.flat_size:
                        raise SparkBamError(SBH_E_NEED_HALO, "the chain leaves the halo")
                    nxt = None if last else int(Pos(*sh.pos_of(x)).to_htsjdk())
                    break
                except SparkBamError as err:
                    if err.code != SBH_E_NEED_HALO or end >= size:
                        raise
                    halo *= 4
                finally:
                    sh.close()
            if cols is not None and cols["flat"].size:
                yield Reads(cols, names)
            if last:
                return
            start, lo = nxt, nxt >> 16
    finally:
        if own_ctx:
            ctx.close()


def load_bam_count(path_or_bytes, split_size=DEFAULT_SPLIT_SIZE, ctx=None, **kw):
    """sc.loadBam(path, splitSize).count (CanLoadBam.scala:196-266; CountReads)."""
    _, counts = load_splits_and_reads(path_or_bytes, split_size, ctx, **kw)
    return sum(counts)


DEFAULT_BLOCKS_SPLIT_SIZE = 2 << 20  # Blocks.apply's maxSplitSize(2 MB) (check/.../check/Blocks.scala:74-78)
STREAM_WINDOW = int(os.environ.get("SBH_STREAM_WINDOW", str(1 << 30)))  # compressed bytes per HBM window


def _file_array(path_or_bytes):
    """The whole file as numpy uint8: memory-mapped for a path (pages are read as windows
    move through HBM, never all at once)."""
    if isinstance(path_or_bytes, np.ndarray):
        return path_or_bytes
    if isinstance(path_or_bytes, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(path_or_bytes), dtype=np.uint8)
    return np.memmap(path_or_bytes, dtype=np.uint8, mode="r")


def file_header(ctx, data):
    """Header(path) (check/.../header/Header.scala:26-60) from the file's leading blocks inflated
    on the device: (contig names, contig lengths, flat end of the header)."""
    size = int(data.size)
    n = min(size, 1 << 20)
    while True:
        sh = ctx.shard(np.ascontiguousarray(data[:n]), file_offset=0, file_size=size)
        try:
            sh.index(0)
            sh.inflate()
            try:
                return parse_bam_header(sh.read_flat(0, sh.flat_size))
            except (IndexError, ValueError):
                if n >= size:
                    raise
        finally:
            sh.close()
        n = min(size, n * 4)


def _in_ranges(ranges, x):
    return ranges is None or any(a <= x < b for a, b in ranges)


def blocks(path_or_bytes, split_size=None, ranges=None, blocks_path=None, ctx=None,
           bgzf_blocks_to_check=DEFAULT_BGZF_BLOCKS_TO_CHECK):
    """Blocks.apply (check/src/main/scala/org/hammerlab/bam/check/Blocks.scala:47-208): the BGZF
    blocks the all-positions modes examine, as (partitions, bounds) -- partitions a list of
    [Metadata, ...] per partition, bounds the [(start, end)] byte range of each.

    With a `.blocks` file (`blocks_path`, default the BAM path + ".blocks"): its blocks whose start
    lies in `ranges`, partitioned by their cumulative compressed size / split_size (:86-139).
    Without one: the file is cut every split_size bytes, the splits that meet `ranges` are kept,
    and each one's blocks are FindBlockStart(split start) then MetadataStream while the block
    start is < the split end (:141-206), found on the device (sbh_find_blocks)."""
    split = int(split_size or DEFAULT_BLOCKS_SPLIT_SIZE)
    if blocks_path is None and isinstance(path_or_bytes, (str, os.PathLike)):
        blocks_path = str(path_or_bytes) + ".blocks"
    if blocks_path is not None and os.path.exists(blocks_path):
        metas = []
        with open(blocks_path) as f:
            for line in f:
                if not line.strip():
                    continue
                parts = line.strip().split(",")
                if len(parts) != 3:
                    raise ValueError(f"Bad blocks-index line: {line.strip()}")
                m = Metadata(int(parts[0]), int(parts[1]), int(parts[2]))
                if _in_ranges(ranges, m.start):
                    metas.append(m)
        # partition = (compressed bytes of the blocks before it) / split_size; the partition count is
        # the last block's partition + 1 (as BlocksTest pins it: "block boundaries" has 5 partitions
        # for blocks at offsets 0, 25228, 50313 of 74344 bytes at a 10 KiB split size)
        out, off = [], 0
        for m in metas:
            k = off // split
            out += [[] for _ in range(k + 1 - len(out))]
            out[k].append(m)
            off += m.compressed_size
        return out, [(i * split, (i + 1) * split) for i in range(len(out))]
    data = _file_array(path_or_bytes)
    size = int(data.size)
    idxs = [i for i in range(-(-size // split))
            if ranges is None or any(a < (i + 1) * split and b > i * split and a < b for a, b in ranges)]
    own_ctx = ctx is None
    ctx = ctx or Context(0)
    try:
        found = ctx.find_blocks(data, [(i * split, min(size, (i + 1) * split)) for i in idxs], bgzf_blocks_to_check)
    finally:
        if own_ctx:
            ctx.close()
    out = [[] for _ in idxs]
    for k, start, cs, us in found:
        if _in_ranges(ranges, start):
            out[k].append(Metadata(start, cs, us))
    return out, [(i * split, (i + 1) * split) for i in idxs]


def _all_positions(path_or_bytes, ranges, ctx, reads_to_check, split_size, blocks_path, window, **kw):
    """Blocks.apply, then every position of those blocks through sbh_check_stream (HBM windows
    of `window` compressed bytes, whatever the file size)."""
    data = _file_array(path_or_bytes)
    own_ctx = ctx is None
    ctx = ctx or Context(0)
    try:
        parts, _ = blocks(path_or_bytes if not isinstance(path_or_bytes, (bytes, bytearray, memoryview))
                          else data, split_size, ranges, blocks_path, ctx)
        starts = [m.start for p in parts for m in p]
        _, contig_len, _ = file_header(ctx, data)
        return ctx.check_stream(data, contig_len, starts, window=window or STREAM_WINDOW,
                                reads_to_check=reads_to_check, **kw)
    finally:
        if own_ctx:
            ctx.close()


def check_bam(path_or_bytes, records=None, ranges=None, ctx=None, reads_to_check=DEFAULT_READS_TO_CHECK,
              split_size=None, blocks_path=None, window=None):
    """CheckBam -s (cli/.../check/eager/CheckBam.scala + CheckerApp.scala:65-227): the eager
    checker at every position of Blocks.apply's blocks vs the `.records` truth.  `records` is a
    list of (blockPos, offset); returns the summary numbers.  Any file size: the blocks move
    through HBM in windows (sbh_check_stream)."""
    truth = None
    if records is not None:
        truth = np.sort(np.asarray([(b << 16) | o for b, o in records], dtype=np.uint64))
    r = _all_positions(path_or_bytes, ranges, ctx, reads_to_check, split_size, blocks_path, window,
                       truth_vpos=truth)
    out = {"positions": r["positions"], "compressed": r["comp_bytes"], "n_windows": r["n_windows"]}
    if truth is None:
        return dict(out, reads=r["n_true"], true_positives=r["n_true"], false_positives=0, false_negatives=0,
                    fp_positions=[], fn_positions=[])
    if r["unknown"]:
        raise SparkBamError(19, f"{r['unknown']} .records positions are not block starts of this file")
    return dict(out, reads=r["tp"] + r["fn"], true_positives=r["tp"], false_positives=r["fp"],
                false_negatives=r["fn"], fp_positions=[Pos.from_htsjdk(int(v)) for v in r["fp_vpos"]],
                fn_positions=[Pos.from_htsjdk(int(v)) for v in r["fn_vpos"]])


def full_check(path_or_bytes, ranges=None, ctx=None, reads_to_check=DEFAULT_READS_TO_CHECK, split_size=None,
               blocks_path=None, window=None):
    """FullCheck (cli/.../check/full/FullCheck.scala:88-329) aggregation over Blocks.apply's
    blocks: Counts per numNonZeroFields, totals, and the critical (1-flag) / close (2-flag)
    positions.  Any file size (sbh_check_stream)."""
    r = _all_positions(path_or_bytes, ranges, ctx, reads_to_check, split_size, blocks_path, window, full=True)
    counts = r["counts"]
    totals = dict(zip(FLAG_NAMES, counts.sum(axis=0).astype(np.int64).tolist()))
    return {"positions": r["positions"], "compressed": r["comp_bytes"], "n_success": r["n_success"],
            "counts_by_nnz": counts, "rbe_by_nnz": r["rbe"], "totals": totals, "n_windows": r["n_windows"],
            "close": [(Pos.from_htsjdk(int(v)), int(w)) for v, w in zip(r["close_vpos"], r["close_word"])]}


def flags_of(word):
    return [FLAG_NAMES[i] for i in range(19) if word & (1 << i)]


def reads_before_error(word):
    return (word >> FULL_N_SHIFT) & 0x3FF


def word_flags_mask(word):
    return word & FULL_FLAGS_MASK


def here():
    return os.path.dirname(os.path.abspath(__file__))


def htsjdk_rewrite(path_or_bytes, out_path=None, read_ranges=None, ctx=None, level=5):
    """HTSJDKRewrite (cli/src/main/scala/org/hammerlab/bam/rewrite/HTSJDKRewrite.scala:40-67):
    the BAM's uncompressed stream -- header, then every record (or only those whose index is
    in `read_ranges`, a collection supporting `in`, like the reference's `-r` IntRanges,
    :48-58) -- re-cut into 65498-byte BGZF members on the GPU (sbh_bgzf_compress) plus the
    EOF member.  Records pass through byte-for-byte (htsjdk's decode/re-encode is the
    identity on the records of a BAM it wrote).  Returns the file bytes (numpy uint8); writes
    them to out_path when given.  The `-b`/`-i` index side-outputs are the CLI's
    `index-blocks` / `index-records` run on the result.

    The members are byte-identical to htsjdk's: cut at 65498 uncompressed bytes and each
    deflated as java.util.zip.Deflater(5, nowrap) = zlib 1.2.11 deflate_slow does (zdeflate.hip),
    so the file, `.blocks` and `.records` equal HTSJDKRewriteTest's fixtures.  `level` picks
    another zlib level (4..9, 0 = stored) or -1 for this library's faster, non-zlib coder."""
    L = _Loaded(path_or_bytes, ctx)
    try:
        sh = L.shard
        if read_ranges is None:
            out, _, _ = L.ctx.bgzf_compress(sh.flat_ptr(), sh.flat_size, level=level)
        else:
            flat = sh.read_flat()
            starts = sh.records(L.header_end, sh.flat_size)["flat"].astype(np.int64)
            ends = np.append(starts[1:], np.int64(sh.flat_size))
            idx = np.arange(starts.size)
            sel = np.asarray(read_ranges, dtype=np.int64) if isinstance(read_ranges, range) else \
                np.fromiter((int(i) for i in read_ranges), dtype=np.int64)  # any collection (IntRanges)
            keep = idx[np.isin(idx, sel)]
            parts = [flat[:L.header_end]] + [flat[starts[i]:ends[i]] for i in keep]
            out, _, _ = L.ctx.bgzf_compress(np.concatenate(parts), level=level)
    finally:
        L.close()
    if out_path is not None:
        with open(out_path, "wb") as f:
            f.write(out.tobytes())
    return out
