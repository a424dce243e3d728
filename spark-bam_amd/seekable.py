"""The seekable BGZF byte view on the GPU: Python twin of jni/Native.scala's `GpuSeekableStream`
(a `SeekableStream` whose blocks the device inflates) under the reference's own
`SeekableUncompressedBytes`, and of `GpuFindRecordStart` reading through the caller's view.

  bgzf/src/main/scala/org/hammerlab/bgzf/block/Stream.scala:79-121        SeekableStream, seek(newPos)
  bgzf/src/main/scala/org/hammerlab/bgzf/block/UncompressedBytes.scala:13-87  UncompressedBytesI /
                                                                          SeekableUncompressedBytes.seek(pos)
  bgzf/src/main/scala/org/hammerlab/bgzf/block/Block.scala:12-46          Block(bytes, start, compressedSize), idx
  check/src/main/scala/org/hammerlab/bam/spark/FindRecordStart.scala:11-63   FindRecordStart(path, start)(view)

The reference inflates one block per `_advance` with java.util.zip.Inflater and keeps the last
100 blocks in an LRU.  Here a WINDOW of blocks (the compressed bytes [p, p + window) plus a halo,
held in one reused shard) is indexed and inflated on the device in one pass, and its inflated
bytes are copied to the host once; the window is the cache -- a seek back into it (the load path
seeks to a split's first record right after FindRecordStart read past it, CanLoadBam.scala:349)
re-inflates nothing.  The channel position, `pos` (the next block's start), the empty block that
ends the stream (Stream.scala:56-58) and `curPos` rolling to Pos(next block, 0) once a block is
used up behave as the reference's.
"""
import numpy as np

from ._lib import SBH_E_NEED_HALO, SparkBamError
from .api import Pos

BLOCK_EMPTY = 1
BLOCK_TRUNCATED = 2


class Block:
    """bgzf Block (Block.scala:12-46): uncompressed bytes, compressed start and size, read index."""

    __slots__ = ("bytes", "start", "compressed_size", "idx")

    def __init__(self, data, start, compressed_size):
        self.bytes, self.start, self.compressed_size, self.idx = data, int(start), int(compressed_size), 0

    @property
    def uncompressed_size(self):
        return int(self.bytes.size)

    @property
    def pos(self):
        return Pos(self.start, self.idx)

    def has_next(self):
        return self.idx < self.bytes.size

    def __repr__(self):
        return f"Block({self.start}:0-{self.uncompressed_size};{self.compressed_size})"


class SeekableStream:
    """SeekableStream (Stream.scala:79-121) with the device inflating a window of blocks at a time.
    `read(lo, hi)` gives the file's compressed bytes [lo, hi) (sharded.file_reader /
    bytes_reader); `contigs` (optional) are the BAM header's contig lengths, for the checks
    FindRecordStart runs on the window's shard."""

    def __init__(self, ctx, read, window=16 << 20, halo=1 << 20, contigs=None):
        self.ctx, self.read, self.size = ctx, read, int(read.size)
        self.window, self.halo = int(window), int(halo)
        self.contigs = None if contigs is None else np.ascontiguousarray(np.asarray(contigs, dtype=np.int32))
        self.position = 0       # compressedBytes.position()
        self._head = None       # SimpleIterator's buffered next block
        self._done = False      # _advance returned None (until clear / seek)
        self.sh = None          # the reused window shard
        self.w_lo = self.w_hi = -1
        self._table = None      # {start: (ustart, csize, usize, flags)} of the window's blocks
        self._flat = None       # the window's inflated bytes, host copy
        self.windows_loaded = 0

    # ---- the window ---------------------------------------------------------------------------
    def _load(self, p, window=None):
        """Index + inflate the blocks from the block start p over [p, p + window + halo)."""
        window = self.window if window is None else window
        hi = min(self.size, p + window + self.halo)
        data = self.read(p, hi)
        if self.sh is None:
            self.sh = self.ctx.shard(data, file_offset=p, file_size=self.size)
        else:
            self.sh.load(data, p)
        if self.contigs is not None:
            self.sh.set_contigs(self.contigs)
        self.sh.index(p)
        self.sh.inflate()
        b = self.sh.block_arrays()
        self._table = {int(s): (int(u), int(c), int(z), int(f)) for s, u, c, z, f in
                       zip(b["start"], b["ustart"], b["csize"], b["usize"], b["flags"])}
        self._flat = self.sh.read_flat(0, self.sh.flat_size) if self.sh.flat_size else np.zeros(0, np.uint8)
        self.w_lo, self.w_hi = p, hi
        self.windows_loaded += 1

    def _block_at(self, p):
        """The window's block starting at p (loading a window there when p is not one of them)."""
        e = self._table.get(p) if self._table is not None else None
        if e is None or (e[3] & BLOCK_TRUNCATED):
            self._load(p)
            e = self._table.get(p)
        return e

    # ---- StreamI ----------------------------------------------------------------------------------
    def _advance(self):
        """StreamI._advance (Stream.scala:31-71): the block at the channel position, or None at EOF
        or at the empty block that ends the stream."""
        start = self.position
        if start >= self.size:
            return None  # (EOFException -> None)
        ustart, csize, usize, flags = self._block_at(start)
        self.position = start + csize
        if flags & BLOCK_EMPTY:
            return None  # dataLength == 2: the empty block at the end of the file
        return Block(self._flat[ustart:ustart + usize], start, csize)

    def has_next(self):
        if self._head is None and not self._done:
            self._head = self._advance()
            self._done = self._head is None
        return self._head is not None

    def next(self):
        if not self.has_next():
            raise StopIteration
        b, self._head = self._head, None
        return b

    def head(self):
        if not self.has_next():
            raise StopIteration
        return self._head

    @property
    def pos(self):
        """The start of the next block to be emitted (`def pos = head.start`)."""
        return self.head().start

    def clear(self):
        self._head, self._done = None, False

    def seek(self, new_pos):
        """Stream.scala:112-121: reposition unless already there; True when it moved."""
        if not self.has_next() or self.pos != new_pos:
            self.clear()
            self.position = int(new_pos)
            return True
        return False

    def __iter__(self):
        while self.has_next():
            yield self.next()

    def close(self):
        if self.sh is not None:
            self.sh.close()
            self.sh = None


class SeekableUncompressedBytes:
    """SeekableUncompressedBytes (UncompressedBytes.scala:13-87): the stream's bytes, flattened,
    with curPos, stopAt and seek(pos); plus the ByteChannel reads the reference's callers use
    (read / get_int / skip / position)."""

    def __init__(self, stream):
        self.block_stream = stream
        self._cur = None
        self._stop_at = None
        self.position = 0  # bytes read through the channel view

    # the flattening `level` iterator: the current block with a byte left, advancing lazily
    def cur_block(self):
        while self._cur is None or not self._cur.has_next():
            if not self.block_stream.has_next():
                self._cur = None
                return None
            self._cur = self.block_stream.next()
        return self._cur

    @property
    def cur_pos(self):
        b = self.cur_block()
        return None if b is None else b.pos

    def stop_at(self, pos):
        self._stop_at = Pos(*pos)

    def reset(self):
        self._stop_at = None

    def clear(self):
        pass  # (no byte is buffered ahead of the current block's index)

    def has_next(self):
        p = self.cur_pos
        if p is None:
            return False
        return not (self._stop_at is not None and tuple(self._stop_at) <= tuple(p))

    def next(self):
        if not self.has_next():
            raise StopIteration
        b = self._cur
        v = int(b.bytes[b.idx])
        b.idx += 1
        self.position += 1
        return v

    def read(self, n):
        """n bytes (fewer at the end of the stream), crossing blocks as needed."""
        out = []
        while n > 0 and self.has_next():
            b = self._cur
            k = min(n, b.uncompressed_size - b.idx)
            if self._stop_at is not None and self._stop_at.block_pos == b.start:
                k = min(k, max(0, self._stop_at.offset - b.idx))
                if k == 0:
                    break
            out.append(b.bytes[b.idx:b.idx + k])
            b.idx += k
            n -= k
            self.position += k
        return np.concatenate(out) if out else np.zeros(0, np.uint8)

    def get_int(self):
        return int(self.read(4).view("<i4")[0])

    def skip(self, n):
        return self.read(n).size

    def seek(self, pos):
        """SeekableUncompressedBytes.seek (UncompressedBytes.scala:65-76)."""
        pos = Pos(*pos)
        self.block_stream.seek(pos.block_pos)
        self._cur = None  # (uncompressedBytes.reset())
        self.clear()
        b = self.cur_block()
        if b is not None:
            b.idx = pos.offset

    def close(self):
        self.block_stream.close()


def seekable_uncompressed_bytes(ctx, read, window=16 << 20, halo=1 << 20, contigs=None):
    """SeekableUncompressedBytes(ch) (UncompressedBytes.scala:79-86) over a GPU SeekableStream."""
    return SeekableUncompressedBytes(SeekableStream(ctx, read, window, halo, contigs))


def find_record_start(path, start, view, reads_to_check=10, max_read_size=100000000):
    """FindRecordStart(path, start)(uncompressedBytes, ...) (FindRecordStart.scala:11-30) through the
    caller's view: the view is seeked to Pos(start, 0) (its window then holds `start`), and the
    first eager-true position within maxReadSize is searched on that window's shard.  The window
    grows x4 while the search needs bytes past it.  Raises NoReadFoundException(path, start,
    maxReadSize) like the reference; leaves the view at the found position."""
    from ._lib import NoReadFoundException
    s = view.block_stream
    if s.contigs is None:
        raise SparkBamError(1, "find_record_start: the view's stream needs the header's contig lengths")
    view.seek(Pos(start, 0))
    window = s.window
    while True:
        try:
            if s.sh is None or start not in (s._table or {}):
                s._load(start, window)
            f0 = s._table[start][0]
            try:
                f, delta = s.sh.find_record_start(f0, reads_to_check, max_read_size)
            except NoReadFoundException as e:
                raise e.with_path(path, start=start)
            bp, off = s.sh.pos_of(f)
            found = Pos(bp, off)
            view.seek(found)
            return found
        except SparkBamError as e:
            if e.code != SBH_E_NEED_HALO or s.w_hi >= s.size:
                raise
            window *= 4
            s._load(start, window)
