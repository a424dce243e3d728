"""Python twin of the Scala load-API facade (jni/Native.scala `GpuCanLoadBam`,
`GpuSplitPartition`, `GpuIntervalsPartition`): the same C-ABI calls in the same order, per
Spark task, so the tests can run the facade's exact call sequence on the GPU.

The reference's partitioning is kept: one task per Hadoop FileSplit (`SplitRDD(FileSplits.
asJava(path, splitSize))`, load/.../CanLoadBam.scala:205,314) for loadBam / loadSplitsAndReads /
loadReadsAndPositions / loadReads, one per `cappedCostGroups` chunk group for loadBamIntervals
(:105-112).  A task's records come back as a columnar `Reads` batch with a `vpos` column (the
Scala facade builds htsjdk SAMRecords from the same record starts and bytes).

Failures are the reference's exceptions: HeaderSearchFailedException(path, start,
positionsAttempted) from FindBlockStart, NoReadFoundException(path, blockStart, maxReadSize) from
FindRecordStart (check/.../spark/FindRecordStart.scala:11-30,66-71).
"""
import os

import numpy as np

from ._lib import (SBH_E_BAD_RECORD, SBH_E_NEED_HALO, SBH_E_NOT_FOUND, HeaderSearchFailedException,
                   NoReadFoundException, SparkBamError)
from .api import (DEFAULT_BGZF_BLOCKS_TO_CHECK, DEFAULT_MAX_READ_SIZE, DEFAULT_READS_TO_CHECK, Pos, Split,
                  file_splits)
from .api import DEFAULT_SPLIT_SIZE as DEFAULT_MAX_SPLIT_SIZE
from .device import Context, PinnedBuffer
from .intervals import (DEFAULT_COMPRESSION_RATIO, _flat_of_pos, capped_cost_groups, chunk_size,
                        get_interval_chunks, parse_loci, read_bai)
from .intervals import DEFAULT_SPLIT_SIZE
from .records import Reads, record_columns


def _reader(path):
    from .sharded import bytes_reader, file_reader
    if isinstance(path, (bytes, bytearray, memoryview, np.ndarray)):
        return bytes_reader(path), "<bytes>"
    return file_reader(path), str(path)


def _empty():
    cols = record_columns()
    cols["vpos"] = np.zeros(0, np.uint64)
    return cols


class SplitWorker:
    """One task thread's reusable device state (jni/Native.scala `GpuSplitWorker`): a page-locked
    buffer the split's bytes are read into and ONE shard whose device buffers (compressed bytes,
    tokens, flat bytes, bitmap, block table, record columns) serve every split the thread runs
    (sbh_shard_load, grow-only), so a split costs no host or device allocation.  A worker belongs
    to one thread at a time (include/sparkbam.h, threading); a context is shared by all of them."""

    def __init__(self, ctx, size, contigs, device_file=None):
        self.ctx, self.size = ctx, int(size)
        self.contigs = np.ascontiguousarray(np.asarray(contigs, dtype=np.int32))
        self.sh = None
        self.pin = None
        self.out_pin = None  # page-locked landing buffer of the record starts / bytes copied out
        # device_file: a device pointer to the whole file's bytes already in HBM (the facade bench's
        # resident mode: the split's bytes are copied device-to-device, no host read or H2D)
        self.device_file = device_file

    def load(self, read, lo, hi):
        """The shard holding file bytes [lo, hi), read into the page-locked buffer first."""
        n = hi - lo
        if self.device_file is not None:
            if self.sh is None:
                self.sh = self.ctx.shard(self.device_file + lo, file_offset=lo, file_size=self.size, on_device=True,
                                         nbytes=n)
                self.sh.set_contigs(self.contigs)
            else:
                self.sh.load(self.device_file + lo, lo, on_device=True, nbytes=n)
            return self.sh
        if self.pin is None or self.pin.array.size < n:
            if self.pin is not None:
                self.pin.close()
            self.pin = PinnedBuffer(max(n, 1 << 20) + (n >> 3))  # (room for a grown halo)
        buf = self.pin.array[:n]
        np.copyto(buf, read(lo, hi))
        if self.sh is None:
            self.sh = self.ctx.shard(buf, file_offset=lo, file_size=self.size)
            self.sh.set_contigs(self.contigs)  # (kept across sbh_shard_load)
        else:
            self.sh.load(buf, lo)
        return self.sh

    def split(self, read, path, start, end, bgzf_blocks_to_check=DEFAULT_BGZF_BLOCKS_TO_CHECK,
              reads_to_check=DEFAULT_READS_TO_CHECK, max_read_size=DEFAULT_MAX_READ_SIZE, decode=True,
              halo0=1 << 20):
        """GpuSplitPartition: loadReadsAndPositions' body for the FileSplit [start, end)
        (CanLoadBam.scala:316-356) in one library call (sbh_split_records), the halo grown x4
        while an answer needs bytes past it.  Returns the split's records (columns + vpos; only
        flat + vpos without decode)."""
        halo = halo0
        while True:
            sh = self.load(read, start, min(self.size, end + halo))
            try:
                info, cols = sh.split_records(start, end, bgzf_blocks_to_check, reads_to_check, max_read_size, decode,
                                          flat_out=None if decode else self._flat_buf)
            except HeaderSearchFailedException as e:
                raise e.with_path(path)
            except NoReadFoundException as e:
                raise e.with_path(path)
            except SparkBamError as e:
                # a record (or the chain's next one) past the resident bytes: more halo
                if e.code not in (SBH_E_NEED_HALO, SBH_E_NOT_FOUND, SBH_E_BAD_RECORD) or end + halo >= self.size:
                    raise
                halo *= 4
                continue
            self.last = info  # (cols["vpos"]: the starts' virtual positions, from the device)
            return cols

    def _flat_buf(self, n):
        """n u64 slots of the worker's page-locked landing buffer (the record starts' copy-out
        lands in page-locked memory: DMA, no runtime staging); returned as a fresh array."""
        self._grow_out(8 * n)
        return self.out_pin.array[:8 * n].view(np.uint64)

    def _grow_out(self, nbytes):
        if self.out_pin is None or self.out_pin.array.size < nbytes:
            if self.out_pin is not None:
                self.out_pin.close()
            self.out_pin = PinnedBuffer(max(int(nbytes * 1.25), 1 << 20))

    def fetch_record_bytes(self, flat):
        """What jni/Native.scala's GpuRecordIterator copies out of HBM: the bytes from the first
        record to the end of the last one (into the worker's page-locked buffer; a view of it).
        `flat` = the split's record starts."""
        sh = self.sh
        last = int(flat[-1])
        l4 = int(sh.read_flat(last, 4).view(np.uint32)[0])
        lo, hi = int(flat[0]), last + 4 + l4
        starts = np.array(flat, copy=True)  # (the starts live in the same landing buffer)
        self._grow_out(hi - lo)
        sh.read_flat_into(lo, hi - lo, self.out_pin.array)
        return starts, self.out_pin.array[:hi - lo]

    def close(self):
        if self.sh is not None:
            self.sh.close()
            self.sh = None
        for b in (self.pin, self.out_pin):
            if b is not None:
                b.close()
        self.pin = self.out_pin = None


def split_partition(ctx, read, size, path, start, end, contigs, bgzf_blocks_to_check=DEFAULT_BGZF_BLOCKS_TO_CHECK,
                    reads_to_check=DEFAULT_READS_TO_CHECK, max_read_size=DEFAULT_MAX_READ_SIZE, halo0=1 << 20,
                    worker=None):
    """GpuSplitPartition: loadReadsAndPositions' body for the FileSplit [start, end)
    (CanLoadBam.scala:316-356).  Returns the split's records (columns + vpos).  `worker`: the
    calling thread's SplitWorker (one is made for the call when absent)."""
    own = worker is None
    w = worker or SplitWorker(ctx, size, contigs)
    try:
        return w.split(read, path, start, end, bgzf_blocks_to_check, reads_to_check, max_read_size, True, halo0)
    finally:
        if own:
            w.close()


def split_partition_calls(ctx, read, size, path, start, end, contigs, bgzf_blocks_to_check=DEFAULT_BGZF_BLOCKS_TO_CHECK,
                          reads_to_check=DEFAULT_READS_TO_CHECK, max_read_size=DEFAULT_MAX_READ_SIZE, halo0=1 << 20):
    """The same split as separate C-ABI calls (round 5's GpuSplitPartition: a shard per split,
    FindBlockStart, index, inflate, flat_bound, FindRecordStart, check_eager, records_scan), kept
    as the cross-check of sbh_split_records and as the facade bench's "before" line."""
    halo = halo0
    while True:
        sh = ctx.shard(read(start, min(size, end + halo)), file_offset=start, file_size=size)
        try:
            sh.set_contigs(contigs)  # (GpuShard's constructor)
            try:
                b = sh.find_block_start(start, bgzf_blocks_to_check)
            except HeaderSearchFailedException as e:
                raise e.with_path(path)
            sh.index(b)  # indexAndInflate
            sh.inflate()
            owned = sh.flat_bound(end)
            at_eof = sh.file_offset + sh.n == size
            if not at_eof and owned == sh.flat_size:
                raise SparkBamError(SBH_E_NEED_HALO, f"no block past {end} in the halo")
            try:
                first, _ = sh.find_record_start(0, reads_to_check, max_read_size)
            except NoReadFoundException as e:
                raise e.with_path(path, start=b)
            if first >= owned:
                return _empty()
            sh.check_eager(0, owned, reads_to_check, want_bits=False)
            cols = sh.records(first, owned)
            return cols
        except SparkBamError as e:
            if e.code not in (SBH_E_NEED_HALO, SBH_E_NOT_FOUND, SBH_E_BAD_RECORD) or end + halo >= size:
                raise
            halo *= 4
        finally:
            sh.close()


def load_reads_and_positions(path, split_size=DEFAULT_MAX_SPLIT_SIZE,
                             bgzf_blocks_to_check=DEFAULT_BGZF_BLOCKS_TO_CHECK,
                             reads_to_check=DEFAULT_READS_TO_CHECK, max_read_size=DEFAULT_MAX_READ_SIZE, ctx=None,
                             threads=1):
    """GpuCanLoadBam.loadReadsAndPositions: one partition per FileSplit, each a Reads batch
    (its vpos column = the reference's Pos keys).  threads > 1 runs the splits on that many
    concurrent task threads sharing the context (a Spark executor's cores)."""
    from .sharded import read_header
    read, name = _reader(path)
    size = read.size
    own = ctx is None
    ctx = ctx or Context(0)
    try:
        names, lens, _ = read_header(ctx, read, size)
        splits = file_splits(size, split_size)
        parts = [None] * len(splits)
        if threads <= 1:
            w = SplitWorker(ctx, size, lens)
            try:
                for i, (start, end) in enumerate(splits):
                    parts[i] = Reads(w.split(read, name, start, end, bgzf_blocks_to_check, reads_to_check,
                                             max_read_size), names)
            finally:
                w.close()
            return parts
        # an executor's concurrent tasks: `threads` task threads share the context, each with its
        # own worker (shard + pinned buffer), taking the splits in order like Spark's task queue
        import threading
        nxt = iter(range(len(splits)))
        lock = threading.Lock()
        errors = []

        def task():
            w = SplitWorker(ctx, size, lens)
            try:
                while True:
                    with lock:
                        i = next(nxt, None)
                    if i is None or errors:
                        return
                    start, end = splits[i]
                    parts[i] = Reads(w.split(read, name, start, end, bgzf_blocks_to_check, reads_to_check,
                                             max_read_size), names)
            except BaseException as e:  # (re-raised on the calling thread)
                errors.append(e)
            finally:
                w.close()

        ts = [threading.Thread(target=task) for _ in range(threads)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if errors:
            raise errors[0]
        return parts
    finally:
        if own:
            ctx.close()


def load_bam(path, split_size=DEFAULT_MAX_SPLIT_SIZE, bgzf_blocks_to_check=DEFAULT_BGZF_BLOCKS_TO_CHECK,
             reads_to_check=DEFAULT_READS_TO_CHECK, max_read_size=DEFAULT_MAX_READ_SIZE, ctx=None, threads=1):
    """GpuCanLoadBam.loadBam = loadReadsAndPositions(...).values: the partitions' records."""
    return load_reads_and_positions(path, split_size, bgzf_blocks_to_check, reads_to_check, max_read_size, ctx,
                                    threads)


def load_splits_and_reads(path, split_size=DEFAULT_MAX_SPLIT_SIZE, bgzf_blocks_to_check=DEFAULT_BGZF_BLOCKS_TO_CHECK,
                          reads_to_check=DEFAULT_READS_TO_CHECK, max_read_size=DEFAULT_MAX_READ_SIZE, ctx=None,
                          threads=1):
    """GpuCanLoadBam.loadSplitsAndReads (CanLoadBam.scala:268-302): BAMRecordRDD(splits, reads),
    splits = the first record of every non-empty partition, sliding2 with Pos(fileSize, 0)."""
    parts = load_reads_and_positions(path, split_size, bgzf_blocks_to_check, reads_to_check, max_read_size, ctx,
                                     threads)
    size = _reader(path)[0].size
    firsts = [Pos.from_htsjdk(int(p.cols["vpos"][0])) for p in parts if p.n]
    splits = [Split(a, b) for a, b in zip(firsts, firsts[1:] + [Pos(size, 0)])]
    return splits, parts


def load_reads(path, bgzf_blocks_to_check=DEFAULT_BGZF_BLOCKS_TO_CHECK, reads_to_check=DEFAULT_READS_TO_CHECK,
               max_read_size=DEFAULT_MAX_READ_SIZE, split_size=DEFAULT_MAX_SPLIT_SIZE, ctx=None):
    """GpuCanLoadBam.loadReads (CanLoadBam.scala:371-405): .bam through loadBam; the reference's
    sam / cram branches are not on the GPU path."""
    if isinstance(path, (str, os.PathLike)) and not str(path).endswith(".bam"):
        raise SparkBamError(1, f"Can't load reads from path on the GPU path: {path} (sam / cram stay the reference's)")
    return load_bam(path, split_size, bgzf_blocks_to_check, reads_to_check, max_read_size, ctx)


def intervals_partition(ctx, read, size, chunks, intervals, contigs, reads_to_check=DEFAULT_READS_TO_CHECK,
                        halo0=1 << 18, merge_gap=1 << 20):
    """GpuIntervalsPartition: one chunk group's records (CanLoadBam.scala:120-154); chunks whose
    block ranges lie within merge_gap share a shard, grown x4 while an answer needs more."""
    groups = []
    for c in chunks:
        lo, hi = c.start.block_pos, c.end.block_pos
        if groups and lo <= groups[-1][1] + merge_gap:
            groups[-1][1] = max(groups[-1][1], hi)
            groups[-1][2].append(c)
        else:
            groups.append([lo, hi, [c]])
    out = []
    for lo, hi, cs in groups:
        halo = halo0
        while True:
            sh = ctx.shard(read(lo, min(size, hi + halo)), file_offset=lo, file_size=size)
            try:
                sh.set_contigs(contigs)  # (GpuShard's constructor)
                sh.index(lo)  # indexAndInflate
                sh.inflate()
                fb = [_flat_of_pos(sh, c.start) for c in cs]
                fe = [min(_flat_of_pos(sh, c.end), sh.flat_size) for c in cs]
                if max(fe) > min(fb):
                    sh.check_eager(min(fb), max(fe), reads_to_check, want_bits=False)
                cols = sh.records_regions(list(zip(fb, fe)), intervals)
                out.append(cols)
                break
            except SparkBamError as e:
                if e.code not in (SBH_E_NEED_HALO, SBH_E_NOT_FOUND, SBH_E_BAD_RECORD) or hi + halo >= size:
                    raise
                halo *= 4
            finally:
                sh.close()
    return out


def load_bam_intervals(path, intervals, split_size=DEFAULT_SPLIT_SIZE,
                       estimated_compression_ratio=DEFAULT_COMPRESSION_RATIO, bai=None,
                       reads_to_check=DEFAULT_READS_TO_CHECK, ctx=None):
    """GpuCanLoadBam.loadBamIntervals(path, LociSet, splitSize, ratio): one partition per
    cappedCostGroups chunk group (getNumPartitions = max(1, groups)), each a Reads batch."""
    from .sharded import read_header
    read, _ = _reader(path)
    size = read.size
    index = read_bai(bai if bai is not None else str(path) + ".bai")
    own = ctx is None
    ctx = ctx or Context(0)
    try:
        names, lens, _ = read_header(ctx, read, size)
        names = list(names)
        loci = parse_loci(intervals, dict(zip(names, (int(x) for x in lens))))
        ivs = sorted((names.index(c), a, e) for c, rs in loci.items() for a, e in rs)
        chunks = get_interval_chunks(index, loci, names)
        groups = capped_cost_groups(chunks, lambda c: chunk_size(c, estimated_compression_ratio), float(split_size))
        parts = []
        for g in groups:
            batches = intervals_partition(ctx, read, size, g, ivs, lens, reads_to_check)
            parts.append(Reads.concat([Reads(b, names) for b in batches], names))
        return parts if parts else [Reads.concat([], names)]
    finally:
        if own:
            ctx.close()
