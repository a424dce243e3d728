"""Context / Shard: thin owners of the C-ABI handles (include/sparkbam.h)."""
import ctypes as C
import weakref

import numpy as np

from .records import record_columns

from ._lib import (SBH_OK, SbhBlock, SbhCheckOpts, SbhCheckResult, SbhRecordsOut, SbhRecordsSizes,
                   SbhShardResult, SbhSplitRecordsResult, SbhStreamOpts, SbhStreamResult, SparkBamError, error_for,
                   lib)


def _check(ctx_handle, rc):
    if rc != SBH_OK:
        msg = lib().sbh_last_error(ctx_handle) if ctx_handle else b""
        fields = ()
        if ctx_handle:
            code, f = C.c_int32(), (C.c_int64 * 4)()
            n = lib().sbh_last_error_detail(ctx_handle, C.byref(code), f, 4)
            if code.value == rc:
                fields = tuple(f[:min(n, 4)])
        raise error_for(rc, (msg or b"").decode(errors="replace"), fields)


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class PinnedBuffer:
    """Page-locked host bytes (sbh_host_alloc) as a numpy uint8 array (`.array`): compressed
    bytes in it stream to HBM with copies that overlap the kernels."""

    def __init__(self, n):
        p = C.c_void_p()
        rc = lib().sbh_host_alloc(int(n), C.byref(p))
        if rc != SBH_OK:
            raise SparkBamError(rc, f"cannot pin {n} host bytes")
        self.p = p
        self.array = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), shape=(int(n),))

    def close(self):
        if self.p:
            self.array = None
            lib().sbh_host_free(self.p)
            self.p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Context:
    """One per device (sbh_ctx_create).  Owns a HIP stream unless one is supplied."""

    def __init__(self, device=0, stream=None):
        h = C.c_void_p()
        rc = lib().sbh_ctx_create(device, C.byref(h))
        if rc != SBH_OK:
            raise SparkBamError(rc, f"cannot create a context on device {device}")
        self.h = h
        self.device = device
        self._shards = weakref.WeakSet()
        if stream is not None:
            _check(self.h, lib().sbh_ctx_set_stream(self.h, C.c_void_p(stream)))

    def synchronize(self):
        _check(self.h, lib().sbh_ctx_synchronize(self.h))

    def close(self):
        """Destroys every live shard first (a shard must not outlive its context)."""
        if self.h:
            for sh in list(self._shards):
                sh.close()
            lib().sbh_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def bgzf_compress(self, data, nbytes=None, level=5):
        """BGZF-compress a flat byte stream (sbh_bgzf_compress_level; htsjdk BlockCompressedOutputStream
        as driven by HTSJDKRewrite.scala:62-67).  level 5 = htsjdk's bytes exactly (zlib 1.2.11
        deflate_slow), 4 / 6..9 = zlib at that level, 0 = stored, -1 = this library's faster coder.
        data: numpy uint8 (host) or a device pointer (int) with nbytes.  Returns (file bytes as
        numpy uint8, number of data members, kernel ms)."""
        on_dev = isinstance(data, int)
        n = int(nbytes) if on_dev else int(data.size)
        cap = lib().sbh_bgzf_compress_bound(n)
        out = np.empty(cap, dtype=np.uint8)
        size, nb, ms = C.c_uint64(), C.c_uint64(), C.c_float()
        src = C.c_void_p(data) if on_dev else _ptr(np.ascontiguousarray(data, dtype=np.uint8))
        _check(self.h, lib().sbh_bgzf_compress_level(self.h, src, n, 1 if on_dev else 0, int(level), _ptr(out), cap,
                                                     C.byref(size), C.byref(nb), C.byref(ms)))
        return out[:size.value], nb.value, ms.value

    def run_stream(self, comp, contig_len, file_offset=0, file_size=None, own_end=None, index_start=None,
                   window=1 << 30, halo=4 << 20, reads_to_check=10, max_read_size=100000000, want_bits=False,
                   splits=None, verify_crc=False, bgzf_blocks_to_check=5):
        """sbh_run_stream2: the per-shard hot path over host-resident compressed bytes `comp`
        (numpy uint8, ideally pinned) = file bytes [file_offset, file_offset + comp.size),
        streamed through HBM in windows.  splits = [(start, end), ...] (file offsets inside the
        owned range): the windows are cut at split starts and every split gets sbh_split's
        (status, first_vpos, count) -> result["split_status" / "split_first_vpos" /
        "split_count"].  verify_crc: every owned block's CRC32 (result["crc_bad_blocks"]).
        Returns (result dict, eager bits or None)."""
        arr = np.ascontiguousarray(comp, dtype=np.uint8) if isinstance(comp, np.ndarray) else comp
        n = int(arr.size)
        file_size = file_offset + n if file_size is None else int(file_size)
        own_end = file_offset + n if own_end is None else int(own_end)
        cl = np.ascontiguousarray(np.asarray(contig_len, dtype=np.int32))
        bits = None
        if want_bits:
            bits = np.zeros(max(1, 4 * n + 64), dtype=np.uint8)  # > (flat + 7) / 8 at any ratio <= 32
        o = SbhStreamOpts()
        o.window, o.halo = int(window), int(halo)
        o.reads_to_check, o.max_read_size = reads_to_check, max_read_size
        o.bgzf_blocks_to_check, o.verify_crc = bgzf_blocks_to_check, 1 if verify_crc else 0
        keep = []
        if splits:
            st = np.ascontiguousarray([a for a, _ in splits], dtype=np.uint64)
            en = np.ascontiguousarray([b for _, b in splits], dtype=np.uint64)
            fv = np.zeros(st.size, np.uint64)
            cn = np.zeros(st.size, np.uint64)
            ss = np.zeros(st.size, np.int32)
            keep = [st, en, fv, cn, ss]
            o.split_start, o.split_end, o.n_splits = _ptr(st).value, _ptr(en).value, st.size
            o.split_first_vpos, o.split_count, o.split_status = _ptr(fv).value, _ptr(cn).value, _ptr(ss).value
        if bits is not None:
            o.out_bits, o.out_bits_cap = _ptr(bits).value, bits.size
        r = SbhStreamResult()
        _check(self.h, lib().sbh_run_stream2(self.h, _ptr(arr), n, int(file_offset), file_size,
                                             0xFFFFFFFFFFFFFFFF if index_start is None else int(index_start),
                                             own_end, _ptr(cl), int(cl.size), C.byref(o), C.byref(r)))
        out = {f: getattr(r, f) for f, _ in SbhStreamResult._fields_ if f != "stage_ms"}
        out["stage_ms"] = list(r.stage_ms)
        for k in ("first_vpos", "exit_vpos"):
            if out[k] == 0xFFFFFFFFFFFFFFFF:
                out[k] = None
        if keep:
            out["split_status"], out["split_first_vpos"], out["split_count"] = keep[4], keep[2], keep[3]
        if bits is not None:
            bits = bits[:(out["flat_bytes"] + 7) // 8]
        return out, bits

    def find_blocks(self, data, splits, bgzf_blocks_to_check=5, window=1 << 30):
        """Blocks.apply's unindexed branch (Blocks.scala:141-206) on the device (sbh_find_blocks):
        data = the whole file (numpy uint8, e.g. a memmap); splits = [(start, end), ...].  Returns
        [(split index, start, compressed size, uncompressed size), ...] in split order."""
        arr = data if isinstance(data, np.ndarray) else np.frombuffer(data, dtype=np.uint8)
        st = np.ascontiguousarray([a for a, _ in splits], dtype=np.uint64)
        en = np.ascontiguousarray([b for _, b in splits], dtype=np.uint64)
        # a realistic first guess (BAM blocks average 15-25 KB compressed); a file of smaller
        # blocks reports the count it needs and is asked again with that capacity
        cap = int(arr.size) // 16384 + 4096
        while True:
            out = (SbhBlock * cap)()
            n = C.c_uint64()
            _check(self.h, lib().sbh_find_blocks(self.h, _ptr(arr), int(arr.size), _ptr(st), _ptr(en), st.size,
                                                 int(bgzf_blocks_to_check), int(window), out, cap, C.byref(n)))
            if n.value <= cap:
                return [(int(b.ustart), int(b.start), int(b.csize), int(b.usize)) for b in out[:n.value]]
            cap = n.value

    def check_stream(self, data, contig_len, blocks, truth_vpos=None, full=False, window=1 << 30, halo=4 << 20,
                     reads_to_check=10, fp_cap=1 << 20, close_cap=1 << 22):
        """check-bam -s / full-check over the listed blocks of a file of any size, streamed through
        HBM in windows (sbh_check_stream): data = the whole file (numpy uint8, e.g. a memmap),
        blocks = file offsets of the block starts to check (ascending), truth_vpos = the `.records`
        positions as htsjdk vpos (ascending) or None.  Returns a dict of the result fields plus
        fp_vpos / fn_vpos and, with full, counts (21 x 19), rbe (21 x 64), close_vpos / close_word."""
        arr = data if isinstance(data, np.ndarray) else np.frombuffer(data, dtype=np.uint8)
        cl = np.ascontiguousarray(np.asarray(contig_len, dtype=np.int32))
        bl = np.ascontiguousarray(blocks, dtype=np.uint64)
        o = SbhCheckOpts()
        o.window, o.halo, o.reads_to_check, o.full = int(window), int(halo), int(reads_to_check), 1 if full else 0
        o.blocks, o.n_blocks = _ptr(bl).value, bl.size
        keep = [bl]
        fp = fn = None
        if truth_vpos is not None:
            tv = np.ascontiguousarray(truth_vpos, dtype=np.uint64)
            fp, fn = np.zeros(max(fp_cap, 1), np.uint64), np.zeros(max(fp_cap, 1), np.uint64)
            keep += [tv, fp, fn]
            o.truth_vpos, o.n_truth = _ptr(tv).value, tv.size
            o.fp_vpos, o.fn_vpos, o.fp_cap, o.fn_cap = _ptr(fp).value, _ptr(fn).value, fp_cap, fp_cap
        counts = rbe = cv = cw = None
        if full:
            counts, rbe = np.zeros(21 * 19, np.uint64), np.zeros(21 * 64, np.uint64)
            cv, cw = np.zeros(max(close_cap, 1), np.uint64), np.zeros(max(close_cap, 1), np.uint32)
            keep += [counts, rbe, cv, cw]
            o.counts, o.rbe_hist = _ptr(counts).value, _ptr(rbe).value
            o.close_vpos, o.close_word, o.close_cap = _ptr(cv).value, _ptr(cw).value, close_cap
        r = SbhCheckResult()
        _check(self.h, lib().sbh_check_stream(self.h, _ptr(arr), int(arr.size), _ptr(cl), int(cl.size), C.byref(o),
                                              C.byref(r)))
        out = {f: getattr(r, f) for f, _ in SbhCheckResult._fields_}
        if fp is not None:
            out["fp_vpos"], out["fn_vpos"] = fp[:min(r.fp, fp_cap)], fn[:min(r.fn, fp_cap)]
        if full:
            k = min(r.n_close, close_cap)
            out.update(counts=counts.reshape(21, 19), rbe=rbe.reshape(21, 64), close_vpos=cv[:k], close_word=cw[:k])
        return out

    def shard(self, comp, file_offset=0, file_size=None, on_device=False, nbytes=None):
        return Shard(self, comp, file_offset, file_size, on_device, nbytes)


class Shard:
    """Compressed bytes [file_offset, file_offset + n) of a BGZF file, resident in HBM."""

    def __init__(self, ctx, comp, file_offset=0, file_size=None, on_device=False, nbytes=None):
        self.ctx = ctx
        if on_device:
            ptr, n = int(comp), int(nbytes)
            src = C.c_void_p(ptr)
        else:
            arr = np.ascontiguousarray(np.frombuffer(comp, dtype=np.uint8)
                                       if not isinstance(comp, np.ndarray) else comp)
            n = int(arr.size)
            src = _ptr(arr)
            self._keep = arr
        self.n = n
        self.file_offset = int(file_offset)
        self.file_size = int(file_size if file_size is not None else file_offset + n)
        h = C.c_void_p()
        _check(ctx.h, lib().sbh_shard_create(ctx.h, src, n, self.file_offset, self.file_size,
                                             1 if on_device else 0, C.byref(h)))
        self.h = h
        self._keep = None
        ctx._shards.add(self)
        self.n_blocks = 0
        self.flat_size = 0

    def _c(self, rc):
        _check(self.ctx.h, rc)

    def close(self):
        if self.h:
            if self.ctx.h:
                lib().sbh_shard_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load(self, comp, file_offset, on_device=False, nbytes=None):
        """Replace the resident bytes with file bytes [file_offset, file_offset + n) of the same
        file, keeping the device buffers (sbh_shard_load): comp = host bytes (numpy uint8), or a
        device pointer (int) with nbytes when on_device."""
        if on_device:
            n = int(nbytes)
            self._c(lib().sbh_shard_load(self.h, C.c_void_p(int(comp)), n, int(file_offset), 1))
        else:
            arr = np.ascontiguousarray(comp, dtype=np.uint8)
            n = int(arr.size)
            self._c(lib().sbh_shard_load(self.h, _ptr(arr), n, int(file_offset), 0))
        self.n, self.file_offset = n, int(file_offset)
        self.n_blocks = self.flat_size = 0

    # -- bgzf --------------------------------------------------------------
    def find_block_start(self, start, bgzf_blocks_to_check=5):
        out = C.c_uint64()
        self._c(lib().sbh_find_block_start(self.h, start, bgzf_blocks_to_check, C.byref(out)))
        return out.value

    def index(self, start=None):
        nb, fs = C.c_uint64(), C.c_uint64()
        s = self.file_offset if start is None else start
        self._c(lib().sbh_index(self.h, s, C.byref(nb), C.byref(fs)))
        self.n_blocks, self.flat_size = nb.value, fs.value
        return self.n_blocks, self.flat_size

    def blocks(self):
        arr = (SbhBlock * max(self.n_blocks, 1))()
        if self.n_blocks:
            self._c(lib().sbh_get_blocks(self.h, 0, self.n_blocks, arr))
        return [(b.start, b.csize, b.usize, b.ustart, b.hsize, b.flags)
                for b in arr[: self.n_blocks]]

    def block_arrays(self):
        """The block table as numpy arrays {start, ustart, usize} (sbh_get_blocks into one
        structured array: no Python object per block)."""
        dt = np.dtype([("start", "<u8"), ("ustart", "<u8"), ("csize", "<u4"), ("hsize", "<u4"), ("usize", "<u4"),
                       ("flags", "<u4")])
        a = np.zeros(max(self.n_blocks, 1), dtype=dt)
        if self.n_blocks:
            self._c(lib().sbh_get_blocks(self.h, 0, self.n_blocks, a.ctypes.data_as(C.c_void_p)))
        a = a[:self.n_blocks]
        return {"start": a["start"], "ustart": a["ustart"], "usize": a["usize"].astype(np.uint64),
                "csize": a["csize"].astype(np.uint64), "flags": a["flags"]}

    def vpos_of_flat(self, flat):
        """Flat positions -> htsjdk virtual offsets over the block table (canonical: a position at
        a block's end is Pos(next block, 0); empty blocks hold no positions)."""
        b = self.block_arrays()
        live = b["usize"] > 0
        starts, ustarts = b["start"][live], b["ustart"][live]
        flat = np.asarray(flat, dtype=np.uint64)
        k = np.searchsorted(ustarts, flat, side="right") - 1
        return (starts[k] << np.uint64(16)) | (flat - ustarts[k])

    def inflate(self):
        bad = C.c_uint64()
        self._c(lib().sbh_inflate(self.h, C.byref(bad)))

    def verify_crc(self):
        """(blocks whose footer CRC32 differs from their inflated bytes, first such block's
        file offset) -- sbh_verify_crc."""
        n, f = C.c_uint64(), C.c_uint64()
        self._c(lib().sbh_verify_crc(self.h, C.byref(n), C.byref(f)))
        return n.value, f.value

    def flat_ptr(self):
        """Device pointer of the inflated flat bytes (sbh_flat_device_ptr)."""
        return lib().sbh_flat_device_ptr(self.h)

    def read_flat(self, flat=0, n=None):
        n = self.flat_size - flat if n is None else n
        out = np.empty(n, dtype=np.uint8)
        if n:
            self._c(lib().sbh_read_flat(self.h, flat, n, _ptr(out)))
        return out

    def read_flat_into(self, flat, n, out):
        """Flat bytes [flat, flat + n) into the host array `out` (e.g. a PinnedBuffer's array)."""
        if n:
            if out.size < n:
                raise ValueError("read_flat_into: buffer too small")
            self._c(lib().sbh_read_flat(self.h, int(flat), int(n), _ptr(out)))

    def flat_of(self, block_pos, offset=0):
        out = C.c_uint64()
        self._c(lib().sbh_flat_of(self.h, block_pos, offset, C.byref(out)))
        return out.value

    def pos_of(self, flat):
        bp, off = C.c_uint64(), C.c_uint32()
        self._c(lib().sbh_pos_of(self.h, flat, C.byref(bp), C.byref(off)))
        return bp.value, off.value

    def flat_bound(self, file_off):
        out = C.c_uint64()
        self._c(lib().sbh_flat_bound(self.h, file_off, C.byref(out)))
        return out.value

    # -- check ---------------------------------------------------------------
    def set_contigs(self, lens):
        a = np.ascontiguousarray(np.asarray(lens, dtype=np.int32))
        self._c(lib().sbh_set_contigs(self.h, _ptr(a), int(a.size)))

    def check_eager(self, begin=0, end=None, reads_to_check=10, want_bits=True):
        end = self.flat_size if end is None else end
        bits = np.zeros((end - begin + 7) // 8, dtype=np.uint8) if want_bits else None
        n = C.c_uint64()
        self._c(lib().sbh_check_eager(self.h, begin, end, reads_to_check, _ptr(bits), C.byref(n)))
        return n.value, bits

    def eager_bits(self, begin=0, end=None):
        """The eager bitmap the last check_eager()/run() left on the device, [begin, end)."""
        end = self.flat_size if end is None else end
        bits = np.zeros((end - begin + 7) // 8, dtype=np.uint8)
        self._c(lib().sbh_eager_bits(self.h, begin, end, _ptr(bits)))
        return bits

    def check_full(self, begin=0, end=None, reads_to_check=10, want_words=False, close_cap=1 << 20):
        end = self.flat_size if end is None else end
        words = np.zeros(end - begin, dtype=np.uint32) if want_words else None
        counts = np.zeros(21 * 19, dtype=np.uint64)
        rbe = np.zeros(21 * 64, dtype=np.uint64)
        close_flat = np.zeros(max(close_cap, 1), dtype=np.uint64)
        close_word = np.zeros(max(close_cap, 1), dtype=np.uint32)
        ns, nclose = C.c_uint64(), C.c_uint64()
        self._c(lib().sbh_check_full(self.h, begin, end, reads_to_check, _ptr(words), _ptr(counts),
                                     _ptr(rbe), C.byref(ns), _ptr(close_flat), _ptr(close_word),
                                     close_cap, C.byref(nclose)))
        k = min(nclose.value, close_cap)
        return {
            "n_success": ns.value, "counts": counts.reshape(21, 19), "rbe": rbe.reshape(21, 64),
            "words": words, "close_flat": close_flat[:k], "close_word": close_word[:k],
            "n_close": nclose.value,
        }

    def find_record_start(self, from_flat, reads_to_check=10, max_read_size=100000000):
        out, d = C.c_uint64(), C.c_int32()
        self._c(lib().sbh_find_record_start(self.h, from_flat, reads_to_check, max_read_size,
                                            C.byref(out), C.byref(d)))
        return out.value, d.value

    def count_records(self, first_flat, end_flat):
        out = C.c_uint64()
        self._c(lib().sbh_count_records(self.h, first_flat, end_flat, C.byref(out)))
        return out.value

    def chain_from(self, first_flat, end_flat):
        """(records of the chain from first_flat starting before end_flat, the chain's exit
        flat position) -- sbh_chain_from."""
        n, x = C.c_uint64(), C.c_uint64()
        self._c(lib().sbh_chain_from(self.h, first_flat, end_flat, C.byref(n), C.byref(x)))
        return n.value, x.value

    def split_starts(self, splits, bgzf_blocks_to_check=5, reads_to_check=10, max_read_size=100000000):
        """Every split [(start, end), ...] at once (sbh_split_starts): numpy arrays
        (status, first_vpos, count) per split, and how many took the per-split path."""
        st = np.ascontiguousarray([a for a, _ in splits], dtype=np.uint64)
        en = np.ascontiguousarray([b for _, b in splits], dtype=np.uint64)
        n = st.size
        v = np.zeros(max(n, 1), np.uint64)
        c = np.zeros(max(n, 1), np.uint64)
        status = np.zeros(max(n, 1), np.int32)
        nh = C.c_uint64()
        self._c(lib().sbh_split_starts(self.h, _ptr(st), _ptr(en), n, bgzf_blocks_to_check, reads_to_check,
                                       max_read_size, _ptr(v), _ptr(c), _ptr(status), C.byref(nh)))
        return status[:n], v[:n], c[:n], nh.value

    def check_records(self, ranges, rec_vpos, reads_to_check=10, cap=1 << 20):
        """check-bam's TP/FP/FN against the `.records` truth on the device (sbh_check_records):
        ranges = sorted disjoint [(begin_flat, end_flat)], rec_vpos = htsjdk vpos of the truth
        records.  Returns (tp, fp, fn, unknown, fp_flat, fn_flat)."""
        rb = np.ascontiguousarray([a for a, _ in ranges], dtype=np.uint64)
        re_ = np.ascontiguousarray([b for _, b in ranges], dtype=np.uint64)
        rv = np.ascontiguousarray(rec_vpos, dtype=np.uint64)
        out = np.zeros(4, np.uint64)
        fp = np.zeros(max(cap, 1), np.uint64)
        fn = np.zeros(max(cap, 1), np.uint64)
        self._c(lib().sbh_check_records(self.h, _ptr(rb), _ptr(re_), rb.size, reads_to_check, _ptr(rv), rv.size,
                                        _ptr(out), _ptr(fp), cap, _ptr(fn), cap))
        tp, nfp, nfn, unk = (int(x) for x in out)
        return tp, nfp, nfn, unk, fp[:min(nfp, cap)], fn[:min(nfn, cap)]

    def split(self, start, end, bgzf_blocks_to_check=5, reads_to_check=10,
              max_read_size=100000000):
        v, n = C.c_uint64(), C.c_uint64()
        self._c(lib().sbh_split(self.h, start, end, bgzf_blocks_to_check, reads_to_check,
                                max_read_size, C.byref(v), C.byref(n)))
        return v.value, n.value

    def run(self, index_start, own_end_file, reads_to_check=10, max_read_size=100000000):
        r = SbhShardResult()
        rc = lib().sbh_run_shard(self.h, index_start, own_end_file, reads_to_check,
                                 max_read_size, C.byref(r))
        self._c(rc)
        return {f: getattr(r, f) for f, _ in SbhShardResult._fields_}

    def exit_vpos(self, result):
        """The htsjdk vpos of a run() result's chain exit (the first record at/after the
        owned end), or None when the chain ran into the end of the resident stream."""
        if not result["count"]:
            return None
        bp, off = C.c_uint64(), C.c_uint32()
        if lib().sbh_pos_of(self.h, result["exit_flat"], C.byref(bp), C.byref(off)) != SBH_OK:
            return None
        return (bp.value << 16) | off.value

    def records(self, first_flat, end_flat):
        """RecordStream + BAMRecordCodec.decode of the records from first_flat while the
        start is < end_flat (RecordStream.scala:16-41), decoded on the GPU: a dict of
        numpy columns (fixed fields per record; names / cigar / seq / qual / aux packed,
        with [n + 1] prefix offsets)."""
        sz = SbhRecordsSizes()
        self._c(lib().sbh_records_scan(self.h, first_flat, end_flat, C.byref(sz)))
        return self._records_fetch(sz)

    def records_regions(self, chunks_flat, intervals):
        """loadBamIntervals' per-chunk record streams + region filter on the GPU
        (CanLoadBam.scala:123-152): chunks_flat = [(begin_flat, end_flat)] in chunk order;
        intervals = [(ref_idx, begin, end)] 0-based half-open, sorted and disjoint.
        Returns the kept records' columns (same layout as records())."""
        cb = np.ascontiguousarray([c[0] for c in chunks_flat], dtype=np.uint64)
        ce = np.ascontiguousarray([c[1] for c in chunks_flat], dtype=np.uint64)
        ir = np.ascontiguousarray([i[0] for i in intervals], dtype=np.int32)
        ib = np.ascontiguousarray([i[1] for i in intervals], dtype=np.int64)
        ie = np.ascontiguousarray([i[2] for i in intervals], dtype=np.int64)
        sz = SbhRecordsSizes()
        self._c(lib().sbh_records_scan_regions(self.h, _ptr(cb), _ptr(ce), cb.size, _ptr(ir), _ptr(ib),
                                               _ptr(ie), ir.size, C.byref(sz)))
        return self._records_fetch(sz)

    def split_records(self, start, end, bgzf_blocks_to_check=5, reads_to_check=10, max_read_size=100000000,
                      decode=True, flat_out=None):
        """One FileSplit of loadReadsAndPositions in one call (sbh_split_records): FindBlockStart,
        index + inflate, the eager check over [Pos(blockStart, 0), Pos(end, 0)), FindRecordStart
        and the split's records.  Returns (info dict, columns): all columns when decode, else
        only `flat` (the record starts)."""
        r = SbhSplitRecordsResult()
        self._c(lib().sbh_split_records(self.h, int(start), int(end), int(bgzf_blocks_to_check), int(reads_to_check),
                                        int(max_read_size), 1 if decode else 0, C.byref(r)))
        info = {f: getattr(r, f) for f, _ in SbhSplitRecordsResult._fields_ if f != "sizes"}
        info["n"] = r.sizes.n
        self.n_blocks, self.flat_size = r.n_blocks, r.flat_size  # (the index the call built: blocks())
        if decode:
            return info, self._records_fetch(r.sizes)
        # flat_out(n) (optional): where the starts and their virtual positions land (e.g. page-locked
        # memory, 2 n u64); copied to fresh arrays
        n = r.sizes.n
        both = np.empty(2 * n, np.uint64) if flat_out is None else flat_out(2 * n)
        if n:
            out = SbhRecordsOut(flat=both.ctypes.data, vpos=both[n:].ctypes.data)
            self._c(lib().sbh_records_fetch(self.h, C.byref(out)))
        if flat_out is None:
            return info, {"flat": both[:n], "vpos": both[n:]}
        return info, {"flat": both[:n].copy(), "vpos": both[n:].copy()}

    def _records_fetch(self, sz):
        cols = record_columns(sz.n, sz.name_bytes, sz.cigar_ops, sz.bases, sz.aux_bytes)
        cols["vpos"] = np.empty(sz.n, np.uint64)  # (computed on the device from the block table)
        out = SbhRecordsOut(**{k: v.ctypes.data if v.size else None for k, v in cols.items()})
        self._c(lib().sbh_records_fetch(self.h, C.byref(out)))
        return cols

    def stage_times(self):
        """[index, inflate+eager pipeline, eager (sum of launches), records, k_huff
        (sum), k_lz (sum)] device ms of the last run() (HIP events on each kernel's
        stream)."""
        ms = (C.c_double * 6)()
        n = lib().sbh_stage_times(self.h, ms, 6)
        return list(ms[:n])
