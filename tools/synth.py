"""ctypes front-end of tools/libsynth.so: deterministic synthetic BAMs (configs B-E)."""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libsynth.so")

SHAPE_SHORT, SHAPE_LONG, SHAPE_ADVERSARIAL = 0, 1, 2
SEEDS = {"B": 0x5B4D0001, "C": 0x5B4D0030, "D": 0x5B4D004C, "E": 0x5B4D00AD}


class Params(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("shape", C.c_int32), ("level", C.c_int32),
                ("payload", C.c_int32), ("threads", C.c_int32), ("empty_every", C.c_int32),
                ("pad", C.c_int32)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(HERE, "synth_bam.c")
        if (not os.path.exists(LIB)) or os.path.getmtime(LIB) < os.path.getmtime(src):
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        L = C.CDLL(LIB)
        P, I64 = C.c_void_p, C.c_int64
        L.synth_header.restype = I64
        L.synth_header.argtypes = [P, I64]
        L.synth_records_size.restype = I64
        L.synth_records_size.argtypes = [P, I64, I64]
        L.synth_records_for_bytes.restype = I64
        L.synth_records_for_bytes.argtypes = [P, I64]
        L.synth_records.restype = I64
        L.synth_records.argtypes = [P, I64, I64, P, I64]
        L.synth_bgzf.restype = I64
        L.synth_bgzf.argtypes = [P, P, I64, I64, C.c_int, P, I64, C.POINTER(I64)]
        L.synth_bam_bound.restype = I64
        L.synth_bam_bound.argtypes = [P, I64]
        L.synth_bam.restype = I64
        L.synth_bam.argtypes = [P, I64, P, I64, C.POINTER(I64), C.POINTER(I64)]
        _lib = L
    return _lib


def params(seed, shape=SHAPE_SHORT, level=6, payload=65498, threads=None, empty_every=0):
    if threads is None:
        threads = min(16, os.cpu_count() or 1)
    return Params(seed, shape, level, payload, threads, empty_every, 0)


def records_for_bytes(p, target_bytes):
    return lib().synth_records_for_bytes(C.byref(p), target_bytes)


def make_bam(p, n_records):
    """Returns (compressed bytes as np.uint8 array, uncompressed size, n data blocks)."""
    L = lib()
    cap = L.synth_bam_bound(C.byref(p), n_records)
    out = np.empty(cap, dtype=np.uint8)
    us, nb = C.c_int64(), C.c_int64()
    n = L.synth_bam(C.byref(p), n_records, out.ctypes.data_as(C.c_void_p), cap, C.byref(us),
                    C.byref(nb))
    if n < 0:
        raise RuntimeError("synth_bam failed")
    return out[:n], us.value, nb.value


def header_bytes():
    L = lib()
    n = L.synth_header(None, 0)
    out = np.empty(n, dtype=np.uint8)
    L.synth_header(out.ctypes.data_as(C.c_void_p), n)
    return out


def records_size(p, a, b):
    return lib().synth_records_size(C.byref(p), a, b)


def records(p, a, b):
    size = records_size(p, a, b)
    out = np.empty(size, dtype=np.uint8)
    n = lib().synth_records(C.byref(p), a, b, out.ctypes.data_as(C.c_void_p), size)
    assert n == size
    return out


def bgzf(p, U, kbase, add_eof):
    """BGZF-compress U (cut into p.payload blocks; levels by global block index)."""
    cap = U.size + (U.size // 32768 + 4) * 128 + 1024
    out = np.empty(cap, dtype=np.uint8)
    nb = C.c_int64()
    n = lib().synth_bgzf(C.byref(p), U.ctypes.data_as(C.c_void_p), U.size, kbase, int(add_eof),
                         out.ctypes.data_as(C.c_void_p), cap, C.byref(nb))
    if n < 0:
        raise RuntimeError("synth_bgzf failed")
    return out[:n], nb.value


def block_sizes(comp):
    """Compressed sizes of consecutive BGZF blocks (BSIZE + 1 of each header)."""
    sizes, pos = [], 0
    while pos + 18 <= comp.size:
        cs = int(comp[pos + 16]) | (int(comp[pos + 17]) << 8)
        sizes.append(cs + 1)
        pos += cs + 1
    return sizes


class Segment:
    """Rank `rank`'s byte-range shard of a synthetic BAM of world * records_per_rank
    records (weak scaling: per-rank work fixed).

    The global uncompressed stream is header + records; it is cut into BGZF blocks
    of `payload` bytes (block k = U[k*P, (k+1)*P)), so records straddle block and
    shard edges exactly as in a real file.  Rank i owns the blocks whose first byte
    lies in its record range, K_i = ceil(U_i / P), and regenerates `halo_blocks`
    blocks of rank i+1 (or the EOF block) as its halo.  Only the per-rank compressed
    sizes must be exchanged to place the shard in the file (see set_offsets)."""

    def __init__(self, p, records_per_rank, world, rank, halo_blocks=16, log=None, alloc=None,
                 chunk_blocks=4096):
        """alloc(n) -> a writable uint8 array of n bytes for the shard's compressed bytes (e.g.
        pinned host memory); records are generated and compressed chunk_blocks blocks at a
        time, so host memory holds the compressed shard plus one chunk."""
        if p.level < 0:
            raise ValueError("segments need a uniform payload size (level >= 0)")
        self.p, self.R, self.world, self.rank = p, records_per_rank, world, rank
        P = p.payload
        hdr = header_bytes()
        h = hdr.size
        # U offset of the first record of each rank (prefix of record sizes)
        self.u_start = [0] * (world + 1)
        acc = h
        for i in range(world):
            self.u_start[i] = h if i == 0 else acc
            acc += records_size(p, i * records_per_rank, (i + 1) * records_per_rank)
        self.u_start[0] = 0
        self.u_total = acc
        ceil = lambda x: (x + P - 1) // P  # noqa: E731
        self.k = [ceil(self.u_start[i]) if i else 0 for i in range(world)] + [ceil(self.u_total)]
        k0, k1 = self.k[rank], self.k[rank + 1]
        k_halo = min(k1 + halo_blocks, self.k[world])
        u0, u1 = k0 * P, min(k_halo * P, self.u_total)
        # records covering [u0, u1), cut into P-aligned chunks of whole blocks as they come:
        # block k is U[kP, (k+1)P) whatever chunk it is compressed in
        first_rec = rank * records_per_rank
        total_recs = world * records_per_rank
        pending = [hdr] if rank == 0 else []
        pend_at = 0 if rank == 0 else self.u_start[rank]  # U offset of pending's first byte
        pend_n = sum(x.size for x in pending)
        rec_end, k, chunks, sizes = first_rec, k0, [], []
        step = max(1024, min(records_per_rank, 200_000))
        done_u = 0
        while k < k_halo:
            need_end = min(u1, (k + chunk_blocks) * P)
            while pend_at + pend_n < need_end and rec_end < total_recs:
                nxt = min(total_recs, rec_end + step)
                pending.append(records(p, rec_end, nxt))
                pend_n += pending[-1].size
                rec_end = nxt
            buf = np.concatenate(pending) if len(pending) > 1 else pending[0]
            lo = k * P - pend_at  # the chunk's first byte within buf
            hi = min(need_end, pend_at + buf.size) - pend_at
            kb = (hi - lo + P - 1) // P
            last = k + kb >= k_halo
            comp, _ = bgzf(p, buf[lo:hi], k, add_eof=last and k_halo == self.k[world])
            chunks.append(comp)
            sizes += block_sizes(comp)
            done_u += hi - lo
            k += kb
            pending, pend_at, pend_n = [buf[hi:]], pend_at + hi, buf.size - hi
            if log and (len(chunks) % 8 == 0 or last):
                log(f"[rank {rank}] generated {done_u / 2**30:.2f} GiB uncompressed, "
                    f"{sum(c.size for c in chunks) / 2**30:.2f} GiB compressed")
        total = sum(c.size for c in chunks)
        comp = alloc(total) if alloc else np.empty(total, dtype=np.uint8)
        o = 0
        while chunks:  # free each chunk once it is placed
            c = chunks.pop(0)
            comp[o:o + c.size] = c
            o += c.size
        self.own_blocks = k1 - k0
        self.own_csize = sum(sizes[:self.own_blocks])
        self.comp = comp
        self.n_records_owned = None  # known only by the chain walk (GPU result)
        self.file_offset = None
        self.file_size = None

    def set_offsets(self, own_csizes):
        """own_csizes: every rank's owned compressed size (the setup allgather)."""
        self.file_offset = sum(own_csizes[:self.rank])
        self.own_end = self.file_offset + own_csizes[self.rank]
        self.file_size = sum(own_csizes) + 28
        return self


class WholeFile:
    """A whole synthetic BAM (header + records + EOF) as rank 0's only shard, for
    parameters without a uniform payload grid (mixed levels)."""

    def __init__(self, p, n_records):
        U = np.concatenate([header_bytes(), records(p, 0, n_records)])
        comp, nb = bgzf(p, U, 0, add_eof=True)
        self.comp = comp
        self.own_csize = comp.size
        self.rank = 0

    def set_offsets(self, own_csizes):
        self.file_offset = 0
        self.own_end = self.file_size = int(self.comp.size)
        return self


class Replicated:
    """configs[2]'s one big file, strong scaling: the BAM header's block(s), then one canonical
    segment of records repeated `copies` times, then the EOF block.  The segment is `records`
    records BGZF-compressed on the htsjdk payload grid with a short last block, so it starts
    with a record at a block start and ends with a record at a block end: the copies join into
    a valid BAM (record chain unbroken across them) whose compressed bytes are a periodic
    pattern.  Any rank materializes its byte range [lo, hi) without generating the rest --
    100 GB of file in seconds of memcpy instead of ~20 minutes of generation.  Block contents
    repeat every segment (~1 GiB compressed, far beyond any cache), so every window still
    inflates and checks its own bytes."""

    def __init__(self, p, records, file_bytes):
        if p.level < 0:
            raise ValueError("a replicated file needs one zlib level")
        hdr = header_bytes()
        self.hdr_comp, _ = bgzf(p, hdr, 0, False)
        recs = records_(p, 0, records)
        self.seg_comp, self.seg_blocks = bgzf(p, recs, 1, False)
        self.seg_flat = int(recs.size)
        del recs
        self.hdr_flat = int(hdr.size)
        self.seg_records = int(records)
        self.copies = max(1, -(-(int(file_bytes) - self.hdr_comp.size - 28) // self.seg_comp.size))
        self.records = self.seg_records * self.copies
        self.eof = np.frombuffer(bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000"),
                                 dtype=np.uint8)
        self.size = int(self.hdr_comp.size + self.copies * self.seg_comp.size + 28)
        self.flat_size = self.hdr_flat + self.copies * self.seg_flat

    def read_into(self, lo, hi, out):
        """Compressed bytes [lo, hi) of the file into out[0: hi - lo]."""
        h, s = self.hdr_comp.size, self.seg_comp.size
        body_end = h + self.copies * s
        o = 0
        p = lo
        while p < hi:
            if p < h:
                n = min(hi, h) - p
                out[o:o + n] = self.hdr_comp[p:p + n]
            elif p < body_end:
                k, r = divmod(p - h, s)
                n = min(hi - p, s - r)
                out[o:o + n] = self.seg_comp[r:r + n]
            else:
                r = p - body_end
                n = min(hi, self.size) - p
                out[o:o + n] = self.eof[r:r + n]
            o += n
            p += n
        return out


records_ = records  # (Replicated's __init__ has a `records` argument)
