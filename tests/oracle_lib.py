"""ctypes binding of the CPU oracle (oracle/liboracle.so) -- TEST INFRASTRUCTURE ONLY.

The oracle is the checker the HIP path is compared against; it is never the thing
measured or shipped.  See oracle/sbam_oracle.h for the reference file:line each
function restates.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "liboracle.so")

OR_OK, OR_END, OR_HEADER_PARSE, OR_TRUNCATED = 0, 1, 2, 3
OR_INFLATE_SIZE, OR_INFLATE_DATA, OR_BAD_ISIZE = 4, 5, 6
OR_SEARCH_FAILED, OR_NO_READ_FOUND = 7, 8
FULL_SUCCESS = 0x80000000
FULL_N_SHIFT = 20
FULL_FLAGS_MASK = 0x7FFFF

FLAG_NAMES = [
    "tooFewFixedBlockBytes", "negativeReadIdx", "tooLargeReadIdx", "negativeReadPos",
    "tooLargeReadPos", "negativeNextReadIdx", "tooLargeNextReadIdx", "negativeNextReadPos",
    "tooLargeNextReadPos", "tooFewBytesForReadName", "nonNullTerminatedReadName",
    "nonASCIIReadName", "noReadName", "emptyReadName", "tooFewBytesForCigarOps",
    "invalidCigarOp", "emptyMappedCigar", "emptyMappedSeq", "tooFewRemainingBytesImplied",
]


class Block(C.Structure):
    _fields_ = [("start", C.c_int64), ("csize", C.c_int32), ("hsize", C.c_int32),
                ("usize", C.c_int32), ("empty", C.c_int32)]


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    src = os.path.join(ORACLE_DIR, "sbam_oracle.c")
    if (not os.path.exists(LIB_PATH)) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
    L = C.CDLL(LIB_PATH)
    P, I32, I64, U32, U64 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint32, C.c_uint64
    sig = {
        "or_header_make": (C.c_int, [P, I64, C.POINTER(I32), C.POINTER(I32)]),
        "or_metadata_stream": (I64, [P, I64, I64, P, I64]),
        "or_find_block_start": (C.c_int, [P, I64, I64, I32, C.POINTER(I64)]),
        "or_stream_open": (P, [P, I64, I64]),
        "or_stream_close": (None, [P]),
        "or_stream_load_all": (C.c_int, [P]),
        "or_stream_size": (I64, [P]),
        "or_stream_error": (I32, [P]),
        "or_stream_data": (P, [P]),
        "or_stream_nblocks": (I64, [P]),
        "or_stream_blocks": (I64, [P, P, I64]),
        "or_stream_flat_of": (I64, [P, I64, I32]),
        "or_stream_pos_of": (C.c_int, [P, I64, C.POINTER(I64), C.POINTER(I32)]),
        "or_eager_check": (C.c_int, [P, I64, P, I32, I32]),
        "or_full_check": (U32, [P, I64, P, I32, I32]),
        "or_eager_check_buf": (C.c_int, [P, I64, I64, P, I32, I32]),
        "or_full_check_buf": (U32, [P, I64, I64, P, I32, I32]),
        "or_eager_range": (I64, [P, I64, I64, P, I32, I32, P]),
        "or_full_range": (I64, [P, I64, I64, P, I32, I32, P, P, P]),
        "or_find_record_start": (C.c_int, [P, I64, P, I32, I32, I32, C.POINTER(I64),
                                           C.POINTER(I32)]),
        "or_parse_header": (I32, [P, P, I32, C.POINTER(I64)]),
        "or_record_chain": (I64, [P, I64, I64, P, I64]),
        "or_file_splits": (I64, [I64, I64, P, P, I64]),
        "or_split": (C.c_int, [P, I64, I64, I64, P, I32, I32, I32, I32, C.POINTER(U64),
                               C.POINTER(I64)]),
        "or_bench_inflate_check": (C.c_double, [P, I64, P, I64, I64, P, I32, I32, I32,
                                                C.POINTER(I64), C.POINTER(I64)]),
        "or_crc32": (U32, [P, I64]),
        "or_zlib_version": (C.c_char_p, []),
        "or_stream_next": (C.c_int, [P, I64, I64, P, P]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


class OracleFile:
    """A BGZF file held in host memory, with a whole-file Stream from offset 0."""

    def __init__(self, data, start=0):
        self.data = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(
            data, np.ndarray) else data
        self.size = int(self.data.size)
        L = lib()
        self._s = L.or_stream_open(_ptr(self.data), self.size, start)
        rc = L.or_stream_load_all(self._s)
        self.error = rc
        self.flat_size = L.or_stream_size(self._s)
        n = L.or_stream_nblocks(self._s)
        blocks = (Block * max(n, 1))()
        L.or_stream_blocks(self._s, blocks, n)
        self.blocks = [(b.start, b.csize, b.usize) for b in blocks[:n]]
        contig = np.zeros(1 << 16, dtype=np.int32)
        end = C.c_int64()
        nref = L.or_parse_header(self._s, _ptr(contig), contig.size, C.byref(end))
        if nref >= 0:
            self.contig_len = contig[:nref].copy()
            self.header_end = end.value
        else:
            self.contig_len = np.zeros(0, dtype=np.int32)
            self.header_end = None

    @classmethod
    def from_path(cls, path):
        with open(path, "rb") as f:
            return cls(f.read())

    def close(self):
        if self._s:
            lib().or_stream_close(self._s)
            self._s = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def uncompressed(self):
        p = lib().or_stream_data(self._s)
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), shape=(self.flat_size,)).copy()

    def uncompressed_range(self, a, b):
        """Flat bytes [a, b) (a copy of just that slice)."""
        p = lib().or_stream_data(self._s)
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), shape=(self.flat_size,))[a:b].copy()

    def flat_of(self, block_pos, offset):
        return lib().or_stream_flat_of(self._s, block_pos, offset)

    def pos_of(self, flat):
        bp, off = C.c_int64(), C.c_int32()
        lib().or_stream_pos_of(self._s, flat, C.byref(bp), C.byref(off))
        return bp.value, off.value

    def eager(self, flat, reads_to_check=10, contig_len=None):
        cl = self.contig_len if contig_len is None else contig_len
        return bool(lib().or_eager_check(self._s, flat, _ptr(cl), cl.size, reads_to_check))

    def full(self, flat, reads_to_check=10, contig_len=None):
        cl = self.contig_len if contig_len is None else contig_len
        return int(lib().or_full_check(self._s, flat, _ptr(cl), cl.size, reads_to_check))

    def eager_range(self, begin, end, reads_to_check=10):
        bits = np.zeros((end - begin + 7) // 8, dtype=np.uint8)
        n = lib().or_eager_range(self._s, begin, end, _ptr(self.contig_len),
                                 self.contig_len.size, reads_to_check, _ptr(bits))
        return n, bits

    def full_range(self, begin, end, reads_to_check=10, want_words=False):
        counts = np.zeros(21 * 19, dtype=np.int64)
        rbe = np.zeros(21 * 64, dtype=np.int64)
        words = np.zeros(end - begin, dtype=np.uint32) if want_words else None
        ns = lib().or_full_range(self._s, begin, end, _ptr(self.contig_len),
                                 self.contig_len.size, reads_to_check, _ptr(words),
                                 _ptr(counts), _ptr(rbe))
        return ns, counts.reshape(21, 19), rbe.reshape(21, 64), words

    def find_record_start(self, from_flat, reads_to_check=10, max_read_size=100000000):
        out, d = C.c_int64(), C.c_int32()
        rc = lib().or_find_record_start(self._s, from_flat, _ptr(self.contig_len),
                                        self.contig_len.size, reads_to_check, max_read_size,
                                        C.byref(out), C.byref(d))
        return rc, out.value, d.value

    def record_chain(self, from_flat, stop_flat=None):
        stop = self.flat_size if stop_flat is None else stop_flat
        n = lib().or_record_chain(self._s, from_flat, stop, None, 0)
        out = np.zeros(max(n, 1), dtype=np.int64)
        lib().or_record_chain(self._s, from_flat, stop, _ptr(out), n)
        return out[:n]

    def find_block_start(self, start, blocks_to_check=5):
        out = C.c_int64()
        rc = lib().or_find_block_start(_ptr(self.data), self.size, start, blocks_to_check,
                                       C.byref(out))
        return rc, out.value

    def split(self, start, end, blocks_to_check=5, reads_to_check=10,
              max_read_size=100000000):
        v, n = C.c_uint64(), C.c_int64()
        rc = lib().or_split(_ptr(self.data), self.size, start, end, _ptr(self.contig_len),
                            self.contig_len.size, blocks_to_check, reads_to_check,
                            max_read_size, C.byref(v), C.byref(n))
        return rc, v.value, n.value


def file_splits(file_size, split_size):
    n = lib().or_file_splits(file_size, split_size, None, None, 0)
    s = np.zeros(n, dtype=np.int64)
    e = np.zeros(n, dtype=np.int64)
    lib().or_file_splits(file_size, split_size, _ptr(s), _ptr(e), n)
    return list(zip(s.tolist(), e.tolist()))


def vpos_str(v):
    return f"{v >> 16}:{v & 0xffff}"


def load_splits_and_reads(of, split_size, **kw):
    """Splits and per-partition counts the way loadSplitsAndReads computes them."""
    firsts, counts = [], []
    for s, e in file_splits(of.size, split_size):
        rc, v, n = of.split(s, e, **kw)
        if rc != OR_OK:
            raise RuntimeError(f"split {s}-{e}: oracle error {rc}")
        counts.append(n)
        if n > 0:
            firsts.append(v)
    ends = firsts[1:] + [of.size << 16]
    splits = [(a, b) for a, b in zip(firsts, ends)]
    return splits, counts
