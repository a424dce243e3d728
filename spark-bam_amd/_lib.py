"""ctypes binding of libsparkbam_hip.so (the C-ABI declared in include/sparkbam.h).

There is no CPU fallback: if the HIP library is missing or cannot be loaded, every
entry point raises.  The library is built in-tree by spark-bam_amd/csrc/Makefile
(``__graft_entry__.build()``).
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SBH_LIB_PATH") or os.path.join(HERE, "libsparkbam_hip.so")

SBH_OK = 0
STATUS_NAMES = {
    0: "SBH_OK", 1: "SBH_E_ARG", 2: "SBH_E_HIP", 3: "SBH_E_NOMEM", 10: "SBH_E_HEADER_PARSE",
    11: "SBH_E_HEADER_SEARCH_FAILED", 12: "SBH_E_TRUNCATED", 13: "SBH_E_INFLATE_SIZE",
    14: "SBH_E_INFLATE_DATA", 15: "SBH_E_BAD_ISIZE", 16: "SBH_E_NO_READ_FOUND",
    17: "SBH_E_NEED_HALO", 18: "SBH_E_STATE", 19: "SBH_E_NOT_FOUND", 20: "SBH_E_BAD_RECORD",
}
SBH_E_ARG, SBH_E_HIP, SBH_E_HEADER_PARSE, SBH_E_HEADER_SEARCH_FAILED = 1, 2, 10, 11
SBH_E_TRUNCATED, SBH_E_INFLATE_SIZE, SBH_E_INFLATE_DATA, SBH_E_BAD_ISIZE = 12, 13, 14, 15
SBH_E_NO_READ_FOUND, SBH_E_NEED_HALO, SBH_E_STATE, SBH_E_NOT_FOUND = 16, 17, 18, 19
SBH_E_BAD_RECORD = 20

FULL_SUCCESS = 0x80000000
FULL_UNKNOWN = 0x40000000
FULL_N_SHIFT = 20
FULL_FLAGS_MASK = 0x7FFFF
BLOCK_EMPTY, BLOCK_TRUNCATED = 1, 2

# Every symbol include/sparkbam.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "sbh_ctx_create", "sbh_ctx_destroy", "sbh_last_error", "sbh_last_error_detail", "sbh_ctx_set_stream",
    "sbh_ctx_synchronize", "sbh_version", "sbh_host_alloc", "sbh_host_free", "sbh_header_make", "sbh_shard_create",
    "sbh_shard_destroy", "sbh_shard_comp_device_ptr", "sbh_find_block_start", "sbh_index",
    "sbh_get_blocks", "sbh_inflate", "sbh_read_flat", "sbh_flat_device_ptr", "sbh_flat_of",
    "sbh_pos_of", "sbh_flat_bound", "sbh_set_contigs", "sbh_check_eager", "sbh_eager_bits", "sbh_check_full",
    "sbh_find_record_start", "sbh_count_records", "sbh_chain_from", "sbh_split", "sbh_split_starts",
    "sbh_check_records", "sbh_run_shard",
    "sbh_stage_times", "sbh_run_stream", "sbh_run_stream2", "sbh_records_scan", "sbh_records_fetch", "sbh_records_scan_regions", "sbh_verify_crc",
    "sbh_bgzf_compress_bound", "sbh_bgzf_compress", "sbh_bgzf_compress_level",
    "sbh_shard_load", "sbh_find_blocks", "sbh_check_stream", "sbh_split_records",
]
LEVEL_HTSJDK, LEVEL_FAST = 5, -1  # sbh_bgzf_compress_level: htsjdk's zlib level 5 / this library's own coder


class SbhBlock(C.Structure):
    _fields_ = [("start", C.c_uint64), ("ustart", C.c_uint64), ("csize", C.c_uint32),
                ("hsize", C.c_uint32), ("usize", C.c_uint32), ("flags", C.c_uint32)]


class SbhShardResult(C.Structure):
    _fields_ = [("n_blocks", C.c_uint64), ("comp_bytes", C.c_uint64), ("flat_bytes", C.c_uint64),
                ("n_true", C.c_uint64), ("first_vpos", C.c_uint64), ("count", C.c_uint64),
                ("exit_flat", C.c_uint64), ("status", C.c_int32), ("anomalies", C.c_int32)]


class SbhStreamResult(C.Structure):
    _fields_ = [("n_windows", C.c_uint64), ("n_blocks", C.c_uint64), ("comp_bytes", C.c_uint64),
                ("flat_bytes", C.c_uint64), ("n_true", C.c_uint64), ("count", C.c_uint64),
                ("first_vpos", C.c_uint64), ("exit_vpos", C.c_uint64), ("status", C.c_int32),
                ("rewalks", C.c_int32), ("host_pinned", C.c_int32), ("pad", C.c_int32),
                ("ms_wall", C.c_double), ("ms_h2d", C.c_double), ("stage_ms", C.c_double * 6),
                ("halo_final", C.c_uint64), ("crc_bad_blocks", C.c_uint64), ("crc_first_bad", C.c_uint64),
                ("splits_host", C.c_uint64), ("ms_splits", C.c_double), ("ms_crc", C.c_double)]


class SbhStreamOpts(C.Structure):
    _fields_ = [("window", C.c_uint64), ("halo", C.c_uint64), ("reads_to_check", C.c_int32),
                ("max_read_size", C.c_int32), ("bgzf_blocks_to_check", C.c_int32), ("verify_crc", C.c_int32),
                ("split_start", C.c_void_p), ("split_end", C.c_void_p), ("n_splits", C.c_uint64),
                ("split_first_vpos", C.c_void_p), ("split_count", C.c_void_p), ("split_status", C.c_void_p),
                ("out_bits", C.c_void_p), ("out_bits_cap", C.c_uint64)]


class SbhCheckOpts(C.Structure):
    _fields_ = [("window", C.c_uint64), ("halo", C.c_uint64), ("reads_to_check", C.c_int32), ("full", C.c_int32),
                ("blocks", C.c_void_p), ("n_blocks", C.c_uint64), ("truth_vpos", C.c_void_p),
                ("n_truth", C.c_uint64), ("fp_vpos", C.c_void_p), ("fn_vpos", C.c_void_p), ("fp_cap", C.c_uint64),
                ("fn_cap", C.c_uint64), ("counts", C.c_void_p), ("rbe_hist", C.c_void_p),
                ("close_vpos", C.c_void_p), ("close_word", C.c_void_p), ("close_cap", C.c_uint64)]


class SbhCheckResult(C.Structure):
    _fields_ = [("n_windows", C.c_uint64), ("positions", C.c_uint64), ("comp_bytes", C.c_uint64),
                ("n_true", C.c_uint64), ("tp", C.c_uint64), ("fp", C.c_uint64), ("fn", C.c_uint64),
                ("unknown", C.c_uint64), ("n_success", C.c_uint64), ("n_close", C.c_uint64),
                ("halo_final", C.c_uint64), ("ms_wall", C.c_double), ("ms_h2d", C.c_double)]


class SbhRecordsSizes(C.Structure):
    _fields_ = [("n", C.c_uint64), ("name_bytes", C.c_uint64), ("cigar_ops", C.c_uint64),
                ("bases", C.c_uint64), ("aux_bytes", C.c_uint64)]


class SbhSplitRecordsResult(C.Structure):
    _fields_ = [("block_start", C.c_uint64), ("n_blocks", C.c_uint64), ("flat_size", C.c_uint64),
                ("owned_flat", C.c_uint64), ("first_flat", C.c_uint64),
                ("first_vpos", C.c_uint64), ("n_true", C.c_uint64), ("sizes", SbhRecordsSizes)]


class SbhRecordsOut(C.Structure):  # host buffers (sbh_records_out); NULL = not copied
    _fields_ = [(f, C.c_void_p) for f in (
        "flat", "ref_id", "pos", "next_ref_id", "next_pos", "tlen", "flag", "bin", "mapq",
        "name_off", "cigar_off", "seq_off", "aux_off", "names", "cigar", "seq", "qual", "aux", "vpos")]


class SparkBamError(RuntimeError):
    """Maps an SBH_E_* status onto the reference's exception vocabulary.  `fields` are the
    values sbh_last_error_detail returned (what the reference's exception is built from)."""

    def __init__(self, code, message="", fields=()):
        self.code = code
        self.fields = tuple(fields)
        super().__init__(f"{STATUS_NAMES.get(code, code)}: {message}")


class HeaderParseException(SparkBamError):
    """bgzf/.../block/HeaderParseException.scala:6-11: HeaderParseException(idx, actual, expected)."""

    def __init__(self, code, message="", fields=()):
        super().__init__(code, message, fields)
        _, self.idx, self.actual, self.expected = (list(fields) + [None] * 4)[:4]


class HeaderSearchFailedException(SparkBamError):
    """bgzf/.../block/HeaderSearchFailedException.scala:7-12: (path, start, positionsAttempted);
    the library knows no path: the caller that does sets it (with_path)."""

    def __init__(self, code, message="", fields=(), path=None):
        super().__init__(code, message, fields)
        self.start, self.positions_attempted = (list(fields) + [None] * 2)[:2]
        self.path = path

    def with_path(self, path):
        self.path = path
        return self


class NoReadFoundException(SparkBamError):
    """check/.../spark/FindRecordStart.scala:66-71: NoReadFoundException(path, start, maxReadSize)."""

    def __init__(self, code, message="", fields=(), path=None):
        super().__init__(code, message, fields)
        self.start, self.max_read_size = (list(fields) + [None] * 2)[:2]
        self.path = path

    def with_path(self, path, start=None):
        self.path = path
        if start is not None:
            self.start = start
        return self


# the status -> exception class the JNI shim throws (jni/sparkbam_jni.c EXCEPTIONS)
EXCEPTION_CLASSES = {}  # filled below, after the status constants


def error_for(code, message="", fields=()):
    return EXCEPTION_CLASSES.get(code, SparkBamError)(code, message, fields)


EXCEPTION_CLASSES.update({SBH_E_HEADER_PARSE: HeaderParseException,
                          SBH_E_HEADER_SEARCH_FAILED: HeaderSearchFailedException,
                          SBH_E_NO_READ_FOUND: NoReadFoundException})

_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise SparkBamError(SBH_E_STATE, f"HIP library not built: {LIB_PATH} "
                                         "(run __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    P, I32, U32, U64 = C.c_void_p, C.c_int32, C.c_uint32, C.c_uint64
    PU64, PI32, PU32 = C.POINTER(U64), C.POINTER(I32), C.POINTER(U32)
    sig = {
        "sbh_ctx_create": [I32, C.POINTER(P)],
        "sbh_ctx_destroy": [P],
        "sbh_ctx_set_stream": [P, P],
        "sbh_ctx_synchronize": [P],
        "sbh_host_alloc": [U64, C.POINTER(P)],
        "sbh_host_free": [P],
        "sbh_header_make": [P, U64, PI32, PI32],
        "sbh_shard_create": [P, P, U64, U64, U64, C.c_int, C.POINTER(P)],
        "sbh_shard_destroy": [P],
        "sbh_find_block_start": [P, U64, I32, PU64],
        "sbh_index": [P, U64, PU64, PU64],
        "sbh_get_blocks": [P, U64, U64, P],
        "sbh_inflate": [P, PU64],
        "sbh_read_flat": [P, U64, U64, P],
        "sbh_flat_of": [P, U64, U32, PU64],
        "sbh_pos_of": [P, U64, PU64, PU32],
        "sbh_flat_bound": [P, U64, PU64],
        "sbh_set_contigs": [P, P, I32],
        "sbh_check_eager": [P, U64, U64, I32, P, PU64],
        "sbh_eager_bits": [P, U64, U64, P],
        "sbh_check_full": [P, U64, U64, I32, P, P, P, PU64, P, P, U64, PU64],
        "sbh_find_record_start": [P, U64, I32, I32, PU64, PI32],
        "sbh_count_records": [P, U64, U64, PU64],
        "sbh_split": [P, U64, U64, I32, I32, I32, PU64, PU64],
        "sbh_chain_from": [P, U64, U64, PU64, PU64],
        "sbh_split_starts": [P, P, P, U64, I32, I32, I32, P, P, P, PU64],
        "sbh_check_records": [P, P, P, U64, I32, P, U64, P, P, U64, P, U64],
        "sbh_run_shard": [P, U64, U64, I32, I32, C.POINTER(SbhShardResult)],
        "sbh_run_stream": [P, P, U64, U64, U64, U64, U64, U64, U64, P, I32, I32, I32, P, U64,
                           C.POINTER(SbhStreamResult)],
        "sbh_run_stream2": [P, P, U64, U64, U64, U64, U64, P, I32, C.POINTER(SbhStreamOpts),
                            C.POINTER(SbhStreamResult)],
        "sbh_records_scan": [P, U64, U64, C.POINTER(SbhRecordsSizes)],
        "sbh_records_fetch": [P, C.POINTER(SbhRecordsOut)],
        "sbh_split_records": [P, U64, U64, I32, I32, I32, I32, C.POINTER(SbhSplitRecordsResult)],
        "sbh_records_scan_regions": [P, P, P, U64, P, P, P, C.c_uint32, C.POINTER(SbhRecordsSizes)],
        "sbh_verify_crc": [P, PU64, PU64],
        "sbh_shard_load": [P, P, U64, U64, C.c_int],
        "sbh_find_blocks": [P, P, U64, P, P, U64, I32, U64, P, U64, PU64],
        "sbh_check_stream": [P, P, U64, P, I32, C.POINTER(SbhCheckOpts), C.POINTER(SbhCheckResult)],
        "sbh_bgzf_compress": [P, P, U64, I32, P, U64, PU64, PU64, C.POINTER(C.c_float)],
        "sbh_bgzf_compress_level": [P, P, U64, I32, I32, P, U64, PU64, PU64, C.POINTER(C.c_float)],
    }
    for name, args in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = C.c_int
    L.sbh_bgzf_compress_bound.argtypes = [U64]
    L.sbh_bgzf_compress_bound.restype = U64
    L.sbh_stage_times.argtypes = [P, C.POINTER(C.c_double), I32]
    L.sbh_stage_times.restype = C.c_int
    L.sbh_last_error.argtypes = [P]
    L.sbh_last_error.restype = C.c_char_p
    L.sbh_last_error_detail.argtypes = [P, PI32, C.POINTER(C.c_int64), I32]
    L.sbh_last_error_detail.restype = I32
    L.sbh_version.argtypes = []
    L.sbh_version.restype = C.c_char_p
    for name in ("sbh_shard_comp_device_ptr", "sbh_flat_device_ptr"):
        getattr(L, name).argtypes = [P]
        getattr(L, name).restype = P
    _lib = L
    return L
