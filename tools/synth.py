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
