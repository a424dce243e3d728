"""CPU-side checks of the drop-in boundary: the C-ABI library builds, loads and exports
every symbol include/sparkbam.h declares; host-only entry points behave like the
reference (no GPU compute here)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from pkg import ROOT, sb


def header_decls():
    with open(os.path.join(ROOT, "include", "sparkbam.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"\b(sbh_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = sb.lib()
    decls = header_decls()
    assert len(decls) >= 20
    for name in decls:
        assert hasattr(L, name), name
    from importlib import import_module  # noqa: F401
    assert sorted(sb._lib.EXPORTS) == decls


def test_version_string():
    assert b"gfx950" in sb.lib().sbh_version()


def test_header_make_host():
    # Header.make (bgzf/.../block/Header.scala:48-83) on 2.bam's first block
    b = np.fromfile(os.path.join(ROOT, "tests/golden/bams/2.bam"), dtype=np.uint8)[:18]
    assert sb.Header.make(b.tobytes()) == (18, 26169)
    bad = bytearray(b.tobytes())
    bad[13] = 0
    with pytest.raises(sb.SparkBamError) as e:
        sb.Header.make(bytes(bad))
    assert e.value.code == 10  # HeaderParseException


def test_header_make_too_short_is_eof():
    with pytest.raises(sb.SparkBamError) as e:
        sb.Header.make(b"\x1f\x8b\x08\x04")
    assert e.value.code == 12


def test_file_splits_matches_oracle():
    from oracle_lib import file_splits as ofs
    for size, split in [(531753, 100000), (597482, 230 * 1024), (1 << 30, 32 << 20), (110, 100)]:
        assert sb.file_splits(size, split) == ofs(size, split)


def test_pos_htsjdk_roundtrip():
    p = sb.Pos(239479, 312)
    assert sb.Pos.from_htsjdk(p.to_htsjdk()) == p and str(p) == "239479:312"
    # Split.length with EstimatedCompressionRatio 3.0 (ComputeSplitsTest elems 224301)
    assert sb.Pos(239479, 312).minus(sb.Pos(0, 45846)) == 224301.0


def test_parse_bam_header_from_oracle_flat():
    from oracle_lib import OracleFile
    of = OracleFile.from_path(os.path.join(ROOT, "tests/golden/bams/2.bam"))
    names, lens, end = sb.parse_bam_header(of.uncompressed()[:65536])
    assert end == 5650 and list(lens) == list(of.contig_len) and names[0] == "1"


def test_no_gpu_context_fails_loudly():
    # a GPU box exposes the KFD device node (torch's check is unreliable once another
    # library in the process has initialised HIP)
    if os.path.exists("/dev/kfd"):
        pytest.skip("GPU present")
    h = C.c_void_p()
    assert sb.lib().sbh_ctx_create(0, C.byref(h)) != 0
