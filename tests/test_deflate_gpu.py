"""The writer's fast, non-zlib coder on the GPU (sbh_bgzf_compress_level(SBH_LEVEL_FAST);
the default, byte-exact htsjdk coder is tests/test_zdeflate_gpu.py).  k_prev + k_deflate run
deflate_core.h's coder one workgroup per member, so the file must equal the host build's
(tools/deflate_host.cpp) byte for byte (test_deflate_cpu.py pins that build against zlib);
the rewritten fixtures re-inflate (zlib and this library's own GPU inflate + CRC check) to the
original stream, with htsjdk's member layout."""
import zlib

import numpy as np
import pytest

from conftest import golden_bam, read_blocks, read_records
from oracle_lib import OracleFile
from pkg import sb
from test_deflate_cpu import PAYLOAD, check_roundtrip, compress, parse_members

pytestmark = pytest.mark.gpu
FAST = -1  # SBH_LEVEL_FAST

FIXTURES = ["2.bam", "1.bam", "5k.bam", "1.2203053-2211029.bam"]


@pytest.fixture(scope="module")
def ctx():
    c = sb.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("n", [0, 1, 3, PAYLOAD, PAYLOAD + 1, 5 * PAYLOAD + 123])
def test_gpu_equals_host_build(ctx, n):
    rng = np.random.default_rng(n)
    for data in (rng.integers(0, 256, n, dtype=np.uint8), np.zeros(n, np.uint8),
                 rng.integers(0, 4, n, dtype=np.uint8)):
        got, nb, _ = ctx.bgzf_compress(data, level=FAST)
        assert nb == (n + PAYLOAD - 1) // PAYLOAD
        assert got.tobytes() == compress(data.tobytes())


def test_batches_of_members(ctx):
    """More members than one batch (DEFLATE_BATCH = 2048): members are independent, so each
    equals the host build of its own 65498-byte piece; every member re-inflates (zlib)."""
    nbatch = 2048
    nb = nbatch + 3
    n = (nb - 1) * PAYLOAD + 777
    rng = np.random.default_rng(11)
    flat = OracleFile(np.fromfile(golden_bam("5k.bam"), dtype=np.uint8)).uncompressed()
    data = np.resize(flat, n)
    data[::4099] = rng.integers(0, 256, data[::4099].size, dtype=np.uint8)  # no two tiles alike
    got, k, _ = ctx.bgzf_compress(data, level=FAST)
    assert k == nb
    m = parse_members(got.tobytes())
    assert len(m) == nb + 1 and m[-1][2] == 0
    for b in [0, 1, nbatch - 1, nbatch, nbatch + 1, nb - 1]:
        piece = data[b * PAYLOAD:(b + 1) * PAYLOAD].tobytes()
        o, c = m[b][0], m[b][1]
        assert got[o:o + c].tobytes() + EOF == compress(piece), b
    assert b"".join(x[3] for x in m) == data.tobytes()


EOF = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


@pytest.mark.parametrize("name", FIXTURES)
def test_htsjdk_rewrite_fixture(ctx, name):
    data = np.fromfile(golden_bam(name), dtype=np.uint8)
    flat = OracleFile(data).uncompressed().tobytes()
    out = sb.htsjdk_rewrite(golden_bam(name), ctx=ctx, level=FAST).tobytes()
    assert out == compress(flat)
    check_roundtrip(flat)
    # the library's own GPU inflate + CRC check reads its writer's output back
    sh = ctx.shard(np.frombuffer(out, dtype=np.uint8))
    sh.index(0)
    sh.inflate()
    assert sh.verify_crc()[0] == 0
    assert sh.read_flat().tobytes() == flat


def test_rewrite_2bam_blocks_and_records(ctx):
    """2.bam was itself written by htsjdk: the rewrite's members have its usize sequence, and
    every .records position maps to the same (member index, offset)."""
    out = sb.htsjdk_rewrite(golden_bam("2.bam"), ctx=ctx, level=FAST).tobytes()
    m = parse_members(out)
    ref_blocks = read_blocks("2.bam")
    assert [x[2] for x in m[:-1]] == [u for _, _, u in ref_blocks]
    def flat_of(starts_usizes, bp, off):
        acc = 0
        for st, u in starts_usizes:
            if st == bp:
                return acc + off
            acc += u
        raise KeyError(bp)
    ref = [(b[0], b[2]) for b in ref_blocks]
    ours = [(x[0], x[2]) for x in m[:-1]]
    for i, (bp, off) in enumerate(read_records("2.bam")):
        mine_bp = ours[[b[0] for b in ref].index(bp)][0]
        assert flat_of(ours, mine_bp, off) == flat_of(ref, bp, off)


def test_rewrite_read_ranges(ctx):
    """-r: header + the selected records only (HTSJDKRewrite.scala:48-58)."""
    data = np.fromfile(golden_bam("2.bam"), dtype=np.uint8)
    flat = OracleFile(data).uncompressed()
    full = sb.load_reads(golden_bam("2.bam"), ctx=ctx)
    starts = full.cols["flat"].astype(np.int64)
    ends = np.append(starts[1:], flat.size)
    keep = set(range(10, 20)) | {100, 2499}
    want = flat[:starts[0]].tobytes() + b"".join(flat[starts[i]:ends[i]].tobytes() for i in sorted(keep))
    out = sb.htsjdk_rewrite(golden_bam("2.bam"), read_ranges=keep, ctx=ctx, level=FAST).tobytes()
    got = b"".join(x[3] for x in parse_members(out))
    assert got == want
    assert len(sb.load_reads(out, ctx=ctx)) == len(keep)


def _vpos_list(records_rows):
    return [(b << 16) | o for b, o in records_rows]


def test_htsjdk_rewrite_test_slice(ctx):
    """HTSJDKRewriteTest's `-r 100-1000` slice through the FAST coder: its compressed bytes are
    not zlib's (the default coder's are: test_zdeflate_gpu.py), everything else is pinned -- the
    uncompressed stream, the member usize column of `.blocks`, and `.records` mapped through
    (member index, offset)."""
    out = sb.htsjdk_rewrite(golden_bam("2.bam"), read_ranges=range(100, 1000), ctx=ctx, level=FAST).tobytes()
    ref = np.fromfile(golden_bam("2.100-1000.bam"), dtype=np.uint8).tobytes()
    m, mr = parse_members(out), parse_members(ref)
    flat, flat_ref = b"".join(x[3] for x in m), b"".join(x[3] for x in mr)
    assert len(flat_ref) == 578330 and flat == flat_ref
    ref_blocks = read_blocks("2.100-1000.bam")
    assert [x[2] for x in m[:-1]] == [u for _, _, u in ref_blocks]  # 8 x 65498, 54346
    assert [x[0] for x in mr[:-1]] == [s for s, _, _ in ref_blocks]
    # .records of the fixture, re-expressed on this file's members
    member_of_ref = {s: i for i, (s, _, _) in enumerate(ref_blocks)}
    want = [(m[member_of_ref[b]][0] << 16) | o for b, o in read_records("2.100-1000.bam")]
    sh = ctx.shard(np.frombuffer(out, dtype=np.uint8))
    try:
        sh.index(0)
        sh.inflate()
        of = OracleFile(np.frombuffer(out, dtype=np.uint8))
        sh.set_contigs(of.contig_len)
        fs = sh.flat_size
        first = sh.find_record_start(of.header_end)[0]
        assert first == of.header_end
        starts = sh.records(first, fs)["flat"]
        got = []
        for f in starts.tolist():
            bp, off = sh.pos_of(int(f))
            got.append((bp << 16) | off)
        assert len(got) == 900 and got == want
    finally:
        sh.close()
