"""BGZF writer on the GPU (sbh_bgzf_compress / htsjdk_rewrite; HTSJDKRewrite.scala:40-67).
k_deflate runs deflate_core.h one lane per block, so its file must equal the host build's
byte for byte (test_deflate_cpu.py pins that build against zlib); the rewritten fixtures
re-inflate (zlib and this library's own GPU inflate + CRC check) to the original stream."""
import zlib

import numpy as np
import pytest

from conftest import golden_bam, read_blocks, read_records
from oracle_lib import OracleFile
from pkg import sb
from test_deflate_cpu import PAYLOAD, check_roundtrip, compress, parse_members

pytestmark = pytest.mark.gpu

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
        got, nb, _ = ctx.bgzf_compress(data)
        assert nb == (n + PAYLOAD - 1) // PAYLOAD
        assert got.tobytes() == compress(data.tobytes())


@pytest.mark.parametrize("name", FIXTURES)
def test_htsjdk_rewrite_fixture(ctx, name):
    data = np.fromfile(golden_bam(name), dtype=np.uint8)
    flat = OracleFile(data).uncompressed().tobytes()
    out = sb.htsjdk_rewrite(golden_bam(name), ctx=ctx).tobytes()
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
    out = sb.htsjdk_rewrite(golden_bam("2.bam"), ctx=ctx).tobytes()
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
    out = sb.htsjdk_rewrite(golden_bam("2.bam"), read_ranges=keep, ctx=ctx).tobytes()
    got = b"".join(x[3] for x in parse_members(out))
    assert got == want
    assert len(sb.load_reads(out, ctx=ctx)) == len(keep)
