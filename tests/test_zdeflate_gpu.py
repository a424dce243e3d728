"""The byte-exact BGZF writer on the GPU (zdeflate.hip; sbh_bgzf_compress / _level) against zlib
1.2.11 driven like htsjdk's Deflater (tests/test_zdeflate_cpu.py's htsjdk_bgzf, which also pins
the host definition zdeflate_core.h) and against the reference's own files.

HTSJDKRewriteTest (cli/src/test/scala/org/hammerlab/bam/rewrite/HTSJDKRewriteTest.scala:14-24)
requires `htsjdk-rewrite -r 100-1000 2.bam` to equal slice/2.100-1000.bam byte for byte; the
htsjdk-written 2.bam / 1.bam / 1.2203053-2211029.bam must come back from their own streams."""
import os
import sys

import numpy as np
import pytest

from conftest import golden_bam, read_blocks, read_records
from oracle_lib import OracleFile
from pkg import sb
from test_zdeflate_cpu import CASES, EOF_MEMBER, PAYLOAD, htsjdk_bgzf, htsjdk_member, members

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


@pytest.fixture(scope="module")
def ctx():
    c = sb.Context(0)
    yield c
    c.close()


def test_htsjdk_rewrite_test_slice(ctx):
    out = sb.htsjdk_rewrite(golden_bam("2.bam"), read_ranges=range(100, 1000), ctx=ctx).tobytes()
    assert out == open(golden_bam("2.100-1000.bam"), "rb").read()
    # .blocks and .records of the output (the CLI's -b / -i) are the fixture's
    sh = ctx.shard(np.frombuffer(out, dtype=np.uint8))
    try:
        sh.index(0)
        sh.inflate()
        blocks = [(b[0], b[1], b[2]) for b in sh.blocks() if b[2]]
        assert blocks == read_blocks("2.100-1000.bam")
        of = OracleFile(np.frombuffer(out, dtype=np.uint8))
        sh.set_contigs(of.contig_len)
        starts = sh.records(of.header_end, sh.flat_size)["flat"]
        assert [sh.pos_of(int(f)) for f in starts.tolist()] == [tuple(r) for r in read_records("2.100-1000.bam")]
    finally:
        sh.close()


@pytest.mark.parametrize("name", ["2.bam", "1.bam", "1.2203053-2211029.bam"])
def test_htsjdk_fixture_reproduced(ctx, name):
    assert sb.htsjdk_rewrite(golden_bam(name), ctx=ctx).tobytes() == open(golden_bam(name), "rb").read()


@pytest.mark.parametrize("name", ["5k.bam", "1.block-aligned.bam"])
def test_level6_members(ctx, name):
    """samtools-written fixtures (zlib level 6): every member's payload, compressed alone at
    level 6, is that member (header, deflate bytes, footer)."""
    data = open(golden_bam(name), "rb").read()
    p = 0
    for u, raw in members(golden_bam(name)):
        bs = (data[p + 16] | data[p + 17] << 8) + 1
        if u:
            got, nb, _ = ctx.bgzf_compress(np.frombuffer(u, dtype=np.uint8), level=6)
            assert nb == 1 and got.tobytes() == data[p:p + bs] + EOF_MEMBER
        p += bs


@pytest.mark.parametrize("name", [k for k in CASES if k not in ("empty",)])
@pytest.mark.parametrize("level", [5, 6])
def test_synthetic_vs_zlib(ctx, name, level):
    data = CASES[name]
    got, _, _ = ctx.bgzf_compress(np.frombuffer(data, dtype=np.uint8), level=level)
    assert got.tobytes() == htsjdk_bgzf(data, level)


@pytest.mark.parametrize("level", [0, 4, 7, 8, 9])
def test_other_levels(ctx, level):
    data = CASES["quality_like"] + CASES["alphabet4"][:40000]
    got, _, _ = ctx.bgzf_compress(np.frombuffer(data, dtype=np.uint8), level=level)
    assert got.tobytes() == htsjdk_bgzf(data, level)


def test_empty_input(ctx):
    got, nb, _ = ctx.bgzf_compress(np.zeros(0, np.uint8))
    assert nb == 0 and got.tobytes() == EOF_MEMBER


def test_synthetic_bam_streams(ctx):
    """Config B / D / E streams (short reads, long reads, adversarial) as htsjdk would write them."""
    import synth
    for seed, shape, nrec in ((synth.SEEDS["B"], 0, 20000), (synth.SEEDS["D"], 1, 80), (synth.SEEDS["E"], 2, 20000)):
        p = synth.params(seed, shape=shape)
        flat = np.concatenate([synth.header_bytes(), synth.records(p, 0, nrec)])
        got, _, _ = ctx.bgzf_compress(flat)
        assert got.tobytes() == htsjdk_bgzf(flat.tobytes()), seed


def test_batches_of_members(ctx, monkeypatch):
    """More members than one batch (here 2048, SBH_ZDEFLATE_BATCH): each member equals htsjdk's
    for its own piece; the input sits on the device (an inflated shard's flat bytes go in this
    way)."""
    monkeypatch.setenv("SBH_ZDEFLATE_BATCH", "2048")
    nb = 2048 + 3
    n = (nb - 1) * PAYLOAD + 777
    rng = np.random.default_rng(11)
    flat = OracleFile(np.fromfile(golden_bam("2.bam"), dtype=np.uint8)).uncompressed()
    data = np.resize(flat, n)
    data[::4099] = rng.integers(0, 256, data[::4099].size, dtype=np.uint8)
    got, k, ms = ctx.bgzf_compress(data)
    assert k == nb and ms > 0
    got = got.tobytes()
    o = 0
    for b in range(nb):
        bs = (got[o + 16] | got[o + 17] << 8) + 1
        if b in (0, 1, 2047, 2048, 2049, nb - 1):
            assert got[o:o + bs] == htsjdk_member(data[b * PAYLOAD:(b + 1) * PAYLOAD].tobytes()), b
        o += bs
    assert got[o:] == EOF_MEMBER
