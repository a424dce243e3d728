"""The index's block chain (sbh_index, MetadataStream._advance: MetadataStream.scala:23-54): the
linear path -- every candidate header from the start on is the previous block's successor, so
marks and ranks are direct and no pointer-jumping rounds run -- against the pointer-jumping path
(SBH_CHAIN_JUMP=1, which every chain whose candidates are not all chained takes) and the
reference's .blocks files, on streams where the linear assumption holds and where it does not: a
header planted inside a block's compressed bytes (a candidate off the chain), a link broken by a
wrong BSIZE, a start past earlier candidates, a shard cut inside a block."""
import os

import numpy as np
import pytest

from conftest import golden_bam, read_blocks
from pkg import sb

pytestmark = pytest.mark.gpu

FIXTURES = ["2.bam", "1.bam", "5k.bam", "2.100-1000.bam"]


@pytest.fixture(scope="module")
def ctx():
    c = sb.Context(0)
    yield c
    c.close()


def index_run(ctx, data, start=0, jump=False):
    """(n_blocks, flat_size, blocks) of one index call, or the exception it raised."""
    old = os.environ.get("SBH_CHAIN_JUMP")
    os.environ["SBH_CHAIN_JUMP"] = "1" if jump else "0"
    sh = ctx.shard(np.ascontiguousarray(data))
    try:
        nb, fs = sh.index(start)
        return nb, fs, sh.blocks()
    except Exception as e:  # (compared by type and message)
        return type(e).__name__, str(e)
    finally:
        sh.close()
        if old is None:
            os.environ.pop("SBH_CHAIN_JUMP", None)
        else:
            os.environ["SBH_CHAIN_JUMP"] = old


def both(ctx, data, start=0):
    a, b = index_run(ctx, data, start, False), index_run(ctx, data, start, True)
    assert a == b
    return a


def data_blocks(blocks):
    return [(s, c, u) for s, c, u, _us, _h, f in blocks if not f & sb.BLOCK_EMPTY]


@pytest.mark.parametrize("name", FIXTURES)
def test_linear_equals_jumping(ctx, name):
    data = np.fromfile(golden_bam(name), dtype=np.uint8)
    nb, fs, bl = both(ctx, data)
    assert data_blocks(bl) == read_blocks(name)


def bgzf_header(csize):
    """An 18-byte BGZF member header (BC subfield, BSIZE = csize - 1)."""
    h = bytes([31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0]) + int(csize - 1).to_bytes(2, "little")
    return np.frombuffer(h, dtype=np.uint8)


def test_planted_header_off_chain(ctx):
    # a valid-looking header inside block 3's compressed bytes: a candidate the chain steps over
    # (the next real header is block 3's start + its BSIZE + 1), so the chain is not linear
    data = np.fromfile(golden_bam("2.bam"), dtype=np.uint8).copy()
    want = read_blocks("2.bam")
    s3, c3, _ = want[3]
    for off, cs in ((100, 1000), (200, c3 - 200), (300, 70000 % 65536)):
        d = data.copy()
        d[s3 + off: s3 + off + 18] = bgzf_header(cs)
        nb, fs, bl = both(ctx, d)
        assert data_blocks(bl) == want  # (the index reads headers and footers only)


def test_start_past_candidates(ctx):
    data = np.fromfile(golden_bam("1.bam"), dtype=np.uint8)
    want = read_blocks("1.bam")
    for k in (1, 5, len(want) - 2):
        nb, fs, bl = both(ctx, data, start=want[k][0])
        assert data_blocks(bl) == want[k:]


def test_broken_link_and_truncation(ctx):
    data = np.fromfile(golden_bam("2.bam"), dtype=np.uint8)
    want = read_blocks("2.bam")
    s5, c5, _ = want[5]
    d = data.copy()
    d[s5 + 16: s5 + 18] = np.frombuffer(int(c5 - 1 - 7).to_bytes(2, "little"), dtype=np.uint8)  # BSIZE 7 short
    both(ctx, d)  # the chain stops at block 5's wrong successor: both paths alike
    for cut in (want[4][0] + 9, want[4][0] + want[4][1] // 2, want[4][0]):
        both(ctx, data[:cut])
