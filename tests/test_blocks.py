"""Blocks.apply (check/src/main/scala/org/hammerlab/bam/check/Blocks.scala:47-208): the blocks the
all-positions modes examine, per partition, against the reference's own BlocksTest
(check/src/test/scala/org/hammerlab/bam/check/BlocksTest.scala): IndexedBlocksTest reads
`1.bam.blocks` (host only, runs here), UnindexedBlocksTest finds the blocks of `1.noblocks.bam`
(the same bytes without `.blocks`) with FindBlockStart per split on the device."""
import pytest

from conftest import golden_bam
from pkg import sb

import spark_bam_amd.api as api  # noqa: E402

ALL_BLOCKS = [
    [0, 14146, 39374, 65429, 89707],
    [113583, 138333, 163285, 188181],
    [213608, 239479, 263656, 287709],
    [312794, 336825, 361204, 386382],
    [410905, 435247, 459832, 484396, 508565],
    [533464, 558458, 583574],
]
ALL_BOUNDS = [(0, 102400), (102400, 204800), (204800, 307200), (307200, 409600), (409600, 512000),
              (512000, 614400)]
# "block boundaries": -i 10k-39374,287709-312795 -m 10k
RANGES = [(10240, 39374), (287709, 312795)]
INDEXED_BOUNDARY_BLOCKS = [[14146], [], [287709], [], [312794]]
INDEXED_BOUNDARY_BOUNDS = [(0, 10240), (10240, 20480), (20480, 30720), (30720, 40960), (40960, 51200)]
UNINDEXED_BOUNDARY_BLOCKS = [[14146], [], [], [287709], [], [312794]]
UNINDEXED_BOUNDARY_BOUNDS = [(10240, 20480), (20480, 30720), (30720, 40960), (286720, 296960), (296960, 307200),
                             (307200, 317440)]


def starts(parts):
    return [[m.start for m in p] for p in parts]


def unindexed(**kw):
    # 1.noblocks.bam is a link to 1.bam in the reference: the same bytes, no `.blocks` beside them
    return api.blocks(golden_bam("1.bam"), blocks_path="/nonexistent/1.noblocks.bam.blocks", **kw)


def test_indexed_all_blocks():
    parts, bounds = api.blocks(golden_bam("1.bam"), split_size=100 * 1024)
    assert starts(parts) == ALL_BLOCKS and bounds == ALL_BOUNDS


@pytest.mark.parametrize("ranges", [[(0, 1)], [(0, 10240)]])  # "-i 0" and "-i 0+10k"
def test_indexed_header_block_only(ranges):
    parts, bounds = api.blocks(golden_bam("1.bam"), ranges=ranges)
    assert starts(parts) == [[0]] and bounds == [(0, 2097152)]


def test_indexed_block_boundaries():
    parts, bounds = api.blocks(golden_bam("1.bam"), split_size=10 * 1024, ranges=RANGES)
    assert starts(parts) == INDEXED_BOUNDARY_BLOCKS and bounds == INDEXED_BOUNDARY_BOUNDS


def test_indexed_metadata_fields():
    parts, _ = api.blocks(golden_bam("2.bam"))
    from conftest import read_blocks
    assert [tuple(m) for p in parts for m in p] == read_blocks("2.bam")


@pytest.mark.gpu
def test_unindexed_all_blocks():
    parts, bounds = unindexed(split_size=100 * 1024)
    assert starts(parts) == ALL_BLOCKS and bounds == ALL_BOUNDS


@pytest.mark.gpu
@pytest.mark.parametrize("ranges", [[(0, 1)], [(0, 10240)]])
def test_unindexed_header_block_only(ranges):
    parts, bounds = unindexed(ranges=ranges)
    assert starts(parts) == [[0]] and bounds == [(0, 2097152)]


@pytest.mark.gpu
def test_unindexed_block_boundaries():
    parts, bounds = unindexed(split_size=10 * 1024, ranges=RANGES)
    assert starts(parts) == UNINDEXED_BOUNDARY_BLOCKS and bounds == UNINDEXED_BOUNDARY_BOUNDS


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["1.bam", "2.bam", "5k.bam", "1.2203053-2211029.bam"])
@pytest.mark.parametrize("split", [2 << 20, 65536, 10000])
def test_unindexed_equals_blocks_file(name, split):
    """Without `.blocks`, the blocks found on the device are the `.blocks` file's, in order, with
    their sizes (every split's FindBlockStart lands on the block chain)."""
    from conftest import read_blocks
    parts, _ = api.blocks(golden_bam(name), split_size=split, blocks_path="/nonexistent")
    assert [tuple(m) for p in parts for m in p] == read_blocks(name)


@pytest.mark.gpu
def test_unindexed_small_windows_and_empty_blocks():
    """sbh_find_blocks with windows of a few splits, on a corpus with empty blocks mid-file:
    MetadataStream stops at an empty block (MetadataStream.scala:43-45), so a split's blocks end
    there and the blocks after it belong to no split until the next split's FindBlockStart --
    checked against a host walk of the device block table."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
    import numpy as np
    import synth
    p = synth.params(0x5B4D00AE, shape=2, level=-1, empty_every=5)
    data = synth.make_bam(p, 30000)[0]
    with sb.Context(0) as ctx:
        sh = ctx.shard(data)
        sh.index(0)
        chain = sh.blocks()  # (start, csize, usize, ustart, hsize, flags)
        sh.close()
        split = 50000
        splits = api.file_splits(data.size, split)
        splits = [(i * split, min(data.size, (i + 1) * split)) for i in range(-(-data.size // split))]
        got = ctx.find_blocks(data, splits, window=150000)
        want = []
        starts_ = [b[0] for b in chain]
        for k, (s, e) in enumerate(splits):
            fbs = sh_fbs(ctx, data, s)
            i = starts_.index(fbs)
            while i < len(chain) and chain[i][0] < e and not (chain[i][5] & sb.BLOCK_EMPTY):
                want.append((k, chain[i][0], chain[i][1], chain[i][2]))
                i += 1
        assert got == want
        assert any(b[5] & sb.BLOCK_EMPTY for b in chain[:-1]), "the corpus should hold empty blocks mid-file"
        assert np.unique([g[1] for g in got]).size == len(got)


def sh_fbs(ctx, data, s):
    sh = ctx.shard(data)
    try:
        return sh.find_block_start(s)
    finally:
        sh.close()
