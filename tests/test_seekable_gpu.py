"""The seekable byte view on the GPU (spark_bam_amd.seekable: the twin of jni/Native.scala's
GpuSeekableStream under the reference's SeekableUncompressedBytes, and of GpuFindRecordStart
reading through the caller's view) against the reference's own ByteStreamTest numbers
(bgzf/src/test/.../block/ByteStreamTest.scala:12-95, on 2.bam) and the CPU oracle:

  * SeekableStream.seek(newPos) (Stream.scala:112-121): True unless already positioned there;
  * the Block sequence: every block of the oracle's stream, and the empty block ending it
    (Stream.scala:56-58), including one in the middle of a file;
  * SeekableUncompressedBytes.seek(pos) + reads across block ends, curPos rolling to
    Pos(next block, 0) when a block is used up, at random positions vs the oracle's bytes;
  * windows much smaller than the file (reloads), and a seek back into the window (no reload);
  * FindRecordStart through the view (FindRecordStart.scala:11-63): 1.bam 239479 -> 239479:312
    (FindRecordStartTest) and random starts vs the oracle."""
import os
import sys

import numpy as np
import pytest

from conftest import golden_bam
from oracle_lib import OR_OK, OracleFile
from pkg import sb

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
sk = __import__(sb.__name__ + ".seekable", fromlist=["x"])
sharded = __import__(sb.__name__ + ".sharded", fromlist=["x"])
Pos = sb.Pos


@pytest.fixture(scope="module")
def ctx():
    c = sb.Context(0)
    yield c
    c.close()


def view(ctx, data, window=16 << 20, contigs=None):
    return sk.seekable_uncompressed_bytes(ctx, sharded.bytes_reader(data), window=window, halo=1 << 16,
                                          contigs=contigs)


def read_string(v, n, includes_null=True):
    b = v.read(n).tobytes()
    return b[:-1].decode() if includes_null else b.decode()


def check_header(v):
    """ByteStreamTest.checkHeader (ByteStreamTest.scala:14-55), 2.bam."""
    v.position = 0  # (a fresh ByteChannel over the view)
    assert read_string(v, 4, includes_null=False) == "BAM\1"
    assert v.get_int() == 4253
    text = v.read(4253).tobytes().decode()
    assert text[:100] == ("@HD\tVN:1.5\tGO:none\tSO:coordinate\n@SQ\tSN:1\tLN:249250621\n"
                          "@SQ\tSN:2\tLN:243199373\n@SQ\tSN:3\tLN:198022430\n@")
    assert v.get_int() == 84
    v.skip(5646 - v.position)
    assert v.cur_pos == Pos(0, 5646)
    assert v.get_int() == 547496
    assert v.cur_pos == Pos(0, 5650)
    assert v.get_int() == 620
    assert v.cur_pos == Pos(0, 5654)
    v.skip(65498 - 4 - v.position)
    v.clear()
    assert v.cur_pos == Pos(0, 65498 - 4)
    v.get_int()
    assert v.cur_pos == Pos(26169, 0)


@pytest.mark.parametrize("window", [16 << 20, 40_000])
def test_seekable_byte_stream(ctx, window):
    """ByteStreamTest "SeekableByteStream": checkHeader, checkRead twice, seek(Pos(0, 0)),
    checkHeader again."""
    data = np.fromfile(golden_bam("2.bam"), dtype=np.uint8)
    v = view(ctx, data, window)
    try:
        check_header(v)

        def check_read():
            v.seek(Pos(26169, 16277))
            assert v.get_int() == 642
            assert v.get_int() == 0
            assert v.get_int() == 12815
            name_len = v.get_int() & 0xff
            v.skip(20)
            assert read_string(v, name_len) == "HWI-ST807:461:C2P0JACXX:4:2311:16471:84756"

        check_read()
        loaded = v.block_stream.windows_loaded
        check_read()
        if window > data.size:  # the seek back lands in the resident window: nothing re-inflated
            assert v.block_stream.windows_loaded == loaded
        v.seek(Pos(0, 0))
        check_header(v)
    finally:
        v.close()


def test_seek_return_values(ctx):
    data = np.fromfile(golden_bam("2.bam"), dtype=np.uint8)
    of = OracleFile(data)
    s = sk.SeekableStream(ctx, sharded.bytes_reader(data))
    try:
        assert s.seek(0) is False          # already there: hasNext and pos == 0
        assert s.pos == 0
        b1 = of.blocks[1][0]
        assert s.seek(b1) is True and s.pos == b1
        assert s.seek(b1) is False
        s.next()
        assert s.pos == of.blocks[2][0]
        # after the stream's end (the EOF empty block) hasNext is false: any seek moves
        for _ in s:
            pass
        assert not s.has_next() and s.seek(0) is True and s.pos == 0
    finally:
        s.close()


@pytest.mark.parametrize("name", ["1.bam", "2.bam", "5k.bam"])
def test_blocks_equal_oracle_stream(ctx, name):
    data = np.fromfile(golden_bam(name), dtype=np.uint8)
    of = OracleFile(data)
    flat = of.uncompressed()
    s = sk.SeekableStream(ctx, sharded.bytes_reader(data), window=100_000, halo=1 << 16)
    try:
        got = [(b.start, b.compressed_size, b.uncompressed_size, bytes(b.bytes)) for b in s]
        want, u = [], 0
        for st, cs, us in of.blocks:
            want.append((st, cs, us, flat[u:u + us].tobytes()))
            u += us
        assert got == want
        assert s.windows_loaded > 1 or data.size < 100_000
    finally:
        s.close()


def test_empty_block_ends_the_stream(ctx):
    """An empty BGZF block in the middle of a file ends the Block stream (Stream.scala:56-58);
    a seek past it starts a new one."""
    import synth
    data = synth.make_bam(synth.params(0x5B4D00AE, shape=2, level=-1, empty_every=5), 3000)[0]
    of = OracleFile(data)
    s = sk.SeekableStream(ctx, sharded.bytes_reader(data), window=200_000)
    try:
        got = [(b.start, b.compressed_size, b.uncompressed_size) for b in s]
        assert got == [(st, cs, us) for st, cs, us in of.blocks]
        end = of.blocks[-1][0] + of.blocks[-1][1]
        assert end < data.size - 28  # (the empty block is mid-file, not the EOF marker)
        nxt = end + 28  # past the empty block (28 bytes)
        of2 = OracleFile(data, start=nxt)
        assert s.seek(nxt) is True
        assert [(b.start, b.compressed_size) for b in s][:5] == [(st, cs) for st, cs, _ in of2.blocks[:5]]
    finally:
        s.close()


@pytest.mark.parametrize("name,window", [("1.bam", 16 << 20), ("1.bam", 50_000), ("5k.bam", 80_000)])
def test_random_seeks_and_reads(ctx, name, window):
    """seek(pos) + read(n) at random positions vs the oracle's bytes; curPos after the read is
    the oracle's canonical Pos of the flat offset reached (Pos(next, 0) at a block's end)."""
    data = np.fromfile(golden_bam(name), dtype=np.uint8)
    of = OracleFile(data)
    flat = of.uncompressed()
    ustarts = np.cumsum([0] + [b[2] for b in of.blocks])
    v = view(ctx, data, window)
    rng = np.random.default_rng(17)
    try:
        for _ in range(60):
            k = int(rng.integers(0, len(of.blocks)))
            st, _, us = of.blocks[k]
            off = int(rng.integers(0, us))
            n = int(rng.choice([1, 4, 37, 300, 70_000]))
            v.seek(Pos(st, off))
            assert v.cur_pos == Pos(st, off)
            f = int(ustarts[k]) + off
            got = v.read(n)
            assert np.array_equal(got, flat[f:f + n])
            f2 = f + got.size
            if f2 < flat.size:
                assert v.cur_pos == Pos(*of.pos_of(f2))
            else:
                assert v.cur_pos is None and not v.has_next()
    finally:
        v.close()


def test_find_record_start_through_the_view(ctx):
    """FindRecordStartTest: 1.bam from block 239479 -> Pos(239479, 312); random block starts vs
    the oracle's FindRecordStart; NoReadFoundException(path, start, maxReadSize)."""
    path = golden_bam("1.bam")
    data = np.fromfile(path, dtype=np.uint8)
    of = OracleFile(data)
    v = view(ctx, data, window=200_000, contigs=of.contig_len)
    try:
        assert sk.find_record_start(path, 239479, v) == Pos(239479, 312)
        assert v.cur_pos == Pos(239479, 312)  # (the view is left at the record)
        rng = np.random.default_rng(3)
        ustarts = np.cumsum([0] + [b[2] for b in of.blocks])
        for k in rng.integers(1, len(of.blocks), 12):
            st = of.blocks[int(k)][0]
            rc, f, _ = of.find_record_start(int(ustarts[int(k)]))
            assert rc == OR_OK
            assert sk.find_record_start(path, st, v) == Pos(*of.pos_of(f))
        with pytest.raises(sb.NoReadFoundException) as e:
            sk.find_record_start(path, 0, v, max_read_size=100)
        assert (e.value.path, e.value.start, e.value.max_read_size) == (path, 0, 100)
    finally:
        v.close()
