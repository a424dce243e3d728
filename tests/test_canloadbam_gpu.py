"""The Scala load-API facade (jni/Native.scala GpuCanLoadBam / GpuSplitPartition /
GpuIntervalsPartition) run through its Python twin (spark_bam_amd.canloadbam: the same C-ABI
calls per Spark task), against the reference's own test answers:

  LoadBAMTest "1e6" / "1e5" / "2e4" partition counts, "indexed all" / "indexed disjoint
  regions" / "indexed intervals empty result" (load/src/test/.../LoadBAMTest.scala:21-113),
  ComputeSplitsTest "eager 230KB" / "compare 240KB" splits (cli/src/test/.../ComputeSplitsTest),
  CountReadsTest (4917 reads of 1.bam);

and the records themselves against the resident decode (every column, vpos included).  Also the
reference's exceptions with their constructor fields: NoReadFoundException(path, start,
maxReadSize), HeaderSearchFailedException(path, start, positionsAttempted),
HeaderParseException(idx, actual, expected).
"""
import numpy as np
import pytest

from conftest import golden_bam
from pkg import sb

pytestmark = pytest.mark.gpu

clb = __import__(sb.__name__ + ".canloadbam", fromlist=["x"])


@pytest.fixture(scope="module")
def ctx():
    c = sb.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("size,expected", [
    (1000000, [2500]),
    (100000, [503, 414, 518, 421, 493, 151]),
    (20000, [96, 102, 105, 101, 99, 102, 101, 106, 0, 105, 105, 102, 104, 103, 104, 106,
             104, 106, 0, 105, 195, 101, 0, 99, 98, 99, 52]),
])
def test_load_bam_partitions(ctx, size, expected):
    # LoadBAMTest 1e6 / 1e5 / 2e4: sc.loadReads(2.bam, splitSize) partition sizes
    parts = clb.load_reads(golden_bam("2.bam"), split_size=size, ctx=ctx)
    assert [p.n for p in parts] == expected


@pytest.mark.parametrize("size,expected", [
    (230 * 1024, ["0:45846-239479:312", "239479:312-484396:25", "484396:25-597482:0"]),
    (240 * 1024, ["0:45846-263656:191", "263656:191-508565:287", "508565:287-597482:0"]),
])
def test_load_splits_and_reads(ctx, size, expected):
    # ComputeSplitsTest "eager 230KB" / "compare 240KB"; CountReadsTest 4917
    splits, parts = clb.load_splits_and_reads(golden_bam("1.bam"), split_size=size, ctx=ctx)
    assert [f"{a}-{b}" for a, b in splits] == expected
    assert sum(p.n for p in parts) == 4917


@pytest.mark.parametrize("name,size", [("2.bam", 20000), ("1.bam", 100000), ("5k.bam", 64 * 1024)])
def test_partition_records_equal_resident_decode(ctx, name, size):
    """The partitions' records, joined, are the file's records (resident decode), every column."""
    parts = clb.load_reads_and_positions(golden_bam(name), split_size=size, ctx=ctx)
    joined = sb.Reads.concat(parts, parts[0].ref_names)
    one = sb.load_reads(golden_bam(name), ctx=ctx)
    assert joined.n == one.n
    for k in one.cols:
        if k != "flat":  # flat offsets are per-partition shard offsets
            assert np.array_equal(joined.cols[k], one.cols[k]), k
    # each record lies in the partition of the split its Pos falls in (vpos < Pos(end, 0))
    for (start, end), p in zip(sb.file_splits(int(np.fromfile(golden_bam(name), np.uint8).size), size), parts):
        if p.n:
            assert int(p.cols["vpos"].max()) < (end << 16)


@pytest.mark.parametrize("intervals,n_parts,count,split", [
    ("1:0-100000", 1, 2450, None),                       # "indexed all"
    ("1:13000-14000,1:60000-61000", 1, 129, None),       # "indexed disjoint regions"
    ("1:13000-14000,1:60000-61000", 2, 129, 10000),      # ... splitSize 10000
    ("1:2000000-3000000", 1, 0, None),                   # "indexed intervals empty result"
])
def test_load_bam_intervals(ctx, intervals, n_parts, count, split):
    kw = {} if split is None else {"split_size": split}
    parts = clb.load_bam_intervals(golden_bam("2.bam"), intervals, ctx=ctx, **kw)
    assert len(parts) == n_parts and sum(p.n for p in parts) == count
    # the same records as the one-device path
    one = sb.load_bam_intervals(golden_bam("2.bam"), intervals, ctx=ctx, **kw)
    joined = sb.Reads.concat(parts, one.reads.ref_names)
    assert joined.n == one.reads.n
    for k in ("vpos", "ref_id", "pos", "flag", "names", "cigar", "seq", "qual"):
        assert np.array_equal(joined.cols[k], one.reads.cols[k]), k


def test_no_read_found_exception(ctx):
    """FindRecordStart.apply throws NoReadFoundException(path, blockStart, maxReadSize) when no
    record starts within maxReadSize positions (FindRecordStart.scala:11-30,66-71): 1.bam's first
    split after the header starts 45846 bytes into its first block."""
    path = golden_bam("1.bam")
    with pytest.raises(sb.NoReadFoundException) as e:
        clb.load_reads_and_positions(path, split_size=1 << 30, max_read_size=1000, ctx=ctx)
    assert e.value.path == path and e.value.start == 0 and e.value.max_read_size == 1000


def test_header_search_failed_exception(ctx):
    """FindBlockStart over bytes with no BGZF header throws HeaderSearchFailedException(path,
    start, positionsAttempted = MAX_BLOCK_SIZE) (FindBlockStart.scala:18-35)."""
    rng = np.random.default_rng(5)
    junk = rng.integers(0, 256, 300_000, dtype=np.uint8)
    junk[junk == 31] = 30  # no gzip magic anywhere
    sh = ctx.shard(junk)
    try:
        with pytest.raises(sb.HeaderSearchFailedException) as e:
            sh.find_block_start(1000)
        assert e.value.start == 1000 and e.value.positions_attempted == 65536
    finally:
        sh.close()


def test_header_parse_exception_fields(ctx):
    """MetadataStream from a position that is not a header throws HeaderParseException(idx,
    actual, expected) for the first byte Header.make rejects (Header.scala:48-71): 2.bam's byte 1
    is 139 (the magic's second byte), read as the signed Byte -117, where 31 is expected."""
    data = np.fromfile(golden_bam("2.bam"), dtype=np.uint8)
    sh = ctx.shard(data)
    try:
        with pytest.raises(sb.HeaderParseException) as e:
            sh.index(1)
        assert (e.value.idx, e.value.actual, e.value.expected) == (0, -117, 31)
    finally:
        sh.close()
