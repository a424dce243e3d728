"""loadBamIntervals: BAI parsing + htsjdk chunk selection on the host,
record streams + region filter on the GPU.

CPU tests pin the host logic and the oracle against LoadBAMTest's "indexed *" goldens
(load/src/test/scala/org/hammerlab/bam/spark/load/LoadBAMTest.scala:46-113) and against a
brute-force property: for any intervals, the records the BAI chunks yield after the
region filter are exactly the records of the whole file whose region overlaps (a BAI is
complete, so chunk selection may only drop records that cannot overlap).  GPU tests run
load_bam_intervals through the C-ABI and compare its columns with the oracle's.
"""
import random

import numpy as np
import pytest

from conftest import golden_bam
from oracle_lib import OracleFile
import oracle_records as orr
from pkg import sb

intervals_mod = __import__(sb.__name__ + ".intervals", fromlist=["x"])
P = sb.Pos


def _chunks(name, text):
    idx = sb.read_bai(golden_bam(name) + ".bai")
    names, lens, _ = _header(name)
    loci = sb.parse_loci(text, dict(zip(names, lens)))
    return sb.get_interval_chunks(idx, loci, names)


_HDR = {}


def _header(name):
    if name not in _HDR:
        data = np.fromfile(golden_bam(name), dtype=np.uint8)
        of = OracleFile(data)
        flat = of.uncompressed()
        names, lens, end = sb.parse_bam_header(flat[:1 << 20])
        _HDR[name] = (names, [int(x) for x in lens], end, of, flat)
    return _HDR[name][:3]


def _oracle(name, text):
    """Oracle: chunk flats from the oracle's own Pos -> flat map, then the chain + region
    filter of oracle_records."""
    names, lens, _ = _header(name)
    of, flat = _HDR[name][3], _HDR[name][4]
    chunks = _chunks(name, text)
    loci = sb.parse_loci(text, dict(zip(names, lens)))
    by_ref = {names.index(c): rs for c, rs in loci.items()}

    def fl(p):
        return flat.size if p.block_pos >= of.data.size else of.flat_of(p.block_pos, p.offset)

    cols, per = orr.interval_records(flat, [(fl(c.start), fl(c.end)) for c in chunks], by_ref)
    return chunks, cols, per


def test_read_bai_2bam():
    idx = sb.read_bai(golden_bam("2.bam") + ".bai")
    assert len(idx.references) == 84
    r0 = idx.references[0]
    assert r0.metadata is not None and r0.metadata.num_mapped + r0.metadata.num_unmapped == 2500
    assert r0.offsets[0] == P(0, 5650)
    assert all(not r.bins for r in idx.references[1:])


def test_read_bai_bad_magic():
    with pytest.raises(IOError):
        sb.read_bai(b"BAM\1" + b"\0" * 16)


@pytest.mark.parametrize("text,want", [
    ("1:0-100000", [(P(0, 5650), P(531725, 0))]),                           # "indexed all"
    ("1:13000-14000,1:60000-61000", [(P(0, 5650), P(314028, 45444)),
                                      (P(439897, 20150), P(439897, 39777))]),  # "indexed disjoint regions"
    ("1:2000000-3000000", []),                                              # "indexed intervals empty result"
])
def test_get_interval_chunks_golden(text, want):
    assert [(c.start, c.end) for c in _chunks("2.bam", text)] == want


@pytest.mark.parametrize("text,split,parts,count", [
    ("1:0-100000", 32 << 20, 1, 2450),
    ("1:13000-14000,1:60000-61000", 32 << 20, 1, 129),
    ("1:13000-14000,1:60000-61000", 10000, 2, 129),
    ("1:2000000-3000000", 32 << 20, 0, 0),
])
def test_partitions_and_oracle_count_golden(text, split, parts, count):
    chunks, cols, per = _oracle("2.bam", text)
    groups = intervals_mod.capped_cost_groups(chunks, intervals_mod.chunk_size, float(split))
    # the reference's RDD has max(1, #groups) partitions (CanLoadBam.scala:114-121)
    assert max(1, len(groups)) == max(1, parts)
    assert cols["flat"].size == sum(per) == count


def _brute(name, by_ref):
    names, lens, end = _header(name)
    flat = _HDR[name][4]
    cols = orr.decode(flat, orr.record_starts(flat, end, flat.size))
    return [int(cols["flat"][i]) for i in range(cols["flat"].size) if orr.region_kept(cols, i, by_ref)]


@pytest.mark.parametrize("name", ["2.bam", "5k.bam"])
def test_chunks_cover_every_overlapping_record(name):
    names, lens, _ = _header(name)
    rng = random.Random(0x5B4D)
    for _ in range(12):
        k = rng.randint(1, 3)
        parts = []
        for _ in range(k):
            a = rng.randint(0, 80000)
            parts.append(f"1:{a}-{a + rng.choice([1, 50, 700, 5000, 30000])}")
        text = ",".join(parts)
        loci = sb.parse_loci(text, dict(zip(names, lens)))
        by_ref = {names.index(c): rs for c, rs in loci.items()}
        _, cols, _ = _oracle(name, text)
        assert sorted(int(x) for x in cols["flat"]) == _brute(name, by_ref), text


def test_parse_loci_forms():
    lens = {"1": 1000, "2": 500}
    assert sb.parse_loci("1:10-20,1:15-30,2:5", lens) == {"1": [(10, 30)], "2": [(5, 6)]}
    assert sb.parse_loci("2", lens) == {"2": [(0, 500)]}
    assert sb.parse_loci("1:900-", lens) == {"1": [(900, 1000)]}
    assert sb.parse_loci("1:20-30,1:30-40", lens) == {"1": [(20, 40)]}
    with pytest.raises(ValueError):
        sb.parse_loci("chrZ:1-2", lens)


def test_optimize_chunk_list_rules():
    opt = intervals_mod.optimize_chunk_list
    # overlapping within a block coalesce; adjacent blocks coalesce; linear-index cut
    assert opt([(10 << 16 | 5, 10 << 16 | 50), (10 << 16 | 40, 12 << 16 | 1)], 0) == [(10 << 16 | 5, 12 << 16 | 1)]
    assert opt([(1 << 16, 5 << 16 | 7), (5 << 16 | 9, 9 << 16)], 0) == [(1 << 16, 9 << 16)]
    assert opt([(1 << 16, 2 << 16), (5 << 16, 6 << 16)], 0) == [(1 << 16, 2 << 16), (5 << 16, 6 << 16)]
    assert opt([(1 << 16, 2 << 16), (5 << 16, 6 << 16)], 3 << 16) == [(5 << 16, 6 << 16)]


# ---------------------------------------------------------------- GPU (through the C-ABI)

COLS = ("ref_id", "pos", "next_ref_id", "next_pos", "tlen", "flag", "bin", "mapq", "name_off",
        "cigar_off", "seq_off", "aux_off", "names", "cigar", "seq", "qual", "aux")


@pytest.fixture(scope="module")
def ctx():
    c = sb.Context(0)
    yield c
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("text,split,parts,count", [
    ("1:0-100000", 32 << 20, 1, 2450),
    ("1:13000-14000,1:60000-61000", 32 << 20, 1, 129),
    ("1:13000-14000,1:60000-61000", 10000, 2, 129),
    ("1:2000000-3000000", 32 << 20, 0, 0),
])
def test_gpu_load_bam_intervals_golden(ctx, text, split, parts, count):
    res = sb.load_bam_intervals(golden_bam("2.bam"), text, split_size=split, ctx=ctx)
    assert len(res.reads) == sum(res.counts) == count
    assert len(res.partitions) == parts
    _, want, per = _oracle("2.bam", text)
    _check_cols("2.bam", res, want)


def _check_cols(name, res, want):
    of = _HDR[name][3]
    vp = [(lambda bp, off: (bp << 16) | off)(*of.pos_of(int(f))) for f in want["flat"]]
    assert [int(v) for v in res.reads.cols["vpos"]] == vp
    for k in COLS:
        assert np.array_equal(res.reads.cols[k], want[k]), k


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["2.bam", "5k.bam"])
def test_gpu_load_bam_intervals_random(ctx, name):
    rng = random.Random(0xB41)
    for _ in range(6):
        parts = []
        for _ in range(rng.randint(1, 4)):
            a = rng.randint(0, 80000)
            parts.append(f"1:{a}-{a + rng.choice([1, 100, 2000, 20000])}")
        text = ",".join(parts)
        res = sb.load_bam_intervals(golden_bam(name), text, ctx=ctx)
        _, want, per = _oracle(name, text)
        assert sum(res.counts) == sum(per)
        _check_cols(name, res, want)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["2.bam", "5k.bam"])
def test_gpu_load_bam_intervals_small_shards(ctx, name):
    """One device shard per chunk (merge_gap 0) starting with a 4 KiB halo: the halo must
    grow until every kept record and eager check is inside its shard."""
    text = "1:100-900,1:13000-14000,1:30000-30100,1:60000-61000"
    res = sb.load_bam_intervals(golden_bam(name), text, ctx=ctx, halo=4096, merge_gap=0)
    _, want, per = _oracle(name, text)
    assert res.counts and sum(res.counts) == sum(per)
    _check_cols(name, res, want)
