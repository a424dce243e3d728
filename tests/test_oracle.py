"""Pins the CPU oracle against the reference's own golden vectors (CPU only).

Each test names the reference test it restates (paths relative to the reference root).
"""
import numpy as np
import pytest

from conftest import GOLDEN, golden_bam, parse_total_error_counts, read_blocks, read_records
from oracle_lib import (FLAG_NAMES, FULL_N_SHIFT, FULL_SUCCESS, OR_OK, OracleFile,
                        file_splits, load_splits_and_reads, vpos_str)

FIXTURES = ["2.bam", "1.bam", "5k.bam", "1.2203053-2211029.bam", "2.100-1000.bam"]


@pytest.fixture(scope="module")
def files():
    return {n: OracleFile.from_path(golden_bam(n)) for n in FIXTURES}


@pytest.mark.parametrize("name", FIXTURES)
def test_blocks_index(files, name):
    # bgzf/src/test/.../index/IndexBlocksTest.scala, MetadataStreamTest.scala
    assert files[name].error == 0
    assert files[name].blocks == read_blocks(name)


@pytest.mark.parametrize("name", FIXTURES)
def test_eager_every_position_equals_records(files, name):
    # cli/src/test/.../CheckBamTest.scala ("eager 1.bam": All calls matched!) for every fixture
    of = files[name]
    n, bits = of.eager_range(0, of.flat_size)
    pos = np.flatnonzero(np.unpackbits(bits, bitorder="little")[: of.flat_size])
    recs = [of.flat_of(b, o) for b, o in read_records(name)]
    assert n == len(recs)
    assert pos.tolist() == recs


@pytest.mark.parametrize("name", FIXTURES)
def test_record_chain_equals_records(files, name):
    # check/src/test/.../index/IndexRecordsTest.scala, PosStreamTest.scala
    of = files[name]
    chain = of.record_chain(of.header_end)
    assert [of.pos_of(int(f)) for f in chain] == read_records(name)


def test_stream_stats_2bam(files):
    # bgzf/src/test/.../block/StreamTest.scala:33-129: 25 blocks, usize 65498 x24, last 34570
    us = [u for _, _, u in files["2.bam"].blocks]
    assert len(us) == 25 and us[:24] == [65498] * 24 and us[24] == 34570


def test_header_end(files):
    # docs/command-line.md: 2.bam 0:5650, 1.bam 0:45846
    assert files["2.bam"].pos_of(files["2.bam"].header_end) == (0, 5650)
    assert files["1.bam"].pos_of(files["1.bam"].header_end) == (0, 45846)


def test_find_block_start(files):
    # bgzf/src/test/.../block/FindBlockStartTest.scala:9-16
    assert files["2.bam"].find_block_start(26170) == (OR_OK, 50249)


def test_find_record_start(files):
    # check/src/test/.../spark/FindRecordStartTest.scala:16-26
    of = files["1.bam"]
    rc, flat, delta = of.find_record_start(of.flat_of(239479, 0))
    assert rc == OR_OK and of.pos_of(flat) == (239479, 312) and delta == 312


def test_full_checker_unit(files):
    # check/src/test/.../check/full/CheckerTest.scala:38-58
    of = files["2.bam"]
    assert of.full(of.flat_of(439897, 52186)) == FULL_SUCCESS | (10 << FULL_N_SHIFT)
    r = of.full(of.flat_of(0, 5649))
    assert r == (1 << FLAG_NAMES.index("noReadName")) | (1 << FLAG_NAMES.index("invalidCigarOp"))


@pytest.mark.parametrize("golden,name,begin,end", [
    ("2.bam", "2.bam", None, None),
    ("2.bam.first", "2.bam", 0, 65498),
    ("1.bam", "1.bam", None, None),
])
def test_full_check_totals(files, golden, name, begin, end):
    # cli/src/test/.../check/full/FullCheckTest.scala + output/full-check/*
    of = files[name]
    b = 0 if begin is None else begin
    e = of.flat_size if end is None else end
    _, counts, rbe, _ = of.full_range(b, e)
    tot = dict(zip(FLAG_NAMES, counts.sum(axis=0).tolist()))
    expected = parse_total_error_counts(f"{GOLDEN}/output/full-check/{golden}")
    for k, v in expected.items():
        assert tot[k] == v, k
    assert rbe.sum() == 0  # no "readsBeforeError" line in the golden totals


@pytest.mark.parametrize("size,expected", [
    (230 * 1024, ["0:45846-239479:312", "239479:312-484396:25", "484396:25-597482:0"]),
    (240 * 1024, ["0:45846-263656:191", "263656:191-508565:287", "508565:287-597482:0"]),
])
def test_compute_splits_1bam(files, size, expected):
    # cli/src/test/.../spark/ComputeSplitsTest.scala:14-88
    splits, counts = load_splits_and_reads(files["1.bam"], size)
    assert [f"{vpos_str(a)}-{vpos_str(b)}" for a, b in splits] == expected
    assert sum(counts) == 4917  # CountReadsTest.scala


@pytest.mark.parametrize("size,expected", [
    (1000000, [2500]),
    (100000, [503, 414, 518, 421, 493, 151]),
    (20000, [96, 102, 105, 101, 99, 102, 101, 106, 0, 105, 105, 102, 104, 103, 104, 106,
             104, 106, 0, 105, 195, 101, 0, 99, 98, 99, 52]),
])
def test_load_bam_partition_counts(files, size, expected):
    # load/src/test/.../load/LoadBAMTest.scala:113-134
    _, counts = load_splits_and_reads(files["2.bam"], size)
    assert counts == expected


def test_load_bam_1bam_300k(files):
    # LoadBAMTest.scala:204-213
    _, counts = load_splits_and_reads(files["1.bam"], 300 * 1024)
    assert sum(counts) == 4917


def test_file_splits_slop():
    assert file_splits(531753, 100000)[-1] == (500000, 531753)
    assert len(file_splits(531753, 1000000)) == 1
    assert file_splits(110, 100) == [(0, 110)]
    assert file_splits(111, 100) == [(0, 100), (100, 111)]
