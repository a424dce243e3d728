"""Record field extraction on the GPU (sbh_records_scan / fetch) vs the CPU oracle's
decode, column for column, and vs the reference's 2.sam as text."""
import os

import numpy as np
import pytest

from conftest import golden_bam
from oracle_lib import OracleFile
import oracle_records as orr
from pkg import sb
from test_records_cpu import sam_golden

pytestmark = pytest.mark.gpu

FIXTURES = ["2.bam", "1.bam", "5k.bam", "1.2203053-2211029.bam", "2.100-1000.bam"]


def assert_cols_equal(got, want):
    assert set(got) == set(want)
    for k in want:
        assert got[k].dtype == want[k].dtype, k
        assert np.array_equal(got[k], want[k]), k


@pytest.mark.parametrize("name", FIXTURES)
def test_load_reads_matches_oracle(name):
    data = np.fromfile(golden_bam(name), dtype=np.uint8)
    flat = OracleFile(data).uncompressed()
    refs, first = orr.bam_refs(flat)
    want = orr.decode(flat, orr.record_starts(flat, first, flat.size))
    reads = sb.load_reads(golden_bam(name))
    assert reads.ref_names == refs
    assert_cols_equal(reads.cols, want)


def test_load_reads_2bam_sam_text():
    assert sb.load_reads(golden_bam("2.bam")).sam_lines() == sam_golden()


def test_records_chain_walk_path_and_subrange():
    # without an eager bitmap the record starts come from the sequential chain walk;
    # a sub-range [first, end) stops at the first record starting at or past end
    data = np.fromfile(golden_bam("1.bam"), dtype=np.uint8)
    flat = OracleFile(data).uncompressed()
    refs, first = orr.bam_refs(flat)
    starts = orr.record_starts(flat, first, flat.size)
    with sb.Context(0) as ctx:
        sh = ctx.shard(data)
        sh.index(0)
        sh.inflate()
        assert_cols_equal(sh.records(first, flat.size), orr.decode(flat, starts))
        lo, hi = starts[100], starts[900] + 1
        assert_cols_equal(sh.records(lo, hi), orr.decode(flat, starts[100:901]))
        empty = sh.records(first, first)
        assert empty["flat"].size == 0 and empty["name_off"].tolist() == [0]
        sh.close()
