"""Record field extraction on the GPU (sbh_records_scan / fetch) vs the CPU oracle's
decode, column for column, and vs the reference's 2.sam as text."""
import os

import numpy as np
import pytest

from conftest import golden_bam
from oracle_lib import OracleFile
import oracle_records as orr
from pkg import sb
SBH_E_BAD_RECORD = sb._lib.SBH_E_BAD_RECORD
from test_records_cpu import sam_golden

pytestmark = pytest.mark.gpu

FIXTURES = ["2.bam", "1.bam", "5k.bam", "1.2203053-2211029.bam", "2.100-1000.bam"]


def assert_cols_equal(got, want):
    got = {k: v for k, v in got.items() if k in want or k != "vpos"}  # (the oracle decode has no vpos)
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
    assert_cols_equal({k: v for k, v in reads.cols.items() if k != "vpos"}, want)
    of = OracleFile(data)
    assert reads.cols["vpos"].tolist() == [(lambda b, o: b << 16 | o)(*of.pos_of(int(f))) for f in want["flat"]]


@pytest.mark.parametrize("name,window", [("1.bam", 100_000), ("5k.bam", 150_000), ("2.bam", 60_000)])
def test_load_reads_windowed(name, window):
    """loadReads a window at a time (api.iter_reads: batches joined) equals the resident decode,
    column for column (flat offsets aside: they are window-relative), vpos included."""
    one = sb.load_reads(golden_bam(name))
    win = sb.load_reads(golden_bam(name), window=window)
    batches = list(sb.api.iter_reads(golden_bam(name), window=window))
    assert len(batches) >= 3
    assert win.n == one.n and win.ref_names == one.ref_names
    for k in one.cols:
        if k != "flat":
            assert np.array_equal(win.cols[k], one.cols[k]), k
    if name == "2.bam":
        assert win.sam_lines() == sam_golden()


def test_load_reads_windowed_synthetic():
    """Long reads (records spanning blocks and windows, a 4 KiB halo grown on demand) and an
    adversarial corpus, windowed vs resident; with an empty block mid-file (the stream ends at
    its start, cutting the record that spans it) both paths raise the same malformed-record error."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
    import synth
    for seed, shape, level, nrec, empty in ((0x5B4D004C, 1, 6, 150, 0), (0x5B4D00AE, 2, -1, 20000, 0),
                                            (0x5B4D00AE, 2, -1, 20000, 5)):
        data = synth.make_bam(synth.params(seed, shape=shape, level=level, empty_every=empty), nrec)[0]

        def windowed():
            with sb.Context(0) as ctx:
                return sb.Reads.concat(list(sb.api.iter_reads(data, window=120_000, halo=4096, ctx=ctx)),
                                       sb.api.file_header(ctx, data)[0])

        if empty:
            with pytest.raises(sb.SparkBamError) as e1:
                sb.load_reads(data)
            with pytest.raises(sb.SparkBamError) as e2:
                windowed()
            assert e1.value.code == e2.value.code == SBH_E_BAD_RECORD
            continue
        one = sb.load_reads(data)
        win = windowed()
        assert win.n == one.n > 0
        for k in one.cols:
            if k != "flat":
                assert np.array_equal(win.cols[k], one.cols[k]), (seed, k)


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


def test_load_reads_windowed_header_only():
    """A BAM with a header and no records: the windowed decode (Reads.concat of no non-empty
    batch) has the resident decode's full column schema, every column empty."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
    import synth
    data = synth.make_bam(synth.params(0x5B4D0001), 0)[0]
    one = sb.load_reads(data)
    win = sb.load_reads(data, window=4096)
    assert one.n == win.n == 0
    assert set(win.cols) == set(one.cols)
    for k in one.cols:
        assert win.cols[k].dtype == one.cols[k].dtype, k
        assert np.array_equal(win.cols[k], one.cols[k]), k


@pytest.mark.parametrize("kind", ["short", "long", "adversarial"])
def test_device_vpos_equals_host_mapping(kind):
    """sbh_records_fetch's vpos column (k_rec_vpos: the last chain block whose first flat byte is
    <= the start, empty blocks skipped) equals the host mapping over the block table (api._vpos_of)
    and the oracle's canonical Pos -- records starting exactly at a block's end take Pos(next, 0)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
    import synth
    kw = {"short": dict(seed=0x5B4D0001, shape=0, level=6), "long": dict(seed=0x5B4D004C, shape=1, level=6),
          "adversarial": dict(seed=0x5B4D00AD, shape=2, level=-1)}[kind]
    data = synth.make_bam(synth.params(kw["seed"], shape=kw["shape"], level=kw["level"]),
                          300 if kind == "long" else 20000)[0]
    of = OracleFile(data)
    with sb.Context(0) as ctx:
        sh = ctx.shard(data)
        sh.index(0)
        sh.inflate()
        sh.set_contigs(of.contig_len)
        sh.check_eager(0, sh.flat_size, want_bits=False)
        first, _ = sh.find_record_start(of.header_end)
        cols = sh.records(first, sh.flat_size)
        host = sb.api._vpos_of(cols["flat"], sh.blocks())
        assert cols["vpos"].size > 0 and np.array_equal(cols["vpos"], host)
        oracle = [(lambda b, o: b << 16 | o)(*of.pos_of(int(f))) for f in cols["flat"][:2000]]
        assert cols["vpos"][:2000].tolist() == oracle
        sh.close()
