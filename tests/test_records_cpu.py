"""Record field extraction, CPU side: the oracle's decoder + SAM renderer and the
package's SAM renderer (host formatting over columns), both pinned against the
reference's test_bams/2.sam (the SAM text of 2.bam)."""
import gzip
import os

from conftest import BAMS, GOLDEN, golden_bam
from oracle_lib import OracleFile
import oracle_records as orr
from pkg import sb

import numpy as np


def sam_golden():
    with gzip.open(os.path.join(GOLDEN, "sam", "2.sam.gz"), "rt", encoding="utf-8") as f:
        return [l.rstrip("\n") for l in f if not l.startswith("@")]


def oracle_cols(name):
    data = np.fromfile(golden_bam(name), dtype=np.uint8)
    flat = OracleFile(data).uncompressed()
    refs, first = orr.bam_refs(flat)
    return orr.decode(flat, orr.record_starts(flat, first, flat.size)), refs


def test_oracle_decoder_matches_2sam():
    cols, refs = oracle_cols("2.bam")
    want = sam_golden()
    assert len(want) == 2500 == cols["flat"].size
    assert [orr.sam_line(cols, i, refs) for i in range(len(want))] == want


def test_reads_renderer_matches_2sam():
    cols, refs = oracle_cols("2.bam")
    assert sb.Reads(cols, refs).sam_lines() == sam_golden()


def test_records_fixture_positions():
    # the chain from the header reproduces the reference's .records fixture (IndexRecordsTest)
    data = np.fromfile(golden_bam("1.bam"), dtype=np.uint8)
    of = OracleFile(data)
    flat = of.uncompressed()
    _, first = orr.bam_refs(flat)
    starts = orr.record_starts(flat, first, flat.size)
    want = [l.strip() for l in open(os.path.join(BAMS, "1.bam.records"))]
    assert len(starts) == len(want) == 4917


def test_tags_text_types():
    import struct
    aux = (b"XAA" + b"q" + b"XCc" + struct.pack("<b", -5) + b"XSS" + struct.pack("<H", 65535) +
           b"XIi" + struct.pack("<i", -70000) + b"XZZhello\0" + b"XHH1AE3\0" +
           b"XBBs" + struct.pack("<ih", 1, -2) + b"XFf" + struct.pack("<f", 1.5))
    assert sb.records.tags_text(np.frombuffer(aux, np.uint8)) == [
        "XA:A:q", "XC:i:-5", "XS:i:65535", "XI:i:-70000", "XZ:Z:hello", "XH:H:1AE3", "XB:B:s,-2",
        "XF:f:1.5"]


def test_reads_concat_empty_has_full_schema():
    """Reads.concat of no non-empty batch keeps every column of a decoded batch:
    the columns sbh_records_fetch fills, zero-length (offset columns one zero), plus vpos."""
    RECORD_COLUMNS, record_columns = sb.records.RECORD_COLUMNS, sb.records.record_columns
    full = record_columns(3, 10, 4, 300, 20)
    full["vpos"] = np.zeros(3, np.uint64)
    empty = sb.Reads.concat([], ["1"])
    assert empty.n == 0 and set(empty.cols) == set(full)
    for k, dt, _ in RECORD_COLUMNS:
        assert empty.cols[k].dtype == dt, k
        want = [0] if k.endswith("_off") else []
        assert empty.cols[k].tolist() == want, k
