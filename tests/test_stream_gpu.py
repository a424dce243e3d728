"""A shard streamed through bounded HBM (sbh_run_stream) must give exactly what the resident
run (sbh_run_shard over the whole shard) gives: the eager bit of every owned position, the
eager-true count, the first record and the stitched record count -- with windows small enough
that records, halos and false-positive bait cross many window edges."""
import os
import sys

import numpy as np
import pytest

from oracle_lib import OracleFile
from pkg import sb

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))

CORPORA = {
    "short_l6": (dict(seed=0x5B4D0001, shape=0, level=6), 30000),
    "wgs_c": (dict(seed=0x5B4D0030, shape=0, level=6), 20000),
    "long": (dict(seed=0x5B4D004C, shape=1, level=6), 200),
    "adversarial": (dict(seed=0x5B4D00AD, shape=2, level=-1), 30000),
}


@pytest.fixture(scope="module")
def ctx():
    c = sb.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def files():
    import synth
    out = {}
    for name, (kw, nrec) in CORPORA.items():
        p = synth.params(kw["seed"], shape=kw["shape"], level=kw["level"])
        out[name] = (synth.make_bam(p, nrec)[0], nrec)
    return out


def resident(ctx, data, contig_len):
    sh = ctx.shard(data)
    try:
        sh.set_contigs(contig_len)
        r = sh.run(0, data.size)
        bits = sh.eager_bits(0, r["flat_bytes"])
        ex = sh.exit_vpos(r)
    finally:
        sh.close()
    return r, bits, ex


@pytest.mark.parametrize("name", list(CORPORA))
@pytest.mark.parametrize("window,halo", [(150_000, 1 << 16), (400_000, 1 << 20)])
def test_stream_equals_resident(ctx, files, name, window, halo):
    data, nrec = files[name]
    of = OracleFile(data)
    r, bits, _ = resident(ctx, data, of.contig_len)
    s, sbits = ctx.run_stream(data, of.contig_len, index_start=0, window=window, halo=halo, want_bits=True)
    assert s["status"] == 0 and s["n_windows"] >= 3
    assert s["flat_bytes"] == r["flat_bytes"] and s["comp_bytes"] == r["comp_bytes"]
    nb = (r["flat_bytes"] + 7) // 8
    d = np.flatnonzero(sbits[:nb] != bits[:nb])
    assert d.size == 0, f"eager bits differ at byte {d[0]}"
    assert s["n_true"] == r["n_true"]
    assert s["count"] == r["count"] == nrec
    assert s["first_vpos"] == r["first_vpos"]


def test_stream_pinned_host_and_halo_growth(ctx, files):
    """Pinned host memory (the overlapped-copy path) and a halo too small for long records
    (grown x4 until every window's records fit)."""
    data, nrec = files["long"]
    of = OracleFile(data)
    buf = sb.PinnedBuffer(data.size)
    buf.array[:] = data
    s, _ = ctx.run_stream(buf.array, of.contig_len, window=300_000, halo=4096)
    buf.close()
    assert s["host_pinned"] == 1 and s["halo_final"] > 4096
    assert s["count"] == nrec and s["ms_h2d"] > 0


def test_stream_subrange_of_a_file(ctx, files):
    """Host bytes = a byte range of a file (file_offset > 0, not at EOF): the owned blocks'
    bits equal the whole-file resident bits at the same flat positions."""
    data, _ = files["wgs_c"]
    of = OracleFile(data)
    sh = ctx.shard(data)
    sh.index(0)
    blocks = sh.blocks()
    k0, k1 = 10, 45  # of 74 data blocks
    lo, own_end, hi = blocks[k0][0], blocks[k1][0], blocks[k1 + 20][0]
    base, E = blocks[k0][3], blocks[k1][3]
    sh.inflate()
    sh.set_contigs(of.contig_len)
    _, want = sh.check_eager(base, E)
    n_ref = sh.count_records(sh.find_record_start(base)[0], E)
    sh.close()
    s, got = ctx.run_stream(data[lo:hi], of.contig_len, file_offset=lo, file_size=data.size, own_end=own_end,
                            window=200_000, halo=1 << 16, want_bits=True)
    assert s["flat_bytes"] == E - base
    assert np.array_equal(np.unpackbits(got, bitorder="little")[:E - base],
                          np.unpackbits(want, bitorder="little")[:E - base])
    assert s["count"] == n_ref


@pytest.mark.parametrize("name", list(CORPORA))
@pytest.mark.parametrize("window,split", [(150_000, 40_000), (400_000, 97_000), (150_000, 400_000),
                                          (150_000, 1 << 40)])
def test_stream_splits_equal_resident_and_oracle(ctx, files, name, window, split):
    """loadSplitsAndReads' per-split answer through bounded HBM (sbh_run_stream2): windows cut
    at split starts, each split decided by the batched split path in its window -- equal to
    the resident batch (sbh_split_starts on the whole file) and to the oracle
    (CanLoadBam.scala:283-297,316-356).  A split larger than a window runs through several (its
    chain followed window by window; the last case is ONE split for the whole file, a rank with a
    single split), so HBM stays bounded.
    The in-run CRC32 check finds no bad block."""
    from oracle_lib import OR_OK, file_splits
    data, nrec = files[name]
    of = OracleFile(data)
    splits = file_splits(data.size, split)
    s, _ = ctx.run_stream(data, of.contig_len, index_start=0, window=window, halo=1 << 16, splits=splits,
                          verify_crc=True)
    assert s["status"] == 0 and s["crc_bad_blocks"] == 0 and s["count"] == nrec
    assert s["n_windows"] >= data.size // window - 1
    sh = ctx.shard(data)
    try:
        sh.index(0)
        sh.inflate()
        sh.set_contigs(of.contig_len)
        st, v, n, _ = sh.split_starts(splits)
    finally:
        sh.close()
    assert s["split_status"].tolist() == st.tolist()
    assert s["split_count"].tolist() == n.tolist()
    assert [int(a) for a, c in zip(s["split_first_vpos"], n) if c] == [int(a) for a, c in zip(v, n) if c]
    assert int(s["split_count"].sum()) == nrec
    if name != "adversarial":
        assert s["splits_host"] == 0
    for i, (a, e) in enumerate(splits):
        rc, vr, nr = of.split(a, e)
        if rc == OR_OK:
            assert int(s["split_status"][i]) == 0 and int(s["split_count"][i]) == nr
            assert nr == 0 or int(s["split_first_vpos"][i]) == vr


def test_stream_crc_detects_a_bad_footer(ctx, files):
    """A damaged footer CRC32 inside the owned range is counted (the data still inflates)."""
    data, _ = files["short_l6"]
    of = OracleFile(data)
    bad = data.copy()
    start, csize, _ = of.blocks[7]
    bad[start + csize - 8] ^= 0xFF
    s, _ = ctx.run_stream(bad, of.contig_len, index_start=0, window=150_000, halo=1 << 16, verify_crc=True)
    assert s["crc_bad_blocks"] == 1 and s["crc_first_bad"] == start


@pytest.mark.parametrize("name", ["short_l6", "long", "adversarial"])
def test_all_positions_streamed_equal_one_window_and_oracle(ctx, files, name):
    """check-bam -s / full-check through bounded HBM (sbh_check_stream, 150 KB windows) equal the
    same pass in one window and the oracle at every position (CallPartition.scala:35-52,
    FullCheck.scala:65-86,142-192); truth = the oracle's record chain with two records dropped
    and one false record added, so the FP / FN lists are exercised."""
    data, _ = files[name]
    of = OracleFile(data)
    chain = [int(f) for f in of.record_chain(of.header_end)]
    truth_flat = sorted(set(chain[:50] + chain[51:-7] + chain[-6:] + [chain[100] + 1]))
    truth = [of.pos_of(f) for f in truth_flat]
    one = sb.check_bam(data, records=truth, ctx=ctx, window=1 << 40)
    many = sb.check_bam(data, records=truth, ctx=ctx, window=150_000)
    assert one["n_windows"] == 1 and many["n_windows"] >= 3
    for k in ("positions", "compressed", "reads", "true_positives", "false_positives", "false_negatives",
              "fp_positions", "fn_positions"):
        assert many[k] == one[k], k
    _, bits = of.eager_range(0, of.flat_size)
    calls = set(np.flatnonzero(np.unpackbits(bits, bitorder="little")[:of.flat_size]).tolist())
    tset = set(truth_flat)
    assert many["positions"] == of.flat_size
    assert many["true_positives"] == len(calls & tset)
    assert [of.flat_of(p.block_pos, p.offset) for p in many["fp_positions"]] == sorted(calls - tset)
    assert [of.flat_of(p.block_pos, p.offset) for p in many["fn_positions"]] == sorted(tset - calls)
    f1 = sb.full_check(data, ctx=ctx, window=1 << 40)
    fm = sb.full_check(data, ctx=ctx, window=150_000)
    ns, counts, rbe, _ = of.full_range(0, of.flat_size)
    assert fm["n_success"] == f1["n_success"] == ns
    assert np.array_equal(fm["counts_by_nnz"], f1["counts_by_nnz"]) and np.array_equal(fm["counts_by_nnz"], counts)
    assert np.array_equal(fm["rbe_by_nnz"], rbe)
    assert fm["close"] == f1["close"] and len(fm["close"]) > 0
