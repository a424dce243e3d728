"""Batched splits (sbh_split_starts), device-side check-bam (sbh_check_records) and the
chain re-walk primitive (sbh_chain_from) against the per-split path and the CPU oracle.

sbh_split_starts must return, for every split, exactly what sbh_split returns (and that is
what the oracle's loadSplitsAndReads restatement returns): CanLoadBam.scala:283-297,
316-356.  sbh_check_records must give CheckerApp's TP/FP/FN (CheckerApp.scala:65-227).
"""
import os
import sys

import numpy as np
import pytest

from conftest import golden_bam, read_records
from oracle_lib import OR_OK, OracleFile, file_splits
from pkg import sb

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))


@pytest.fixture(scope="module")
def ctx():
    c = sb.Context(0)
    yield c
    c.close()


SYN = {
    "short_l6": (dict(seed=0x5B4D0001, shape=0, level=6), 30000),
    "wgs_c": (dict(seed=0x5B4D0030, shape=0, level=6), 30000),
    "long": (dict(seed=0x5B4D004C, shape=1, level=6), 150),
    "adversarial": (dict(seed=0x5B4D00AD, shape=2, level=-1), 30000),
    "adversarial_empty": (dict(seed=0x5B4D00AE, shape=2, level=-1, empty_every=5), 30000),
}


@pytest.fixture(scope="module")
def files():
    import synth
    out = {}
    for name, (kw, nrec) in SYN.items():
        p = synth.params(kw["seed"], shape=kw["shape"], level=kw["level"], empty_every=kw.get("empty_every", 0))
        out[name] = synth.make_bam(p, nrec)[0]
    for name in ("1.bam", "2.bam", "5k.bam"):
        out[name] = np.fromfile(golden_bam(name), dtype=np.uint8)
    return out


def loaded(ctx, data):
    of = OracleFile(data)
    sh = ctx.shard(data)
    sh.index(0)
    sh.inflate()
    sh.set_contigs(of.contig_len)
    return of, sh


@pytest.mark.parametrize("name", ["1.bam", "2.bam", "5k.bam", "short_l6", "wgs_c", "long", "adversarial",
                                  "adversarial_empty"])
@pytest.mark.parametrize("div", [3, 11, 40])
def test_split_starts_equals_per_split_and_oracle(ctx, files, name, div):
    data = files[name]
    of, sh = loaded(ctx, data)
    try:
        size = max(data.size // div, 20000)
        splits = file_splits(data.size, size)
        status, v, n, n_host = sh.split_starts(splits)
        for i, (s, e) in enumerate(splits):
            try:
                v1, n1 = sh.split(s, e)
                st1 = 0
            except sb.SparkBamError as err:
                st1, v1, n1 = err.code, 0, 0
            assert (int(status[i]), int(n[i])) == (st1, n1), (i, s, e)
            if n1:
                assert int(v[i]) == v1, (i, s, e)
            rc, vr, nr = of.split(s, e)
            if rc == OR_OK:
                assert int(status[i]) == 0 and int(n[i]) == nr and (nr == 0 or int(v[i]) == vr), (i, s, e)
        if name in ("1.bam", "2.bam", "5k.bam", "short_l6", "wgs_c"):
            assert n_host == 0, f"{n_host} of {len(splits)} splits left the device path"
    finally:
        sh.close()


def test_split_starts_after_run_shard_owned_range(ctx, files):
    """After sbh_run_shard the bitmap covers the owned range only: the batch reuses it."""
    data = files["wgs_c"]
    of, sh = loaded(ctx, data)
    try:
        r = sh.run(0, data.size)
        splits = file_splits(data.size, data.size // 9)
        status, v, n, n_host = sh.split_starts(splits)
        assert n_host == 0 and not status.any()
        assert int(n.sum()) == r["count"] == 30000
        for i, (s, e) in enumerate(splits):
            rc, vr, nr = of.split(s, e)
            assert rc == OR_OK and int(n[i]) == nr and int(v[i]) == vr
    finally:
        sh.close()


@pytest.mark.parametrize("name,div", [("2.bam", 13), ("short_l6", 13), ("long", 13), ("adversarial", 13),
                                      ("adversarial_empty", 13), ("short_l6", 150), ("adversarial_empty", 150)])
def test_split_starts_fast_path_after_run(ctx, files, name, div):
    """After sbh_run_shard (chain proof + chunk counts resident) sbh_split_starts takes its one-
    round-trip path: counts written by the count kernel, a range leaving the proven chain (the
    empty blocks' later segments, bait) sent down the general path.  Twice in a row, against
    sbh_split per split and the oracle."""
    data = files[name]
    of, sh = loaded(ctx, data)
    try:
        try:
            sh.run(0, data.size)
        except sb.SparkBamError:
            pass  # (a corpus whose owned range has no record: the splits still decide alone)
        # (div 150: more than 64 splits, so the ranges go over by a copy, not kernel arguments)
        splits = file_splits(data.size, max(data.size // div, 20000))
        for _ in range(2):
            status, v, n, n_host = sh.split_starts(splits)
            for i, (s, e) in enumerate(splits):
                rc, vr, nr = of.split(s, e)
                if rc == OR_OK:
                    assert int(status[i]) == 0 and int(n[i]) == nr and (nr == 0 or int(v[i]) == vr), (i, s, e)
                else:  # as the per-split path decides it
                    try:
                        v1, n1 = sh.split(s, e)
                        st1 = 0
                    except sb.SparkBamError as err:
                        st1, v1, n1 = err.code, 0, 0
                    assert (int(status[i]), int(n[i])) == (st1, n1), (i, s, e)
    finally:
        sh.close()


def test_chain_from(ctx, files):
    data = files["2.bam"]
    of, sh = loaded(ctx, data)
    try:
        first = sh.flat_of(0, 5650)
        assert sh.chain_from(first, sh.flat_size) == (2500, sh.flat_size)
        chain = of.record_chain(first, of.flat_size)
        E = int(chain[1000])
        n, ex = sh.chain_from(int(chain[10]), E)
        assert (n, ex) == (990, E)
    finally:
        sh.close()


def _bits_positions(bits, base, n):
    return np.flatnonzero(np.unpackbits(bits, bitorder="little")[:n]) + base


@pytest.mark.parametrize("name", ["1.bam", "5k.bam", "adversarial"])
def test_check_records_matches_host_sets(ctx, files, name):
    data = files[name]
    of, sh = loaded(ctx, data)
    try:
        if name.endswith(".bam"):
            recs = [(b << 16) | o for b, o in read_records(name)]
        else:  # the true chain (the adversarial corpus carries false-positive bait)
            chain = of.record_chain(of.header_end, of.flat_size)
            recs = []
            for r in chain:
                bp, off = of.pos_of(int(r))
                recs.append((bp << 16) | off)
        rng = np.random.default_rng(7)
        recs = np.asarray(recs, dtype=np.uint64)
        drop = rng.choice(recs.size, 5, replace=False)
        truth = np.delete(recs, drop)
        # bogus truth: one byte past 3 records (never eager-true there)
        bogus = [int(x) + 1 for x in recs[rng.choice(recs.size, 3, replace=False)]]
        truth = np.concatenate([truth, np.asarray(bogus, dtype=np.uint64)])
        blocks = [b for b in sh.blocks() if b[2] and not b[5] & sb.BLOCK_EMPTY]
        for ranges in ([(blocks[0][3], blocks[-1][3] + blocks[-1][2])],
                       [(b[3], b[3] + b[2]) for b in blocks[1::3]]):
            tp, fp, fn, unk, fpl, fnl = sh.check_records(ranges, truth)
            called, tset = [], set()
            for a, b in ranges:
                _, bits = sh.check_eager(a, b)
                called += _bits_positions(bits, a, b - a).tolist()
            for v in truth.tolist():
                try:
                    f = sh.flat_of(v >> 16, v & 0xFFFF)
                except sb.SparkBamError:
                    continue
                if any(a <= f < b for a, b in ranges):
                    tset.add(f)
            cset = set(called)
            assert unk == 0
            assert (tp, fp, fn) == (len(cset & tset), len(cset - tset), len(tset - cset))
            assert fpl.tolist() == sorted(cset - tset) and fnl.tolist() == sorted(tset - cset)
    finally:
        sh.close()


def test_check_bam_api_golden(ctx):
    # CheckBamTest "eager 1.bam" through the device comparison, and a damaged truth
    recs = read_records("1.bam")
    r = sb.check_bam(golden_bam("1.bam"), records=recs, ctx=ctx)
    assert (r["positions"], r["reads"], r["false_positives"], r["false_negatives"]) == (1608257, 4917, 0, 0)
    r = sb.check_bam(golden_bam("1.bam"), records=recs[:100] + recs[101:], ctx=ctx)
    assert r["false_positives"] == 1 and r["false_negatives"] == 0
    assert r["fp_positions"] == [sb.Pos(*recs[100])]


@pytest.mark.parametrize("name,split_size", [("1.bam", 230 * 1024), ("2.bam", 102400)])
def test_load_splits_and_reads_streamed(ctx, monkeypatch, name, split_size):
    """api.load_splits_and_reads on a file over the resident budget: streamed through HBM in
    windows (sharded.RankRun over sbh_run_stream2), same splits and counts as the oracle."""
    import spark_bam_amd.sharded as sharded
    from conftest import golden_bam
    from oracle_lib import load_splits_and_reads as oracle_load
    monkeypatch.setattr(sharded, "RESIDENT_MAX", 1)
    monkeypatch.setattr(sharded, "STREAM_WINDOW", 120_000)
    splits, counts = sb.load_splits_and_reads(golden_bam(name), split_size, ctx=ctx)
    of = OracleFile.from_path(golden_bam(name))
    ref_splits, ref_counts = oracle_load(of, split_size)
    assert counts == ref_counts
    assert [(a.to_htsjdk(), b.to_htsjdk()) for a, b in splits] == ref_splits
