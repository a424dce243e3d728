"""The Scala drop-in checkers' call sequence on the GPU (jni/Native.scala GpuEagerChecker /
GpuFullChecker, mirrored call for call by spark_bam_amd.checkers).

The reference asks its checkers one position at a time, block by block
(CallPartition.scala:35-52 over PosIterator(block)): here `apply(pos)` is called at EVERY
position of every block of short-read, long-read and adversarial corpora, through windows of
1 MiB of compressed bytes starting with a 4 KiB halo (grown x4 on SBH_E_NEED_HALO), and each
answer is compared with the CPU oracle (eager/Checker.scala:24-126, full/Checker.scala:22-184).
nextReadStart (eager/Checker.scala:134-147) is checked from every block start."""
import os
import sys

import numpy as np
import pytest

from oracle_lib import OR_OK, OracleFile
from pkg import sb

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))

CORPORA = {
    "short": (dict(seed=0x5B4D0001, shape=0, level=6), 30000),
    "long": (dict(seed=0x5B4D004C, shape=1, level=6), 200),
    "adversarial": (dict(seed=0x5B4D00AD, shape=2, level=-1), 30000),
}
WINDOW, HALO = 1 << 20, 4 << 10


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
        data = synth.make_bam(p, nrec)[0]
        out[name] = (data, OracleFile(data))
    return out


def positions(of):
    """Every Pos of every data block of the oracle's stream, in file order (PosIterator)."""
    for start, _, usize in of.blocks:
        for off in range(usize):
            yield start, off


@pytest.mark.parametrize("name", list(CORPORA))
def test_eager_checker_every_position(ctx, files, name):
    from spark_bam_amd.checkers import WindowedEagerChecker
    data, of = files[name]
    _, bits_ref = of.eager_range(0, of.flat_size)
    want = np.unpackbits(bits_ref, bitorder="little")[:of.flat_size].astype(bool)
    Pos = sb.Pos
    with WindowedEagerChecker(data, of.contig_len, window=WINDOW, halo=HALO, ctx=ctx) as ck:
        got = np.fromiter((ck.apply(Pos(b, o)) for b, o in positions(of)), dtype=bool, count=of.flat_size)
        assert ck.loads >= 3, "the corpus should span several windows"
        assert ck.halo >= HALO
    d = np.flatnonzero(got != want)
    assert d.size == 0, f"{d.size} positions differ, first at flat {d[0]} ({of.pos_of(int(d[0]))})"


@pytest.mark.parametrize("name", list(CORPORA))
def test_eager_checker_next_read_start(ctx, files, name):
    """nextReadStart from every block start (FindRecordStart's question, FindRecordStart.scala:40-46)."""
    from spark_bam_amd.checkers import WindowedEagerChecker
    data, of = files[name]
    Pos = sb.Pos
    with WindowedEagerChecker(data, of.contig_len, window=WINDOW, halo=HALO, ctx=ctx) as ck:
        for start, _, usize in of.blocks:
            if not usize:
                continue
            rc, want, d = of.find_record_start(of.flat_of(start, 0))
            got = ck.next_read_start_with_delta(Pos(start, 0))
            if rc == OR_OK:
                assert got is not None and got[0] == Pos(*of.pos_of(want)) and got[1] == d, (name, start)
            else:
                assert got is None, (name, start)


@pytest.mark.parametrize("name", list(CORPORA))
def test_full_checker_every_position(ctx, files, name):
    from spark_bam_amd.checkers import WindowedFullChecker
    data, of = files[name]
    _, _, _, want = of.full_range(0, of.flat_size, want_words=True)
    Pos = sb.Pos
    with WindowedFullChecker(data, of.contig_len, window=WINDOW, halo=HALO, ctx=ctx) as ck:
        got = np.fromiter((ck.apply(Pos(b, o)) for b, o in positions(of)), dtype=np.uint32, count=of.flat_size)
        assert ck.loads >= 3
    d = np.flatnonzero(got != want)
    assert d.size == 0, f"{d.size} words differ, first at flat {d[0]}: {hex(got[d[0]])} vs {hex(want[d[0]])}"


def test_full_checker_result_decoding(ctx, files):
    """Result words back to the reference's Success(n) / Flags(..., readsBeforeError)."""
    from spark_bam_amd.checkers import WindowedFullChecker
    data, of = files["short"]
    rc, first, _ = of.find_record_start(of.header_end)
    assert rc == OR_OK
    with WindowedFullChecker(data, of.contig_len, window=WINDOW, halo=HALO, ctx=ctx) as ck:
        assert ck.result(ck.apply(sb.Pos(*of.pos_of(first)))) == ("success", 10)
        kind, flags, n = ck.result(ck.apply(sb.Pos(*of.pos_of(first + 1))))
        assert kind == "flags" and flags and n == 0
