"""GPU parity: the HIP path (through the C-ABI) vs the CPU oracle and the reference's
golden fixtures.  Bit-exact for every byte, bit and count.

Reference tests restated are named per test (paths relative to the reference root).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden_bam, parse_total_error_counts, read_blocks, read_records
from oracle_lib import FLAG_NAMES, OR_OK, OracleFile, file_splits, lib as olib
from pkg import sb

pytestmark = pytest.mark.gpu

FIXTURES = ["2.bam", "1.bam", "5k.bam", "1.2203053-2211029.bam", "2.100-1000.bam"]


@pytest.fixture(scope="module")
def ctx():
    c = sb.Context(0)
    yield c
    c.close()


def load(ctx, data, contigs=None):
    sh = ctx.shard(data)
    sh.index(0)
    sh.inflate()
    if contigs is not None:
        sh.set_contigs(contigs)
    return sh


def first_diff(a, b):
    n = min(a.size, b.size)
    d = np.flatnonzero(a[:n] != b[:n])
    return int(d[0]) if d.size else (n if a.size != b.size else -1)


@pytest.fixture(scope="module")
def golden(ctx):
    out = {}
    for name in FIXTURES:
        data = np.fromfile(golden_bam(name), dtype=np.uint8)
        of = OracleFile(data)
        sh = load(ctx, data, of.contig_len)
        out[name] = (data, of, sh)
    yield out
    for _, _, sh in out.values():
        sh.close()


@pytest.mark.parametrize("name", FIXTURES)
def test_index_blocks(golden, name):
    # IndexBlocksTest / MetadataStreamTest: (start, csize, usize) of every data block
    data, of, sh = golden[name]
    bl = [(s, c, u) for s, c, u, _us, _h, f in sh.blocks() if not f & sb.BLOCK_EMPTY]
    assert bl == read_blocks(name)
    assert sh.flat_size == of.flat_size


@pytest.mark.parametrize("name", FIXTURES)
def test_inflate_bytes(golden, name):
    # StreamTest: inflated bytes identical to java.util.zip.Inflater (zlib)
    data, of, sh = golden[name]
    got, want = sh.read_flat(), of.uncompressed()
    i = first_diff(got, want)
    assert i < 0, f"first differing flat byte {i} at Pos {of.pos_of(i) if i < want.size else 'end'}"


@pytest.mark.parametrize("name", FIXTURES)
def test_eager_every_position(golden, name):
    # CheckBamTest "eager 1.bam": eager at every position == .records (All calls matched!)
    data, of, sh = golden[name]
    n, bits = sh.check_eager(0, sh.flat_size)
    n_ref, bits_ref = of.eager_range(0, of.flat_size)
    i = first_diff(np.unpackbits(bits, bitorder="little"), np.unpackbits(bits_ref, bitorder="little"))
    assert i < 0, f"first differing position {i}"
    assert n == n_ref == len(read_records(name))


@pytest.mark.parametrize("golden_name,name,end", [("2.bam", "2.bam", None),
                                                  ("2.bam.first", "2.bam", 65498),
                                                  ("1.bam", "1.bam", None)])
def test_full_check_totals(golden, golden_name, name, end):
    # FullCheckTest + output/full-check/*: "Total error counts", per-nnz Counts == oracle
    data, of, sh = golden[name]
    e = sh.flat_size if end is None else end
    r = sh.check_full(0, e)
    _, counts_ref, rbe_ref, _ = of.full_range(0, e)
    assert np.array_equal(r["counts"].astype(np.int64), counts_ref)
    assert np.array_equal(r["rbe"].astype(np.int64), rbe_ref)
    tot = dict(zip(FLAG_NAMES, r["counts"].sum(axis=0).tolist()))
    for k, v in parse_total_error_counts(f"{GOLDEN}/output/full-check/{golden_name}").items():
        assert tot[k] == v, k


def test_full_words_match_oracle(golden):
    data, of, sh = golden["2.bam"]
    r = sh.check_full(0, 200000, want_words=True)
    _, _, _, w_ref = of.full_range(0, 200000, want_words=True)
    i = first_diff(r["words"], w_ref)
    assert i < 0, f"position {i}: {hex(r['words'][i])} vs {hex(w_ref[i])}"


def test_full_close_calls_2bam(golden):
    # output/full-check/2.bam: 2880 positions where exactly two checks failed, no 1-flag
    data, of, sh = golden["2.bam"]
    r = sh.check_full(0, sh.flat_size)
    words = r["close_word"]
    nnz = np.array([bin(int(w) & 0x7FFFF).count("1") + (((int(w) >> 20) & 0x3FF) > 0) for w in words])
    assert (nnz == 2).sum() == 2880 and (nnz == 1).sum() == 0
    first = [str(sb.Pos(*sh.pos_of(int(f)))) for f in r["close_flat"][:3]]
    assert first == ["0:5649", "0:6273", "0:6893"]


def test_full_checker_unit(golden):
    # check/.../full/CheckerTest.scala
    data, of, sh = golden["2.bam"]
    p = sh.flat_of(439897, 52186)
    r = sh.check_full(p, p + 1, want_words=True)
    assert r["words"][0] == sb.FULL_SUCCESS | (10 << sb.FULL_N_SHIFT)
    p = sh.flat_of(0, 5649)
    r = sh.check_full(p, p + 1, want_words=True)
    assert r["words"][0] == (1 << 12) | (1 << 15)


def test_find_block_start(golden):
    # FindBlockStartTest: FindBlockStart(2.bam, 26170, 5) == 50249
    data, of, sh = golden["2.bam"]
    assert sh.find_block_start(26170) == 50249
    rng = np.random.default_rng(7)
    for s in rng.integers(0, data.size - 1, 25).tolist() + [0, 1, data.size - 28, data.size - 30]:
        rc, want = of.find_block_start(int(s))
        if rc == OR_OK:
            assert sh.find_block_start(int(s)) == want, s
        else:
            with pytest.raises(sb.SparkBamError):
                sh.find_block_start(int(s))


def test_find_record_start(golden):
    # FindRecordStartTest: FindRecordStart(1.bam, 239479) == Pos(239479, 312)
    data, of, sh = golden["1.bam"]
    f, delta = sh.find_record_start(sh.flat_of(239479, 0))
    assert sh.pos_of(f) == (239479, 312) and delta == 312


@pytest.mark.parametrize("size,expected", [
    (230 * 1024, ["0:45846-239479:312", "239479:312-484396:25", "484396:25-597482:0"]),
    (240 * 1024, ["0:45846-263656:191", "263656:191-508565:287", "508565:287-597482:0"]),
])
def test_compute_splits_1bam(ctx, size, expected):
    # ComputeSplitsTest "eager 230KB" / "compare 240KB"
    splits, counts = sb.load_splits_and_reads(golden_bam("1.bam"), size, ctx=ctx)
    assert [f"{a}-{b}" for a, b in splits] == expected
    assert sum(counts) == 4917  # CountReadsTest


@pytest.mark.parametrize("size,expected", [
    (1000000, [2500]),
    (100000, [503, 414, 518, 421, 493, 151]),
    (20000, [96, 102, 105, 101, 99, 102, 101, 106, 0, 105, 105, 102, 104, 103, 104, 106,
             104, 106, 0, 105, 195, 101, 0, 99, 98, 99, 52]),
])
def test_load_bam_partition_counts(ctx, size, expected):
    # LoadBAMTest 1e6 / 1e5 / 2e4
    _, counts = sb.load_splits_and_reads(golden_bam("2.bam"), size, ctx=ctx)
    assert counts == expected


def test_check_bam_summary(ctx):
    # CheckBamTest "eager 1.bam": 1608257 positions, 4917 reads, All calls matched!
    r = sb.check_bam(golden_bam("1.bam"), records=read_records("1.bam"), ctx=ctx)
    assert r["positions"] == 1608257 and r["reads"] == 4917
    assert r["false_positives"] == 0 and r["false_negatives"] == 0


def test_run_shard_whole_file(golden):
    data, of, sh = golden["1.bam"]
    r = sh.run(0, data.size)
    assert r["status"] == 0 and r["count"] == 4917 and r["n_true"] == 4917
    assert sb.Pos.from_htsjdk(r["first_vpos"]) == (0, 45846)
    sh.index(0)  # run() re-indexed: restore for other tests
    sh.inflate()
    sh.set_contigs(of.contig_len)


# ------------------------------------------------------------- synthetic corpora
SYN = [
    ("short_l6", dict(seed=0x5B4D0001, shape=0, level=6), 30000),
    ("short_l1", dict(seed=0x5B4D0002, shape=0, level=1), 20000),
    ("short_l9", dict(seed=0x5B4D0003, shape=0, level=9), 20000),
    ("short_l0", dict(seed=0x5B4D0004, shape=0, level=0), 8000),
    ("long", dict(seed=0x5B4D004C, shape=1, level=6), 150),
    ("adversarial", dict(seed=0x5B4D00AD, shape=2, level=-1), 30000),
    ("adversarial_empty", dict(seed=0x5B4D00AE, shape=2, level=-1, empty_every=5), 30000),
]


@pytest.fixture(scope="module")
def synth_files():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
    import synth
    out = {}
    for name, kw, nrec in SYN:
        p = synth.params(kw["seed"], shape=kw["shape"], level=kw["level"],
                         empty_every=kw.get("empty_every", 0))
        data, _, _ = synth.make_bam(p, nrec)
        out[name] = data
    return out


@pytest.mark.parametrize("name", [s[0] for s in SYN])
def test_synthetic_inflate_and_eager(ctx, synth_files, name):
    data = synth_files[name]
    of = OracleFile(data)
    sh = load(ctx, data, of.contig_len)
    try:
        # the GPU index covers every segment; the oracle stream from 0 stops at the
        # first empty block: compare that prefix (later segments: see the next test)
        got = sh.read_flat(0, of.flat_size)
        i = first_diff(got, of.uncompressed())
        assert i < 0, f"inflate differs at flat {i}"
        n, bits = sh.check_eager(0, of.flat_size)
        n_ref, bits_ref = of.eager_range(0, of.flat_size)
        i = first_diff(np.unpackbits(bits, bitorder="little"), np.unpackbits(bits_ref, bitorder="little"))
        assert i < 0 and n == n_ref, f"eager differs at {i} ({n} vs {n_ref})"
        e = min(of.flat_size, 300000)
        r = sh.check_full(0, e, want_words=True)
        _, counts_ref, _, w_ref = of.full_range(0, e, want_words=True)
        i = first_diff(r["words"], w_ref)
        assert i < 0, f"full word differs at {i}: {hex(r['words'][i])} vs {hex(w_ref[i])}"
    finally:
        sh.close()


@pytest.mark.parametrize("name", ["long", "adversarial", "short_l6"])
def test_synthetic_find_record_start(ctx, synth_files, name):
    # FindRecordStart from random offsets through the eager bitmap (k_first_set's chunked
    # grid walk: long reads put the next record start tens of KiB, i.e. chunks, ahead) and
    # through fresh eager windows (a shard with no bitmap yet), against the oracle
    data = synth_files[name]
    of = OracleFile(data)
    rng = np.random.default_rng(len(name))
    offs = rng.integers(0, of.flat_size - 1, 16).tolist() + [0, of.flat_size - 40]
    for covered in (False, True):
        sh = load(ctx, data, of.contig_len)
        try:
            if covered:
                sh.check_eager(0, of.flat_size)
            for f in offs:
                rc, want, d = of.find_record_start(int(f))
                if rc == OR_OK:
                    assert sh.find_record_start(int(f)) == (want, d), (name, covered, f)
                else:
                    with pytest.raises(sb.SparkBamError):
                        sh.find_record_start(int(f))
        finally:
            sh.close()


def test_synthetic_empty_block_segments(ctx, synth_files):
    # empty BGZF blocks end the stream (Stream.scala:56-58): a stream opened after the
    # k-th empty block sees only that segment
    data = synth_files["adversarial_empty"]
    sh = load(ctx, data)
    of0 = OracleFile(data)
    sh.set_contigs(of0.contig_len)
    blocks = sh.blocks()
    empties = [i for i, b in enumerate(blocks) if b[5] & sb.BLOCK_EMPTY]
    assert len(empties) >= 3
    try:
        for k in empties[:3]:
            nxt = blocks[k + 1] if k + 1 < len(blocks) else None
            if nxt is None or nxt[5] & sb.BLOCK_EMPTY:
                continue
            of = OracleFile(data, start=nxt[0])
            base = nxt[3]
            got = sh.read_flat(base, of.flat_size)
            assert np.array_equal(got, of.uncompressed())
            n, bits = sh.check_eager(base, base + of.flat_size)
            # oracle stream positions are relative to its start block
            cl = of0.contig_len
            ref = np.zeros(of.flat_size, dtype=bool)
            for p in range(of.flat_size):
                ref[p] = of.eager(p, contig_len=cl)
            assert np.array_equal(np.unpackbits(bits, bitorder="little")[:of.flat_size].astype(bool), ref)
    finally:
        sh.close()


@pytest.mark.parametrize("name", ["short_l6", "long", "adversarial"])
def test_synthetic_splits(ctx, synth_files, name):
    data = synth_files[name]
    of = OracleFile(data)
    size = max(data.size // 7, 70000)
    splits, counts = sb.load_splits_and_reads(data, size, ctx=ctx)
    ref_counts, firsts = [], []
    for s, e in file_splits(data.size, size):
        rc, v, n = of.split(s, e)
        assert rc == OR_OK
        ref_counts.append(n)
        if n:
            firsts.append(v)
    assert counts == ref_counts
    assert [a.to_htsjdk() for a, _ in splits] == firsts


def test_inflate_corrupt_matches_zlib(ctx, synth_files):
    """Flip bytes inside deflate data: the per-block outcome (ok / size / data error)
    must be what zlib (Inflater) reports for that block."""
    data0 = synth_files["short_l1"]
    of = OracleFile(data0)
    L = olib()
    import ctypes as C
    rng = np.random.default_rng(3)
    mism = []
    for trial in range(40):
        data = data0.copy()
        b = of.blocks[int(rng.integers(0, len(of.blocks)))]
        start, csize = b[0], b[1]
        off = start + 18 + int(rng.integers(0, csize - 26))
        data[off] ^= np.uint8(1 << int(rng.integers(0, 8)))
        out = np.zeros(65536, dtype=np.uint8)
        blk = (C.c_int64 * 3)()
        rc_ref = L.or_stream_next(data.ctypes.data_as(C.c_void_p), data.size, start,
                                  out.ctypes.data_as(C.c_void_p), blk)
        sh = ctx.shard(data)
        sh.index(0)
        try:
            sh.inflate()
            rc = 0
        except sb.SparkBamError as e:
            rc = e.code
        sh.close()
        want = {0: 0, 1: 0, 4: 13, 5: 14, 6: 15}.get(rc_ref, -1)
        if rc != want:
            mism.append((trial, off, rc, rc_ref))
    assert not mism, mism


def test_shard_with_halo_matches_whole_file(ctx, synth_files):
    """A byte-range shard (not at EOF) with a halo: eager bits of its owned blocks equal
    the whole-file result; with no halo the call reports SBH_E_NEED_HALO."""
    data = synth_files["short_l6"]
    of = OracleFile(data)
    whole = load(ctx, data, of.contig_len)
    blocks = whole.blocks()
    try:
        k0, k1 = 10, 30
        s0 = blocks[k0][0]
        own_end = blocks[k1][0]
        halo_end = blocks[k1 + 3][0]
        sh = ctx.shard(data[s0:halo_end], file_offset=s0, file_size=data.size)
        sh.index(s0)
        sh.inflate()
        sh.set_contigs(of.contig_len)
        E = sh.flat_bound(own_end)
        n, bits = sh.check_eager(0, E)
        base = blocks[k0][3]
        n2, bits2 = whole.check_eager(base, base + E)
        assert n == n2 and np.array_equal(bits, bits2)
        with pytest.raises(sb.SparkBamError) as e:
            sh.check_eager(0, sh.flat_size)
        assert e.value.code == 17
        sh.close()
    finally:
        whole.close()


@pytest.mark.parametrize("name,batch_blocks", [("short_l6", 4), ("long", 2), ("adversarial", 3)])
def test_pipelined_run_matches_separate_calls(ctx, synth_files, name, batch_blocks):
    """run() inflates and checks in a pipeline over block batches (eager tiles launched
    behind the inflate frontier, positions whose exact check crosses it deferred).  With
    tiny batches (many frontiers; long reads cross them) it must equal inflate() +
    check_eager() + the record walk."""
    data = synth_files[name]
    of = OracleFile(data)
    sh = ctx.shard(data)
    sh.set_contigs(of.contig_len)
    old = os.environ.get("SBH_PIPE_MIN_BLOCKS")
    os.environ["SBH_PIPE_MIN_BLOCKS"] = str(batch_blocks)
    try:
        r = sh.run(0, data.size)
        got = sh.read_flat(0, of.flat_size)
        i = first_diff(got, of.uncompressed())
        assert i < 0, f"inflate differs at flat {i}"
        E = r["flat_bytes"]
        bits_pipe = sh.eager_bits(0, E)
    finally:
        if old is None:
            del os.environ["SBH_PIPE_MIN_BLOCKS"]
        else:
            os.environ["SBH_PIPE_MIN_BLOCKS"] = old
    assert r["status"] == 0
    # the same shard, unpipelined, over the same range
    sh.index(0)
    sh.inflate()
    n, bits = sh.check_eager(0, E)
    assert r["n_true"] == n
    i = first_diff(np.unpackbits(bits_pipe, bitorder="little"), np.unpackbits(bits, bitorder="little"))
    assert i < 0, f"pipelined eager differs at {i}"
    # and the first stream segment against the oracle
    n_ref, bits_ref = of.eager_range(0, of.flat_size)
    k = of.flat_size
    assert np.array_equal(np.unpackbits(bits_pipe, bitorder="little")[:k], np.unpackbits(bits_ref, bitorder="little")[:k])
    sh.close()


@pytest.mark.parametrize("marking", ["peel", "doubling"])
@pytest.mark.parametrize("name", ["adversarial", "short_l6", "long"])
def test_chain_count_with_false_positive_bits(ctx, synth_files, name, marking, monkeypatch):
    """Record counts / exits / record starts over an eager bitmap that holds false
    positives (config E's bait): the chain marker -- off-chain nodes peeled from the nodes no
    record steps to (default), or pointer doubling (SBH_CM_DOUBLING=1) -- must give exactly
    the PosStream chain (oracle walk), for ranges starting at true records."""
    monkeypatch.setenv("SBH_CM_DOUBLING", "1" if marking == "doubling" else "0")
    data = synth_files[name]
    of = OracleFile(data)
    sh = load(ctx, data, of.contig_len)
    try:
        n_true, _ = sh.check_eager(0, of.flat_size)
        _, _, first = sb.parse_bam_header(sh.read_flat(0, min(of.flat_size, 1 << 20)))
        chain = of.record_chain(first)
        if name == "adversarial":
            assert n_true > len(chain)  # the bitmap really holds false positives
        rng = np.random.default_rng(7)
        cases = [(0, len(chain), of.flat_size)]
        for _ in range(6):
            i = int(rng.integers(0, len(chain) - 1))
            e = int(rng.integers(int(chain[i]) + 1, of.flat_size + 1))
            cases.append((i, None, e))
        for i, _, e in cases:
            f = int(chain[i])
            want = [int(x) for x in chain[i:] if x < e]
            assert sh.count_records(f, e) == len(want), (name, f, e)
            got = sh.records(f, e)["flat"]
            assert [int(x) for x in got] == want, (name, f, e)
    finally:
        sh.close()


@pytest.mark.parametrize("name", ["adversarial", "short_l6", "short_l0", "long"])
def test_chain_proof_tile_summaries(ctx, synth_files, name, monkeypatch):
    """The chain proof (k_verify_chain_w) reading k_eager's per-tile summaries gives the same
    counts, exits and anomaly counts as reading every true position's length from U
    (SBH_TSUM=1 vs 0), over the whole file (sbh_run_shard, pipelined eager) and over sub-ranges
    that start and end inside tiles or on tile edges (sbh_check_eager's bitmap)."""
    data = synth_files[name]
    of = OracleFile(data)
    tile = 16384

    def run(flag):
        monkeypatch.setenv("SBH_TSUM", flag)
        sh = load(ctx, data, of.contig_len)
        try:
            r = sh.run(0, data.size)
            _, _, first = sb.parse_bam_header(sh.read_flat(0, min(of.flat_size, 1 << 20)))
            chain = of.record_chain(first)
            sh.check_eager(0, of.flat_size)
            out = [(r["count"], r["exit_flat"], r["anomalies"], r["n_true"])]
            rng = np.random.default_rng(11)
            for _ in range(8):
                i = int(rng.integers(0, len(chain) - 1))
                f = int(chain[i])
                for e in (int(rng.integers(f + 1, of.flat_size + 1)), (f // tile + 3) * tile, of.flat_size):
                    e = min(e, of.flat_size)
                    want = int(np.count_nonzero((chain >= f) & (chain < e)))
                    got = sh.count_records(f, e)
                    assert got == want, (name, flag, f, e)
                    out.append((f, e, got, sh.chain_from(f, e)))
            return out, len(chain)
        finally:
            sh.close()

    on, n_chain = run("1")
    off, _ = run("0")
    assert on == off
    assert on[0][0] == n_chain


@pytest.mark.parametrize("name", FIXTURES)
def test_verify_crc_fixtures(ctx, name):
    """Every inflated block's bytes match its BGZF footer CRC32 (sbh_verify_crc)."""
    data = np.fromfile(golden_bam(name), dtype=np.uint8)
    sh = load(ctx, data)
    try:
        assert sh.verify_crc()[0] == 0
    finally:
        sh.close()


def test_verify_crc_synthetic_and_corrupt_footer(ctx, synth_files):
    for name in ("short_l6", "short_l0", "long", "adversarial_empty"):
        sh = load(ctx, synth_files[name])
        try:
            assert sh.verify_crc()[0] == 0, name
        finally:
            sh.close()
    # a flipped footer CRC byte: inflate is unaffected (the reference never reads CRC32),
    # the check names exactly that block
    data = np.fromfile(golden_bam("2.bam"), dtype=np.uint8).copy()
    blocks = read_blocks("2.bam")
    start, csize = blocks[3][0], blocks[3][1]
    data[start + csize - 8] ^= 0x5A
    sh = load(ctx, data)
    try:
        assert sh.verify_crc() == (1, start)
    finally:
        sh.close()


# readsToCheck (CheckerApp / CanLoadBam `--reads-to-check`, default 10) and
# bgzfBlocksToCheck (`-z`, default 5) away from their defaults: the device honours any value
# the ABI accepts (rtc 0..1023), bit for bit with the oracle at each.
RTCS = [0, 1, 2, 3, 25, 100, 1023]


@pytest.mark.parametrize("rtc", RTCS)
@pytest.mark.parametrize("name", ["2.bam", "5k.bam"])
def test_eager_reads_to_check(golden, name, rtc):
    data, of, sh = golden[name]
    end = min(sh.flat_size, 400000)
    n, bits = sh.check_eager(0, end, reads_to_check=rtc)
    n_ref, bits_ref = of.eager_range(0, end, reads_to_check=rtc)
    i = first_diff(np.unpackbits(bits, bitorder="little"), np.unpackbits(bits_ref, bitorder="little"))
    assert i < 0, f"rtc {rtc}: first differing position {i}"
    assert n == n_ref


@pytest.mark.parametrize("rtc", RTCS)
def test_full_reads_to_check(golden, rtc):
    data, of, sh = golden["2.bam"]
    r = sh.check_full(0, 150000, reads_to_check=rtc, want_words=True)
    _, counts_ref, rbe_ref, w_ref = of.full_range(0, 150000, reads_to_check=rtc, want_words=True)
    i = first_diff(r["words"], w_ref)
    assert i < 0, f"rtc {rtc}: position {i}"
    assert np.array_equal(r["counts"].astype(np.int64), counts_ref)
    assert np.array_equal(r["rbe"].astype(np.int64), rbe_ref)


@pytest.mark.parametrize("rtc", [0, 1, 3, 100, 1023])
def test_find_record_start_reads_to_check(golden, rtc):
    data, of, sh = golden["1.bam"]
    rng = np.random.default_rng(rtc)
    for f in rng.integers(0, sh.flat_size - 1, 12).tolist() + [0, sh.flat_of(239479, 0)]:
        rc, want, d = of.find_record_start(int(f), reads_to_check=rtc)
        if rc == OR_OK:
            assert sh.find_record_start(int(f), reads_to_check=rtc) == (want, d), (f, rtc)
        else:
            with pytest.raises(sb.SparkBamError):
                sh.find_record_start(int(f), reads_to_check=rtc)


@pytest.mark.parametrize("z", [1, 2, 3, 10])
def test_find_block_start_blocks_to_check(golden, z):
    data, of, sh = golden["2.bam"]
    rng = np.random.default_rng(z)
    for s in rng.integers(0, data.size - 1, 20).tolist() + [0, 26170, data.size - 28]:
        rc, want = of.find_block_start(int(s), blocks_to_check=z)
        if rc == OR_OK:
            assert sh.find_block_start(int(s), bgzf_blocks_to_check=z) == want, (s, z)
        else:
            with pytest.raises(sb.SparkBamError):
                sh.find_block_start(int(s), bgzf_blocks_to_check=z)


@pytest.mark.parametrize("z,rtc", [(1, 1), (2, 0), (10, 3), (5, 100)])
def test_split_parameters(golden, z, rtc):
    data, of, sh = golden["1.bam"]
    for s, e in file_splits(data.size, 100 * 1024):
        rc, v, n = of.split(s, e, blocks_to_check=z, reads_to_check=rtc)
        if rc == OR_OK:
            got = sh.split(s, e, bgzf_blocks_to_check=z, reads_to_check=rtc)
            assert got[1] == n and (n == 0 or got[0] == v), (s, e, z, rtc)
        else:
            with pytest.raises(sb.SparkBamError):
                sh.split(s, e, bgzf_blocks_to_check=z, reads_to_check=rtc)
    # the batched path (sbh_split_starts) agrees at the same parameters
    sp = [(s, e) for s, e in file_splits(data.size, 100 * 1024)]
    status, v, c, _ = sh.split_starts(sp, bgzf_blocks_to_check=z, reads_to_check=rtc)
    for k, (s, e) in enumerate(sp):
        rc, want_v, want_n = of.split(s, e, blocks_to_check=z, reads_to_check=rtc)
        if rc == OR_OK:
            assert status[k] == 0 and int(c[k]) == want_n and (want_n == 0 or int(v[k]) == want_v), (s, e, z, rtc)
        else:
            assert status[k] != 0, (s, e, z, rtc)


def test_shard_lifecycle_frees_hbm(ctx):
    """Creating and destroying shards (index, inflate, eager pass, whole run) leaves device
    memory where it was: every buffer a shard grows is released by sbh_shard_destroy (ADVICE r04:
    the eager tile-summary buffer was not)."""
    import ctypes as C
    # the HIP runtime libsparkbam_hip.so itself links (torch, when imported earlier in the run,
    # brings its own libamdhip64.so: a second runtime instance with no device state of ours)
    hip = C.CDLL("libamdhip64.so.7")
    free, total = C.c_size_t(), C.c_size_t()

    def free_now():
        assert hip.hipMemGetInfo(C.byref(free), C.byref(total)) == 0
        return free.value

    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
    import synth
    data = synth.make_bam(synth.params(0x5B4D0001), 100_000)[0]  # ~33 MB flat
    of = OracleFile(data)

    def cycle():
        sh = load(ctx, data, of.contig_len)
        sh.check_eager(0, of.flat_size)
        sh.run(0, data.size)
        sh.close()

    cycle()
    before = free_now()
    for _ in range(12):
        cycle()
    assert before - free_now() < (1 << 20), (before, free_now())
