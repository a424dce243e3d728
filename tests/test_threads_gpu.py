"""One context shared by concurrent task threads (include/sparkbam.h, threading): a Spark
executor runs its tasks on concurrent threads, every one calling the same device context
(jni/Native.scala Device), each task with its own shard -- the reference's own model, where each
task builds its own channel and checker (load/.../CanLoadBam.scala:316-320,
check/.../PosChecker.scala:19-20).

Four threads start together on one Context and run, at the same time:
  * the per-split load path (canloadbam.SplitWorker = GpuSplitPartition: sbh_split_records over a
    reused shard) and the round-5 sequence of separate calls (split_partition_calls), over the
    splits of the configs[1] (short reads) and configs[3] (long reads) generators;
  * sbh_run_stream2 with per-split results (the pooled window caches);
  * calls that fail -- FindBlockStart over junk, FindRecordStart with a tiny maxReadSize -- whose
    exception class and constructor fields must come back intact while the others succeed.
Every answer is checked against the CPU oracle (record starts as vpos, per split)."""
import os
import sys
import threading

import numpy as np
import pytest

from oracle_lib import OR_OK, OracleFile, file_splits
from pkg import sb

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
clb = __import__(sb.__name__ + ".canloadbam", fromlist=["x"])

CORPORA = {
    "short": (dict(seed=0x5B4D0001, shape=0, level=6), 60000, 400_000),  # configs[1] shape
    "long": (dict(seed=0x5B4D004C, shape=1, level=6), 300, 700_000),     # configs[3] shape
}


@pytest.fixture(scope="module")
def ctx():
    c = sb.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def corpora():
    import synth
    out = {}
    for name, (kw, nrec, split) in CORPORA.items():
        data = synth.make_bam(synth.params(kw["seed"], shape=kw["shape"], level=kw["level"]), nrec)[0]
        of = OracleFile(data)
        splits = file_splits(of.size, split)
        want = []  # per split: the record starts as htsjdk vpos (oracle: FindBlockStart, FindRecordStart, chain)
        for s, e in splits:
            rc, v, n = of.split(s, e)
            assert rc == OR_OK
            if n == 0:
                want.append(np.zeros(0, np.uint64))
                continue
            f0 = of.flat_of(v >> 16, v & 0xffff)
            chain = of.record_chain(f0)[:n]
            want.append(np.array([(lambda bp, o: (bp << 16) | o)(*of.pos_of(int(f))) for f in chain], np.uint64))
        out[name] = (data, of, splits, want, nrec)
    return out


def _run_threads(targets):
    """Start every target at once (a barrier), join, re-raise the first failure."""
    bar = threading.Barrier(len(targets))
    errs = []

    def wrap(fn):
        def run():
            try:
                bar.wait()
                fn()
            except BaseException as e:  # noqa: B902 (re-raised below)
                errs.append(e)
        return run

    ts = [threading.Thread(target=wrap(f)) for f in targets]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        raise errs[0]


def test_concurrent_split_tasks(ctx, corpora):
    """Four task threads over the splits of two corpora at once: two with reused workers
    (sbh_split_records), one with the separate-call sequence, one streaming its corpus with
    per-split results -- each answer equal to the oracle's."""
    got = {}

    def worker_task(name, parity):
        data, of, splits, want, _ = corpora[name]
        read = sb_reader(data)
        w = clb.SplitWorker(ctx, data.size, of.contig_len)
        try:
            for i in range(parity, len(splits), 2):
                s, e = splits[i]
                got[(name, i, "worker")] = w.split(read, name, s, e)["vpos"]
        finally:
            w.close()

    def calls_task(name):
        data, of, splits, want, _ = corpora[name]
        read = sb_reader(data)
        for i, (s, e) in enumerate(splits):
            got[(name, i, "calls")] = clb.split_partition_calls(ctx, read, data.size, name, s, e, of.contig_len)["vpos"]

    def stream_task(name):
        data, of, splits, want, _ = corpora[name]
        for rep in range(2):  # (two calls: the pooled cache is taken and given back)
            r, _ = ctx.run_stream(data, of.contig_len, index_start=0, window=300_000, halo=1 << 16, splits=splits)
            got[(name, rep, "stream")] = r

    _run_threads([lambda: worker_task("short", 0), lambda: worker_task("short", 1),
                  lambda: calls_task("long"), lambda: stream_task("short")])
    _run_threads([lambda: worker_task("long", 0), lambda: worker_task("long", 1),
                  lambda: calls_task("short"), lambda: stream_task("long")])
    for name, (data, of, splits, want, nrec) in corpora.items():
        for i in range(len(splits)):
            for how in ("worker", "calls"):
                v = got[(name, i, how)]
                assert np.array_equal(np.asarray(v, np.uint64), want[i]), (name, i, how)
        assert sum(w.size for w in want) == nrec
        for rep in range(2):
            r = got[(name, rep, "stream")]
            assert r["status"] == 0 and r["count"] == nrec
            assert list(r["split_count"]) == [w.size for w in want], (name, rep)
            firsts = [int(w[0]) for w in want if w.size]
            assert [int(v) for v, n in zip(r["split_first_vpos"], r["split_count"]) if n] == firsts


def test_concurrent_failures_keep_their_fields(ctx, corpora):
    """Failing calls on some threads while others succeed on the same context: each thread's
    exception is its own (class, message and the reference constructor's fields), and the
    succeeding threads' answers equal the oracle's."""
    rng = np.random.default_rng(7)
    junk = rng.integers(0, 256, 200_000, dtype=np.uint8)
    junk[junk == 31] = 30  # no gzip magic anywhere
    data, of, splits, want, _ = corpora["short"]
    out = {}

    def search_failed(start):
        def run():
            for _ in range(20):
                sh = ctx.shard(junk)
                try:
                    with pytest.raises(sb.HeaderSearchFailedException) as e:
                        sh.find_block_start(start)
                    out.setdefault(("hsf", start), []).append((e.value.start, e.value.positions_attempted))
                finally:
                    sh.close()
        return run

    def no_read_found():
        # the first split starts inside the BAM header block; 100 positions hold no record start
        w = clb.SplitWorker(ctx, data.size, of.contig_len)
        try:
            for _ in range(20):
                with pytest.raises(sb.NoReadFoundException) as e:
                    w.split(sb_reader(data), "short.bam", 0, splits[0][1], max_read_size=100)
                out.setdefault("nrf", []).append((e.value.path, e.value.start, e.value.max_read_size))
        finally:
            w.close()

    def good():
        w = clb.SplitWorker(ctx, data.size, of.contig_len)
        try:
            for rep in range(3):
                for i, (s, e) in enumerate(splits):
                    out[("good", rep, i)] = w.split(sb_reader(data), "short.bam", s, e)["vpos"]
        finally:
            w.close()

    _run_threads([search_failed(1000), search_failed(5000), no_read_found, good])
    assert out[("hsf", 1000)] == [(1000, 65536)] * 20
    assert out[("hsf", 5000)] == [(5000, 65536)] * 20
    assert out["nrf"] == [("short.bam", 0, 100)] * 20
    for rep in range(3):
        for i in range(len(splits)):
            assert np.array_equal(np.asarray(out[("good", rep, i)], np.uint64), want[i])


def sb_reader(data):
    from importlib import import_module
    return import_module(sb.__name__ + ".sharded").bytes_reader(data)
