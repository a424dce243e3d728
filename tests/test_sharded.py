"""Byte-range sharding across ranks (spark-bam_amd/sharded.py).

CPU tests (gloo, world_size 2 and 3) drive the product's exchange + stitch with per-rank
parts that the oracle computes for each rank's Hadoop splits, and compare the stitched
result with the single-process oracle's loadSplitsAndReads and the reference goldens
(LoadBAMTest / ComputeSplitsTest values restated in SURVEY.md §8c).  The GPU test runs
the whole sharded path (sharded.load_splits_and_reads) in 2 processes on cuda:0.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT, golden_bam
from pkg import sb
from oracle_lib import OracleFile, file_splits, load_splits_and_reads as oracle_splits

import spark_bam_amd.sharded as sharded  # noqa: E402  (pkg registered the package)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _oracle_part(of, rank, world, split_size):
    """What run_rank computes on a device, computed by the oracle (the checker)."""
    a, mine = sharded.rank_splits(of.size, split_size, world, rank)
    if not mine:
        return sharded.RankPart(rank, a, [], [], None, 0, None)
    firsts, counts = [], []
    for s, e in mine:
        rc, v, n = of.split(s, e)
        assert rc == 0
        firsts.append(v if n else None)
        counts.append(n)
    lo, hi = mine[0][0], mine[-1][1]
    rc, b = of.find_block_start(lo)
    assert rc == 0
    rc, first, _ = of.find_record_start(of.flat_of(b, 0))
    E = next((of.flat_of(s, 0) for s, _c, _u in of.blocks if s >= hi), of.flat_size)
    chain = of.record_chain(first, of.flat_size)
    inside = [r for r in chain if r < E]
    after = [r for r in chain if r >= E]
    exit_vpos = None
    if after:
        bp, off = of.pos_of(int(after[0]))
        exit_vpos = (bp << 16) | off
    bp, off = of.pos_of(first)
    return sharded.RankPart(rank, a, firsts, counts, (bp << 16) | off if inside else None,
                            len(inside), exit_vpos)


def _oracle_rewalk(of, rank, world, split_size):
    """RankRun.rewalk computed by the oracle: the chain from a vpos, counted while the record
    starts before the rank's owned end, and its exit vpos."""
    _, mine = sharded.rank_splits(of.size, split_size, world, rank)
    hi = mine[-1][1]
    E = next((of.flat_of(s, 0) for s, _c, _u in of.blocks if s >= hi), of.flat_size)

    def rewalk(v):
        chain = of.record_chain(of.flat_of(v >> 16, v & 0xFFFF), of.flat_size)
        after = [r for r in chain if r >= E]
        ex = None
        if after:
            bp, off = of.pos_of(int(after[0]))
            ex = (bp << 16) | off
        return int(sum(1 for r in chain if r < E)), ex
    return rewalk


def _gloo_worker(rank, world, port, path, split_size, fail_rank, out_dir):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        of = OracleFile.from_path(path)
        part = _oracle_part(of, rank, world, split_size)
        if rank == fail_rank:
            part = sb.SparkBamError(17, "injected")
        try:
            splits, counts, st = sharded.stitch(sharded.exchange(part), of.size)
            res = {"splits": [[a.to_htsjdk(), b.to_htsjdk()] for a, b in splits], "counts": counts,
                   "ok": st["ok"]}
        except sb.SparkBamError as e:
            res = {"error": e.code}
        with open(os.path.join(out_dir, f"r{rank}.json"), "w") as f:
            json.dump(res, f)
    finally:
        dist.destroy_process_group()


def _run_gloo(world, path, split_size, tmp_path, fail_rank=-1):
    import torch.multiprocessing as mp

    mp.spawn(_gloo_worker, args=(world, _free_port(), path, split_size, fail_rank, str(tmp_path)),
             nprocs=world, join=True)
    return [json.load(open(tmp_path / f"r{r}.json")) for r in range(world)]


def test_rank_splits_partition_the_file():
    for size, split, world in [(531753, 102400, 2), (531753, 102400, 4), (597482, 300 * 1024, 3),
                               (10, 100, 4), (1 << 30, (1 << 30) // 8, 8)]:
        got = []
        for r in range(world):
            a, mine = sharded.rank_splits(size, split, world, r)
            assert a == len(got)
            got += mine
        assert got == sb.file_splits(size, split)


@pytest.mark.parametrize("name,split_size,world,expect_counts", [
    ("2.bam", 102400, 2, [503, 519, 413, 518, 495, 52]),
    ("2.bam", 102400, 3, [503, 519, 413, 518, 495, 52]),
    ("1.bam", 300 * 1024, 2, [2536, 2381]),
    ("2.bam", None, 2, None),  # one byte-range shard per rank
])
def test_gloo_exchange_and_stitch(tmp_path, name, split_size, world, expect_counts):
    path = golden_bam(name)
    of = OracleFile.from_path(path)
    ss = split_size or -(-of.size // world)
    ref_splits, ref_counts = oracle_splits(of, ss)
    res = _run_gloo(world, path, ss, tmp_path)
    for r in res:  # identical on every rank, equal to the single-process reference answer
        assert r == res[0]
        assert r["counts"] == ref_counts
        assert [tuple(s) for s in r["splits"]] == ref_splits
        assert r["ok"]
    if expect_counts:
        assert res[0]["counts"] == expect_counts


def test_gloo_rank_failure_reaches_every_rank(tmp_path):
    res = _run_gloo(2, golden_bam("2.bam"), 102400, tmp_path, fail_rank=1)
    assert [r.get("error") for r in res] == [17, 17]


def _gloo_fp_worker(rank, world, port, path, split_size, out_dir):
    """Rank 1's part as if its FindRecordStart had stopped on a false positive one record
    past its true first record: the stitch must re-walk rank 1 from rank 0's exit."""
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        of = OracleFile.from_path(path)
        part = _oracle_part(of, rank, world, split_size)
        true_count = part.count
        if rank == 1:
            chain = of.record_chain(of.flat_of(part.first_vpos >> 16, part.first_vpos & 0xFFFF), of.flat_size)
            bp, off = of.pos_of(int(chain[1]))
            part = part._replace(first_vpos=(bp << 16) | off, count=part.count - 1)
        splits, counts, st = sharded.reconcile(sharded.exchange(part), of.size, rank,
                                               _oracle_rewalk(of, rank, world, split_size))
        with open(os.path.join(out_dir, f"r{rank}.json"), "w") as f:
            json.dump({"st": {k: st[k] for k in ("ok", "chain_ok", "chain_count")},
                       "rewalk": {str(k): v for k, v in st["rewalk"].items()}, "true_count": true_count,
                       "counts": counts}, f)
    finally:
        dist.destroy_process_group()


def test_gloo_stitch_rewalks_a_false_positive_first(tmp_path):
    path = golden_bam("2.bam")
    of = OracleFile.from_path(path)
    ss = -(-of.size // 2)
    import torch.multiprocessing as mp

    mp.spawn(_gloo_fp_worker, args=(2, _free_port(), path, ss, str(tmp_path)), nprocs=2, join=True)
    res = [json.load(open(tmp_path / f"r{r}.json")) for r in range(2)]
    _, ref_counts = oracle_splits(of, ss)
    for r in res:
        assert r["st"]["ok"] is False and r["st"]["chain_ok"] is True
        assert r["st"]["chain_count"] == 2500 == sum(ref_counts)
        assert r["rewalk"]["1"]["count"] == res[1]["true_count"]
        assert r["counts"] == ref_counts  # the per-split answer is untouched


def _gloo_raise_worker(rank, world, port, path, out_dir):
    """load_splits_and_reads with rank 1 failing by a plain ValueError (not a SparkBamError)
    before its run: rank 0 (whose run is the oracle's part) must not block in the exchange."""
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        of = OracleFile.from_path(path)

        def read_header(ctx, read, file_size):
            if rank == 1:
                raise ValueError("injected header failure")
            return [], of.contig_len, of.header_end

        class FakeRun:
            def __init__(self, ctx, read, file_size, a, mine, contig_len, r, halo, **kw):
                self.part = _oracle_part(of, r, world, -(-of.size // world))

            def rewalk(self, v):
                raise AssertionError("no re-walk expected")

            def close(self):
                pass

        sharded.read_header, sharded.RankRun = read_header, FakeRun
        try:
            sharded.load_splits_and_reads(path, ctx=object())
            res = {"error": None}
        except sb.SparkBamError as e:
            res = {"error": "SparkBamError", "code": e.code, "msg": str(e)}
        except ValueError as e:
            res = {"error": "ValueError", "msg": str(e)}
        with open(os.path.join(out_dir, f"r{rank}.json"), "w") as f:
            json.dump(res, f)
    finally:
        dist.destroy_process_group()


def test_gloo_non_sparkbam_failure_reaches_every_rank(tmp_path):
    import torch.multiprocessing as mp

    mp.spawn(_gloo_raise_worker, args=(2, _free_port(), golden_bam("2.bam"), str(tmp_path)), nprocs=2, join=True)
    r0, r1 = (json.load(open(tmp_path / f"r{r}.json")) for r in range(2))
    assert r1 == {"error": "ValueError", "msg": "injected header failure"}
    assert r0["error"] == "SparkBamError" and r0["code"] == -1 and "ValueError" in r0["msg"]


def test_stitch_reports_mismatch():
    P = sharded.RankPart
    parts = [P(1, 2, [900 << 16], [5], 900 << 16, 5, None),
             P(0, 0, [10 << 16, None], [7, 0], 10 << 16, 7, 899 << 16)]
    splits, counts, st = sharded.stitch(parts, 1000)
    assert counts == [7, 0, 5]
    assert [(a.to_htsjdk(), b.to_htsjdk()) for a, b in splits] == [(10 << 16, 900 << 16),
                                                                    (900 << 16, 1000 << 16)]
    assert not st["ok"] and st["mismatches"][0]["rank"] == 0


GPU_WORKER = r"""
import json, os, sys
sys.path.insert(0, os.environ["SBH_ROOT"])
import torch.distributed as dist
from __graft_entry__ import load_package
sb = load_package()
import spark_bam_amd.sharded as sharded
if os.environ.get("SBH_TEST_BACKEND", "gloo") == "nccl":  # RCCL on the box's one device
    import torch
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
else:
    dist.init_process_group("gloo")
path, ss = sys.argv[1], (int(sys.argv[2]) or None)
if os.environ.get("SBH_TEST_FP_RANK"):
    # rank k's chain as if its FindRecordStart had stopped on a false positive one record
    # past its true first record: the stitch must re-walk it from the upstream exit
    fp_rank = int(os.environ["SBH_TEST_FP_RANK"])

    class FPRun(sharded.RankRun):
        def __init__(self, *a, **kw):
            super().__init__(*a, **kw)
            p = self.part
            if self.rank == fp_rank and p.count > 1:
                if self.sh is not None:
                    sh = self.sh
                    f = sh.flat_of(p.first_vpos >> 16, p.first_vpos & 0xFFFF)
                    nxt = f + 4 + int(sh.read_flat(f, 4).view("<i4")[0])
                    bp, off = sh.pos_of(nxt)
                else:  # a streamed rank keeps no shard: the checker's view of the file
                    sys.path.insert(0, os.path.join(os.environ["SBH_ROOT"], "tests"))
                    from oracle_lib import OracleFile
                    of = OracleFile.from_path(path)
                    f = of.flat_of(p.first_vpos >> 16, p.first_vpos & 0xFFFF)
                    nxt = f + 4 + int(of.uncompressed_range(f, f + 4).view("<i4")[0])
                    bp, off = of.pos_of(nxt)
                self.true_count = p.count
                self.part = p._replace(first_vpos=(bp << 16) | off, count=p.count - 1)
    sharded.RankRun = FPRun
with sb.Context(0) as ctx:  # every rank shares the one device of the box
    splits, counts, st = sharded.load_splits_and_reads(path, ss, ctx=ctx, halo=int(sys.argv[3]))
json.dump({"splits": [[a.to_htsjdk(), b.to_htsjdk()] for a, b in splits], "counts": counts,
           "ok": st["ok"], "rank_counts": st["rank_counts"], "mismatches": st["mismatches"],
           "chain_ok": st["chain_ok"], "chain_count": st["chain_count"],
           "rewalk": {str(k): v for k, v in st["rewalk"].items()}},
          open(os.path.join(sys.argv[4], "r%d.json" % dist.get_rank()), "w"))
dist.destroy_process_group()
"""


def _run_gpu_ranks(tmp_path, path, split_size, halo, world=2, env_extra=None, timeout=150):
    script = tmp_path / "w.py"
    script.write_text(GPU_WORKER)
    env = dict(os.environ, SBH_ROOT=ROOT, MASTER_ADDR="127.0.0.1", **(env_extra or {}))
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
                    "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(script), path,
                    str(split_size), str(halo), str(tmp_path)], env=env, check=True, timeout=timeout)
    return [json.load(open(tmp_path / f"r{r}.json")) for r in range(world)]


@pytest.mark.gpu
@pytest.mark.parametrize("name,split_size,halo", [("2.bam", 0, 1 << 20), ("2.bam", 102400, 4096),
                                                   ("1.bam", 300 * 1024, 1 << 20),
                                                   ("1.bam", 0, 4096)])
def test_gpu_two_ranks_on_one_device(tmp_path, name, split_size, halo):
    """Two processes (gloo exchange) share cuda:0, each running its shard's hot path; a
    4 KiB starting halo forces the NEED_HALO growth loop."""
    path = golden_bam(name)
    res = _run_gpu_ranks(tmp_path, path, split_size, halo)
    of = OracleFile.from_path(path)
    ref_splits, ref_counts = oracle_splits(of, split_size or -(-of.size // 2))
    for r in res:
        assert r["counts"] == ref_counts
        assert [tuple(s) for s in r["splits"]] == ref_splits
        assert r["ok"], (r, [_oracle_part(of, k, 2, split_size or -(-of.size // 2)) for k in range(2)])


@pytest.mark.gpu
@pytest.mark.parametrize("name,split_size", [("2.bam", 102400), ("1.bam", 0)])
def test_gpu_rccl_exchange_one_rank(tmp_path, name, split_size):
    """The load path's exchange over RCCL (backend "nccl": device tensors, all_gather_object)
    with the one rank a one-GPU box allows; the splits and counts equal the oracle's."""
    path = golden_bam(name)
    res = _run_gpu_ranks(tmp_path, path, split_size, 1 << 20, world=1, env_extra={"SBH_TEST_BACKEND": "nccl"})
    of = OracleFile.from_path(path)
    ref_splits, ref_counts = oracle_splits(of, split_size or of.size)
    assert res[0]["counts"] == ref_counts and [tuple(x) for x in res[0]["splits"]] == ref_splits
    assert res[0]["ok"]


def _synth_file(tmp_path, seed, shape, nrec, name):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import synth
    data = synth.make_bam(synth.params(seed, shape=shape, level=6), nrec)[0]
    path = str(tmp_path / name)
    data.tofile(path)
    return path, data


@pytest.mark.gpu
def test_gpu_four_ranks_wgs_shape(tmp_path):
    """configs[2]'s generator shape (seed 0x5B4D0030, 30x-WGS short reads) byte-range
    sharded over 4 ranks on cuda:0, each rank several Hadoop splits, vs the oracle."""
    path, data = _synth_file(tmp_path, 0x5B4D0030, 0, 50000, "wgs.bam")
    of = OracleFile(data)
    ss = data.size // 10
    res = _run_gpu_ranks(tmp_path, path, ss, 1 << 18, world=4)
    ref_splits, ref_counts = oracle_splits(of, ss)
    assert sum(ref_counts) == 50000
    for r in res:
        assert r["counts"] == ref_counts and [tuple(s) for s in r["splits"]] == ref_splits
        assert r["ok"] and r["chain_ok"] and r["chain_count"] == 50000


def _edges_inside_long_records(of, world, min_len=65536):
    """A split size whose rank edges (the first split start of ranks 1..world-1) all land inside records
    longer than min_len (configs[3]: records straddle every shard edge): FindBlockStart from
    the edge reaches a block whose first byte lies strictly inside such a record, so the
    rank's FindRecordStart starts in the middle of it."""
    chain = of.record_chain(of.header_end, of.flat_size).tolist() + [of.flat_size]
    big = [(a, b) for a, b in zip(chain, chain[1:]) if b - a > min_len]
    good, prev = [], None  # compressed offsets whose next block start is inside a big record
    for s, c, u in of.blocks:
        f0 = of.flat_of(s, 0)
        if prev is not None and u and any(a < f0 < b for a, b in big):
            good.append((prev + 1, s + 1))
        prev = s
    for size in range(of.size // world, of.size // (10 * world), -97):
        edges = [sharded.rank_splits(of.size, size, world, r)[1][0][0] for r in range(1, world)]
        if all(any(a <= e < b for a, b in good) for e in edges):
            return size
    return None


@pytest.mark.gpu
def test_gpu_four_ranks_long_reads_edges_inside_records(tmp_path):
    """configs[3]: long reads (10-50 kb, some records > 64 KiB spanning BGZF blocks); every
    rank edge lies inside such a record, so each rank's FindRecordStart skips the rest of a
    >64 KiB record and the stitch joins the chain across the edge."""
    path, data = _synth_file(tmp_path, 0x5B4D004C, 1, 500, "long.bam")
    of = OracleFile(data)
    ss = _edges_inside_long_records(of, 4)
    assert ss is not None, "no split size puts every edge inside a > 64 KiB record"
    res = _run_gpu_ranks(tmp_path, path, ss, 4096, world=4)
    ref_splits, ref_counts = oracle_splits(of, ss)
    for r in res:
        assert r["counts"] == ref_counts and [tuple(s) for s in r["splits"]] == ref_splits
        assert r["ok"] and r["chain_ok"] and r["chain_count"] == 500


@pytest.mark.gpu
def test_gpu_stitch_rewalk_after_false_positive(tmp_path):
    """Rank 1 reports a first record one past its true one (an injected false positive):
    the stitch re-walks rank 1 on its device from rank 0's exit and reconciles the count."""
    path = golden_bam("2.bam")
    res = _run_gpu_ranks(tmp_path, path, 0, 1 << 20, world=3, env_extra={"SBH_TEST_FP_RANK": "1"})
    for r in res:
        assert not r["ok"] and r["chain_ok"] and r["chain_count"] == 2500
        assert r["rewalk"]["1"]["count"] == r["rank_counts"][1] + 1


STREAMED = {"SBH_RESIDENT_MAX": "1", "SBH_STREAM_WINDOW": "150000"}


@pytest.mark.gpu
def test_gpu_four_ranks_wgs_shape_streamed(tmp_path):
    """The same 4-rank configs[2] run with every rank streamed through HBM (RankRun over
    sbh_run_stream2: windows of 150 KB cut at split starts, per-split results per window)."""
    path, data = _synth_file(tmp_path, 0x5B4D0030, 0, 50000, "wgs.bam")
    of = OracleFile(data)
    ss = data.size // 23
    res = _run_gpu_ranks(tmp_path, path, ss, 1 << 18, world=4, env_extra=STREAMED)
    ref_splits, ref_counts = oracle_splits(of, ss)
    for r in res:
        assert r["counts"] == ref_counts and [tuple(s) for s in r["splits"]] == ref_splits
        assert r["ok"] and r["chain_ok"] and r["chain_count"] == 50000


@pytest.mark.gpu
def test_gpu_long_reads_streamed_edges_inside_records(tmp_path):
    path, data = _synth_file(tmp_path, 0x5B4D004C, 1, 500, "long.bam")
    of = OracleFile(data)
    ss = _edges_inside_long_records(of, 2)
    assert ss is not None
    res = _run_gpu_ranks(tmp_path, path, ss, 4096, world=2, env_extra=STREAMED)
    ref_splits, ref_counts = oracle_splits(of, ss)
    for r in res:
        assert r["counts"] == ref_counts and [tuple(s) for s in r["splits"]] == ref_splits
        assert r["ok"] and r["chain_ok"] and r["chain_count"] == 500


@pytest.mark.gpu
def test_gpu_stitch_rewalk_streamed(tmp_path):
    """The stitch fix-up on streamed ranks: rank 1 re-walks window by window (each window's
    eager bitmap, then the chain) from rank 0's exit."""
    path, data = _synth_file(tmp_path, 0x5B4D0030, 0, 20000, "wgs_fp.bam")
    res = _run_gpu_ranks(tmp_path, path, 0, 1 << 20, world=3,
                         env_extra=dict(STREAMED, SBH_TEST_FP_RANK="1"))
    for r in res:
        assert not r["ok"] and r["chain_ok"] and r["chain_count"] == 20000
        assert r["rewalk"]["1"]["count"] == r["rank_counts"][1] + 1


@pytest.mark.gpu
@pytest.mark.parametrize("tasks", [1, 2, 3, 5])
def test_gpu_tasks_mirror_of_scala_facade(tasks):
    """jni/Native.scala GpuLoadBam's call sequence (sharded.load_splits_and_reads_tasks): the
    Hadoop splits dealt to Spark tasks, each task's shard closed when it ends, the driver's
    stitch: ComputeSplitsTest's 230k splits and LoadBAMTest's counts of 1.bam for every task
    count."""
    splits, counts, st = sharded.load_splits_and_reads_tasks(golden_bam("1.bam"), 230 * 1024, tasks)
    assert [(str(a), str(b)) for a, b in splits] == [("0:45846", "239479:312"), ("239479:312", "484396:25"),
                                                    ("484396:25", "597482:0")]
    assert sum(counts) == 4917 and st["ok"] and st["chain_ok"]


@pytest.mark.gpu
def test_gpu_tasks_rewalk_reads_bytes_again(tmp_path):
    """A task whose first record is a false positive (injected) is re-walked by the driver from
    the upstream task's exit, re-reading that task's bytes (the task's shard is gone)."""
    path, data = _synth_file(tmp_path, 0x5B4D0030, 0, 20000, "wgs_tasks.bam")
    of = OracleFile(data)
    ss = data.size // 7
    ref_splits, ref_counts = oracle_splits(of, ss)
    orig = sharded.RankRun._part

    def fp_part(self, split_index, splits, status, v, n, first, count, exit_vpos):
        if self.rank == 2:  # rank 2 reports its first record one byte later and one record fewer
            first, count = first + 1, count - 1
        return orig(self, split_index, splits, status, v, n, first, count, exit_vpos)

    sharded.RankRun._part = fp_part
    try:
        splits, counts, st = sharded.load_splits_and_reads_tasks(path, ss, 4)
    finally:
        sharded.RankRun._part = orig
    assert counts == ref_counts and [(a.to_htsjdk(), b.to_htsjdk()) for a, b in splits] == ref_splits
    assert not st["ok"] and st["chain_ok"] and st["chain_count"] == 20000 and 2 in st["rewalk"]


@pytest.mark.gpu
def test_gpu_streamed_rank_with_one_split(tmp_path, monkeypatch):
    """one split per rank (split_size = the whole file) streamed through 150 KB windows:
    the split runs through every window (its chain followed window by window), HBM stays bounded,
    and the answer equals the oracle."""
    path, data = _synth_file(tmp_path, 0x5B4D0030, 0, 20000, "wgs_one.bam")
    of = OracleFile(data)
    monkeypatch.setattr(sharded, "RESIDENT_MAX", 1)
    monkeypatch.setattr(sharded, "STREAM_WINDOW", 150_000)
    splits, counts, st = sharded.load_splits_and_reads(path, None, world=1, rank=0)
    ref_splits, ref_counts = oracle_splits(of, data.size)
    assert counts == ref_counts == [20000]
    assert [(a.to_htsjdk(), b.to_htsjdk()) for a, b in splits] == ref_splits
