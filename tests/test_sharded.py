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
from oracle_lib import OracleFile, load_splits_and_reads as oracle_splits

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
dist.init_process_group("gloo")
path, ss = sys.argv[1], (int(sys.argv[2]) or None)
with sb.Context(0) as ctx:  # both ranks share the one device of the box
    splits, counts, st = sharded.load_splits_and_reads(path, ss, ctx=ctx, halo=int(sys.argv[3]))
json.dump({"splits": [[a.to_htsjdk(), b.to_htsjdk()] for a, b in splits], "counts": counts,
           "ok": st["ok"], "rank_counts": st["rank_counts"], "mismatches": st["mismatches"]},
          open(os.path.join(sys.argv[4], "r%d.json" % dist.get_rank()), "w"))
dist.destroy_process_group()
"""


@pytest.mark.gpu
@pytest.mark.parametrize("name,split_size,halo", [("2.bam", 0, 1 << 20), ("2.bam", 102400, 4096),
                                                   ("1.bam", 300 * 1024, 1 << 20),
                                                   ("1.bam", 0, 4096)])
def test_gpu_two_ranks_on_one_device(tmp_path, name, split_size, halo):
    """Two processes (gloo exchange) share cuda:0, each running its shard's hot path; a
    4 KiB starting halo forces the NEED_HALO growth loop."""
    path = golden_bam(name)
    script = tmp_path / "w.py"
    script.write_text(GPU_WORKER)
    env = dict(os.environ, SBH_ROOT=ROOT, MASTER_ADDR="127.0.0.1")
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                    "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(script), path,
                    str(split_size), str(halo), str(tmp_path)], env=env, check=True, timeout=100)
    of = OracleFile.from_path(path)
    ref_splits, ref_counts = oracle_splits(of, split_size or -(-of.size // 2))
    res = [json.load(open(tmp_path / f"r{r}.json")) for r in range(2)]
    for r in res:
        assert r["counts"] == ref_counts
        assert [tuple(s) for s in r["splits"]] == ref_splits
        assert r["ok"], (r, [_oracle_part(of, k, 2, split_size or -(-of.size // 2)) for k in range(2)])
