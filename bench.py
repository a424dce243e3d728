#!/usr/bin/env python3
"""Benchmark: BGZF inflate + eager record-boundary check at every uncompressed offset
(+ record split/count and RCCL stitching) on MI355X.

Workload (BASELINE.json configs[1]): a synthetic BAM of 100 bp Illumina-like short
reads, BGZF level 6, ~1 GiB compressed PER GPU (weak scaling: N GPUs process an
N-GiB file, each rank one byte-range shard resident in HBM).  One step = the whole
per-shard hot path (sbh_run_shard: block index -> inflate -> eager check at every
owned position -> first record + record count) followed by the RCCL allgather of the
per-shard {first_vpos, count, exit} records that stitches the splits.

Run: python bench.py --gpus N --steps K --warmup W   (N>1 under torch.distributed.run)
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

METRIC = "decompressed GB/s + records/sec (inflate+boundary check) at 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


CONFIGS = {  # BASELINE.json configs; SURVEY 8d
    "B": dict(seed=0x5B4D0001, shape=0, level=6, records=12_400_000, fp_free=True,
              workload="configs[1]: synthetic ~1 GiB-compressed BAM per GPU, 100 bp short reads, BGZF level 6 "
                       "(htsjdk 65498 B payloads)"),
    "C": dict(seed=0x5B4D0030, shape=0, level=6, records=155_000_000, fp_free=True, stream=True,
              workload="configs[2] per-GPU shard: 12.5 GiB compressed (the 100 GB WGS file / 8 GPUs), 100 bp "
                       "short reads, level 6, streamed from pinned host memory through HBM in 1 GiB windows"),
    "D": dict(seed=0x5B4D004C, shape=1, level=6, records=71_000, fp_free=True,
              workload="configs[3]: ~1 GiB-compressed long-read BAM per GPU (10-50 kb records spanning BGZF "
                       "blocks and shard edges), level 6"),
    "E": dict(seed=0x5B4D00AD, shape=2, level=-1, records=7_600_000, fp_free=False,
              workload="configs[4]: ~1 GiB-compressed adversarial BAM (per-block levels 0/1/9, unmapped and "
                       "zero-length reads, false-positive bait), N=1"),
}


def launch_ranks(n):
    """torch.distributed.run --nproc-per-node n over this script with the same arguments, on
    127.0.0.1 and a free port, as a child process; returns its exit code."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    log(f"launching {n} ranks: {' '.join(cmd)}")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="B",
                    help="B (default, the metric's config): 1 GiB short reads per GPU; C: the 100 GB WGS "
                         "file's per-GPU shard at N=8 (12.5 GiB); D: long reads; E: adversarial (N=1 only)")
    ap.add_argument("--records-per-gpu", type=int, default=None,
                    help="~1.0 GiB compressed per GPU at level 6 (config B)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="CPU baseline threads (default: every host core this process may use)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-full", action="store_true", help="skip the full-checker side measurement")
    ap.add_argument("--stream", action="store_true",
                    help="stream the shard from pinned host memory through HBM (sbh_run_stream; default for C)")
    ap.add_argument("--window", type=int, default=1 << 30, help="stream window, compressed bytes")
    ap.add_argument("--e2e-window", type=int, default=256 << 20,
                    help="window of the H2D-inclusive side measurement of the resident configs")
    ap.add_argument("--no-e2e", action="store_true", help="skip the H2D-inclusive side measurement")
    ap.add_argument("--file-gib", type=float, default=None,
                    help="strong scaling over ONE file of this many GiB compressed (configs[2]: --config C "
                         "--file-gib 100): the N ranks split its Hadoop splits and stream their ranges")
    ap.add_argument("--split-mib", type=float, default=32.0, help="Hadoop split size of the --file-gib file")
    ap.add_argument("--no-crc", action="store_true", help="--file-gib: skip the in-run CRC32 check")
    ap.add_argument("--no-pin", action="store_true", help="--file-gib: pageable host memory for the rank's bytes")
    ap.add_argument("--no-facade", action="store_true",
                    help="skip the load-API facade side measurement (loadReadsAndPositions per 32 MiB split)")
    ap.add_argument("--facade-threads", type=int, default=8,
                    help="concurrent task threads of the facade measurement (a Spark executor's cores)")
    ap.add_argument("--facade-modes", default="hbm,pinned_host,hbm_records,calls_r05",
                    help="facade modes to run (comma list; see facade_bench)")
    ap.add_argument("--facade-only", action="store_true",
                    help="skip full-check / e2e / CPU baseline side lines (facade iteration)")
    ap.add_argument("--traffic", type=float, default=None,
                    help="HBM bytes per launch of the dominant kernel (default: the committed "
                         "rocprofv3 --pmc summary, profiles/*_pmc_traffic.json)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N` outside a launcher: start the N ranks as a CHILD process
        # group (torch.distributed.run), before anything here has touched the GPU, and hand back
        # its exit code; rank 0's JSON line reaches stdout through the inherited descriptors.
        sys.exit(launch_ranks(args.gpus))

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: WORLD_SIZE={world} but --gpus={args.gpus}; the line reports ranks_seen and exits non-zero")

    import torch
    import torch.distributed as dist

    # One rank per GPU over RCCL.  More ranks than devices (a rehearsal of the N>1 path on
    # a one-GPU box) share the devices round-robin and exchange over gloo instead.
    ndev = max(1, torch.cuda.device_count())
    backend = "nccl" if world <= ndev else "gloo"
    device = local_rank % ndev
    xdev = "cuda" if backend == "nccl" else "cpu"
    torch.cuda.set_device(device)
    # SBH_BENCH_COLLECTIVES=1: run the N>1 collectives (RCCL) even at WORLD_SIZE=1, so a
    # one-GPU box exercises the nccl code path end to end (torch.distributed.run --nproc-per-node 1)
    coll = world > 1 or os.environ.get("SBH_BENCH_COLLECTIVES") == "1"
    if coll:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            log(f"note: {world} ranks on {ndev} device(s): gloo exchange (rehearsal, not a scaling run)")
            dist.init_process_group("gloo")

    import synth
    from __graft_entry__ import load_package

    sb = load_package()
    import spark_bam_amd.sharded as sharded

    if args.file_gib is not None:
        return main_strong(args, rank, world, local_rank, device, backend, xdev, coll, dist, torch, synth, sb,
                           sharded)

    # ---- input generation (not timed) ----
    t0 = time.time()
    cfg = CONFIGS[args.config]
    if args.records_per_gpu is None:
        args.records_per_gpu = cfg["records"]
    p = synth.params(cfg["seed"], shape=cfg["shape"], level=cfg["level"],
                     threads=min(16, os.cpu_count() or 1))
    streaming = args.stream or cfg.get("stream", False)
    pins = []

    def pinned(n):  # page-locked host memory for the streamed shard (overlapped H2D copies)
        pins.append(sb.PinnedBuffer(n))
        return pins[-1].array

    if cfg["level"] < 0:  # mixed levels: no uniform payload grid, so one whole file (N=1)
        if world != 1:
            raise SystemExit(f"config {args.config} runs at N=1 only")
        seg = synth.WholeFile(p, args.records_per_gpu)
    else:
        seg = synth.Segment(p, args.records_per_gpu, world, rank, halo_blocks=64 if streaming else 16, log=log,
                            alloc=pinned if streaming else None)
    own = torch.tensor([seg.own_csize], dtype=torch.int64, device=xdev)
    if coll:
        gathered = [torch.zeros_like(own) for _ in range(world)]
        dist.all_gather(gathered, own)
        own_sizes = [int(g.item()) for g in gathered]
    else:
        own_sizes = [seg.own_csize]
    seg.set_offsets(own_sizes)
    log(f"[rank {rank}] generated shard: {seg.comp.size / 2**30:.3f} GiB compressed "
        f"(owned {seg.own_csize / 2**30:.3f} GiB, file {seg.file_size / 2**30:.3f} GiB) "
        f"in {time.time() - t0:.1f}s")

    ctx = sb.Context(device)
    header = synth.header_bytes()
    names, contig_len, _ = sb.parse_bam_header(header)
    shard = None
    if not streaming:
        shard = ctx.shard(seg.comp, file_offset=seg.file_offset, file_size=seg.file_size)
        shard.set_contigs(contig_len)

    result_t = torch.zeros(5, dtype=torch.int64, device=xdev)
    stream_last = {}

    # the streamed shard's Hadoop splits (32 MiB, SplitRDD's partitions): per-split first record
    # and count come back from every window (sbh_run_stream2)
    # (resident shards too: the step returns every owned split's first record and count, the
    # north star's "split virtual offsets", from sbh_split_starts on the run's bitmap)
    sp = sb.file_splits(seg.own_end - seg.file_offset, 32 << 20)
    stream_splits = [(seg.file_offset + x, seg.file_offset + y) for x, y in sp]
    split_last = {}

    def run_once():
        if streaming:  # windows through HBM; copies of window w+1 overlap window w's kernels
            r, _ = ctx.run_stream(seg.comp, contig_len, file_offset=seg.file_offset, file_size=seg.file_size,
                                  own_end=seg.own_end, index_start=seg.file_offset, window=args.window,
                                  halo=4 << 20, splits=stream_splits, verify_crc=True)
            stream_last.update(r)
            first = r["first_vpos"] or 0
            ex = r["exit_vpos"]
            return dict(r, first_vpos=first), r["stage_ms"], ex
        r = shard.run(seg.file_offset, seg.own_end)
        stages = shard.stage_times()
        st, v, n, nh = shard.split_starts(stream_splits)
        split_last.update(split_status=st, split_vpos=v, split_count=n, splits_host=nh)
        return r, stages, shard.exit_vpos(r)  # exit: None when the chain hit the stream end

    def step():
        r, stages, ex = run_once()
        if r["status"] != 0:
            raise RuntimeError(f"run status {r['status']}")
        ex = -1 if ex is None else ex
        r["stages"] = stages
        mine = [r["first_vpos"], r["count"], r["n_true"], r["flat_bytes"], ex]
        if coll:  # RCCL allgather of the per-shard split records (stitching)
            result_t.copy_(torch.tensor(mine, dtype=torch.int64))
            out = [torch.zeros_like(result_t) for _ in range(world)]
            dist.all_gather(out, result_t)
            return r, [o.cpu().tolist() for o in out]
        return r, [mine]

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if coll:
        dist.barrier()
    torch.cuda.synchronize()
    stage_acc = np.zeros(6)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        r, allr = step()
        stage_acc += np.asarray(r["stages"])
    torch.cuda.synchronize()
    if coll:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    if coll:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=xdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    # ---- correctness of the stitched result (every rank) ----
    total_records = sum(x[1] for x in allr)
    total_true = sum(x[2] for x in allr)
    total_flat = sum(x[3] for x in allr)
    expect = world * args.records_per_gpu
    parts = [sharded.RankPart(i, i, [x[0] if x[1] else None], [x[1]], x[0] if x[1] else None, x[1],
                              None if x[4] < 0 else x[4]) for i, x in enumerate(allr)]
    _, _, stitch = sharded.stitch(parts, seg.file_size)
    # eager-true positions equal the records except where the input carries false-positive
    # bait (config E), whose exact bits are pinned by the parity tests, not here
    # every inflated block of the last step against its BGZF footer CRC32 (full-size
    # bit-exactness of the inflate), outside the timed region
    # (stream mode: every window's owned blocks were CRC-checked in the run, sbh_run_stream2)
    crc_bad = shard.verify_crc()[0] if shard is not None else stream_last.get("crc_bad_blocks", 0)
    sl = stream_last if streaming else split_last
    split_ok = (int(np.count_nonzero(sl["split_status"])) == 0 and int(sl["split_count"].sum()) == r["count"])
    ok = (total_records == expect and (total_true == expect or not cfg["fp_free"]) and stitch["ok"] and crc_bad == 0
          and split_ok)
    firsts = [x[0] for x in allr if x[1] > 0]

    stage_ms = stage_acc / args.steps
    comp_bytes = r["comp_bytes"]
    flat_bytes = r["flat_bytes"]
    # Roofline of the dominant kernel.  run() is one pipeline over block batches on three
    # streams (k_huff | k_lz | k_eager); each kernel's time is the sum of its launches,
    # timed with HIP events on its own stream.  Algorithmic bytes per unit follow SURVEY
    # 8(d): k_huff reads C, k_lz writes U, k_eager reads U and writes U/8 (the 4 B/token
    # intermediate is this design's overhead, not algorithmic).
    kern = {
        "k_huff": (comp_bytes, stage_ms[4], "C read"),
        "k_lz": (flat_bytes, stage_ms[5], "U written"),
        "k_eager": (flat_bytes * 1.125, stage_ms[2], "U read + U/8 bitmap written"),
    }
    dom = max(kern, key=lambda k: kern[k][1])
    alg_bytes, dom_ms, dom_units = kern[dom]
    achieved = alg_bytes / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0

    traffic, traffic_src, traffic_fresh = args.traffic, "--traffic" if args.traffic is not None else None, None
    if traffic is None:
        tj, tsrc = latest_pmc("traffic.json")
        kt = tj["kernels"].get(dom) if tj else None
        if kt:
            traffic, traffic_src = stage_traffic(tj, dom), tsrc
            traffic_fresh = tj.get("src_hash") == kernel_src_hash()

    def gbps(nbytes, ms):
        return round(nbytes / (ms * 1e-3) / 1e9, 2) if ms > 0 else None

    # Full-checker mode, reported separately: full.Checker at every owned
    # position with the FullCheck Counts aggregation (no per-position words), on the
    # inflated shard the last step left; wall time of the synchronous call, best of 2.
    if args.facade_only:
        args.no_full = args.no_e2e = args.no_cpu_baseline = True
    facade = None
    if (not args.no_facade and rank == 0 and world == 1 and shard is not None and not seg.file_offset
            and seg.comp.size == seg.file_size):
        facade = facade_bench(sb, ctx, seg.comp, seg.file_size, contig_len, args.facade_threads, torch, r,
                              split_last, stream_splits, value_ref=total_flat * args.steps / elapsed / 1e9,
                              modes=args.facade_modes.split(","))

    full = None
    if not args.no_full and shard is not None:
        f0 = max(0, shard.flat_bound(seg.file_offset)) if seg.file_offset else 0
        f1 = shard.flat_bound(seg.own_end)
        best = None
        for _ in range(2):
            torch.cuda.synchronize()
            t0f = time.perf_counter()
            fr = shard.check_full(f0, f1, want_words=False, close_cap=1 << 16)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0f
            best = dt if best is None else min(best, dt)
        full = {"positions": int(f1 - f0), "ms": round(best * 1e3, 3),
                "GBps_decompressed": round((f1 - f0) / best / 1e9, 2),
                "n_success": int(fr["n_success"]), "close_calls": int(fr["n_close"]),
                "note": "sbh_check_full over the owned flat range (Counts + rbe histograms + close calls), "
                        "inflated shard already resident; not part of `value`"}

    # End-to-end rate with the compressed shard starting in (pinned) host memory: the same
    # per-shard path streamed through HBM in windows, H2D copies overlapped with the kernels
    # (sbh_run_stream).  Reported beside `value` (which has the inputs resident in HBM).
    e2e = None
    if streaming:
        e2e = {"GBps_decompressed": round(total_flat * args.steps / elapsed / 1e9, 2),
               "windows": stream_last.get("n_windows"), "window_bytes": args.window,
               "h2d_ms_per_step": round(stream_last.get("ms_h2d", 0), 3),
               "h2d_GBps": round(stream_last["comp_bytes"] / (stream_last["ms_h2d"] * 1e-3) / 1e9, 2)
               if stream_last.get("ms_h2d") else None,
               "device_ms_per_step": round(float(stage_acc[1] + stage_acc[0] + stage_acc[3]) / args.steps, 3),
               "host_pinned": bool(stream_last.get("host_pinned")),
               "crc_ms_per_step": round(stream_last.get("ms_crc", 0), 3),
               "splits": len(stream_splits), "splits_host_path": int(stream_last.get("splits_host", 0)),
               "split_counts_sum": int(stream_last["split_count"].sum()),
               "note": "value IS the streamed rate here: shard in pinned host memory, windows through HBM cut at "
                       "split starts; per-split first record + count and every block's CRC32 in the timed run"}
    elif not args.no_e2e and seg.file_offset is not None:
        buf = sb.PinnedBuffer(seg.comp.size)
        buf.array[:] = seg.comp
        best, sr = None, None
        for _ in range(2):
            t0e = time.perf_counter()
            sr, _ = ctx.run_stream(buf.array, contig_len, file_offset=seg.file_offset, file_size=seg.file_size,
                                   own_end=seg.own_end, index_start=seg.file_offset, window=args.e2e_window,
                                   halo=4 << 20)
            dt = time.perf_counter() - t0e
            best = dt if best is None else min(best, dt)
        buf.close()
        e2e = {"GBps_decompressed": round(sr["flat_bytes"] / best / 1e9, 2),
               "compressed_GBps": round(sr["comp_bytes"] / best / 1e9, 2),
               "ms": round(best * 1e3, 3), "windows": sr["n_windows"], "window_bytes": args.e2e_window,
               "h2d_ms": round(sr["ms_h2d"], 3),
               "h2d_GBps": round(sr["comp_bytes"] / (sr["ms_h2d"] * 1e-3) / 1e9, 2) if sr["ms_h2d"] else None,
               "records_match": sr["count"] == r["count"] and sr["n_true"] == r["n_true"],
               "note": "rank-local shard from pinned host memory, streamed through HBM in windows (sbh_run_stream); "
                       "not `value`"}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(seg.comp, seg.file_offset or 0, contig_len, args.cpu_seconds, args.cpu_threads)

    ranks_seen = dist.get_world_size() if coll else 1
    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        value = total_flat * args.steps / elapsed / 1e9
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GB/s decompressed (whole job)",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": f"synthetic (tools/synth_bam.c, seed {cfg['seed']:#x}), generated per rank",
            "config": {
                "workload": cfg["workload"] + ("" if args.records_per_gpu == cfg["records"] else
                                               f" [run at --records-per-gpu {args.records_per_gpu}: "
                                               f"{sum(own_sizes) / world / 2**30:.2f} GiB compressed per GPU]"),
                "records_per_gpu": args.records_per_gpu,
                "compressed_bytes": int(sum(own_sizes)),
                "decompressed_bytes": int(total_flat),
                "parallelism": f"dp{world} byte-range shards + "
                               f"{'RCCL' if backend == 'nccl' else 'gloo (rehearsal)'} allgather stitch",
            },
            "records_per_s": round(total_records * args.steps / elapsed, 1),
            "compressed_GBps": round(sum(own_sizes) * args.steps / elapsed / 1e9, 3),
            "correct": bool(ok),
            "ranks_seen": ranks_seen,
            "backend": backend if coll else "none (one rank)",
            "stitch_ok": bool(stitch["ok"]),
            "splits_rank0": {"n": len(stream_splits), "split_bytes": 32 << 20,
                             "host_path": int(sl.get("splits_host", 0)),
                             "counts_sum": int(sl["split_count"].sum()),
                             "note": "every owned Hadoop split's first-record vpos and count "
                                     "(sbh_split_starts) inside the timed step"},
            "crc_bad_blocks_rank0": int(crc_bad),
            "records": int(total_records),
            "eager_true": int(total_true),
            "stages_ms_rank0": {"index": round(stage_ms[0], 3),
                                "inflate+eager pipeline": round(stage_ms[1], 3),
                                "k_huff (sum)": round(stage_ms[4], 3), "k_lz (sum)": round(stage_ms[5], 3),
                                "k_eager (sum)": round(stage_ms[2], 3),
                                "split_count": round(stage_ms[3], 3)},
            "roofline": {
                "kernel": (f"{dom} (summed launches of the pipelined run, HIP events on its stream"
                           + ("; with its k_hdr header pre-pass)" if dom == "k_huff" else ")")),
                "bound": "hbm",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 5),
                "traffic": traffic,
                "traffic_unit": "HBM bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)",
                "traffic_source": traffic_src,
                "traffic_matches_kernels": traffic_fresh,  # collected from these kernel sources (hash)
                # tools/pmc_collect.sh runs the default workload (config B): for another config the
                # per-launch bytes are config B's
                "traffic_workload": "B" if traffic_src and traffic_src != "--traffic" else None,
                "traffic_same_workload": (args.config == "B") if traffic_src and traffic_src != "--traffic"
                else None,
                "alg_bytes_per_step": int(alg_bytes),
                "alg_units": dom_units,
                "limiter": limiter_text(dom, dom_ms, traffic),
                "path": {  # B_alg = C + U (inflate write) + U (checker read) + U/8 (bitmap) per step
                    "alg_bytes_per_step": int(sum(own_sizes) / world + 2.125 * flat_bytes),
                    "achieved": round((sum(own_sizes) / world + 2.125 * flat_bytes) * args.steps / elapsed / 1e9, 2),
                    "frac": round((sum(own_sizes) / world + 2.125 * flat_bytes) * args.steps / elapsed / 1e9
                                  / HBM_PEAK_GBPS, 5),
                },
                "per_kernel_GBps": {k: gbps(v[0], v[1]) for k, v in kern.items()},
            },
            "full_check": full,
            "facade": facade,
            "e2e_h2d": e2e,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if shard is not None:
        shard.close()
    ctx.close()
    for b in pins:
        b.close()
    if coll:
        dist.destroy_process_group()
    if not ok:
        log(f"STITCH CHECK FAILED: records {total_records} true {total_true} expected {expect}; "
            f"stitch {stitch}")
        sys.exit(3)
    if ranks_seen != args.gpus:
        log(f"ranks_seen {ranks_seen} != --gpus {args.gpus}")
        sys.exit(4)


def main_strong(args, rank, world, local_rank, device, backend, xdev, coll, dist, torch, synth, sb, sharded):
    """configs[2] as BASELINE.json states it: ONE file of --file-gib GiB compressed, its Hadoop
    splits dealt to the N ranks as contiguous runs (sharded.rank_splits), every rank streaming
    its byte range from pinned host memory through HBM (sbh_run_stream2: windows cut at split
    starts, per-split first record + count, in-run CRC32 of every owned block), one RCCL
    allgather of the per-rank chain records per step.  Strong scaling: total work is fixed."""
    cfg = CONFIGS[args.config]
    if cfg["level"] < 0:
        raise SystemExit("--file-gib needs a single-level config (B, C or D)")
    t0 = time.time()
    p = synth.params(cfg["seed"], shape=cfg["shape"], level=cfg["level"], threads=min(16, os.cpu_count() or 1))
    seg_records = args.records_per_gpu or CONFIGS["B"]["records"]  # ~1 GiB compressed canonical segment
    F = synth.Replicated(p, seg_records, int(args.file_gib * 2**30))
    split = int(args.split_mib * 2**20)
    a, mine = sharded.rank_splits(F.size, split, world, rank)
    nsplits = len(sharded.rank_splits(F.size, split, 1, 0)[1])
    lo, hi = mine[0][0], mine[-1][1]
    end = min(F.size, hi + (64 << 20))
    pins = []
    if args.no_pin:
        comp = np.empty(end - lo, dtype=np.uint8)
    else:
        pins.append(sb.PinnedBuffer(end - lo))
        comp = pins[-1].array
    F.read_into(lo, end, comp)
    log(f"[rank {rank}] file {F.size / 2**30:.2f} GiB ({F.copies} x {F.seg_comp.size / 2**30:.3f} GiB segment, "
        f"{F.records} records, {nsplits} splits); rank range [{lo}, {hi}) = {(hi - lo) / 2**30:.2f} GiB, "
        f"{len(mine)} splits; ready in {time.time() - t0:.1f}s")
    ctx = sb.Context(device)
    _, contig_len, _ = sb.parse_bam_header(synth.header_bytes())
    res_t = torch.zeros(5, dtype=torch.int64, device=xdev)
    last = {}

    def step():
        r, _ = ctx.run_stream(comp, contig_len, file_offset=lo, file_size=F.size, own_end=hi, window=args.window,
                              halo=4 << 20, splits=mine, verify_crc=not args.no_crc)
        last.clear()
        last.update(r)
        mine_rec = [r["first_vpos"] or 0, r["count"], r["n_true"], r["flat_bytes"],
                    -1 if r["exit_vpos"] is None else r["exit_vpos"]]
        if coll:
            res_t.copy_(torch.tensor(mine_rec, dtype=torch.int64))
            out = [torch.zeros_like(res_t) for _ in range(world)]
            dist.all_gather(out, res_t)
            return [o.cpu().tolist() for o in out]
        return [mine_rec]

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if coll:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        allr = step()
    torch.cuda.synchronize()
    if coll:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    if coll:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=xdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    # per-split results -> the reference's splits (sliding2 over non-empty firsts) and counts
    r = last
    part = sharded.RankPart(rank, a, [int(v) if c else None for v, c in zip(r["split_first_vpos"], r["split_count"])],
                            [int(c) for c in r["split_count"]], r["first_vpos"] if r["count"] else None, r["count"],
                            r["exit_vpos"])
    parts = sharded.exchange(part) if coll else [part]
    splits, counts, st = sharded.stitch(parts, F.size)
    crc_bad = [r["crc_bad_blocks"]]
    split_bad = int(np.count_nonzero(r["split_status"]))
    if coll:
        g = [None] * world
        dist.all_gather_object(g, (int(r["crc_bad_blocks"]), split_bad, int(r["splits_host"])))
        crc_bad, split_bad, host = [x[0] for x in g], sum(x[1] for x in g), sum(x[2] for x in g)
    else:
        host = int(r["splits_host"])
    total_records = sum(x[1] for x in allr)
    total_flat = sum(x[3] for x in allr)
    ok = (total_records == F.records and sum(counts) == F.records and st["ok"] and sum(crc_bad) == 0
          and split_bad == 0 and len(counts) == nsplits)
    ranks_seen = dist.get_world_size() if coll else 1
    if rank == 0:
        value = total_flat * args.steps / elapsed / 1e9
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GB/s decompressed (whole job)",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u8",
            "data": (f"synthetic (tools/synth_bam.c seed {cfg['seed']:#x}): one {seg_records}-record segment "
                     f"replicated x{F.copies} into one file (synth.Replicated)"),
            "config": {
                "workload": (f"configs[2]: ONE {F.size / 2**30:.1f} GiB-compressed WGS-shaped BAM ({F.records} records,"
                             f" {F.flat_size / 1e9:.1f} GB flat), its {nsplits} Hadoop splits of {args.split_mib:g} MiB "
                             f"dealt to {world} rank(s), each streamed from {'pinned' if not args.no_pin else 'pageable'}"
                             f" host memory through HBM in {args.window / 2**30:g} GiB windows"),
                "file_bytes": F.size, "decompressed_bytes": int(total_flat), "splits": nsplits,
                "parallelism": f"dp{world} byte-range shards (Hadoop split runs) + "
                               f"{'RCCL' if backend == 'nccl' else 'gloo'} allgather stitch",
            },
            "records_per_s": round(total_records * args.steps / elapsed, 1),
            "compressed_GBps": round(F.size * args.steps / elapsed / 1e9, 3),
            "correct": bool(ok),
            "ranks_seen": ranks_seen,
            "backend": backend if coll else "none (one rank)",
            "stitch_ok": bool(st["ok"]),
            "records": int(total_records),
            "splits_nonempty": len(splits),
            "split_counts_sum": int(sum(counts)),
            "splits_host_path": int(host),
            "crc_bad_blocks": int(sum(crc_bad)),
            "crc_checked": not args.no_crc,
            "rank0": {"windows": r["n_windows"], "h2d_ms": round(r["ms_h2d"], 2), "wall_ms": round(r["ms_wall"], 2),
                      "crc_ms": round(r["ms_crc"], 2), "splits_ms": round(r["ms_splits"], 2),
                      "stages_ms": [round(x, 2) for x in r["stage_ms"]], "host_pinned": bool(r["host_pinned"])},
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    for b in pins:
        b.close()
    if coll:
        dist.destroy_process_group()
    if not ok:
        log(f"CHECK FAILED: records {total_records}/{F.records}, counts {sum(counts)}, stitch {st['ok']}, "
            f"crc {crc_bad}, split errors {split_bad}, splits {len(counts)}/{nsplits}")
        sys.exit(3)
    if ranks_seen != args.gpus:
        log(f"ranks_seen {ranks_seen} != --gpus {args.gpus}")
        sys.exit(4)


def facade_bench(sb, ctx, comp, file_size, contig_len, threads, torch, run, split_last, splits, value_ref,
                 modes=("hbm", "pinned_host", "hbm_records", "calls_r05")):
    """The load-API drop-in path (GpuCanLoadBam.loadReadsAndPositions, CanLoadBam.scala:316-356;
    its twin spark_bam_amd.canloadbam): one task per 32 MiB Hadoop FileSplit, `threads` task threads
    sharing the context (a Spark executor's cores), each with its own reused shard + pinned buffer
    (SplitWorker) and ONE library call per split (sbh_split_records).  Modes:
      hbm           the file's bytes already in HBM (device-to-device per split): the per-split
                    overhead against `value`'s one resident shard
      pinned_host   the file's bytes in page-locked host memory (a host read + H2D per split)
      hbm_records   as hbm, plus what jni/Native.scala's GpuRecordIterator copies out of HBM to build
                    htsjdk SAMRecords: the record starts and the records' bytes (into the task
                    thread's page-locked buffer)
      calls_r05     round 5's sequence (a shard per split, seven calls), one thread, from host memory
    Wall time over every split; record starts -> vpos on the host; the per-split counts and first
    records must equal the resident run's sbh_split_starts (checked against the oracle in tests/)."""
    import threading

    clb = __import__(sb.__name__ + ".canloadbam", fromlist=["x"])
    read = __import__(sb.__name__ + ".sharded", fromlist=["x"]).bytes_reader(comp)
    want_n = [int(x) for x in split_last["split_count"]]
    want_v = [int(v) for v in split_last["split_vpos"]]
    flat_total = int(run["flat_bytes"])
    dev = torch.from_numpy(comp).to("cuda")
    torch.cuda.synchronize()
    pin = sb.PinnedBuffer(comp.size)
    pin.array[:] = comp
    pread = __import__(sb.__name__ + ".sharded", fromlist=["x"]).bytes_reader(pin.array)

    # one SplitWorker per task thread, kept across passes like jni/Native.scala's ThreadLocal
    # GpuSplitWorker (its shard's device buffers and pinned buffers reach their size in the warm
    # pass; a hipMalloc / hipFree in a timed pass would synchronize the whole device)
    pools = {}

    def workers(mode, n):
        key = (mode.startswith("hbm"), n)
        if key not in pools:
            pools[key] = [clb.SplitWorker(ctx, file_size, contig_len,
                                          device_file=dev.data_ptr() if mode.startswith("hbm") else None)
                          for _ in range(n)]
        return pools[key]

    def one_pass(mode, nthreads):
        got = [None] * len(splits)
        tm = [None] * len(splits)
        it = iter(range(len(splits)))
        lock = threading.Lock()
        errs = []

        def task(w):
            try:
                while True:
                    with lock:
                        i = next(it, None)
                    if i is None:
                        return
                    a, e = splits[i]
                    t0 = time.perf_counter()
                    cols = w.split(pread if mode == "pinned_host" else read, "bench.bam", a, e, decode=False)
                    if mode == "hbm_records" and cols["flat"].size:
                        # GpuRecordIterator: [first record, end of the last record) in one copy
                        w.fetch_record_bytes(cols["flat"])
                    got[i] = (int(cols["vpos"].size), int(cols["vpos"][0]) if cols["vpos"].size else None)
                    tm[i] = time.perf_counter() - t0
            except BaseException as ex:  # noqa: B902 (reported below)
                errs.append(ex)

        t0 = time.perf_counter()
        if mode == "calls_r05":
            for i, (a, e) in enumerate(splits):
                ts = time.perf_counter()
                cols = clb.split_partition_calls(ctx, read, file_size, "bench.bam", a, e, contig_len)
                got[i] = (int(cols["vpos"].size), int(cols["vpos"][0]) if cols["vpos"].size else None)
                tm[i] = time.perf_counter() - ts
        else:
            ts = [threading.Thread(target=task, args=(w,)) for w in workers(mode, nthreads)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
        wall = time.perf_counter() - t0
        if errs:
            raise errs[0]
        return wall, got, tm

    out = {"splits": len(splits), "split_bytes": 32 << 20, "threads": threads, "value_ref_GBps": round(value_ref, 2)}
    for mode in modes:
        nth = 1 if mode == "calls_r05" else threads
        reps = 1 if mode == "calls_r05" else 3
        best = None
        if mode != "calls_r05":
            one_pass(mode, nth)  # warm: each thread's shard and pinned buffer reach their size
        for _ in range(reps):
            wall, got, tm = one_pass(mode, nth)
            if best is None or wall < best[0]:
                best = (wall, got, tm)
        wall, got, tm = best
        counts = [g[0] for g in got]
        firsts = [g[1] for g in got]
        ok = (counts == want_n and sum(counts) == int(run["count"]) and
              all(f == v for f, v, n in zip(firsts, want_v, want_n) if n))
        out[mode] = {"GBps_decompressed": round(flat_total / wall / 1e9, 2),
                     "compressed_GBps": round(comp.size / wall / 1e9, 2),
                     "records_per_s": round(sum(counts) / wall, 1), "ms": round(wall * 1e3, 2),
                     "per_split_ms": {"mean": round(1e3 * float(np.mean(tm)), 3),
                                      "max": round(1e3 * float(np.max(tm)), 3)},
                     "threads": nth, "records": int(sum(counts)), "records_match": bool(ok),
                     "frac_of_value": round(flat_total / wall / 1e9 / value_ref, 3) if value_ref else None}
        log(f"facade {mode}: {out[mode]}")
    # per-split device stages of one split (HIP events of its sbh_run_shard), one thread
    w = workers("hbm", 1)[0]
    a, e = splits[len(splits) // 2]
    w.split(read, "bench.bam", a, e, decode=False)
    t0 = time.perf_counter()
    w.split(read, "bench.bam", a, e, decode=False)
    out["one_split_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
    # the same split's host-side phases, one thread: shard refill (device-to-device), the one
    # library call, the starts + vpos copy-out
    t0 = time.perf_counter()
    sh = w.load(read, a, min(file_size, e + (1 << 20)))
    t1 = time.perf_counter()
    info, cols = sh.split_records(a, e, decode=False, flat_out=w._flat_buf)
    t2 = time.perf_counter()
    out["one_split_phases_ms"] = {"shard_load": round((t1 - t0) * 1e3, 3),
                                  "split_records+fetch": round((t2 - t1) * 1e3, 3)}
    out["one_split_stages_ms"] = dict(zip(["index", "inflate+eager", "k_eager", "split/count", "k_huff", "k_lz"],
                                          [round(x, 3) for x in w.sh.stage_times()]))
    for ws in pools.values():
        for w in ws:
            w.close()
    pin.close()
    del dev
    out["note"] = ("GpuCanLoadBam.loadReadsAndPositions' per-split path (sbh_split_records per FileSplit, per-thread "
                   "reused shard + pinned buffer, record starts -> vpos); not `value`")
    return out


def kernel_src_hash():
    """Content hash of the kernel sources (spark-bam_amd/csrc/*.hip, *.h): counter summaries
    record it when collected (tools/pmc_collect.sh), so a bench line can tell whether its
    `traffic` / `limiter` still describe the kernels it ran."""
    import glob
    import hashlib
    h = hashlib.sha256()
    for f in sorted(glob.glob(os.path.join(ROOT, "spark-bam_amd", "csrc", "*.hip")) +
                    glob.glob(os.path.join(ROOT, "spark-bam_amd", "csrc", "*.h"))):
        h.update(os.path.basename(f).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def latest_pmc(name):
    """The committed counter summary `profiles/r*_pmc/<name>` (tools/pmc_collect.sh) collected
    from the kernel sources this run uses (its `src_hash`), else the last by name."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc", name)))
    if not files:
        return None, None
    cur = kernel_src_hash()
    fresh = []
    for f in files:
        try:
            with open(os.path.join(os.path.dirname(f), "src_hash")) as fh:
                if fh.read().strip() == cur:
                    fresh.append(f)
        except OSError:
            pass
    files = fresh or files
    with open(files[-1]) as fh:
        return json.load(fh), os.path.relpath(files[-1], ROOT)


# The launches each timed stage's HIP events bracket: launch_huff is the k_hdr header pre-pass,
# k_huff, the k_huff_tail finish of deferred final deflate blocks and the serial fallback.
STAGE_KERNELS = {"k_huff": ("k_hdr", "k_huff", "k_hdr_tail", "k_huff_tail", "k_huff_serial")}


def stage_traffic(tj, dom):
    """HBM bytes per launch of the stage timed as `dom`, from a traffic.json (tools/pmc_traffic.py):
    the sum over the kernels that stage launches that the counter passes saw."""
    ks = tj["kernels"]
    return sum(ks[k]["hbm_bytes"] for k in STAGE_KERNELS.get(dom, (dom,)) if ks.get(k))


def limiter_text(kernel, ms=None, traffic=None):
    """What bounds `kernel`, worded from its own counters (tools/pmc_derived.py over the
    rocprofv3 passes of tools/pmc_collect.sh) and its measured HBM traffic."""
    d, src = latest_pmc("derived.json")
    if not d:
        return "no counter data committed"
    k = d["kernels"].get(kernel)
    if not k:
        return f"no counter data for {kernel} in {src}"
    parts = []
    if traffic and ms:
        bw = traffic / (ms * 1e-3) / 1e9
        parts.append(f"{'HBM-bound' if bw > 0.6 * HBM_PEAK_GBPS else 'not HBM-bound'}: its measured traffic "
                     f"moves at {bw:.0f} GB/s ({100 * bw / HBM_PEAK_GBPS:.0f}% of peak) while it runs")
    parked, issuing = k.get("parked_waitcnt_barrier_frac") or 0, k.get("issuing_frac") or 0
    if parked >= 0.4:
        parts.append(f"latency-bound: waves parked on s_waitcnt/barrier {100 * parked:.0f}% of wave cycles, "
                     f"issuing {100 * issuing:.0f}%")
    else:
        parts.append(f"issue-bound: waves issuing {100 * issuing:.0f}% of wave cycles, parked {100 * parked:.0f}%")
    bc = k.get("lds_bank_conflict_frac")
    if bc is not None:
        parts.append(f"LDS bank conflicts {100 * bc:.0f}% of LDS-array cycles")
    parts.append(f"VALU active {100 * k['valu_active_frac']:.0f}%")
    fresh = d.get("src_hash") == kernel_src_hash()
    return "; ".join(parts) + f" -- {src}" + ("" if fresh else " (collected before the last kernel change)")


def host_cores():
    """(cores this process may run on, what limits it): the scheduler affinity mask capped by
    the cgroup CPU quota (a GPU box's share of the host), so no thread waits for a core."""
    n, why = len(os.sched_getaffinity(0)), "sched_getaffinity"
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max" and int(quota) // int(period) < n:
            n, why = max(1, int(quota) // int(period)), f"cgroup cpu.max {quota}/{period}"
    except (OSError, ValueError):
        pass
    return n, why


def host_block_table(comp, limit=None):
    """(start, csize, hsize, usize) of the consecutive BGZF blocks of `comp` (host-side header
    walk for the CPU baseline's sample; empty blocks skipped)."""
    out, pos, n = [], 0, comp.size
    while pos + 18 <= n and (limit is None or len(out) < limit):
        xlen = int(comp[pos + 10]) | int(comp[pos + 11]) << 8
        cs = (int(comp[pos + 16]) | int(comp[pos + 17]) << 8) + 1
        if pos + cs > n:
            break
        us = int.from_bytes(comp[pos + cs - 4:pos + cs].tobytes(), "little")
        if us:
            out.append((pos, cs, 18 + xlen - 6, us))
        pos += cs
    return out


def cpu_baseline(comp, base, contig_len, budget_s, threads):
    """The oracle (C restatement of the reference path: zlib inflate + eager check at
    every offset) on the host cores, over a bounded sample of the same shard's
    blocks.  Reported beside the GPU number; it is a baseline, not the target."""
    import ctypes

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import Block, lib as olib  # the CPU oracle, timed as the baseline

    lib = olib()
    limit = None
    if threads is None:
        threads, limit = host_cores()
    blocks = host_block_table(comp)
    arr = (Block * len(blocks))()
    nb = 0
    for start, csize, hsize, usize in blocks:
        arr[nb].start, arr[nb].csize, arr[nb].hsize, arr[nb].usize = start, csize, hsize, usize
        nb += 1
    cl = np.ascontiguousarray(contig_len, dtype=np.int32)
    pos, tr = ctypes.c_int64(), ctypes.c_int64()
    # pilot on 64 blocks, then size the sample to the time budget
    pilot = min(64, nb)
    tp = lib.or_bench_inflate_check(comp.ctypes.data_as(ctypes.c_void_p), comp.size, arr, 0, pilot,
                                    cl.ctypes.data_as(ctypes.c_void_p), cl.size, 10, threads,
                                    ctypes.byref(pos), ctypes.byref(tr))
    n = min(nb, max(pilot, int(pilot * budget_s / max(tp, 1e-3))))
    ts = lib.or_bench_inflate_check(comp.ctypes.data_as(ctypes.c_void_p), comp.size, arr, 0, n,
                                    cl.ctypes.data_as(ctypes.c_void_p), cl.size, 10, threads,
                                    ctypes.byref(pos), ctypes.byref(tr))
    return {
        "value": round(pos.value / ts / 1e9, 4),
        "unit": "GB/s decompressed",
        "cores": threads,
        "cores_limit": limit or "--cpu-threads",
        "host_cpus_visible": os.cpu_count(),
        "zlib_version": lib.or_zlib_version().decode(),
        "kind": "port",
        "sample": f"first {n} of {nb} BGZF blocks of the rank-0 shard ({pos.value / 1e6:.0f} MB "
                  f"uncompressed): zlib inflate + eager check at every offset, {threads} pthreads, "
                  f"{ts:.1f} s; CPU restatement (oracle/), not the JVM reference",
        "records_found": int(tr.value),
    }


if __name__ == "__main__":
    main()
