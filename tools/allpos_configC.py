#!/usr/bin/env python3
"""check-bam -s (and optionally full-check) over configs[2]'s ONE ~100 GiB file, streamed through
HBM in windows (sbh_check_stream): the all-positions mode on a file far larger than HBM.

The file is synth.Replicated (the bench's configs[2] strong-scaling file: one canonical
12.4 M-record segment repeated); its `.records` truth is the CPU oracle's record chain over ONE
copy of the segment (tests/oracle_lib.py, the checker), shifted to every copy's blocks.  Prints
CheckerApp's summary lines (CheckerApp.scala:150-227) and one JSON line with the timings.
usage: python tools/allpos_configC.py [--file-gib 100] [--window-gib 1] [--full]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--file-gib", type=float, default=100.0)
    ap.add_argument("--records", type=int, default=12_400_000, help="records per replicated segment")
    ap.add_argument("--window-gib", type=float, default=1.0)
    ap.add_argument("--full", action="store_true", help="full-check's aggregation in the same pass")
    a = ap.parse_args()
    import synth
    from oracle_lib import OracleFile  # the checker: truth records of one segment copy
    from __graft_entry__ import load_package
    sb = load_package()
    t0 = time.time()
    p = synth.params(0x5B4D0030, shape=0, level=6, threads=min(16, os.cpu_count() or 1))
    F = synth.Replicated(p, a.records, int(a.file_gib * 2**30))
    log(f"segment: {F.seg_comp.size / 2**30:.3f} GiB compressed, {F.copies} copies, file {F.size / 2**30:.2f} GiB "
        f"({time.time() - t0:.0f} s)")
    data = np.empty(F.size, dtype=np.uint8)
    step = 4 << 30
    for lo in range(0, F.size, step):
        F.read_into(lo, min(F.size, lo + step), data[lo:min(F.size, lo + step)])
        log(f"file bytes {min(F.size, lo + step) / 2**30:.0f} GiB ({time.time() - t0:.0f} s)")
    # the truth: one copy's record chain (the oracle), shifted by k segment sizes per copy
    one = np.concatenate([F.hdr_comp, F.seg_comp, F.eof])
    of = OracleFile(one)
    flat = of.record_chain(of.header_end).astype(np.int64)
    starts = np.asarray([b[0] for b in of.blocks], dtype=np.int64)
    usizes = np.asarray([b[2] for b in of.blocks], dtype=np.int64)
    ustarts = np.concatenate([[0], np.cumsum(usizes)[:-1]])
    bi = np.searchsorted(ustarts, flat, side="right") - 1
    while True:  # canonical Pos: a record at a block's end is Pos(next block, 0); empty blocks skipped
        over = flat - ustarts[bi] >= usizes[bi]
        if not over.any():
            break
        bi[over] += 1
    v0 = (starts[bi].astype(np.uint64) << np.uint64(16)) | (flat - ustarts[bi]).astype(np.uint64)
    assert v0.size == a.records, (v0.size, a.records)
    h, s = F.hdr_comp.size, F.seg_comp.size
    shift = (np.arange(F.copies, dtype=np.uint64) * np.uint64(s)) << np.uint64(16)
    truth = (v0[None, :] + shift[:, None]).ravel()
    del shift
    # the blocks Blocks.apply reads from the file's `.blocks` (every data block, in order)
    hb = synth.block_sizes(F.hdr_comp)
    sb_ = np.asarray(synth.block_sizes(F.seg_comp), dtype=np.int64)
    seg_starts = np.concatenate([[0], np.cumsum(sb_)[:-1]])
    hstarts = np.concatenate([[0], np.cumsum(hb)[:-1]]).astype(np.int64)
    blocks = np.concatenate([hstarts] + [h + k * s + seg_starts for k in range(F.copies)]).astype(np.uint64)
    log(f"truth: {truth.size} records, blocks: {blocks.size} ({time.time() - t0:.0f} s)")
    _, contig_len, _ = sb.parse_bam_header(synth.header_bytes())
    with sb.Context(0) as ctx:
        t1 = time.perf_counter()
        r = ctx.check_stream(data, contig_len, blocks, truth_vpos=truth, full=a.full,
                             window=int(a.window_gib * 2**30), fp_cap=1000, close_cap=1 << 16)
        dt = time.perf_counter() - t1
    tp, fp, fn = r["tp"], r["fp"], r["fn"]
    print(f"{r['positions']} uncompressed positions")
    print(f"{r['comp_bytes'] / 2**30:.1f}G compressed")
    print(f"Compression ratio: {r['positions'] / r['comp_bytes']:.2f}")
    print(f"{tp + fn} reads")
    print("All calls matched!" if not fp and not fn and not r["unknown"] else f"{fp} false positives, {fn} false negatives")
    out = {"file_bytes": int(F.size), "records": int(F.records), "positions": int(r["positions"]),
           "tp": int(tp), "fp": int(fp), "fn": int(fn), "unknown": int(r["unknown"]), "windows": int(r["n_windows"]),
           "ms": round(dt * 1e3, 1), "ms_h2d": round(r["ms_h2d"], 1),
           "GBps_decompressed": round(r["positions"] / dt / 1e9, 2), "halo_final": int(r["halo_final"]),
           "all_matched": bool(not fp and not fn and not r["unknown"] and tp == F.records)}
    if a.full:
        out["n_success"] = int(r["n_success"])
        out["n_close"] = int(r["n_close"])
        out["counts_total"] = int(r["counts"].sum())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
