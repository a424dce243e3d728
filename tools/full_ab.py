#!/usr/bin/env python3
"""A/B timing of sbh_check_full (k_full) on a synthetic short-read shard: the library given by
SBH_LIB_PATH (default: the in-tree build), a few readsToCheck values.
usage: SBH_LIB_PATH=build/variants/lib_fnh.so python tools/full_ab.py [--records N]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def counts_digest(r):
    """sha1 prefix of Counts, rbe, success / close-call counts and the sorted close calls
    (their order is atomic-slot order): variants must agree."""
    import hashlib
    import numpy as np
    h = hashlib.sha1()
    for k in ("counts", "rbe"):
        h.update(np.ascontiguousarray(r[k]).tobytes())
    h.update(f"{r['n_success']},{r['n_close']}".encode())
    if r["n_close"] <= len(r["close_flat"]):  # (past close_cap, which calls are kept varies)
        order = np.lexsort((r["close_word"], r["close_flat"]))
        h.update(r["close_flat"][order].tobytes() + r["close_word"][order].tobytes())
    return h.hexdigest()[:12]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=2_000_000)
    ap.add_argument("--rtc", default="10,1")
    ap.add_argument("--config", default="B", choices=["B", "D", "E"])
    a = ap.parse_args()
    import synth
    from __graft_entry__ import load_package
    sb = load_package()
    seed, shape, level = {"B": (0x5B4D0001, 0, 6), "D": (0x5B4D004C, 1, 6), "E": (0x5B4D00AD, 2, -1)}[a.config]
    p = synth.params(seed, shape=shape, level=level)
    data, usize, nb = synth.make_bam(p, a.records)
    with sb.Context(0) as ctx:
        sh = ctx.shard(data)
        _, cl, _ = sb.parse_bam_header(synth.header_bytes())
        sh.set_contigs(cl)
        sh.index(0)
        sh.inflate()
        for rtc in (int(x) for x in a.rtc.split(",")):
            best = None
            for _ in range(3):
                t0 = time.perf_counter()
                r = sh.check_full(0, sh.flat_size, reads_to_check=rtc, close_cap=1 << 10)
                dt = time.perf_counter() - t0
                best = dt if best is None else min(best, dt)
            # the digest from an untimed run that keeps every close call (a large close_cap
            # costs host allocation and copy-back time, so the timed runs keep 1 Ki)
            r = sh.check_full(0, sh.flat_size, reads_to_check=rtc, close_cap=1 << 22)
            print(f"{os.path.basename(os.environ.get('SBH_LIB_PATH', '') or 'in-tree')} config {a.config} rtc {rtc}: {best * 1e3:.2f} ms for "
                  f"{sh.flat_size} positions ({sh.flat_size / best / 1e9:.1f} GB/s), success {r['n_success']}, "
                  f"counts {counts_digest(r)}",
                  flush=True)


if __name__ == "__main__":
    main()
