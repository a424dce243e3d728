#!/usr/bin/env python3
"""Time sbh_verify_crc (k_block_crc: every inflated block's bytes against its BGZF footer
CRC32) on a synthetic config-B shard; the library given by SBH_LIB_PATH (default in-tree).
usage: python tools/crc_bench.py [--records N]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=4_000_000)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import synth
    from __graft_entry__ import load_package
    sb = load_package()
    p = synth.params(synth.SEEDS["B"])
    data, usize, nb = synth.make_bam(p, a.records)
    with sb.Context(0) as ctx:
        sh = ctx.shard(data)
        sh.index(0)
        sh.inflate()
        best, res = None, None
        for _ in range(a.reps):
            t0 = time.perf_counter()
            res = sh.verify_crc()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        print(json.dumps({"lib": os.path.basename(os.environ.get("SBH_LIB_PATH", "") or "in-tree"),
                          "blocks": int(nb), "flat_bytes": int(sh.flat_size), "ms": round(best * 1e3, 3),
                          "GBps": round(sh.flat_size / best / 1e9, 1), "bad": list(res)}), flush=True)


if __name__ == "__main__":
    main()
