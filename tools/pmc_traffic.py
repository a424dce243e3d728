#!/usr/bin/env python3
"""Per-kernel HBM traffic per launch from two rocprofv3 --pmc passes over bench.py
(FETCH_SIZE and WRITE_SIZE, separate runs as the microarchitecture guide prescribes).

Both counters are in KiB.  On gfx950 FETCH_SIZE tallies 128-byte requests at 64 B, i.e.
reports half the bytes of a wide coalesced stream (MI355X_MICROARCH.md, HBM section):
the read side is doubled.  WRITE_SIZE is exact for 16-B-per-lane stores.  The median
launch of each kernel is taken.

usage: python tools/pmc_traffic.py FETCH.csv WRITE.csv > profiles/rNN_pmc_traffic.json
"""
import collections
import csv
import json
import os
import re
import sys


def src_hash(d):
    """bench.kernel_src_hash() of the kernels the passes ran (tools/pmc_collect.sh writes it)."""
    p = os.path.join(d, "src_hash")
    return open(p).read().strip() if os.path.exists(p) else None


def per_kernel(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        m = re.search(r"(k_\w+)", r["Kernel_Name"].replace("k_hdr<true>", "k_hdr_tail"))
        if m:
            agg[m.group(1)].append(float(r["Counter_Value"]))
    return {k: sorted(v)[len(v) // 2] for k, v in agg.items()}


def main(fetch, write):
    f, w = per_kernel(fetch), per_kernel(write)
    out = {}
    for k in sorted(set(f) | set(w)):
        rd = 2 * f.get(k, 0.0) * 1024
        wr = w.get(k, 0.0) * 1024
        out[k] = {"read_bytes": int(rd), "write_bytes": int(wr), "hbm_bytes": int(rd + wr)}
    json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE over `bench.py --no-cpu-baseline "
                         "--steps 2 --warmup 1` (median launch; FETCH_SIZE doubled, gfx950)",
               "src_hash": src_hash(os.path.dirname(fetch)), "kernels": out}, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
