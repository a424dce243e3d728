#!/usr/bin/env python3
"""Counter calibration report: per calibration kernel (tools/calib_counters.hip) the raw
FETCH_SIZE / WRITE_SIZE (KiB, median launch) against the bytes the kernel is known to move, as
the factor that turns the counter into bytes for that access pattern.

usage: python tools/calib_report.py FETCH.csv WRITE.csv KNOWN.json-line"""
import collections
import csv
import json
import re
import sys


def per_kernel(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        m = re.search(r"(k_cal_\w+)", r["Kernel_Name"])
        if m:
            agg[m.group(1)].append(float(r["Counter_Value"]))
    return {k: sorted(v)[len(v) // 2] for k, v in agg.items()}


def main(fetch, write, known):
    f, w = per_kernel(fetch), per_kernel(write)
    kb = json.loads(open(known).read().strip().splitlines()[-1])["bytes"]
    reads = {"k_cal_read16", "k_cal_tok12", "k_cal_tok8"}
    out = {}
    for k, b in kb.items():
        raw = (f if k in reads else w).get(k)
        cnt = "FETCH_SIZE" if k in reads else "WRITE_SIZE"
        out[k] = {"counter": cnt, "raw_bytes": None if raw is None else raw * 1024, "known_bytes": b,
                  "bytes_per_counted_byte": None if not raw else round(b / (raw * 1024), 4),
                  "other_counter_bytes": (w if k in reads else f).get(k, 0.0) * 1024}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
