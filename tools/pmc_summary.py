#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 --pmc CSV (counter_collection.csv): counter totals
and the SQ wave-cycle split (parked on waitcnt/barrier, issue-stalled, issuing).

usage: python tools/pmc_summary.py gpurun_out/pmc/p1_counter_collection.csv"""
import collections
import csv
import re
import sys


def main(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    ndisp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        m = re.search(r"(k_\w+)", r["Kernel_Name"].replace("k_hdr<true>", "k_hdr_tail"))
        k = m.group(1) if m else r["Kernel_Name"][:40]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        ndisp[k].add(r["Dispatch_Id"])
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        line = f"{k} (dispatches {len(ndisp[k])}): " + " ".join(f"{c}={x:.3g}" for c, x in sorted(v.items()))
        wc = v.get("SQ_WAVE_CYCLES", 0)
        if wc:
            line += " | wait_any %.0f%% wait_inst %.0f%% active %.0f%%" % (
                100 * v.get("SQ_WAIT_ANY", 0) / wc, 100 * v.get("SQ_WAIT_INST_ANY", 0) / wc,
                100 * v.get("SQ_ACTIVE_INST_ANY", 0) / wc)
        print(line)


if __name__ == "__main__":
    main(sys.argv[1])
