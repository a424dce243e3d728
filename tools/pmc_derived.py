#!/usr/bin/env python3
"""Derived per-kernel counter ratios from the rocprofv3 passes of tools/pmc_collect.sh: the
SQ wave-cycle split (parked on s_waitcnt / barrier, issue-stalled, issuing), VALU-active
share, LDS bank-conflict share of the LDS-array cycles, LDS-issue stalls, instructions per
wave.  SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* count quad-cycles on gfx950; only ratios are
used.  usage: python tools/pmc_derived.py DIR > DIR/derived.json (DIR holds sq_lds.csv, sq_wait.csv)"""
import collections
import csv
import json
import os
import re
import sys


def load(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        m = re.search(r"(k_\w+)", r["Kernel_Name"].replace("k_hdr<true>", "k_hdr_tail"))
        if m:
            agg[m.group(1)][r["Counter_Name"]] += float(r["Counter_Value"])
    return agg


def main(d):
    a, b = load(os.path.join(d, "sq_lds.csv")), load(os.path.join(d, "sq_wait.csv"))
    out = {}
    for k in sorted(set(a) & set(b), key=lambda k: -a[k].get("SQ_WAVE_CYCLES", 0)):
        x, y = a[k], b[k]
        wc, wc2 = x.get("SQ_WAVE_CYCLES", 0), y.get("SQ_WAVE_CYCLES", 0)
        if wc < 1e8:
            continue
        lds = x.get("SQ_LDS_IDX_ACTIVE", 0)
        out[k] = {
            "wave_cycles": wc,
            "valu_active_frac": round(x.get("SQ_ACTIVE_INST_VALU", 0) / wc, 3),
            "parked_waitcnt_barrier_frac": round(y.get("SQ_WAIT_ANY", 0) / wc2, 3) if wc2 else None,
            "issue_stalled_frac": round(y.get("SQ_WAIT_INST_ANY", 0) / wc2, 3) if wc2 else None,
            "issuing_frac": round(y.get("SQ_ACTIVE_INST_ANY", 0) / wc2, 3) if wc2 else None,
            "lds_bank_conflict_frac": round(x.get("SQ_LDS_BANK_CONFLICT", 0) / lds, 3) if lds else None,
            "lds_issue_stall_frac": round(x.get("SQ_WAIT_INST_LDS", 0) / wc, 3),
            "valu_insts_per_wave": round(x.get("SQ_INSTS_VALU", 0) / y["SQ_WAVES"], 1) if y.get("SQ_WAVES") else None,
            "lds_insts_per_wave": round(x.get("SQ_INSTS_LDS", 0) / y["SQ_WAVES"], 1) if y.get("SQ_WAVES") else None,
            "salu_insts_per_wave": round(y.get("SQ_INSTS_SALU", 0) / y["SQ_WAVES"], 1) if y.get("SQ_WAVES") else None,
        }
    hp = os.path.join(d, "src_hash")
    json.dump({"source": f"rocprofv3 --pmc passes in {d} (tools/pmc_collect.sh over bench.py)",
               "src_hash": open(hp).read().strip() if os.path.exists(hp) else None, "kernels": out},
              sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
