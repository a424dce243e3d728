#!/usr/bin/env python3
"""Dump the per-kernel summary of a rocprofv3 rocpd database (`--kernel-trace --stats`,
ROCm 7 default output) as CSV: name, calls, total/average duration (us), share.

usage: python tools/prof_stats.py gpurun_out/prof/run_results.db > profiles/rNN_kernel_stats.csv
"""
import csv
import sqlite3
import sys


def main(path):
    con = sqlite3.connect(path)
    cur = con.execute("select name, total_calls, total_duration, average, percentage from top_kernels")
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"])
    for row in cur:
        w.writerow(row)


if __name__ == "__main__":
    main(sys.argv[1])
