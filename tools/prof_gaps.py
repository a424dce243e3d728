#!/usr/bin/env python3
"""Device-idle gaps between consecutive kernels of a rocprofv3 `--kernel-trace` database
(rocpd sqlite, ROCm 7 default output): the busy / idle split of the trace's last N ms and the
largest gaps with the kernels on either side -- where a step waits on the host.

usage: python tools/prof_gaps.py RUN_results.db [--last-ms 100] [--top 15]
"""
import argparse
import sqlite3


def load(con):
    names = [r[0] for r in con.execute("select name from sqlite_master where type in ('table','view')")]
    for view in ("kernels", "kernel_dispatch", "rocpd_kernel_dispatch"):
        if view not in names:
            continue
        cols = [r[1] for r in con.execute(f"pragma table_info({view})")]
        start = next((c for c in ("start", "start_ns", "begin") if c in cols), None)
        end = next((c for c in ("end", "end_ns", "stop") if c in cols), None)
        name = next((c for c in ("name", "kernel_name", "kernel") if c in cols), None)
        if start and end and name:
            return [(int(a), int(b), str(n)) for a, b, n in
                    con.execute(f'select "{start}", "{end}", "{name}" from {view} order by "{start}"')]
    raise SystemExit(f"no kernel view with start/end/name among: {names}")


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    return n.split("(")[0].split("::")[-1][:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last-ms", type=float, default=100.0)
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--step-kernel", default=None,
                    help="a kernel launched once per step (e.g. k_lz): analyse the last --steps periods "
                         "between its launches instead of the last --last-ms")
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    ks = load(sqlite3.connect(a.db))
    if a.step_kernel:
        marks = [s for s, _, n in ks if short(n) == a.step_kernel]
        t0, t1 = marks[-a.steps - 1], marks[-1]
        ks = [k for k in ks if t0 <= k[0] < t1]
    else:
        t_end = max(e for _, e, _ in ks)
        t0 = t_end - int(a.last_ms * 1e6)
        ks = [k for k in ks if k[0] >= t0]
    busy, gaps, last_end, prev = 0, [], None, None
    for s, e, n in ks:
        if last_end is not None and s > last_end:
            gaps.append((s - last_end, short(prev), short(n)))
        busy += max(0, e - max(s, last_end or s))
        last_end = e if last_end is None else max(last_end, e)
        prev = n
    span = last_end - ks[0][0]
    print(f"{len(ks)} kernels over {span / 1e6:.2f} ms: busy {busy / 1e6:.2f} ms, idle {(span - busy) / 1e6:.2f} ms "
          f"in {len(gaps)} gaps")
    for g, p, n in sorted(gaps, reverse=True)[:a.top]:
        print(f"  {g / 1e3:9.1f} us  after {p:40s} before {n}")


if __name__ == "__main__":
    main()
