#!/usr/bin/env python3
"""A/B the inflate-kernel variants (spark-bam_amd/build/ab/lib_*.so) on one
synthetic shard: per-variant k_inflate time (HIP events) and output identity vs the
in-tree library.  Each variant runs in its own process (the library path is bound at
import).  Usage: python tools/ab_inflate.py [--records N] [--config B|D|E] [variant ...]"""
import argparse
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


CONFIGS = {"B": (0x5B4D0001, 0, 6), "D": (0x5B4D004C, 1, 6), "E": (0x5B4D00AD, 2, -1)}


def child(lib, records, reps, config="B"):
    if lib:
        os.environ["SBH_LIB_PATH"] = lib
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import hashlib

    import numpy as np
    import synth
    from __graft_entry__ import load_package
    sb = load_package()
    seed, shape, level = CONFIGS[config]
    p = synth.params(seed, shape=shape, level=level)
    data, usize, nb = synth.make_bam(p, records)
    with sb.Context(0) as ctx:
        sh = ctx.shard(data)
        names, cl, _ = sb.parse_bam_header(synth.header_bytes())
        sh.set_contigs(cl)
        if os.environ.get("AB_INFLATE_ONLY"):  # variants whose tokens are wrong: time index + inflate only
            import time
            sh.index(0)
            wall = []
            for _ in range(reps + 1):
                t0 = time.perf_counter()
                sh.inflate()
                wall.append((time.perf_counter() - t0) * 1e3)
            print(json.dumps({"lib": os.path.basename(lib or "in-tree"), "inflate_wall_ms": sorted(wall[1:])}))
            return
        times = []
        for _ in range(reps):
            r = sh.run(0, data.size)
            times.append(sh.stage_times())
        sh.index(0)
        sh.inflate()
        h = hashlib.sha1(sh.read_flat().tobytes()).hexdigest()
        t = np.median(np.asarray(times), axis=0).tolist()
        print(json.dumps({"lib": os.path.basename(lib or "in-tree"), "comp": int(data.size),
                          "usize": int(usize), "blocks": int(nb), "stage_ms": t,
                          "inflate_GBps": usize / (t[1] * 1e-3) / 1e9, "sha1": h,
                          "count": r["count"]}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=2_000_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--child", default=None)
    ap.add_argument("--config", default="B", choices=sorted(CONFIGS))
    ap.add_argument("--rounds", type=int, default=1,
                    help="run the library list this many times, alternating its order (ABBA), and "
                         "print each library's per-stage median over the rounds at the end")
    ap.add_argument("variants", nargs="*")
    a = ap.parse_args()
    if a.child is not None:
        return child(a.child, a.records, a.reps, a.config)
    vdir = os.path.join(ROOT, "spark-bam_amd/build/ab")
    named = [v if v.endswith(".so") else os.path.join(vdir, f"lib_{v}.so") for v in a.variants]
    libs = [""] + (named or sorted(glob.glob(os.path.join(vdir, "lib_*.so"))))
    got = {}
    for rnd in range(a.rounds):
        for lib in (libs if rnd % 2 == 0 else libs[::-1]):
            r = subprocess.run([sys.executable, __file__, "--child", lib, "--records", str(a.records),
                                "--reps", str(a.reps), "--config", a.config], capture_output=True, text=True,
                               timeout=900)
            print(r.stdout.strip() or r.stderr[-2000:], flush=True)
            if r.stderr and r.stdout:  # probe variants print their counters on stderr/stdout
                print(r.stderr[-4000:], flush=True)
            try:
                d = json.loads(r.stdout.strip().splitlines()[-1])
                got.setdefault(d["lib"], []).append((d["stage_ms"], d.get("sha1")))
            except (ValueError, IndexError, KeyError):
                pass
    if a.rounds > 1:
        import numpy as np
        for lib, v in got.items():
            med = np.median(np.asarray([x[0] for x in v]), axis=0).round(4).tolist()
            print(json.dumps({"summary": lib, "rounds": len(v), "stage_ms_median": med,
                              "sha1": sorted({x[1] for x in v})}), flush=True)


if __name__ == "__main__":
    main()
