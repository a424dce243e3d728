#!/usr/bin/env python3
"""Inflate each golden fixture through the in-tree (or SBH_LIB_PATH) library and compare
with the oracle; prints one line per fixture.  Debug aid for k_lz changes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
from conftest import golden_bam  # noqa: E402
from oracle_lib import OracleFile  # noqa: E402
from pkg import sb  # noqa: E402

for name in sys.argv[1:] or ["2.bam", "1.bam", "5k.bam", "1.2203053-2211029.bam", "2.100-1000.bam"]:
    data = np.fromfile(golden_bam(name), dtype=np.uint8)
    with sb.Context(0) as ctx:
        sh = ctx.shard(data)
        sh.index(0)
        print(name, "indexed", flush=True)
        sh.inflate()
        flat = sh.read_flat()
        ref = OracleFile(data).uncompressed()
        d = np.flatnonzero(flat[:min(flat.size, ref.size)] != ref[:min(flat.size, ref.size)])
        print(name, flat.size, ref.size, "first diff", int(d[0]) if d.size else -1, flush=True)
        sh.close()
