"""Side measurement of the BGZF writer (sbh_bgzf_compress_level): the 5k.bam fixture's
uncompressed stream tiled to --mib MiB, resident on the device, compressed on the GPU at
--level (5 = htsjdk's bytes exactly, -1 = the fast coder).  Reports the writer kernels'
HIP-event time (GB/s of uncompressed input) and the whole call (incl. gather and the D2H of
the file).  Every member is inflated by zlib and compared with the source; with
--exact-every K every K-th member is also compared byte for byte with what htsjdk writes
(java.util.zip.Deflater = zlib 1.2.11 here, tests/test_zdeflate_cpu.htsjdk_member)."""
import argparse
import json
import os
import sys
import time
import zlib

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from pkg import sb  # noqa: E402
from oracle_lib import OracleFile  # noqa: E402
from test_zdeflate_cpu import htsjdk_member  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--mib", type=int, default=512)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--level", type=int, default=5)
ap.add_argument("--exact-every", type=int, default=0, help="byte-compare every K-th member with htsjdk's (level >= 0)")
a = ap.parse_args()
bam = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "bams", "5k.bam")
flat = OracleFile(np.fromfile(bam, dtype=np.uint8)).uncompressed()
n = a.mib << 20
src = np.resize(flat, n)
dev = torch.from_numpy(src).to("cuda:0")
torch.cuda.synchronize()
ctx = sb.Context(0)
best = None
for r in range(a.reps + 1):
    t0 = time.perf_counter()
    out, nb, ms = ctx.bgzf_compress(dev.data_ptr(), n, level=a.level)
    wall = time.perf_counter() - t0
    if r and (best is None or ms < best[0]):
        best = (ms, wall)
# full check: every member inflates (zlib) to the source bytes
o, pos, bad = out.tobytes(), 0, 0
f = k = exact_n = exact_bad = 0
while f < len(o):
    bsize = int.from_bytes(o[f + 16:f + 18], "little") + 1
    d = zlib.decompressobj(-15).decompress(o[f + 18:f + bsize - 8])
    if d != src[pos:pos + len(d)].tobytes() or zlib.crc32(d) != int.from_bytes(o[f + bsize - 8:f + bsize - 4], "little"):
        bad += 1
    if a.exact_every and a.level >= 0 and d and k % a.exact_every == 0:
        exact_n += 1
        exact_bad += htsjdk_member(d, a.level) != o[f:f + bsize]
    pos += len(d)
    f += bsize
    k += 1
print(json.dumps({"what": f"bgzf_compress level {a.level}", "input_bytes": n, "blocks": nb, "out_bytes": int(out.size),
                  "ratio": round(n / out.size, 3), "writer_ms": round(best[0], 3),
                  "writer_GBps": round(n / best[0] / 1e6, 2), "call_s_incl_d2h": round(best[1], 3),
                  "bad_members": bad, "roundtrip_ok": bad == 0 and pos == n,
                  "exact_checked": exact_n, "exact_bad": exact_bad}))
