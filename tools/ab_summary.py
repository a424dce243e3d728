#!/usr/bin/env python3
"""Summarize tools/ab_inflate.py logs: k_huff / k_lz / pipeline ms per library, output sha1, count."""
import json
import sys

for f in sys.argv[1:]:
    for line in open(f):
        line = line.strip()
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        if "stage_ms" not in d:
            print(f, d)
            continue
        t = d["stage_ms"]
        print(f"{f.split('/')[-1]:24s} {d['lib']:18s} huff {t[4]:.3f} lz {t[5]:.3f} pipe {t[1]:.3f} "
              f"{d['sha1'][:10]} {d['count']}")
