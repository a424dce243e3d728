#!/usr/bin/env python3
"""LZ77 token statistics of BGZF blocks (a design aid for the token format between k_huff and
k_lz): per block, literals / matches / match lengths, and how many tokens a format that packs up
to K consecutive literals into one token would need.  A small pure-Python DEFLATE decoder
(RFC 1951) over the first N blocks of a synthetic config-B BAM.

usage: python tools/token_stats.py [--blocks 8] [--records 20000] [--level 6]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195,
         227, 258]
LEXT = [0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0]
DBASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073,
         4097, 6145, 8193, 12289, 16385, 24577]
DEXT = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]


class Bits:
    def __init__(self, b):
        self.b, self.p = b, 0

    def get(self, n):
        v = 0
        for i in range(n):
            v |= ((self.b[self.p >> 3] >> (self.p & 7)) & 1) << i
            self.p += 1
        return v


def huff(lens):
    """canonical code -> {(len, code): sym}"""
    mx = max(lens) if lens else 0
    bl = [0] * (mx + 1)
    for L in lens:
        if L:
            bl[L] += 1
    code, nxt = 0, [0] * (mx + 2)
    for b in range(1, mx + 1):
        code = (code + bl[b - 1]) << 1
        nxt[b] = code
    t = {}
    for s, L in enumerate(lens):
        if L:
            t[(L, nxt[L])] = s
            nxt[L] += 1
    return t


LAST_LEN = [0]  # code length of the last symbol sym() decoded


def sym(br, t):
    code = L = 0
    while True:
        code = (code << 1) | br.get(1)
        L += 1
        if (L, code) in t:
            LAST_LEN[0] = L
            return t[(L, code)]


def tokens(raw):
    """DEFLATE stream -> list of tokens: ('L', byte) or ('M', length, distance)"""
    br, out = Bits(raw), []
    while True:
        final, typ = br.get(1), br.get(2)
        if typ == 0:
            br.p = (br.p + 7) & ~7
            n = br.get(16)
            br.get(16)
            for _ in range(n):
                out.append(("L", br.get(8), 8))
        else:
            if typ == 1:
                lit = huff([8] * 144 + [9] * 112 + [7] * 24 + [8] * 8)
                dist = huff([5] * 30)
            else:
                hlit, hdist, hclen = br.get(5) + 257, br.get(5) + 1, br.get(4) + 4
                order = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
                cl = [0] * 19
                for i in range(hclen):
                    cl[order[i]] = br.get(3)
                ct, lens = huff(cl), []
                while len(lens) < hlit + hdist:
                    s = sym(br, ct)
                    if s < 16:
                        lens.append(s)
                    elif s == 16:
                        lens += [lens[-1]] * (3 + br.get(2))
                    elif s == 17:
                        lens += [0] * (3 + br.get(3))
                    else:
                        lens += [0] * (11 + br.get(7))
                lit, dist = huff(lens[:hlit]), huff(lens[hlit:])
            while True:
                s = sym(br, lit)
                if s < 256:
                    out.append(("L", s, LAST_LEN[0]))
                elif s == 256:
                    break
                else:
                    s -= 257
                    cl = LAST_LEN[0] + LEXT[s]
                    L = LBASE[s] + br.get(LEXT[s])
                    d = sym(br, dist)
                    D = DBASE[d] + br.get(DEXT[d])
                    out.append(("M", L, D, cl, LAST_LEN[0] + DEXT[d]))
            out.append(("E",))  # end of a deflate block
        if final:
            return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=8)
    ap.add_argument("--records", type=int, default=20000)
    ap.add_argument("--level", type=int, default=6)
    a = ap.parse_args()
    import synth
    data = synth.make_bam(synth.params(0x5B4D0001, level=a.level), a.records)[0]
    sizes = synth.block_sizes(data)
    starts = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    tot = {"tok": 0, "lit": 0, "match": 0, "bytes": 0, "pack2": 0, "pack3": 0, "pack4": 0, "mlen1": 0}
    runs = {}
    for bi in range(1, min(len(sizes) - 1, a.blocks + 1)):  # (block 0: the header)
        s, n = int(starts[bi]), int(sizes[bi])
        blk = bytes(data[s:s + n])
        xlen = blk[10] | blk[11] << 8
        raw = blk[12 + xlen:n - 8]
        t = tokens(raw)
        # two literals per table lookup: a pair of consecutive literal codes (same deflate block)
        # whose lengths sum to <= W bits is decodable from one W-bit lookup
        i = 0
        while i < len(t):
            x = t[i]
            if x[0] == "L":
                for W in (10, 11, 12):
                    if i + 1 < len(t) and t[i + 1][0] == "L" and x[2] + t[i + 1][2] <= W:
                        tot["pair%d" % W] = tot.get("pair%d" % W, 0) + 1
                tot["litbits"] = tot.get("litbits", 0) + x[2]
            elif x[0] == "M":
                tot["lenbits"] = tot.get("lenbits", 0) + x[3]
                tot["distbits"] = tot.get("distbits", 0) + x[4]
            i += 1
        # greedy pairing at W bits: lookups needed for the literals
        for W in (10, 11, 12):
            i = look = 0
            while i < len(t):
                if t[i][0] == "L" and i + 1 < len(t) and t[i + 1][0] == "L" and t[i][2] + t[i + 1][2] <= W:
                    i += 2
                elif t[i][0] == "E":
                    i += 1
                    continue
                else:
                    i += 1
                look += 1
            tot["look%d" % W] = tot.get("look%d" % W, 0) + look
        t = [x for x in t if x[0] != "E"]
        lit = sum(1 for x in t if x[0] == "L")
        tot["tok"] += len(t)
        tot["lit"] += lit
        tot["match"] += len(t) - lit
        tot["bytes"] += sum(1 if x[0] == "L" else x[1] for x in t)
        run = 0
        for x in t + [("M", 0, 0)]:
            if x[0] == "L":
                run += 1
                continue
            if run:
                runs[run] = runs.get(run, 0) + 1
                for k in (2, 3, 4):
                    tot["pack%d" % k] += (run + k - 1) // k
            run = 0
    m = tot["match"]
    print(f"blocks {a.blocks}: tokens {tot['tok']}, literals {tot['lit']} ({tot['lit'] / tot['tok']:.1%}), "
          f"matches {m}, bytes {tot['bytes']} ({tot['bytes'] / tot['tok']:.2f} per token, "
          f"{(tot['bytes'] - tot['lit']) / max(m, 1):.1f} per match)")
    for k in (2, 3, 4):
        n = m + tot["pack%d" % k]
        print(f"  literals packed {k} per token: {n} tokens ({n / tot['tok']:.1%} of today's)")
    print(f"  mean code bits: literal {tot['litbits'] / tot['lit']:.2f}, length {tot['lenbits'] / max(m, 1):.2f}, "
          f"distance {tot['distbits'] / max(m, 1):.2f}")
    for W in (10, 11, 12):
        print(f"  {W}-bit lookups decoding two literals when both codes fit: {tot['look%d' % W]} lookups for "
              f"{tot['tok']} tokens ({tot['look%d' % W] / tot['tok']:.1%})")
    hist = sorted(runs.items())
    tot_runs = sum(runs.values())
    print("  literal runs:", tot_runs, "; length histogram (len: share of runs):",
          ", ".join(f"{k}: {v / tot_runs:.1%}" for k, v in hist[:12]))


if __name__ == "__main__":
    main()
