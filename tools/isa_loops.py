#!/usr/bin/env python3
"""Instruction counts of the innermost loops of a kernel in a gfx950 .s file (hipcc -S):
per loop (grouped by the compiler's 'in Loop: Header=BB.. Depth=N' block comments) and per
basic block, VALU / SALU / LDS / VMEM / other.  Loops are listed when they contain every
--must mnemonic.  usage: isa_loops.py FILE.s KERNEL_SUBSTR [--must v_alignbit_b32 ...]"""
import re
import sys
from collections import OrderedDict, defaultdict


def kind(m):
    if m.startswith("v_"):
        return "valu"
    if m.startswith("ds_"):
        return "lds"
    if m.startswith(("global_", "buffer_", "scratch_", "flat_")):
        return "vmem"
    if m.startswith("s_waitcnt") or m.startswith("s_nop"):
        return "wait"
    if m.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if m.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, kern = sys.argv[1], sys.argv[2]
    must = [m for m in sys.argv[sys.argv.index("--must") + 1:] if not m.startswith("--")] if "--must" in sys.argv else []
    lines = open(path).read().split("\n")
    # the kernel's function body
    start = next(i for i, l in enumerate(lines) if re.match(rf"^\S*{kern}\S*:", l))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith("s_endpgm"))
    blocks = OrderedDict()
    cur = None
    body = lines[start:end + 1]
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\S+|; %bb\.\d+):?\s*(?:;\s*(.*))?$", l)
        if m:
            cur = m.group(1).rstrip(":")
            c = m.group(2) or ""
            h = re.search(r"Header=(BB\S+) Depth=(\d+)", c)
            nxt = body[i + 1] if i + 1 < len(body) else ""
            is_hdr = "Loop Header" in nxt and "=>" in nxt and "This" in nxt
            blocks[cur] = {"hdr": h.group(1) if h else None, "depth": int(h.group(2)) if h else 0,
                           "is_header": is_hdr, "inner": "Inner Loop Header" in nxt, "ins": []}
            continue
        s = l.strip()
        if cur and s and not s.startswith((";", ".")):
            blocks[cur]["ins"].append(s.split()[0])
    loops = defaultdict(list)
    inner = {"BB" + n.split("BB")[-1] for n, b in blocks.items() if b["inner"]}
    for name, b in blocks.items():
        key = b["hdr"]
        if b["is_header"]:
            key = "BB" + name.split("BB")[-1]
        if key in inner or (key and "--all" in sys.argv):
            loops[key].append((name, b))
    for key, bl in loops.items():
        allm = [m for _, b in bl for m in b["ins"]]
        if any(not any(x == mm for x in allm) for mm in must):
            continue
        tot = defaultdict(int)
        for m in allm:
            tot[kind(m)] += 1
        print(f"loop {key}: {len(bl)} blocks, " + " ".join(f"{k} {v}" for k, v in sorted(tot.items())))
        for name, b in bl:
            c = defaultdict(int)
            for m in b["ins"]:
                c[kind(m)] += 1
            print(f"   {name:10s} " + " ".join(f"{k} {v}" for k, v in sorted(c.items())))


if __name__ == "__main__":
    main()
