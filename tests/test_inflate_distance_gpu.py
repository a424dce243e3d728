"""Distances at and past the bytes before their match (zlib's "invalid distance too far back",
java.util.zip.DataFormatException at Stream.scala:49-51): a BGZF member whose deflate stream
(fixed Huffman codes, written here token by token) carries a match reaching exactly to the
member's first byte inflates to zlib's bytes; one byte further is SBH_E_INFLATE_DATA, as zlib
fails it -- in a member's first deflate block (k_huff's lane-parallel passes), in a short final
deflate block (k_huff_tail), and in the second member of a file whose first is sound.  The
lane-parallel passes leave that test to k_lz, which sees every match token once."""
import struct
import zlib

import numpy as np
import pytest

from pkg import sb

pytestmark = pytest.mark.gpu

LEN_BASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163,
            195, 227, 258]
LEN_EXTRA = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DIST_BASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049,
             3073, 4097, 6145, 8193, 12289, 16385, 24577]
DIST_EXTRA = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]
EOF_MEMBER = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
SBH_E_INFLATE_DATA = 14


class Bits:
    def __init__(self):
        self.v, self.n = 0, 0

    def put(self, value, nbits):  # LSB first
        self.v |= (value & ((1 << nbits) - 1)) << self.n
        self.n += nbits

    def code(self, c, nbits):  # Huffman codes go most significant bit first
        self.put(int(format(c, f"0{nbits}b")[::-1], 2), nbits)

    def bytes(self):
        return self.v.to_bytes((self.n + 7) // 8, "little")


def fixed_lit(w, sym):
    if sym < 144:
        w.code(0x30 + sym, 8)
    elif sym < 256:
        w.code(0x190 + sym - 144, 9)
    elif sym < 280:
        w.code(sym - 256, 7)
    else:
        w.code(0xC0 + sym - 280, 8)


def fixed_block(w, tokens, final):
    """tokens: ints (literal bytes) or (length, distance) pairs."""
    w.put(1 if final else 0, 1)
    w.put(1, 2)  # BTYPE 01: fixed codes
    for t in tokens:
        if isinstance(t, tuple):
            ln, d = t
            c = max(i for i in range(29) if LEN_BASE[i] <= ln)
            fixed_lit(w, 257 + c)
            w.put(ln - LEN_BASE[c], LEN_EXTRA[c])
            dc = max(i for i in range(30) if DIST_BASE[i] <= d)
            w.code(dc, 5)
            w.put(d - DIST_BASE[dc], DIST_EXTRA[dc])
        else:
            fixed_lit(w, t)
    fixed_lit(w, 256)


def expand(tokens, out=None):
    """The bytes the tokens stand for (None when a distance reaches before the first byte)."""
    out = bytearray() if out is None else out
    for t in tokens:
        if isinstance(t, tuple):
            ln, d = t
            if d > len(out):
                return None
            for _ in range(ln):
                out.append(out[-d])
        else:
            out.append(t)
    return out


def member(blocks, isize):
    """A BGZF member of deflate blocks (lists of tokens); ISIZE / CRC of `isize` bytes when the
    stream is invalid (nothing reads them before the error)."""
    w = Bits()
    for i, toks in enumerate(blocks):
        fixed_block(w, toks, i == len(blocks) - 1)
    raw = w.bytes()
    u = expand([t for b in blocks for t in b])
    body = raw + struct.pack("<II", zlib.crc32(bytes(u)) if u is not None else 0, len(u) if u is not None else isize)
    total = 18 + len(body)
    hdr = bytes([31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0]) + struct.pack("<H", total - 1)
    return hdr + body, raw, u


def literals(n, seed):
    rng = np.random.default_rng(seed)
    return [int(x) for x in rng.integers(0, 256, n)]


@pytest.fixture(scope="module")
def ctx():
    c = sb.Context(0)
    yield c
    c.close()


def inflate(ctx, data):
    """(None, bytes) or (error code, None)."""
    sh = ctx.shard(np.frombuffer(data, dtype=np.uint8).copy())
    try:
        _, flat = sh.index(0)
        sh.inflate()
        return None, bytes(sh.read_flat(0, flat))
    except sb.SparkBamError as e:
        return e.code, None
    finally:
        sh.close()


def zlib_outcome(raws):
    try:
        return None, b"".join(zlib.decompress(r, -15) for r in raws)
    except zlib.error:
        return SBH_E_INFLATE_DATA, None


@pytest.mark.parametrize("at", [0, 3000, 5990])
@pytest.mark.parametrize("extra", [0, 1, 700])
def test_first_deflate_block(ctx, at, extra):
    # `at` literals, a match whose distance is the bytes before it plus `extra`, then literals to
    # 6000+ bytes: the lane-parallel path (usize >= 4096, staged)
    lead = literals(max(at, 1), 1)
    toks = lead + [(40, len(lead) + extra)] + literals(6000 - len(lead), 2)
    data, raw, u = member([toks], 6040)
    got = inflate(ctx, data + EOF_MEMBER)
    want = zlib_outcome([raw])
    assert got == want
    assert (got[0] is None) == (extra == 0) and (u is None) == (extra > 0)


@pytest.mark.parametrize("extra", [0, 1])
def test_short_final_block(ctx, extra):
    # a long first deflate block and a short last one (k_huff_tail's) whose match reaches to the
    # member's first byte, or one past it
    b1 = literals(7000, 3)
    b2 = literals(300, 4) + [(10, 7300 + extra)] + literals(50, 5)
    data, raw, u = member([b1, b2], 7360)
    got = inflate(ctx, data + EOF_MEMBER)
    assert got == zlib_outcome([raw])
    assert (got[0] is None) == (extra == 0)


def test_second_member(ctx):
    good, raw1, _ = member([literals(6000, 6) + [(100, 6000)]], 6100)
    bad, raw2, _ = member([literals(5000, 7) + [(20, 5001)] + literals(1000, 8)], 6020)
    got = inflate(ctx, good + bad + EOF_MEMBER)
    assert got == (SBH_E_INFLATE_DATA, None) == zlib_outcome([raw1, raw2])
    got = inflate(ctx, good + good + EOF_MEMBER)
    assert got[0] is None and got[1] == zlib.decompress(raw1, -15) * 2


@pytest.mark.parametrize("at,extra", [(3000, 0), (3000, 1), (3000, 20000), (10, 32768 - 10)])
def test_long_far_match(ctx, at, extra):
    # a 258-byte match (k_lz marks it with a start every 32 bytes) reaching exactly to the first
    # byte, one byte past it, far past it, and distance 32768 at a small offset
    lead = literals(at, 9)
    toks = lead + [(258, len(lead) + extra)] + literals(6000, 10)
    data, raw, u = member([toks], at + 6258)
    got = inflate(ctx, data + EOF_MEMBER)
    assert got == zlib_outcome([raw])
    assert (got[0] is None) == (extra == 0)


@pytest.mark.parametrize("extra", [0, 1, 5000])
def test_far_match_after_carried_cut(ctx, extra):
    # long matches fill k_lz's 6656-byte pointer pass before the chunk's 1536 tokens are used up,
    # so the chunk is cut and carried; the (far) match comes after several such cuts
    lead = literals(400, 11)
    toks = list(lead)
    for i in range(60):  # ~15 KB of 258-byte matches (several passes' worth), literals between
        toks += [(258, 300 + i)] + literals(3, 100 + i)
    n = len(expand(toks))
    toks += [(100, n + extra)] + literals(4000, 12)
    data, raw, u = member([toks], n + 4100)
    got = inflate(ctx, data + EOF_MEMBER)
    assert got == zlib_outcome([raw])
    assert (got[0] is None) == (extra == 0)
