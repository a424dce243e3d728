"""Short final deflate blocks with dynamic Huffman headers (k_huff_tail's work): since round 6
their headers are decoded and tabled by k_hdr<true> between k_huff and k_huff_tail whenever the
header record fits between the tail's two leading words and the end of the block's token region
(`tail_hdr_room`, inflate.hip); otherwise k_huff_tail decodes the header itself.  Members are
built with zlib (level 6, `Z_BLOCK` between parts, so each part ends a deflate block) and every
one must inflate to zlib's own bytes: a tail with room (the pre-decoded header), a tail without
room (a literal-heavy first part: about one token per byte), a tail of two deflate blocks (the
second header decoded inside k_huff_tail), and a fixed-code tail (no record)."""
import struct
import zlib

import numpy as np
import pytest

from pkg import sb

pytestmark = pytest.mark.gpu

EOF_MEMBER = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


def deflate_parts(parts, level=6):
    """Raw deflate of the concatenated parts, each part ending its own deflate block(s)."""
    co = zlib.compressobj(level, zlib.DEFLATED, -15)
    out = b""
    for i, p in enumerate(parts):
        out += co.compress(p)
        out += co.flush(zlib.Z_FINISH if i == len(parts) - 1 else zlib.Z_BLOCK)
    return out


def member(raw, u):
    body = raw + struct.pack("<II", zlib.crc32(u), len(u))
    total = 18 + len(body)
    assert total <= 65536
    return bytes([31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0]) + struct.pack("<H", total - 1) + body


def repetitive(n, seed):
    """~n bytes of a 1 KB random motif repeated with point mutations: long matches, few tokens."""
    rng = np.random.default_rng(seed)
    motif = rng.integers(65, 91, 1024, dtype=np.uint8)
    reps = np.tile(motif, n // 1024 + 1)[:n].copy()
    idx = rng.integers(0, n, n // 200)
    reps[idx] = rng.integers(65, 91, len(idx), dtype=np.uint8)
    return reps.tobytes()


def literal_heavy(n, seed):
    """bytes over 128 symbols: dynamic codes (7 bits of entropy), almost no 3-byte repeats."""
    return np.random.default_rng(seed).integers(0, 128, n, dtype=np.uint8).tobytes()


def acgt(n, seed):
    return np.random.default_rng(seed).choice(np.frombuffer(b"ACGT", np.uint8), n).tobytes()


@pytest.fixture(scope="module")
def ctx():
    c = sb.Context(0)
    yield c
    c.close()


def inflate(ctx, data):
    sh = ctx.shard(np.frombuffer(data, dtype=np.uint8).copy())
    try:
        _, flat = sh.index(0)
        sh.inflate()
        return bytes(sh.read_flat(0, flat))
    finally:
        sh.close()


CASES = {
    # few tokens before the tail: the tail's header record fits (k_hdr<true>)
    "room": lambda: [repetitive(58000, 1), acgt(1000, 2)],
    # ~1 token per byte before a 500-byte tail: no room, k_huff_tail decodes its header
    "no_room": lambda: [literal_heavy(40000, 3), literal_heavy(16383, 4), acgt(500, 9)],
    # the tail is two deflate blocks: the second header is decoded inside k_huff_tail
    "two_block_tail": lambda: [repetitive(60000, 5), acgt(500, 6), literal_heavy(300, 7)],
    # a small tail zlib codes with the fixed code (no dynamic header for k_hdr<true>)
    "fixed_tail": lambda: [repetitive(60000, 8), b"ACGT" * 5],
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_tail_headers_inflate_to_zlib_bytes(ctx, case):
    parts = CASES[case]()
    raw = deflate_parts(parts)
    u = b"".join(parts)
    assert zlib.decompress(raw, -15) == u
    got = inflate(ctx, member(raw, u) + EOF_MEMBER)
    assert got == u


def test_many_members_mixed_tails(ctx):
    # every kind of tail in one file, repeated, so k_hdr<true> and k_huff_tail see many blocks
    # in one launch (a record left by one block must never be read by another)
    data, want = b"", b""
    for i in range(12):
        for case in sorted(CASES):
            parts = CASES[case]()
            if i % 2:
                parts = parts[::-1] if case != "two_block_tail" else parts
            raw = deflate_parts(parts)
            u = b"".join(parts)
            data += member(raw, u)
            want += u
    assert inflate(ctx, data + EOF_MEMBER) == want
