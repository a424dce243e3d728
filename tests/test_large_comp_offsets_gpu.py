"""Compressed offsets past 2^31.  A configs[2] rank shard holds 12.5 GiB of compressed bytes,
so every kernel that handles shard-relative compressed offsets (the index, inflate's stream
addressing, FindBlockStart, the batched split prologue) must be right past 2 GiB -- a lane
broadcast that sign-extends a 32-bit half (splits.hip's FindBlockStart result once did) sends
those splits off the device path.

The file: the synthetic BAM header (level 6), then 2^31 + 1 MiB of random bytes stored in
level-0 BGZF blocks (so the COMPRESSED offsets of everything after them exceed 2^31), then
short reads (config B) and long reads (config D) at level 6 and the EOF block.  Against the
CPU oracle (the reference's semantics: MetadataStream.scala:23-54, Stream.scala:31-71,
FindBlockStart.scala:8-36, eager/Checker.scala:24-126, CanLoadBam.scala:283-297,316-356):
the block table, the inflated bytes (and every block's CRC32), the eager bits across the
region, FindBlockStart from offsets past 2 GiB, and every split's first record and count from
sbh_split_starts, all of them decided on the device (n_host == 0)."""
import os
import sys

import numpy as np
import pytest

from oracle_lib import OR_OK, OracleFile, file_splits
from pkg import sb

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import synth  # noqa: E402

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

PAD = (1 << 31) + (1 << 20)
N_SHORT, N_LONG = 30000, 40


@pytest.fixture(scope="module")
def big():
    p6 = synth.params(synth.SEEDS["B"], shape=synth.SHAPE_SHORT, level=6)
    p0 = synth.params(synth.SEEDS["B"], shape=synth.SHAPE_SHORT, level=0)
    pl = synth.params(synth.SEEDS["D"], shape=synth.SHAPE_LONG, level=6)
    hdr = synth.header_bytes()
    recs = np.concatenate([synth.records(p6, 0, N_SHORT), synth.records(pl, 0, N_LONG)])
    pad = np.random.default_rng(0x5B4D2000).integers(0, 256, PAD, dtype=np.uint8)
    c_hdr, _ = synth.bgzf(p6, hdr, 0, False)
    c_pad, _ = synth.bgzf(p0, pad, 0, False)
    del pad
    c_rec, _ = synth.bgzf(p6, recs, 0, True)
    comp = np.concatenate([c_hdr, c_pad, c_rec])
    rec_comp = c_hdr.size + c_pad.size  # compressed offset of the records' first block
    del c_pad
    assert rec_comp > (1 << 31) + (1 << 20)
    of = OracleFile(comp)
    assert of.error == 0
    r0 = hdr.size + PAD  # flat offset of the first record
    assert of.flat_size == r0 + recs.size
    yield comp, of, r0, rec_comp
    of.close()


@pytest.fixture(scope="module")
def loaded(big):
    comp, of, r0, rec_comp = big
    ctx = sb.Context(0)
    sh = ctx.shard(comp)
    sh.index(0)
    sh.inflate()
    sh.set_contigs(of.contig_len)
    yield sh
    sh.close()
    ctx.close()


def test_index_and_inflate(big, loaded):
    comp, of, r0, rec_comp = big
    sh = loaded
    assert [(b[0], b[1], b[2]) for b in sh.blocks() if not b[5] & sb.BLOCK_EMPTY] == \
        [tuple(b) for b in of.blocks if b[2]]
    assert sh.flat_size == of.flat_size
    assert sh.verify_crc() == (0, 0)
    # the bytes around the pad's end and the records (flat offsets past 2^31, compressed too)
    a = r0 - (1 << 20)
    assert np.array_equal(sh.read_flat(a, of.flat_size - a), of.uncompressed_range(a, of.flat_size))


def test_eager_and_count(big, loaded):
    comp, of, r0, rec_comp = big
    sh = loaded
    a = r0 - (1 << 20)
    n_ref, bits_ref = of.eager_range(a, of.flat_size)
    n, bits = sh.check_eager(a, of.flat_size)
    assert n == n_ref == N_SHORT + N_LONG
    assert np.array_equal(bits, bits_ref)
    assert sh.find_record_start(a)[0] == r0
    assert sh.count_records(r0, of.flat_size) == N_SHORT + N_LONG


def test_find_block_start_past_2g(big, loaded):
    comp, of, r0, rec_comp = big
    sh = loaded
    rng = np.random.default_rng(3)
    offs = [(1 << 31) + 17, (1 << 31) + 65536 * 3 + 1, rec_comp - 70000, rec_comp - 5, rec_comp, rec_comp + 1,
            comp.size - 200000] + [int(x) for x in rng.integers(1 << 31, comp.size - 100, 12)]
    for o in offs:
        rc, want = of.find_block_start(o)
        assert rc == OR_OK
        assert sh.find_block_start(o) == want, o


def test_split_starts_past_2g(big, loaded):
    """Every 1 MiB split starting at or past 2^31 (the pad's last blocks, whose first record is
    the file's first, then the records; their starts' shard-relative compressed offsets all
    have bit 31 set) on the device path, equal to the oracle."""
    comp, of, r0, rec_comp = big
    sh = loaded
    splits = [(s, e) for s, e in file_splits(comp.size, 1 << 20) if s >= (1 << 31)]
    assert len(splits) >= 5 and any(s < rec_comp for s, _ in splits)
    status, v, n, n_host = sh.split_starts(splits)
    assert n_host == 0, f"{n_host} of {len(splits)} splits left the device path"
    for i, (s, e) in enumerate(splits):
        rc, vr, nr = of.split(s, e)
        assert rc == OR_OK and int(status[i]) == 0, (i, s, e)
        assert int(n[i]) == nr and (nr == 0 or int(v[i]) == vr), (i, s, e)
    assert int(n.sum()) == N_SHORT + N_LONG


def test_run_shard_past_2g(big, loaded):
    """The whole per-shard path indexed from the records' first block (compressed offset past
    2^31; from offset 0 the first record lies 2 GiB past the start, beyond maxReadSize)."""
    comp, of, r0, rec_comp = big
    sh = loaded
    r = sh.run(rec_comp, comp.size)
    assert r["status"] == 0 and r["count"] == N_SHORT + N_LONG
    assert r["first_vpos"] == (rec_comp << 16)
