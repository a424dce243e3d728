"""Flat offsets past 2^31.  A configs[2]/[3] shard holds 3+ GB of flat bytes per GPU, so
every kernel's 64-bit position arithmetic is on the path; a 32-bit slip (a sign-extended
lane broadcast in k_eager's wave-cooperative CIGAR test once sent a wave to a wild
address, at config D's full size only) shows up only past 2 GiB.

The file: the synthetic BAM header, then 2^31 + 1 MiB of zero bytes (BGZF-compressed to a
few MB), then config-D long reads (10-50 kb, CIGARs of 50-500 ops), so the long-read
records sit at flat offsets above 2^31.  The eager call at every position of that region
and the record chain through it equal the CPU oracle's (parity at the reference's
semantics: eager/Checker.scala:24-126, PosStream.scala:14-22)."""
import os
import sys

import numpy as np
import pytest

from oracle_lib import OracleFile
from pkg import sb

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import synth  # noqa: E402

pytestmark = pytest.mark.gpu

N_REC = 120


@pytest.fixture(scope="module")
def past_2g():
    p = synth.params(synth.SEEDS["D"], shape=synth.SHAPE_LONG)
    hdr = synth.header_bytes()
    recs = synth.records(p, 0, N_REC)
    pad = (1 << 31) + (1 << 20)
    flat = np.zeros(hdr.size + pad + recs.size, dtype=np.uint8)
    flat[:hdr.size] = hdr
    flat[hdr.size + pad:] = recs
    r0 = hdr.size + pad
    comp, _ = synth.bgzf(p, flat, 0, True)
    del flat
    of = OracleFile(comp)
    assert of.flat_size == r0 + recs.size
    yield comp, of, r0
    of.close()


def test_eager_and_chain_past_2g(past_2g):
    comp, of, r0 = past_2g
    end = of.flat_size
    n_ref, bits_ref = of.eager_range(r0 - 4096, end)
    chain_ref = of.record_chain(r0)
    assert len(chain_ref) == N_REC
    with sb.Context(0) as ctx:
        sh = ctx.shard(comp)
        nb, fs = sh.index(0)
        assert fs == end
        sh.inflate()
        sh.set_contigs(of.contig_len)
        n, bits = sh.check_eager(r0 - 4096, end)
        assert n == n_ref == N_REC
        assert np.array_equal(bits, bits_ref)
        # the first record from inside the zero region, and the count over the region
        first = sh.find_record_start(r0 - 4096)
        assert first[0] == r0
        assert sh.count_records(r0, end) == N_REC
        sh.close()
