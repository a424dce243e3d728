"""bench.py's roofline `traffic`: the committed PMC summary's bytes for the whole timed stage."""
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _tj(**kb):
    return {"kernels": {k: {"hbm_bytes": v} for k, v in kb.items()}}


def test_huffman_stage_sums_its_launches():
    tj = _tj(k_hdr=5, k_huff=100, k_huff_tail=7, k_huff_serial=1, k_lz=1000)
    assert bench.stage_traffic(tj, "k_huff") == 113
    assert bench.stage_traffic(_tj(k_huff=100), "k_huff") == 100  # passes that saw no tail launch


def test_single_kernel_stages():
    tj = _tj(k_huff=100, k_lz=1000, k_eager=400)
    assert bench.stage_traffic(tj, "k_lz") == 1000
    assert bench.stage_traffic(tj, "k_eager") == 400


def test_latest_pmc_prefers_the_kernel_sources_in_the_tree():
    tj, src = bench.latest_pmc("traffic.json")
    assert tj is not None and src.startswith("profiles/")
    for k in ("k_hdr", "k_huff", "k_huff_tail", "k_lz", "k_eager"):
        assert tj["kernels"][k]["hbm_bytes"] > 0
    cur = bench.kernel_src_hash()
    dirs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc", "src_hash")))
    if any(open(d).read().strip() == cur for d in dirs):  # counters collected from these sources exist
        assert tj.get("src_hash") == cur
