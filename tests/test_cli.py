"""CLI parity: `spark-bam <cmd>` output vs the reference's golden CLI outputs
(cli/src/test/resources/output/**, ComputeSplitsTest, CheckBamTest, FullCheckTest)."""
import os
import subprocess

import pytest

from conftest import BAMS, GOLDEN, ROOT

pytestmark = pytest.mark.gpu
CLI = os.path.join(ROOT, "cli", "spark-bam")


def run(*args):
    r = subprocess.run([CLI, *args], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return r.stdout


def test_compute_splits_230k():
    # ComputeSplitsTest "eager 230KB"
    out = run("compute-splits", "-s", "-m", "230k", os.path.join(BAMS, "1.bam")).splitlines()
    assert out[0].startswith("Get spark-bam splits: ") and out[0].endswith("ms")
    assert out[1:] == [
        "", "Split-size distribution:", "N: 3, μ/σ: 1.9e5/57877, med/mad: 2.2e5/20521",
        " elems: 224301 244822 113078", "sorted: 113078 224301 244822", "", "3 splits:",
        "\t0:45846-239479:312", "\t239479:312-484396:25", "\t484396:25-597482:0", ""]


def test_compute_splits_240k():
    # ComputeSplitsTest "compare 240KB" (the spark-bam half)
    out = run("compute-splits", "-s", "-m", "240k", os.path.join(BAMS, "1.bam")).splitlines()
    assert out[2:] == [
        "Split-size distribution:", "N: 3, μ/σ: 1.9e5/74433, med/mad: 2.4e5/3497",
        " elems: 248438 244941 88822", "sorted: 88822 244941 248438", "", "3 splits:",
        "\t0:45846-263656:191", "\t263656:191-508565:287", "\t508565:287-597482:0", ""]


def test_compute_splits_and_count_streamed():
    # the same ComputeSplitsTest / CountReadsTest answers when the file is streamed through
    # HBM (SBH_RESIDENT_MAX below the file size: sbh_run_stream2 with every split)
    env = dict(os.environ, SBH_RESIDENT_MAX="1")
    r = subprocess.run([CLI, "compute-splits", "-s", "-m", "230k", os.path.join(BAMS, "1.bam")], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    assert r.stdout.splitlines()[-4:] == ["\t0:45846-239479:312", "\t239479:312-484396:25", "\t484396:25-597482:0", ""]
    r = subprocess.run([CLI, "count-reads", "-m", "100k", os.path.join(BAMS, "1.bam")], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    assert "spark-bam found 4917 reads" in r.stdout


def test_check_bam_eager_1bam():
    # CheckBamTest "eager 1.bam"
    out = run("check-bam", "-s", "-m", "200k", os.path.join(BAMS, "1.bam"))
    assert out == ("1608257 uncompressed positions\n583K compressed\nCompression ratio: 2.69\n"
                   "4917 reads\nAll calls matched!\n")


@pytest.mark.parametrize("golden,args", [
    ("2.bam", ["2.bam"]),
    ("2.bam.first", ["-i", "0", "2.bam"]),
    ("2.bam.second", ["-i", "26169", "2.bam"]),
    ("2.bam.200k", ["-i", "0-200k", "-m", "100k", "2.bam"]),
    ("1.bam", ["-m", "200k", "1.bam"]),
])
def test_full_check_outputs(golden, args):
    # FullCheckTest: whole output files (with -l 10, as the reference test passes)
    args = args[:-1] + [os.path.join(BAMS, args[-1])]
    out = run("full-check", "-l", "10", *args)
    with open(os.path.join(GOLDEN, "output", "full-check", golden), encoding="utf-8") as f:
        want = f.read()
    assert out.splitlines() == want.splitlines()


@pytest.fixture(scope="module")
def noblocks(tmp_path_factory):
    """1.noblocks.bam: 1.bam's bytes with no `.blocks` / `.records` beside them (in the reference it
    is a link to 1.bam, test_bams/src/main/resources)."""
    import shutil
    d = tmp_path_factory.mktemp("noblocks")
    p = d / "1.noblocks.bam"
    shutil.copyfile(os.path.join(BAMS, "1.bam"), p)
    return str(p)


def test_full_check_noblocks(noblocks):
    # FullCheckTest "1.bam without indexed records": Blocks.apply without `.blocks` (FindBlockStart
    # per 200k split on the device, Blocks.scala:141-206) and no records summary
    out = run("full-check", "-l", "10", "-m", "200k", noblocks)
    with open(os.path.join(GOLDEN, "output", "full-check", "1.noblocks.bam"), encoding="utf-8") as f:
        assert out.splitlines() == f.read().splitlines()


def test_check_bam_noblocks(noblocks):
    # CheckBamTest's eager summary on the unindexed file (truth records given with -r)
    out = run("check-bam", "-s", "-m", "200k", "-r", os.path.join(BAMS, "1.bam.records"), noblocks)
    assert out == ("1608257 uncompressed positions\n583K compressed\nCompression ratio: 2.69\n"
                   "4917 reads\nAll calls matched!\n")


@pytest.mark.parametrize("window", ["100000", "30000"])
def test_all_positions_streamed_windows(window, noblocks):
    """check-bam -s and every full-check golden with the file moved through HBM in windows of
    `window` compressed bytes (sbh_check_stream; SBH_STREAM_WINDOW): byte-identical outputs."""
    env = dict(os.environ, SBH_STREAM_WINDOW=window)

    def run_env(*args):
        r = subprocess.run([CLI, *args], capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, r.stderr
        return r.stdout
    assert run_env("check-bam", "-s", "-m", "200k", os.path.join(BAMS, "1.bam")).endswith("All calls matched!\n")
    cases = [("2.bam", ["2.bam"]), ("2.bam.first", ["-i", "0", "2.bam"]), ("2.bam.second", ["-i", "26169", "2.bam"]),
             ("2.bam.200k", ["-i", "0-200k", "-m", "100k", "2.bam"]), ("1.bam", ["-m", "200k", "1.bam"])]
    for golden, args in cases:
        out = run_env("full-check", "-l", "10", *args[:-1], os.path.join(BAMS, args[-1]))
        with open(os.path.join(GOLDEN, "output", "full-check", golden), encoding="utf-8") as f:
            assert out.splitlines() == f.read().splitlines(), golden
    out = run_env("full-check", "-l", "10", "-m", "200k", noblocks)
    with open(os.path.join(GOLDEN, "output", "full-check", "1.noblocks.bam"), encoding="utf-8") as f:
        assert out.splitlines() == f.read().splitlines()


def test_count_reads_1bam():
    out = run("count-reads", "-m", "100k", os.path.join(BAMS, "1.bam"))
    assert "spark-bam found 4917 reads" in out


def test_index_blocks_and_records(tmp_path):
    # IndexBlocksTest / IndexRecordsTest: byte-exact .blocks / .records
    for name in ("2.bam", "1.bam"):
        ob, orc = tmp_path / (name + ".blocks"), tmp_path / (name + ".records")
        run("index-blocks", os.path.join(BAMS, name), str(ob))
        run("index-records", os.path.join(BAMS, name), str(orc))
        assert ob.read_text() == open(os.path.join(BAMS, name + ".blocks")).read()
        assert orc.read_text() == open(os.path.join(BAMS, name + ".records")).read()


def _golden_check_blocks(name):
    with open(os.path.join(GOLDEN, "output", "check-blocks", name), encoding="utf-8") as f:
        return f.read()


def test_check_blocks_spark_bam_1bam():
    # CheckBlocksTest "1.bam spark-bam": indexed (.records) vs eager, byte-exact
    assert run("check-blocks", "-s", os.path.join(BAMS, "1.bam")) == _golden_check_blocks("1.bam.s")


@pytest.mark.parametrize("name", ["2.bam", "1.block-aligned.bam"])
def test_check_blocks_matched_outputs(name, tmp_path):
    # CheckBlocksTest "2.bam" / "1.block-aligned.bam" are default-mode (eager vs hadoop-bam)
    # runs that matched everywhere, so eager's first-read offsets are the records'; the -s
    # run (indexed vs eager) prints the same text.  1.block-aligned.bam has no .records in
    # the reference: it is generated with index-records (IndexRecordsTest-pinned).
    bam = os.path.join(BAMS, name)
    recs = bam + ".records"
    if not os.path.exists(recs):
        recs = str(tmp_path / (name + ".records"))
        run("index-records", bam, recs)
    assert run("check-blocks", "-s", "-r", recs, bam) == _golden_check_blocks(name)


def test_check_blocks_mismatch_report(tmp_path):
    # The mismatch report (CheckBlocksTest "1.bam"): make the indexed side disagree at
    # block 239479 by replacing its first record 239479:312 with 239479:311 in a copy
    # of the records file; the counts, ratio and block line follow the golden's format.
    recs = tmp_path / "1.bam.records"
    lines = open(os.path.join(BAMS, "1.bam.records")).read().splitlines()
    lines[lines.index("239479,312")] = "239479,311"
    recs.write_text("\n".join(lines) + "\n")
    out = run("check-blocks", "-s", "-r", str(recs), os.path.join(BAMS, "1.bam")).splitlines()
    want = _golden_check_blocks("1.bam.default").splitlines()
    assert out[:3] == want[:3]  # "... mismatched in 1 of 25 ...", "", "25871 of 597482 (0.0433...) ..."
    assert out[-2:] == ["1 mismatched blocks:", "\t239479 (prev block size: 25871):\t239479:311\t239479:312"]


def test_check_blocks_needs_spark_bam_mode():
    r = subprocess.run([CLI, "check-blocks", os.path.join(BAMS, "1.bam")], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode != 0 and "hadoop-bam" in r.stderr


def _members(path):
    """[(offset, usize, payload)] of a BGZF file's data members."""
    import struct
    import zlib
    b = open(path, "rb").read()
    out, o = [], 0
    while o < len(b):
        bs = struct.unpack_from("<H", b, o + 16)[0] + 1
        d = zlib.decompressobj(-15).decompress(b[o + 18:o + bs - 8])
        if d:
            out.append((o, len(d), d))
        o += bs
    return out


@pytest.mark.parametrize("rng", [None, "100-1000"])
def test_htsjdk_rewrite(tmp_path, rng):
    # HTSJDKRewriteTest (cli/src/test/scala/org/hammerlab/bam/rewrite/HTSJDKRewriteTest.scala:14-24):
    # `-r 100-1000 -b -i 2.bam` -> dirMatch with slice/2.100-1000.bam{,.blocks,.records}: the
    # BAM and both index files byte-equal; without -r the rewrite reproduces 2.bam itself
    # (htsjdk wrote it) and its .blocks / .records.
    ref = os.path.join(BAMS, "2.100-1000.bam" if rng else "2.bam")
    out = tmp_path / "out.bam"
    args = ["htsjdk-rewrite"] + (["-r", rng] if rng else []) + ["-b", "-i", os.path.join(BAMS, "2.bam"), str(out)]
    run(*args)
    for ext in ("", ".blocks", ".records"):
        assert open(str(out) + ext, "rb").read() == open(ref + ext, "rb").read(), ext
    mine = _members(str(out))
    assert [u for _, u, _ in mine] == [u for _, u, _ in _members(ref)]
