"""SURVEY.md §5 sanitizers: the CPU-side C/C++ code built with -fsanitize=address,undefined and
run, so a memory or UB error aborts the test -- the oracle restatement over the reference's
fixtures and a synthetic corpus, the BGZF writer's host coder (the code k_deflate runs), and
the CLI's argument handling.  Also a syntax check of the JNI shim (jni/sparkbam_jni.c) against
the harness header in tests/jni_compile/ (the shim itself is built by jni/Makefile where a
JDK exists)."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT, golden_bam

SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")


@pytest.fixture(scope="module")
def build(tmp_path_factory):
    d = tmp_path_factory.mktemp("san")
    o = str(d / "oracle_driver")
    subprocess.run(["gcc", *SAN, "-I", os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests", "sanitize",
                    "oracle_driver.c"), os.path.join(ROOT, "oracle", "sbam_oracle.c"), "-lz", "-lpthread", "-o", o],
                   check=True)
    w = str(d / "deflate_driver")
    subprocess.run(["g++", *SAN, "-std=c++17", os.path.join(ROOT, "tests", "sanitize", "deflate_driver.cpp"),
                    os.path.join(ROOT, "tools", "deflate_host.cpp"), "-lz", "-o", w], check=True)
    return d, o, w


@pytest.mark.parametrize("name", ["2.bam", "1.bam", "5k.bam", "1.block-aligned.bam", "2.100-1000.bam"])
def test_oracle_under_asan_ubsan(build, name):
    _, o, _ = build
    r = subprocess.run([o, golden_bam(name)], env=ENV, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "flat " in r.stdout


def test_oracle_under_asan_ubsan_adversarial(build, tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import synth
    data = synth.make_bam(synth.params(0x5B4D00AE, shape=2, level=-1, empty_every=5), 4000)[0]
    p = tmp_path / "adv.bam"
    data.tofile(p)
    _, o, _ = build
    r = subprocess.run([o, str(p)], env=ENV, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]


def test_deflate_host_under_asan_ubsan(build):
    _, _, w = build
    r = subprocess.run([w, golden_bam("2.bam"), golden_bam("5k.bam")], env=ENV, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert "0 failed" in r.stdout


def test_cli_arguments_under_asan_ubsan(tmp_path):
    """The CLI's host code (argument parsing, byte-size and range syntax, error paths) built
    with the sanitizers; without a GPU every command stops at context creation."""
    exe = str(tmp_path / "spark-bam-san")
    subprocess.run(["g++", *SAN, "-std=c++17", "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "cli",
                    "spark_bam.cpp"), "-L", os.path.join(ROOT, "spark-bam_amd"), "-lsparkbam_hip",
                    f"-Wl,-rpath,{os.path.join(ROOT, 'spark-bam_amd')}", "-o", exe], check=True)
    bam = golden_bam("2.bam")
    for args in (["compute-splits", "-m", "100k", bam], ["count-reads", "-m", "230KB", bam],
                 ["check-bam", "-s", "-i", "0-200k,300k+10k", bam], ["full-check", "-i", "0-200k", bam],
                 ["nonsense"], [], ["compute-splits"], ["compute-splits", "-m"]):
        r = subprocess.run([exe, *args], env=dict(ENV, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1"),
                           capture_output=True, text=True, timeout=120)
        assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, (args, r.stderr[-2000:])
        assert r.returncode in (0, 1, 2), (args, r.returncode, r.stderr[-2000:])


def test_jni_shim_compiles():
    subprocess.run(["gcc", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter",
                    "-I", os.path.join(ROOT, "tests", "jni_compile"), "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "jni", "sparkbam_jni.c")], check=True)
