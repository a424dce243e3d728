import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.join(ROOT, "tests")
GOLDEN = os.path.join(TESTS, "golden")
BAMS = os.path.join(GOLDEN, "bams")
for p in (ROOT, TESTS):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C-ABI)")
    config.addinivalue_line("markers", "slow: larger CPU-side cases")


@pytest.fixture(scope="session")
def bams():
    return BAMS


def golden_bam(name):
    return os.path.join(BAMS, name)


def read_blocks(name):
    with open(os.path.join(BAMS, name + ".blocks")) as f:
        return [tuple(map(int, l.split(","))) for l in f if l.strip()]


def read_records(name):
    with open(os.path.join(BAMS, name + ".records")) as f:
        return [tuple(map(int, l.split(","))) for l in f if l.strip()]


def parse_total_error_counts(path):
    """'Total error counts:' section of a reference full-check output file."""
    out, on = {}, False
    with open(path, encoding="utf-8") as f:
        for line in f:
            if line.startswith("Total error counts:"):
                on = True
                continue
            if on:
                s = line.strip()
                if not s:
                    break
                k, v = s.split(":")
                out[k.strip()] = int(v.strip())
    return out
