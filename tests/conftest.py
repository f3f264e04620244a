"""Shared test setup.

- `gpu` marker: tests that need a real MI355X (run with `-m gpu`).
- oracle/ (the CPU restatement) is importable here: tests use it as the checker.
- the product package lives in huff-encoding_amd/ (hyphenated dir, so it is
  put on sys.path rather than imported as a dotted path).
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "huff-encoding_amd")
ORACLE = os.path.join(ROOT, "oracle")
for p in (PKG, ORACLE, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")


def _ensure_built():
    """`make` is incremental: always run it, so a test never loads a library
    older than its sources (a pushed tree without build/ rebuilds from
    scratch, which takes ~30 s)"""
    subprocess.run(["make", "-s", "-C", PKG, "-j8"], check=True)
    subprocess.run(["make", "-s", "-C", ORACLE], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def O():
    import oracle

    return oracle


@pytest.fixture(scope="session")
def H():
    import huff_coding

    return huff_coding


@pytest.fixture(scope="session")
def golden():
    import json

    d = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(d, "reference_pinned.json")) as f:
        pinned = json.load(f)
    with open(os.path.join(d, "derived.json")) as f:
        derived = json.load(f)
    return pinned, derived


@pytest.fixture(scope="session")
def ctx(H):
    """the GPU context (gpu tests only)"""
    return H.Context(0)
