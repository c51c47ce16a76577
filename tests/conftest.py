"""Shared test set-up.

-m "not gpu": oracle vs the reference-pinned goldens, host logic (rtc parser,
OBJ loader, kd build == oracle kd build), C-ABI library loading / exports, and
the multi-rank tile protocol on gloo.  -m gpu: parity of the HIP path against
the oracle, through the C-ABI (libchiaro_hip.so).
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "chiaroscuro-raytracer_amd"
for p in (str(PKG), str(ROOT / "oracle"), str(ROOT / "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)
os.environ.setdefault("CHIARO_QUIET", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libchiaro_hip.so)")
    config.addinivalue_line("markers", "slow: full-size scene (several seconds on CPU)")


def _ensure_built():
    """The libraries under test are the ones built from this tree's sources: `make -q`
    asks whether any target is older than its sources (a no-op check when the
    pushed binaries are current) and only then rebuilds incrementally."""
    for d, jobs in ((PKG, "-j8"), (ROOT / "oracle", "-j1")):
        if subprocess.run(["make", "-q", "-C", str(d)], stdout=subprocess.DEVNULL).returncode != 0:
            sys.stderr.write("conftest: %s is stale or unbuilt; running make\n" % d)
            subprocess.run(["make", "-s", jobs, "-C", str(d)], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def ca():
    import chiaroscuro_amd
    return chiaroscuro_amd


@pytest.fixture(scope="session")
def po():
    import pyoracle
    return pyoracle


@pytest.fixture(scope="session")
def scenes():
    from chiaroscuro_amd import scenes as s
    return s
