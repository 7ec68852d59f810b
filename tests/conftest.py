"""Shared pytest setup.

* ``-m gpu`` tests need an MI355X (run via gpurun); everything else runs on
  CPU.  The oracle (oracle/) is imported only here in tests, as the checker.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "toy-heaan-ckks_amd")
for p in (REPO, PKG, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def kats():
    with open(os.path.join(GOLDEN, "reference_kats.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def vectors():
    return np.load(os.path.join(GOLDEN, "vectors.npz"))


@pytest.fixture(scope="session")
def manifest():
    with open(os.path.join(GOLDEN, "vectors_manifest.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def gpu():
    """Skip unless a GPU is visible; returns the rns_ntt module."""
    import rns_ntt

    rns_ntt.load()
    if not os.path.exists("/dev/kfd"):
        pytest.skip("no GPU on this host")
    # on a GPU host the HIP path must run: never skip silently
    assert rns_ntt.device_count() > 0, "a GPU host without a visible HIP device"
    return rns_ntt
