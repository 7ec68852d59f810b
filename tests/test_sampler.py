"""Device-sampler restatement (oracle/sampler.py) pinned on CPU.

* Philox4x32-10 against the Random123 known-answer vectors
  (kat_vectors: philox4x32_10 for zero, all-ones and pi-digit inputs).
* The three samplers against the reference's own statistical sampler tests
  (math/sampling.rs:98-242, poly.rs:841-851, 978-987): ranges, balance,
  mean/variance, exact Hamming weight including the extremes.
"""
from __future__ import annotations

import numpy as np
import pytest

import sampler as smp

KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,want", KAT)
def test_philox_known_answers(ctr, key, want):
    got = smp.philox(*[np.array([c], dtype=np.uint64) for c in ctr], *key)
    assert tuple(int(x[0]) for x in got) == want


def test_uniform_in_range_and_balanced():
    """sampling.rs:98-135 / poly.rs:841-851: every residue < q; roughly balanced."""
    mods = [17, 97, 2147483137, (1 << 61) - 1]
    u = smp.uniform(mods, 1024, 2, seed=5, stream=0)
    for li, q in enumerate(mods):
        assert np.all(u[:, li] < np.uint64(q))
    big = u[:, 2].astype(np.float64) / 2147483137
    assert abs(big.mean() - 0.5) < 0.03
    # two streams differ, the same stream repeats
    assert not np.array_equal(u, smp.uniform(mods, 1024, 2, seed=5, stream=1))
    assert np.array_equal(u, smp.uniform(mods, 1024, 2, seed=5, stream=0))


def test_gaussian_mean_and_variance():
    """sampling.rs:172-205: mean near 0, variance near sigma^2."""
    sigma = 3.2
    e = smp.gaussian_ints(4096, 4, sigma, seed=11, stream=2).astype(np.float64)
    assert abs(e.mean()) < 0.1
    assert abs(e.var() - (sigma ** 2 + 1 / 12)) < 0.6  # rounding adds ~1/12
    assert np.abs(e).max() < 10 * sigma


@pytest.mark.parametrize("h", [0, 1, 3, 32, 64])
def test_ternary_exact_hamming_weight(h):
    """sampling.rs:210-238 / poly.rs:978-987, including the extremes."""
    t = smp.ternary_ints(64, 3, h, seed=3, stream=4)
    assert np.all(np.isin(t, [-1, 0, 1]))
    assert all(int(np.count_nonzero(row)) == h for row in t)


def test_ternary_signs_and_positions_are_spread():
    t = smp.ternary_ints(4096, 2, 2048, seed=9, stream=0)
    nz = t[t != 0]
    assert abs(nz.mean()) < 0.1
    assert 900 < np.count_nonzero(t[0, :2048]) < 1150  # positions not clustered
