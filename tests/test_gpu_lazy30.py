"""The Harvey-lazy product path for 30-bit bases (rnt_modarith.hpp Mod30;
k_colt_fwd / k_row<2> / k_colt_inv with LZ = true), bit-exact against the
oracle (MulAssign, poly.rs:277-331).

The lazy path keeps forward values in [0, 4q) and inverse values in
[0, 2q), so the cases stress the bounds: uniform residues, all q - 1
(every sum at its maximum), all zero, and single monomials, at every ring
size that takes the tiled column path (N >= 2^10) up to 2^17.  A basis with
one 31-bit prime must fall back to the canonical path and stay exact.
"""
from __future__ import annotations

import numpy as np
import pytest

import pyoracle as orc

pytestmark = pytest.mark.gpu


def _check(rn, mods, n, a, b, sample=None):
    B = rn.RnsBasis(mods, n)
    got = (rn.RnsPoly.from_channels(a, B) * rn.RnsPoly.from_channels(b, B)).channels()
    if got.ndim == 2:
        got = got[None]
    ob = orc.Basis(mods, n)
    for p in (range(a.shape[0]) if sample is None else sample):
        assert np.array_equal(got[p], orc.mul(ob, a[p], b[p])), p


@pytest.mark.parametrize("log_n,L", [(10, 3), (11, 2), (12, 4), (13, 3), (14, 2), (16, 4), (17, 2)])
def test_lazy30_product_matches_oracle(gpu, log_n, L):
    rn = gpu
    n = 1 << log_n
    mods = rn.generate_primes(30, L, n)
    assert max(mods) < (1 << 30)
    rng = np.random.default_rng(log_n)
    B = 3 if log_n <= 14 else 2
    a = orc.uniform_poly(mods, n, rng, batch=B)
    b = orc.uniform_poly(mods, n, rng, batch=B)
    # pair 1: every residue q - 1 (the largest sums the lazy bounds allow)
    qm1 = np.array(mods, dtype=np.uint64)[:, None] - np.uint64(1)
    a[1] = qm1
    b[1] = qm1
    _check(rn, mods, n, a, b, sample=None if log_n <= 14 else [0, 1])


def test_lazy30_edge_polys(gpu):
    rn = gpu
    n = 1 << 12
    mods = rn.generate_primes(30, 3, n)
    L = len(mods)
    z = np.zeros((2, L, n), dtype=np.uint64)
    one = z.copy()
    one[:, :, 0] = 1
    xn = z.copy()
    xn[:, :, n - 1] = 1  # X^(N-1) * X^(N-1) = -X^(N-2)
    _check(rn, mods, n, z.copy(), one.copy())
    _check(rn, mods, n, one.copy(), one.copy())
    _check(rn, mods, n, xn.copy(), xn.copy())


def test_mixed_basis_falls_back_to_canonical(gpu):
    """One 31-bit prime disables the lazy path for the whole basis."""
    rn = gpu
    n = 1 << 12
    mods = rn.generate_primes(30, 2, n) + rn.generate_primes(31, 1, n)
    rng = np.random.default_rng(5)
    a = orc.uniform_poly(mods, n, rng, batch=2)
    b = orc.uniform_poly(mods, n, rng, batch=2)
    _check(rn, mods, n, a, b)
