"""The Harvey-lazy product path for u64 bases of primes below 2^62
(rnt_modarith.hpp Mod62; k_colt_fwd / k_row<2> / k_colt_inv and the
whole-plane k_row<2, WHOLE> with LZ = true on 64-bit words), bit-exact
against the oracle (MulAssign, poly.rs:277-331).

The lazy ranges are forward values in [0, 4q) and inverse values in
[0, 2q), which need 4q < 2^64: the cases take the largest primes that
qualify (62-bit, just under 2^62, the reference's integration_mul.rs
width), the horner_chain.rs 61-bit shape and 40-bit primes, with uniform,
all-(q - 1), zero and monomial operands, on the whole-plane (2^10..2^14)
and four-step (2^15..2^17) products.  A basis with one 63-bit prime must
take the canonical kernels and stay exact; RNT_LAZY62=0 likewise.
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


@pytest.mark.parametrize("bits,log_n,L", [(62, 10, 2), (62, 12, 2), (61, 13, 7), (62, 14, 2), (40, 13, 3),
                                          (62, 15, 2), (62, 16, 3), (61, 17, 2)])
def test_lazy62_product_matches_oracle(gpu, bits, log_n, L):
    rn = gpu
    n = 1 << log_n
    mods = rn.generate_primes(bits, L, n)
    assert max(mods) < (1 << 62)
    rng = np.random.default_rng(62 * log_n + bits)
    B = 3 if log_n <= 14 else 2
    a = orc.uniform_poly(mods, n, rng, batch=B)
    b = orc.uniform_poly(mods, n, rng, batch=B)
    # pair 1: every residue q - 1 (the largest sums the lazy bounds allow)
    qm1 = np.array(mods, dtype=np.uint64)[:, None] - np.uint64(1)
    a[1] = qm1
    b[1] = qm1
    _check(rn, mods, n, a, b, sample=None if log_n <= 14 else [0, 1])


@pytest.mark.parametrize("log_n", [12, 16])
def test_lazy62_edge_polys(gpu, log_n):
    rn = gpu
    n = 1 << log_n
    mods = rn.generate_primes(62, 2, n)
    L = len(mods)
    z = np.zeros((2, L, n), dtype=np.uint64)
    one = z.copy()
    one[:, :, 0] = 1
    xn = z.copy()
    xn[:, :, n - 1] = 1  # X^(N-1) * X^(N-1) = -X^(N-2)
    _check(rn, mods, n, z.copy(), one.copy())
    _check(rn, mods, n, one.copy(), one.copy())
    _check(rn, mods, n, xn.copy(), xn.copy())


@pytest.mark.parametrize("log_n", [13, 16])
def test_lazy62_canonical_fallbacks(gpu, monkeypatch, log_n):
    """One 63-bit prime keeps the whole basis on the canonical kernels, and
    RNT_LAZY62=0 does the same for a 62-bit basis: both exact."""
    rn = gpu
    n = 1 << log_n
    rng = np.random.default_rng(63 + log_n)
    mods = rn.generate_primes(62, 1, n) + rn.generate_primes(63, 1, n)
    a = orc.uniform_poly(mods, n, rng, batch=2)
    b = orc.uniform_poly(mods, n, rng, batch=2)
    _check(rn, mods, n, a, b)
    monkeypatch.setenv("RNT_LAZY62", "0")
    mods = rn.generate_primes(62, 2, n)
    a = orc.uniform_poly(mods, n, rng, batch=2)
    b = orc.uniform_poly(mods, n, rng, batch=2)
    _check(rn, mods, n, a, b)
