"""The whole-plane row path (rnt_kernels.hip k_row<..., WHOLE>) at
2^10 <= N <= 2^14: every (poly, limb) plane is one row, so rnt_mul is one
launch (3 planes of HBM traffic) and rnt_ntt_fwd / rnt_ntt_inv one launch
each, on u32 and u64 bases.  Bit-exact against the oracle on the BASELINE
configs' rings and the reference's own u64 shapes:

* config 2: N = 2^12, 4 x 31-bit primes (fwd/inv NTT + products);
* config 3: N = 2^14, 8 x 31-bit primes;
* examples/horner_chain.rs:61,73: N = 2^13, 7 x 61-bit primes;
* tests/integration_mul.rs:16-25: N = 2^10, 2 x 62-bit primes;
* 30-bit primes (the Harvey-lazy product arithmetic) and two odd sizes
  (2^11, 2^14 x 61-bit: one partial radix-16 pass, the largest u64 row).

Reference: poly.rs:307-329 (coefficient MulAssign), poly.rs:136-166
(to_ntt_domain / to_coeff_domain).  Every poly of each batch is compared
(first and last included); the products cover random, all-(q-1), zero and
negacyclic-monomial operands and both in-place forms.  RNT_PLANE=0 runs the
same checks through the four-step kernels, and the cross-path test feeds
one path's NTT-domain output to the other's inverse.
"""
from __future__ import annotations

import numpy as np
import pytest

import pyoracle as orc

pytestmark = pytest.mark.gpu

RINGS = [
    (12, 31, 4),  # config 2
    (14, 31, 8),  # config 3
    (13, 61, 7),  # horner_chain.rs
    (10, 62, 2),  # integration_mul.rs
    (12, 30, 4),  # 30-bit: lazy arithmetic
    (11, 31, 3),
    (14, 61, 3),
]


def _ctx(rn, mod, n, monkeypatch, plane):
    if plane is None:
        monkeypatch.delenv("RNT_PLANE", raising=False)
    else:
        monkeypatch.setenv("RNT_PLANE", plane)
    return rn.RnsBasis(mod, n)


def _operands(mod, n, seed):
    L = len(mod)
    rng = np.random.default_rng(seed)
    q = np.array(mod, dtype=np.uint64)[:, None]
    full = np.broadcast_to(q - 1, (L, n)).copy()
    mono = np.zeros((L, n), dtype=np.uint64)
    mono[:, n - 1] = 1
    r = orc.uniform_poly(mod, n, rng, batch=4)
    pairs = [(r[0], r[1]), (full, full), (full, r[2]), (np.zeros_like(full), r[3]), (mono, mono), (mono, r[1]),
             (r[2], r[3])]
    return pairs, orc.uniform_poly(mod, n, rng, batch=3)


@pytest.mark.parametrize("plane", [None, "0"])
@pytest.mark.parametrize("logn,bits,L", RINGS)
def test_product_matches_oracle(gpu, monkeypatch, logn, bits, L, plane):
    rn = gpu
    n = 1 << logn
    mod = rn.generate_primes(bits, L, n)
    Bd, Bo = _ctx(rn, mod, n, monkeypatch, plane), orc.Basis(mod, n)
    pairs, _ = _operands(mod, n, 1000 * logn + bits)
    a_h = np.stack([p[0] for p in pairs])
    b_h = np.stack([p[1] for p in pairs])
    want = [orc.mul(Bo, x, y) for x, y in pairs]
    a = rn.RnsPoly.from_channels(a_h, Bd)
    b = rn.RnsPoly.from_channels(b_h, Bd)
    got = (a * b).channels()
    for i in range(len(pairs)):
        assert np.array_equal(got[i], want[i]), i
    a *= b  # out aliases a
    assert np.array_equal(a.channels(), got)
    a2 = rn.RnsPoly.from_channels(a_h, Bd)
    b2 = rn.RnsPoly.from_channels(b_h, Bd)
    rn.check(rn.load().rnt_mul(b2.handle, a2.handle, b2.handle))  # out aliases b
    assert np.array_equal(b2.channels(), got)


@pytest.mark.parametrize("plane", [None, "0"])
@pytest.mark.parametrize("logn,bits,L", RINGS)
def test_transforms_match_oracle(gpu, monkeypatch, logn, bits, L, plane):
    rn = gpu
    n = 1 << logn
    mod = rn.generate_primes(bits, L, n)
    Bd, Bo = _ctx(rn, mod, n, monkeypatch, plane), orc.Basis(mod, n)
    pairs, x_h = _operands(mod, n, 7 * logn + bits)
    a_h = np.stack([p[0] for p in pairs])
    t = rn.RnsPoly.from_channels(a_h, Bd)
    t.to_ntt_domain()
    got = t.channels()
    for i in range(len(pairs)):
        assert np.array_equal(got[i], orc.to_ntt(Bo, a_h[i])), i
    t.to_coeff_domain()
    assert np.array_equal(t.channels(), a_h)
    # random NTT-domain uploads through the inverse
    u = rn.RnsPoly.from_channels(x_h, Bd, in_ntt_domain=True)
    u.to_coeff_domain()
    got = u.channels()
    for i in range(len(x_h)):
        assert np.array_equal(got[i], orc.to_coeff(Bo, x_h[i])), i


@pytest.mark.parametrize("logn,bits,L", [(12, 31, 4), (13, 61, 7), (14, 31, 8)])
def test_cross_path_device_order(gpu, monkeypatch, logn, bits, L):
    """One path's NTT-domain device words, as they lie in memory, through
    the other path's inverse (rnt_buf_wrap of the same storage in a second
    context): the whole-plane kernels and the four-step kernels keep the
    same bit-reversed device order, in both directions."""
    rn = gpu
    n = 1 << logn
    mod = rn.generate_primes(bits, L, n)
    Bo = orc.Basis(mod, n)
    pairs, _ = _operands(mod, n, 31 * logn + bits)
    a_h = np.stack([p[0] for p in pairs])
    Bw = _ctx(rn, mod, n, monkeypatch, None)
    B4 = _ctx(rn, mod, n, monkeypatch, "0")
    for fwd_ctx, inv_ctx in ((Bw, B4), (B4, Bw)):
        t = rn.RnsPoly.from_channels(a_h, fwd_ctx)
        t.to_ntt_domain()
        assert np.array_equal(t.channels()[-1], orc.to_ntt(Bo, a_h[-1]))
        fwd_ctx.sync()
        ptr, _ = t.device_ptr()
        u = rn.RnsPoly.wrap(inv_ctx, ptr, len(pairs), in_ntt_domain=True, owner=t)
        u.to_coeff_domain()
        inv_ctx.sync()
        assert np.array_equal(u.channels(), a_h)
