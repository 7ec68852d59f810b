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


KS_RINGS = [(10, 31, 2), (11, 31, 3), (12, 31, 4), (12, 30, 4), (13, 31, 5), (14, 31, 8)]


@pytest.mark.parametrize("plane", [None, "0"])
@pytest.mark.parametrize("logn,bits,L", KS_RINGS)
def test_keyswitch_matches_oracle(gpu, monkeypatch, logn, bits, L, plane):
    """The whole-plane key-switch (k_ks_whole: one workgroup per row block
    and target limb forward-transforms each source limb in registers and
    accumulates both gadget sums, no S in HBM) against the oracle's gadget
    sum (engine.rs:505-528), every poly of the batch, including an
    all-(q-1) input; keyswitch_ext over a limb shard of the targets; the
    relinearised ct-mul, whose key-switch adds the tensor's d0/d1 in its
    epilogue.  RNT_PLANE=0 runs the same checks through the four-step
    key-switch (S, k_ks_rows, k_colt_inv); at 2^14 both runs take the
    four-step kernels (ks_whole_ok: N <= 2^13)."""
    rn = gpu
    n = 1 << logn
    mod = rn.generate_primes(bits, L, n)
    Bd, Bo = _ctx(rn, mod, n, monkeypatch, plane), orc.Basis(mod, n)
    rng = np.random.default_rng(77 * logn + bits)
    q = np.array(mod, dtype=np.uint64)[:, None]
    d = orc.uniform_poly(mod, n, rng, batch=3)
    d[1] = np.broadcast_to(q - 1, (L, n))
    ka, kb = orc.uniform_poly(mod, n, rng, batch=L), orc.uniform_poly(mod, n, rng, batch=L)
    key = rn.RnsGadgetKey.from_channels(ka, kb, Bd)
    a0, a1 = rn.keyswitch(rn.RnsPoly.from_channels(d, Bd), key)
    g0, g1 = a0.channels(), a1.channels()
    want = [orc.keyswitch(Bo, d[p], ka, kb) for p in range(3)]
    for p in range(3):
        assert np.array_equal(g0[p], want[p][0]) and np.array_equal(g1[p], want[p][1]), p
    Lt = max(1, L - 1)
    Bt = rn.RnsBasis(mod[:Lt], n)
    key_t = rn.RnsGadgetKey.from_channels(np.ascontiguousarray(ka[:, :Lt]), np.ascontiguousarray(kb[:, :Lt]), Bt)
    src = rn.RnsPoly.from_channels(d, Bd)
    ptr, _ = src.device_ptr()
    e0, e1 = rn.keyswitch_ext(ptr, L, key_t, Bt, 3)
    h0, h1 = e0.channels(), e1.channels()
    for p in range(3):
        assert np.array_equal(h0[p], want[p][0][:Lt]) and np.array_equal(h1[p], want[p][1][:Lt]), p
    c = orc.uniform_poly(mod, n, rng, batch=4)
    up = lambda x: rn.RnsPoly.from_channels(x[None], Bd)  # noqa: E731
    out = rn.mul_ciphertexts_gadget(rn.Ciphertext(up(c[0]), up(c[1])), rn.Ciphertext(up(c[2]), up(c[3])), key)
    w0, w1 = orc.mul_ciphertexts_gadget(Bo, c[0], c[1], c[2], c[3], ka, kb)
    assert np.array_equal(out.c0.channels()[0], w0) and np.array_equal(out.c1.channels()[0], w1)


@pytest.mark.parametrize("logn,bits,L", [(10, 31, 2), (12, 31, 4), (12, 61, 3), (13, 31, 5), (13, 31, 8)])
def test_tensor_matches_four_step_and_oracle(gpu, monkeypatch, logn, bits, L):
    """The whole-plane tensor (k_tensor_rows<..., WHOLE>, engine.rs:480-493):
    d2 = c1 c1' in coefficient domain against the oracle's product; the
    NTT-resident key-switch seeds d0^, d1^ (Montgomery-scaled, as the
    key-switch sums they seed) word for word equal to the four-step tensor's
    (RNT_PLANE=0), every poly of the batch.  A 1 MiB key-switch workspace
    (RNT_KS_WS_MB=1) at 2^12 x 4 runs the relinearised ct-mul one ciphertext a
    chunk: the tensor reads the ciphertexts at their full limb stride and
    writes chunk-local planes."""
    rn = gpu
    n = 1 << logn
    mod = rn.generate_primes(bits, L, n)
    Bo = orc.Basis(mod, n)
    rng = np.random.default_rng(5 * logn + bits)
    B = 3
    c = [orc.uniform_poly(mod, n, rng, batch=B) for _ in range(4)]
    q = np.array(mod, dtype=np.uint64)[:, None]
    c[1][2] = np.broadcast_to(q - 1, (L, n))
    c[3][2] = np.broadcast_to(q - 1, (L, n))
    outs = {}
    for plane in (None, "0"):
        Bd = _ctx(rn, mod, n, monkeypatch, plane)
        d = rn.ct_tensor(*(rn.RnsPoly.from_channels(x, Bd) for x in c))
        outs[plane] = [x.channels() for x in d]
    for p in range(B):
        assert np.array_equal(outs[None][2][p], orc.mul(Bo, c[1][p], c[3][p])), p
    for i in range(3):
        assert np.array_equal(outs[None][i], outs["0"][i]), i
    if (logn, bits, L) == (12, 31, 4):
        monkeypatch.setenv("RNT_KS_WS_MB", "1")
        Bd = _ctx(rn, mod, n, monkeypatch, None)
        ka, kb = orc.uniform_poly(mod, n, rng, batch=L), orc.uniform_poly(mod, n, rng, batch=L)
        key = rn.RnsGadgetKey.from_channels(ka, kb, Bd)
        up = lambda x: rn.RnsPoly.from_channels(x, Bd)  # noqa: E731
        big = [np.concatenate([x] * 40) for x in c]  # 120 cts: > 1 MiB of D0..D2
        out = rn.mul_ciphertexts_gadget(rn.Ciphertext(up(big[0]), up(big[1])),
                                        rn.Ciphertext(up(big[2]), up(big[3])), key)
        o0, o1 = out.c0.channels(), out.c1.channels()
        for p in (0, 2, 118, 119):
            w0, w1 = orc.mul_ciphertexts_gadget(Bo, big[0][p], big[1][p], big[2][p], big[3][p], ka, kb)
            assert np.array_equal(o0[p], w0) and np.array_equal(o1[p], w1), p
