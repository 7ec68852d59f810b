"""The default N = 2^16 transform path (k_mf_ntt, the MFMA whole-plane
transforms: rnt_ntt_fwd / rnt_ntt_inv and every NTT-domain op that runs
through them) against the oracle on random operands, at the metric's ring
(N = 2^16, L = 16 x 31-bit), in the default mode and with RNT_PLANE=0
(four-step kernels).

Reference: to_ntt_domain / to_coeff_domain (poly.rs:136-166), the
NTT-domain MulAssign branch (poly.rs:297-306), rescale_into from the NTT
domain (poly.rs:187-228) and automorphism of NTT-domain input
(poly.rs:492-569).  Every poly of a batch of B = 4 is compared (the first
and last of the batch included), so a poly-offset or layout error shared by
the forward and inverse kernels cannot hide behind a round trip.  The
cross-path tests feed one path's NTT-domain output to the other path's
inverse (both contexts use the device's bit-reversed order).
"""
from __future__ import annotations

import numpy as np
import pytest

import pyoracle as orc

pytestmark = pytest.mark.gpu

N, L, B = 1 << 16, 16, 4


@pytest.fixture(scope="module")
def ring(gpu):
    rn = gpu
    mod = rn.generate_primes(31, L, N)
    Bo = orc.Basis(mod, N)
    rng = np.random.default_rng(0x2_0016)
    a_h = orc.uniform_poly(mod, N, rng, batch=B)
    b_h = orc.uniform_poly(mod, N, rng, batch=B)
    # NTT-domain operands drawn directly (random natural-order evaluations)
    x_h = orc.uniform_poly(mod, N, rng, batch=B)
    y_h = orc.uniform_poly(mod, N, rng, batch=B)
    want = {
        "fwd": [orc.to_ntt(Bo, a_h[i]) for i in range(B)],
        "inv": [orc.to_coeff(Bo, x_h[i]) for i in range(B)],
        "nmul": [orc.mul(Bo, x_h[i], y_h[i], ntt=True) for i in range(B)],
        "rescale": [orc.rescale(Bo, x_h[i], in_ntt=True) for i in range(B)],
    }
    return rn, mod, Bo, a_h, b_h, x_h, y_h, want


def _basis(rn, mod, monkeypatch, plane):
    if plane is not None:
        monkeypatch.setenv("RNT_PLANE", plane)
    else:
        monkeypatch.delenv("RNT_PLANE", raising=False)
    return rn.RnsBasis(mod, N)


@pytest.mark.parametrize("plane", [None, "0"])
def test_forward_random_batch(ring, monkeypatch, plane):
    rn, mod, Bo, a_h, _, _, _, want = ring
    Bd = _basis(rn, mod, monkeypatch, plane)
    t = rn.RnsPoly.from_channels(a_h, Bd)
    t.to_ntt_domain()
    assert t.is_ntt_domain()
    got = t.channels()
    for i in range(B):
        assert np.array_equal(got[i], want["fwd"][i]), i


@pytest.mark.parametrize("plane", [None, "0"])
def test_inverse_random_ntt_upload(ring, monkeypatch, plane):
    rn, mod, Bo, _, _, x_h, _, want = ring
    Bd = _basis(rn, mod, monkeypatch, plane)
    t = rn.RnsPoly.from_channels(x_h, Bd, in_ntt_domain=True)
    # natural-order NTT-domain upload / download is the identity on the host view
    assert np.array_equal(t.channels(), x_h)
    t.to_coeff_domain()
    assert not t.is_ntt_domain()
    got = t.channels()
    for i in range(B):
        assert np.array_equal(got[i], want["inv"][i]), i


@pytest.mark.parametrize("plane", [None, "0"])
def test_ntt_domain_mul_assign(ring, monkeypatch, plane):
    rn, mod, Bo, _, _, x_h, y_h, want = ring
    Bd = _basis(rn, mod, monkeypatch, plane)
    x = rn.RnsPoly.from_channels(x_h, Bd, in_ntt_domain=True)
    y = rn.RnsPoly.from_channels(y_h, Bd, in_ntt_domain=True)
    z = x * y
    assert z.is_ntt_domain()
    got = z.channels()
    for i in range(B):
        assert np.array_equal(got[i], want["nmul"][i]), i
    x *= y  # in place
    assert np.array_equal(x.channels(), got)


@pytest.mark.parametrize("plane", [None, "0"])
def test_rescale_and_automorphism_from_ntt(ring, monkeypatch, plane):
    rn, mod, Bo, _, _, x_h, _, want = ring
    Bd = _basis(rn, mod, monkeypatch, plane)
    x = rn.RnsPoly.from_channels(x_h, Bd, in_ntt_domain=True)
    r = x.rescale().channels()
    for i in range(B):
        assert np.array_equal(r[i], want["rescale"][i]), i
    for g in (5, 2 * N - 1, 6):
        out = x.automorphism(g)
        got = out.channels()
        for i in (0, B - 1):
            w, f = orc.automorphism(Bo, x_h[i], g, in_ntt=True)
            assert np.array_equal(got[i], w), (g, i)
            assert out.is_ntt_domain() == f


def test_cross_path_forward_inverse(ring, monkeypatch):
    """Four-step forward output through the whole-plane inverse and the other
    way round, and both forwards equal on the device order (downloaded
    through the same natural-order permutation)."""
    rn, mod, Bo, a_h, _, _, _, want = ring
    B0 = _basis(rn, mod, monkeypatch, "0")
    B3 = _basis(rn, mod, monkeypatch, None)
    for src, dst in ((B0, B3), (B3, B0)):
        t = rn.RnsPoly.from_channels(a_h, src)
        t.to_ntt_domain()
        nt = t.channels()
        for i in range(B):
            assert np.array_equal(nt[i], want["fwd"][i]), i
        u = rn.RnsPoly.from_channels(nt, dst, in_ntt_domain=True)
        u.to_coeff_domain()
        assert np.array_equal(u.channels(), a_h)


def test_mf_tensor_matches_four_step_and_oracle(ring, monkeypatch):
    """The matrix-core tensor (k_mf_tensor, engine.rs:480-493) at the
    metric's ring: d2 = c1 c1' (coefficient domain) against the oracle for
    every poly of the batch, and the NTT-resident key-switch seeds d0^, d1^
    word for word equal to the four-step tensor's (RNT_PLANE=0), including an
    all-(q-1) ciphertext."""
    rn, mod, Bo, a_h, b_h, x_h, y_h, _ = ring
    q = np.array(mod, dtype=np.uint64)[:, None]
    c = [a_h.copy(), b_h.copy(), x_h.copy(), y_h.copy()]
    c[1][B - 1] = np.broadcast_to(q - 1, (L, N))
    c[3][B - 1] = np.broadcast_to(q - 1, (L, N))
    outs = {}
    for plane in (None, "0"):
        Bd = _basis(rn, mod, monkeypatch, plane)
        d = rn.ct_tensor(*(rn.RnsPoly.from_channels(x, Bd) for x in c))
        outs[plane] = [x.channels() for x in d]
    for p in range(B):
        assert np.array_equal(outs[None][2][p], orc.mul(Bo, c[1][p], c[3][p])), p
    for i in range(3):
        assert np.array_equal(outs[None][i], outs["0"][i]), i


def _seeds_want(Bo, mod, c0, c1, c0p, c1p):
    """Oracle d0^, d1^ (NTT domain, times 2^-32 as the device's seeds) and d2."""
    q = np.array(mod, dtype=object)[:, None]
    rinv = np.array([pow(2, -32, int(x)) for x in mod], dtype=object)[:, None]
    d0 = orc.to_ntt(Bo, orc.mul(Bo, c0, c0p))
    d1 = orc.to_ntt(Bo, orc.add(Bo, orc.mul(Bo, c0, c1p), orc.mul(Bo, c1, c0p)))
    scale = lambda x: ((x.astype(object) * rinv) % q).astype(np.uint64)  # noqa: E731
    return scale(d0), scale(d1), orc.mul(Bo, c1, c1p)


def test_mf_tensor_slot_scratch_batch(ring, monkeypatch):
    """128 ciphertexts x 16 limbs = 2048 (poly, limb) pairs: the tensor's c1^
    temporary goes to the CU-indexed scratch slots (kPlaneSlots).  Sampled
    ciphertexts' d0^, d1^ (Montgomery-scaled NTT-domain seeds) and d2 against
    the oracle, on both paths."""
    rn, mod, Bo, *_ = ring
    Bc = 128
    picks = (0, 1, 63, 64, 127)
    for plane in (None, "0"):
        Bd = _basis(rn, mod, monkeypatch, plane)
        drng = rn.DeviceRng(128)
        c = [rn.RnsPoly.sample_uniform(Bd, drng, Bc) for _ in range(4)]
        d = rn.ct_tensor(*c)
        for p in picks:
            ch = [x.channels_of(p)[0] for x in c]
            want = _seeds_want(Bo, mod, *ch)
            for i in range(3):
                assert np.array_equal(d[i].channels_of(p)[0], want[i]), (plane, i, p)


@pytest.mark.parametrize("Bc", [32, 128])
def test_mf_tensor_full_output(ring, monkeypatch, Bc):
    """Every word of d0^, d1^ and d2 equal to the four-step tensor's, for 32
    ciphertexts (512 (poly, limb) pairs: c1^ in the pairs' own scratch
    planes) and 128 (2048 pairs: the CU-indexed scratch slots, kPlaneSlots).
    The check that caught r04's MFMA hazard (16-300 wrong words per 2^26
    before the tiles were made hazard-free by construction, DESIGN.md §3
    "MFMA hazards")."""
    rn, mod, *_ = ring
    outs = {}
    for plane in (None, "0"):
        Bd = _basis(rn, mod, monkeypatch, plane)
        drng = rn.DeviceRng(4242 + Bc)
        c = [rn.RnsPoly.sample_uniform(Bd, drng, Bc) for _ in range(4)]
        outs[plane] = rn.ct_tensor(*c)
    for i in range(3):
        a, b = outs[None][i].channels_batch(), outs["0"][i].channels_batch()
        bad = int((a != b).sum())
        assert bad == 0, (i, bad)
        del a, b


def test_mf_ntt_full_output_1024_planes(ring, monkeypatch):
    """k_mf_ntt forward and inverse, every word of 64 polys x 16 limbs = 1024
    planes against the four-step kernels (RNT_PLANE=0) on the same
    device-drawn data: the forward on coefficient-domain input, the inverse
    on the same words taken as NTT-domain input (device order), and
    inverse(forward) = identity on the default path."""
    rn, mod, *_ = ring
    Bp = 64
    fwd, inv, x0 = {}, {}, None
    for plane in (None, "0"):
        Bd = _basis(rn, mod, monkeypatch, plane)
        x = rn.RnsPoly.sample_uniform(Bd, rn.DeviceRng(0x1024), Bp)
        if plane is None:
            x0 = x.channels_batch()
        x.to_ntt_domain()
        fwd[plane] = x.channels_batch()
        if plane is None:
            x.to_coeff_domain()
            back = x.channels_batch()
            assert int((back != x0).sum()) == 0
            del back
        del x
        # the same sampled words as NTT-domain input: a fresh draw, relabelled
        y = rn.RnsPoly.sample_uniform(Bd, rn.DeviceRng(0x1025), Bp)
        z = rn.RnsPoly.wrap(Bd, y.device_ptr()[0], Bp, in_ntt_domain=True)
        z.to_coeff_domain()
        inv[plane] = y.channels_batch()
        del z, y
    bad_f = int((fwd[None] != fwd["0"]).sum())
    bad_i = int((inv[None] != inv["0"]).sum())
    assert bad_f == 0 and bad_i == 0, (bad_f, bad_i)
