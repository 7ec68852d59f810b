"""GPU parity: the HIP backend (through the C-ABI, via the rns_ntt mirror)
against the CPU oracle, the reference's KATs and the committed big-integer
vectors.  Bit-exact everywhere: this path is integer arithmetic only."""
from __future__ import annotations

import numpy as np
import pytest

import pyoracle as orc

pytestmark = pytest.mark.gpu


def _basis(rn, moduli, n):
    return rn.RnsBasis(moduli, n), orc.Basis(moduli, n)


# --------------------------------------------------------------------------
# reference KATs (poly.rs / basis.rs #[test] blocks, N = 8)
# --------------------------------------------------------------------------


def test_reference_poly_kats(gpu, kats):
    rn = gpu
    k = kats["poly_n8"]
    B2 = rn.RnsBasis([17, 97], 8)
    B3 = rn.RnsBasis([17, 97, 113], 8)

    c = k["from_coeffs_reduces_correctly"]
    ch = rn.RnsPoly.from_coeffs(c["coeffs"], B2).channels()
    for i, j, v in c["expect"]:
        assert ch[i, j] == v
    with pytest.raises(rn.RnsNttError) as e:
        rn.RnsPoly.from_channels(k["from_channels_rejects_unreduced_coefficient"]["channels"], B2)
    assert e.value.kind == "NonReducedCoefficient"
    with pytest.raises(rn.RnsNttError) as e:
        rn.RnsPoly.from_channels(k["from_channels_rejects_wrong_channel_count"]["channels"], B2)
    assert e.value.kind == "ChannelCountMismatch"

    c = k["ntt_roundtrip_preserves_coefficients"]
    p = rn.RnsPoly.from_coeffs(c["coeffs"], B2)
    orig = p.channels()
    p.to_ntt_domain()
    assert p.is_ntt_domain()
    p.to_coeff_domain()
    assert not p.is_ntt_domain()
    assert np.array_equal(p.channels(), orig)

    c = k["to_ntt_is_idempotent"]
    p = rn.RnsPoly.from_coeffs(c["coeffs"], B2)
    p.to_ntt_domain()
    first = p.channels()
    p.to_ntt_domain()
    assert np.array_equal(p.channels(), first)

    c = k["mod_drop_removes_last_channels"]
    d = rn.RnsPoly.from_coeffs(c["coeffs"], B3).mod_drop_last(c["drop"])
    assert d.basis.channel_count() == c["expect_channels"] and d.channels().shape[0] == 2

    c = k["add_assign_computes_correct_sum"]
    a = rn.RnsPoly.from_coeffs(c["a"], B2)
    a += rn.RnsPoly.from_coeffs(c["b"], B2)
    assert (a.channels() == c["expect_all"]).all()
    c = k["add_assign_wraps_at_modulus"]
    a = rn.RnsPoly.from_coeffs(c["a"], B2)
    a += rn.RnsPoly.from_coeffs(c["b"], B2)
    assert a.channels()[0, 0] == 1
    c = k["neg_negates_coefficients"]
    n = -rn.RnsPoly.from_coeffs(c["a"], B2)
    assert n.channels()[0, 0] == 14 and n.channels()[0, 1] == 0

    for name in ("mul_assign_schoolbook_small", "mul_assign_wraps_around_quotient"):
        c = k[name]
        a = rn.RnsPoly.from_coeffs(c["a"], B2)
        a *= rn.RnsPoly.from_coeffs(c["b"], B2)
        assert list(a.to_coeffs()) == c["expect_coeffs"], name

    c = k["to_coeffs_roundtrips_from_coeffs"]
    assert list(rn.RnsPoly.from_coeffs(c["coeffs"], B2).to_coeffs()) == c["coeffs"]
    c = k["to_coeffs_works_from_ntt_domain"]
    p = rn.RnsPoly.from_coeffs(c["coeffs"], B2)
    p.to_ntt_domain()
    assert list(p.to_coeffs()) == c["coeffs"] and p.is_ntt_domain()

    c = k["mul_assign_ntt_domain_matches_coeff_domain"]
    a = rn.RnsPoly.from_coeffs(c["a"], B2)
    a *= rn.RnsPoly.from_coeffs(c["b"], B2)
    expected = a.to_coeffs()
    an, bn = rn.RnsPoly.from_coeffs(c["a"], B2), rn.RnsPoly.from_coeffs(c["b"], B2)
    an.to_ntt_domain()
    bn.to_ntt_domain()
    an *= bn
    assert an.is_ntt_domain()
    assert np.array_equal(an.to_coeffs(), expected)

    c = k["automorphism_identity_preserves_coefficients"]
    p = rn.RnsPoly.from_coeffs(c["coeffs"], B2)
    for g in c["exponents"]:
        assert list(p.automorphism(g).to_coeffs()) == c["coeffs"]
    c = k["automorphism_applies_sign_change_correctly"]
    r = rn.RnsPoly.from_coeffs(c["coeffs"], B2).automorphism(c["exponent"]).to_coeffs()
    assert list(r) == c["expect_coeffs"]
    for name in ("rotate_slots_works_for_simple_case", "rotate_slots_negative_uses_conjugate"):
        c = k[name]
        assert len(rn.RnsPoly.from_coeffs(c["coeffs"], B2).rotate_slots(c["k"]).to_coeffs()) == 8
    c = k["automorphism_preserves_ntt_domain_flag"]
    p = rn.RnsPoly.from_coeffs(c["coeffs"], B2)
    p.to_ntt_domain()
    assert p.automorphism(c["exponent"]).is_ntt_domain() == c["expect_ntt"]

    c = k["mul_assign_matches_naive"]
    Bo = orc.Basis([17, 97], 8)
    a = rn.RnsPoly.from_coeffs(c["a"], B2)
    a *= rn.RnsPoly.from_coeffs(c["b"], B2)
    naive = orc.mul_naive(Bo, orc.from_coeffs(Bo, c["a"]), orc.from_coeffs(Bo, c["b"]))
    assert np.array_equal(a.channels(), naive)

    c = k["rescale_drops_channel_count"]
    r = rn.RnsPoly.from_coeffs(c["coeffs"], B3).rescale()
    assert r.basis.channel_count() == 2 and not r.is_ntt_domain()
    with pytest.raises(rn.RnsNttError) as e:
        rn.RnsPoly.from_coeffs(c["coeffs"], rn.RnsBasis([17], 8)).rescale()
    assert e.value.kind == "InvalidModDrop"
    c = k["rescale_is_exact_division_by_last_prime"]
    assert list(rn.RnsPoly.from_coeffs(c["coeffs"], B3).rescale().to_coeffs()) == c["expect_coeffs"]
    c = k["rescale_from_ntt_domain_matches_coeff_domain"]
    want = rn.RnsPoly.from_coeffs(c["coeffs"], B3).rescale().to_coeffs()
    p = rn.RnsPoly.from_coeffs(c["coeffs"], B3)
    p.to_ntt_domain()
    assert np.array_equal(p.rescale().to_coeffs(), want)


def test_reference_basis_kats(gpu, kats):
    rn = gpu
    k = kats["basis_n8"]
    b = rn.RnsBasis([17, 97, 113], 8)
    assert b.drop_last(1).moduli() == [17, 97]
    with pytest.raises(rn.RnsNttError) as e:
        rn.RnsBasis([17, 97], 8).drop_last(2)
    assert e.value.kind == "InvalidModDrop"
    for case in ("reconstruct_centered_single_channel", "reconstruct_centered_two_channels"):
        c = k[case]
        bb = rn.RnsBasis(c["moduli"], 8)
        for res, want in c["cases"]:
            assert bb.reconstruct_centered_coeff(res) == want


# --------------------------------------------------------------------------
# committed big-integer vectors
# --------------------------------------------------------------------------


def test_golden_ring_vectors(gpu, vectors, manifest):
    rn = gpu
    for name, m in manifest.items():
        if f"{name}/a" not in vectors:
            continue
        mod = [int(x) for x in vectors[f"{name}/moduli"]]
        B = rn.RnsBasis(mod, m["n"])
        assert [B.psi(i) for i in range(len(mod))] == [int(x) for x in vectors[f"{name}/psi"]]
        a = rn.RnsPoly.from_channels(vectors[f"{name}/a"], B)
        b = rn.RnsPoly.from_channels(vectors[f"{name}/b"], B)
        assert np.array_equal((a * b).channels(), vectors[f"{name}/mul"]), name
        assert np.array_equal((a + b).channels(), vectors[f"{name}/add"]), name
        an = a.clone()
        an.to_ntt_domain()
        assert np.array_equal(an.channels(), vectors[f"{name}/ntt_a"]), name  # natural order
        # NTT-domain upload of the natural-order vector round-trips to a
        up = rn.RnsPoly.from_channels(vectors[f"{name}/ntt_a"], B, in_ntt_domain=True)
        up.to_coeff_domain()
        assert np.array_equal(up.channels(), vectors[f"{name}/a"]), name
        if f"{name}/rescale_a" in vectors:
            assert np.array_equal(a.rescale().channels(), vectors[f"{name}/rescale_a"]), name
        for key in vectors.files:
            if key.startswith(f"{name}/auto_"):
                g = int(key.split("_")[-1])
                assert np.array_equal(a.automorphism(g).channels(), vectors[key]), key


def test_golden_ciphertext_vectors(gpu, vectors, manifest):
    rn = gpu
    for name, m in manifest.items():
        if not name.startswith("ks_"):
            continue
        mod = [int(x) for x in vectors[f"{name}/moduli"]]
        B = rn.RnsBasis(mod, m["n"])
        P = lambda k: rn.RnsPoly.from_channels(vectors[f"{name}/{k}"], B)  # noqa: E731
        rlk = rn.RnsGadgetKey(P("key_a"), P("key_b"))
        ct1 = rn.Ciphertext(P("c0"), P("c1"), 20, 60)
        ct2 = rn.Ciphertext(P("c0p"), P("c1p"), 20, 60)
        out = rn.mul_ciphertexts_gadget(ct1, ct2, rlk)
        assert np.array_equal(out.c0.channels(), vectors[f"{name}/relin_out0"]), name
        assert np.array_equal(out.c1.channels(), vectors[f"{name}/relin_out1"]), name
        assert out.logp == 40
        for k in (1, -1, 3):
            rotk = rn.RnsGadgetKey(P("key_a"), P("key_b"), rotation=k)
            r = rn.rotate_ciphertext(ct1, rotk)
            assert np.array_equal(r.c0.channels(), vectors[f"{name}/rot{k}_out0"]), (name, k)
            assert np.array_equal(r.c1.channels(), vectors[f"{name}/rot{k}_out1"]), (name, k)


# --------------------------------------------------------------------------
# seeded random parity vs the oracle, across ring sizes and prime widths
# --------------------------------------------------------------------------

SHAPES = [
    # (log_n, bits, L, batch)
    (0, 20, 2, 3),
    (1, 20, 2, 3),
    (2, 31, 2, 5),
    (3, 31, 3, 7),
    (4, 31, 3, 3),
    (5, 40, 2, 3),
    (6, 31, 3, 5),
    (7, 62, 2, 3),
    (8, 31, 3, 3),
    (9, 61, 2, 2),
    (10, 31, 3, 3),
    (11, 62, 2, 2),
    (12, 31, 4, 8),   # BASELINE config 2 (N=2^12, 4 primes)
    (13, 31, 2, 2),
    (14, 40, 2, 2),
    (15, 31, 2, 2),
]


def _rand(rng, mod, n, batch):
    return orc.uniform_poly(mod, n, rng, batch=batch)


@pytest.mark.parametrize("log_n,bits,L,batch", SHAPES)
def test_ring_ops_vs_oracle(gpu, log_n, bits, L, batch):
    rn = gpu
    n = 1 << log_n
    mod = rn.generate_primes(bits, L, max(n, 2)) if n >= 2 else rn.generate_primes(bits, L, 2)
    B, Bo = _basis(rn, mod, n)
    rng = np.random.default_rng(1000 + log_n)
    a_h, b_h = _rand(rng, mod, n, batch), _rand(rng, mod, n, batch)
    a = rn.RnsPoly.from_channels(a_h, B)
    b = rn.RnsPoly.from_channels(b_h, B)
    prod = (a * b).channels().reshape(batch, L, n)
    ntt = a.clone()
    ntt.to_ntt_domain()
    ntt_h = ntt.channels().reshape(batch, L, n)
    ssum = (a + b).channels().reshape(batch, L, n)
    diff = a.clone()
    diff -= b
    diff = diff.channels().reshape(batch, L, n)
    neg = (-a).channels().reshape(batch, L, n)
    for i in range(batch):
        assert np.array_equal(prod[i], orc.mul(Bo, a_h[i], b_h[i])), i
        assert np.array_equal(ntt_h[i], orc.to_ntt(Bo, a_h[i])), i
        assert np.array_equal(ssum[i], orc.add(Bo, a_h[i], b_h[i])), i
        assert np.array_equal(neg[i], orc.neg(Bo, a_h[i])), i
        mods = np.array(mod, dtype=np.uint64)[:, None]
        assert np.array_equal(diff[i], (a_h[i] + mods - b_h[i]) % mods), i
    # NTT-domain mul stays NTT and equals the oracle's pointwise product
    bn = b.clone()
    bn.to_ntt_domain()
    pn = ntt * bn
    assert pn.is_ntt_domain()
    pnh = pn.channels().reshape(batch, L, n)
    for i in range(batch):
        assert np.array_equal(pnh[i], orc.mul(Bo, orc.to_ntt(Bo, a_h[i]), orc.to_ntt(Bo, b_h[i]), ntt=True))
    # inverse brings it back to the coefficient product
    pn.to_coeff_domain()
    assert np.array_equal(pn.channels().reshape(batch, L, n), prod)
    # rescale from both domains (poly.rs:187-228)
    r = a.rescale().channels().reshape(batch, L - 1, n)
    rn_ = ntt.rescale().channels().reshape(batch, L - 1, n)
    for i in range(batch):
        want = orc.rescale(Bo, a_h[i])
        assert np.array_equal(r[i], want) and np.array_equal(rn_[i], want)
    # automorphisms: odd, even (non-automorphism quirk), zero, from NTT domain
    for g in (1, 3, 5 ** 7, 2 * n - 1, 2, 6, n, 2 * n, 4 * n + 3):
        if n == 1 and g % 2 == 0:
            continue
        out = a.automorphism(g)
        outn = ntt.automorphism(g)
        oh = out.channels().reshape(batch, L, n)
        onh = outn.channels().reshape(batch, L, n)
        for i in range(batch):
            want, f = orc.automorphism(Bo, a_h[i], g)
            assert np.array_equal(oh[i], want), (g, i)
            wantn, fn = orc.automorphism(Bo, orc.to_ntt(Bo, a_h[i]), g, in_ntt=True)
            assert np.array_equal(onh[i], wantn), (g, i)
            assert outn.is_ntt_domain() == fn
    for k in (1, 2, -1, -3):
        rh = a.rotate_slots(k).channels().reshape(batch, L, n)
        for i in range(batch):
            assert np.array_equal(rh[i], orc.rotate_slots(Bo, a_h[i], k)[0]), (k, i)


def test_errors_domain_and_basis(gpu):
    rn = gpu
    mod = rn.generate_primes(31, 3, 64)
    B = rn.RnsBasis(mod, 64)
    a = rn.RnsPoly.from_coeffs(np.arange(64), B)
    b = rn.RnsPoly.from_coeffs(np.arange(64), B)
    b.to_ntt_domain()
    with pytest.raises(rn.RnsNttError) as e:
        a *= b
    assert e.value.kind == "DomainMismatch"
    with pytest.raises(rn.RnsNttError) as e:
        a += b
    assert e.value.kind == "DomainMismatch"
    B2 = rn.RnsBasis(mod, 64)  # equal moduli, different Arc
    c = rn.RnsPoly.from_coeffs(np.arange(64), B2)
    with pytest.raises(rn.RnsNttError) as e:
        a *= c
    assert e.value.kind == "BasisMismatch"
    big = np.full((3, 64), mod[0], dtype=np.uint64)
    with pytest.raises(rn.RnsNttError) as e:
        rn.RnsPoly.from_channels(big, B)
    assert e.value.kind == "NonReducedCoefficient"
    assert str(mod[0]) in str(e.value)


def test_from_coeffs_extremes(gpu):
    rn = gpu
    for bits in (31, 62):
        mod = rn.generate_primes(bits, 2, 16)
        B, Bo = _basis(rn, mod, 16)
        c = np.array([-(2 ** 63), 2 ** 63 - 1, -1, 0, 1, -mod[0], mod[0], mod[1] - 1] + list(range(-4, 4)), dtype=np.int64)
        assert np.array_equal(rn.RnsPoly.from_coeffs(c, B).channels(), orc.from_coeffs(Bo, c))


# --------------------------------------------------------------------------
# BASELINE configs
# --------------------------------------------------------------------------


def test_config3_mul_relin_rescale(gpu, vectors):
    """Config 3: N=2^14, 8 primes -- ct x ct + gadget relin + rescale vs oracle."""
    rn = gpu
    n = 1 << 14
    mod = [int(x) for x in vectors["cfg3_n16384/moduli"]]
    B, Bo = _basis(rn, mod, n)
    L = len(mod)
    rng = np.random.default_rng(3)
    batch = 2
    c0, c1, c0p, c1p = (_rand(rng, mod, n, batch) for _ in range(4))
    ka, kb = _rand(rng, mod, n, L), _rand(rng, mod, n, L)
    rlk = rn.RnsGadgetKey.from_channels(ka, kb, B)
    ct1 = rn.Ciphertext(rn.RnsPoly.from_channels(c0, B), rn.RnsPoly.from_channels(c1, B), 31, 248)
    ct2 = rn.Ciphertext(rn.RnsPoly.from_channels(c0p, B), rn.RnsPoly.from_channels(c1p, B), 31, 248)
    out = rn.mul_ciphertexts_gadget(ct1, ct2, rlk)
    res = rn.rescale_ciphertext(out)
    o0 = out.c0.channels()
    o1 = out.c1.channels()
    r0 = res.c0.channels()
    r1 = res.c1.channels()
    assert res.logp == 62 - 31 and res.c0.basis.channel_count() == L - 1
    for i in range(batch):
        w0, w1 = orc.mul_ciphertexts_gadget(Bo, c0[i], c1[i], c0p[i], c1p[i], ka, kb)
        assert np.array_equal(o0[i], w0) and np.array_equal(o1[i], w1), i
        assert np.array_equal(r0[i], orc.rescale(Bo, w0)) and np.array_equal(r1[i], orc.rescale(Bo, w1)), i


def test_config4_metric_shape_polymul(gpu, vectors):
    """The metric's workload (N=2^16, 16 primes): poly-mul bit-exact vs the
    oracle on sampled pairs, plus size-independent properties on a batch."""
    rn = gpu
    n = 1 << 16
    mod = [int(x) for x in vectors["cfg4_n65536/moduli"]]
    B, Bo = _basis(rn, mod, n)
    assert B.psi(0) == 1615402923
    rng = np.random.default_rng(4)
    batch = 6
    a_h, b_h, c_h = (_rand(rng, mod, n, batch) for _ in range(3))
    a, b, c = (rn.RnsPoly.from_channels(x, B) for x in (a_h, b_h, c_h))
    ab = a * b
    abh = ab.channels()
    for i in (0, batch - 1):  # sampled bit-exact against the oracle
        assert np.array_equal(abh[i], orc.mul(Bo, a_h[i], b_h[i])), i
    # commutativity, distributivity, round trip (whole batch)
    assert np.array_equal((b * a).channels(), abh)
    lhs = (a + b) * c
    rhs = a * c + b * c
    assert np.array_equal(lhs.channels(), rhs.channels())
    t = a.clone()
    t.to_ntt_domain()
    t.to_coeff_domain()
    assert np.array_equal(t.channels(), a_h)
    # in-place aliasing forms of MulAssign
    x = a.clone()
    x *= b
    assert np.array_equal(x.channels(), abh)
    y = b.clone()
    y *= y
    assert np.array_equal(y.channels(), (b * b).channels())


def test_config5_rotation_keyswitch_sample(gpu, vectors):
    """Config 5 ring (N=2^17, 32 primes): rotation key-switch on one
    ciphertext vs oracle for a sampled Galois element."""
    rn = gpu
    n = 1 << 17
    mod = [int(x) for x in vectors["cfg5_n131072/moduli"]][:4]  # oracle time bound: 4 limbs
    B, Bo = _basis(rn, mod, n)
    L = len(mod)
    rng = np.random.default_rng(5)
    c0, c1 = _rand(rng, mod, n, 1), _rand(rng, mod, n, 1)
    ka, kb = _rand(rng, mod, n, L), _rand(rng, mod, n, L)
    rotk = rn.RnsGadgetKey.from_channels(ka, kb, B, rotation=5)
    ct = rn.Ciphertext(rn.RnsPoly.from_channels(c0[0], B), rn.RnsPoly.from_channels(c1[0], B))
    r = rn.rotate_ciphertext(ct, rotk)
    w0, w1 = orc.rotate_ciphertext(Bo, c0[0], c1[0], 5, ka, kb)
    assert np.array_equal(r.c0.channels(), w0)
    assert np.array_equal(r.c1.channels(), w1)


def test_config5_full_limbs_ntt_roundtrip(gpu, vectors):
    rn = gpu
    n = 1 << 17
    mod = [int(x) for x in vectors["cfg5_n131072/moduli"]]
    B, Bo = _basis(rn, mod, n)
    rng = np.random.default_rng(6)
    a_h = _rand(rng, mod, n, 2)
    a = rn.RnsPoly.from_channels(a_h, B)
    t = a.clone()
    t.to_ntt_domain()
    th = t.channels()
    assert np.array_equal(th[1][:2], orc.to_ntt(orc.Basis(mod[:2], n), a_h[1][:2]))
    t.to_coeff_domain()
    assert np.array_equal(t.channels(), a_h)


# ---------------------------------------------------------------------------
# decode-side CRT (basis.rs:158-180, poly.rs:404-427)
# ---------------------------------------------------------------------------


def _centered_crt(mods, residues):
    """Exact centred CRT in Python ints (the reference's math without its
    u128 limit)."""
    Q = 1
    for q in mods:
        Q *= q
    x = 0
    for r, q in zip(residues, mods):
        Qi = Q // q
        x += (int(r) * pow(Qi % q, -1, q) % q) * Qi
    x %= Q
    return x - Q if x > Q // 2 else x


@pytest.mark.gpu
@pytest.mark.parametrize("log_n,bits,L", [(3, 20, 2), (4, 31, 3), (6, 40, 3), (8, 61, 2), (10, 31, 4)])
def test_to_coeffs_matches_oracle(gpu, log_n, bits, L):
    """Q < 2^128: bit-exact against the oracle's restatement of to_coeffs."""
    rn = gpu
    n = 1 << log_n
    mods = rn.generate_primes(bits, L, n)
    Bo = orc.Basis(mods, n)
    rng = np.random.default_rng(log_n * 7 + L)
    a = orc.uniform_poly(mods, n, rng, batch=3)
    p = rn.RnsPoly.from_channels(a, rn.RnsBasis(mods, n))
    got = p.to_coeffs()
    for i in range(3):
        assert np.array_equal(got[i], orc.to_coeffs(Bo, a[i])), i
    # NTT-domain input decodes through a temporary copy, unchanged
    p.to_ntt_domain()
    assert np.array_equal(p.to_coeffs(), got)
    assert p.is_ntt_domain()


@pytest.mark.gpu
@pytest.mark.parametrize("log_n,L", [(16, 16), (17, 32)])
def test_crt_centered_large_q(gpu, log_n, L):
    """Q >= 2^128 (configs 4, 5): exact centred values against Python ints
    on sampled coefficients, and small signed coefficients round-trip."""
    rn = gpu
    n = 1 << log_n
    mods = rn.generate_primes(31, L, n)
    B = rn.RnsBasis(mods, n)
    rng = np.random.default_rng(L)
    a = orc.uniform_poly(mods, n, rng, batch=1)
    p = rn.RnsPoly.from_channels(a[0], B)  # the reference's single polynomial: [N] views
    exact = p.to_coeffs_exact()
    for i in rng.integers(0, n, size=64):
        assert exact[i] == _centered_crt(mods, a[0, :, i]), i
    # i64 path = the low 64 bits of the same values
    low = p.to_coeffs()
    for i in rng.integers(0, n, size=64):
        v = exact[i] & ((1 << 64) - 1)
        assert int(low[i]) == (v - (1 << 64) if v >> 63 else v)
    # from_coeffs -> to_coeffs is the identity on i64 inputs
    c = rng.integers(-(1 << 62), 1 << 62, size=n, dtype=np.int64)
    c[:4] = [0, 1, -1, (1 << 62) - 1]
    assert np.array_equal(rn.RnsPoly.from_coeffs(c, B).to_coeffs(), c)
