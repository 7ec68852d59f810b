"""The CPU oracle pinned by the reference's own known-answer tests
(tests/golden/reference_kats.json) and by the independent big-integer
restatement (tests/golden/vectors.npz).  CPU only."""
from __future__ import annotations

import numpy as np
import pytest

import pyoracle as orc

U64 = (1 << 64) - 1


def test_primes_kats(kats):
    k = kats["primes"]
    L = orc.lib()
    for p in k["known_small_primes"]["values"]:
        assert L.or_is_prime(p) and L.or_is_prime_reference(p)
    for c in k["known_small_composites"]["values"]:
        assert not L.or_is_prime(c) and not L.or_is_prime_reference(c)
    m = k["mul_mod_matches_widened_reference"]
    assert L.or_mul_mod(m["a"], m["b"], m["modulus"]) == (m["a"] * m["b"]) % m["modulus"]
    for b, e, q, want in k["mod_pow_handles_edge_cases"]["cases"]:
        assert L.or_mod_pow(b, e, q) == want
    for p in k["is_prime_large"]["prime"] + k["near_u64_limit"]["prime"]:
        assert L.or_is_prime(p)
    for c in k["is_prime_large"]["composite"] + k["tricky_composites"]["composite"] + k["near_u64_limit"]["composite"]:
        assert not L.or_is_prime(c)
    for lo, hi in k["miller_rabin_matches_reference_ranges"]["ranges"]:
        for n in range(lo, hi + 1):
            assert L.or_is_prime(n) == L.or_is_prime_reference(n), n
    f = k["ntt_friendly_condition"]
    assert all(L.or_is_ntt_friendly_prime(p, f["n"]) for p in f["friendly"])
    assert not any(L.or_is_ntt_friendly_prime(p, f["n"]) for p in f["not_friendly"])
    u = k["first_prime_up_matches_reference"]
    assert L.or_get_first_prime_up(u["logq"], u["n"]) == u["expect"]
    d = k["prime_down_descends"]
    p = L.or_get_first_prime_up(d["logq"], d["n"])
    below = L.or_get_first_prime_down(p, d["n"])
    assert 0 < below < p and L.or_is_ntt_friendly_prime(below, d["n"])
    pb = k["prime_down_basic"]
    p = L.or_get_first_prime_down(pb["bound"], pb["n"])
    assert p < pb["bound"] and L.or_is_ntt_friendly_prime(p, pb["n"])
    for b in pb["none_bounds"]:
        assert L.or_get_first_prime_down(b, pb["n"]) == 0
    g = k["generates_ntt_primes_in_range"]
    ps = orc.generate_primes(g["bits"], g["count"], g["degree"])
    assert all((1 << (g["bits"] - 1)) <= q < (1 << g["bits"]) and L.or_is_ntt_friendly_prime(q, g["degree"]) for q in ps)
    g = k["panics_when_not_enough_primes"]
    with pytest.raises(orc.OracleError):
        orc.generate_primes(g["bits"], g["count"], g["degree"])
    g = k["doctest_generate_primes"]
    assert all(L.or_is_ntt_friendly_prime(q, g["degree"]) for q in orc.generate_primes(g["bits"], g["count"], g["degree"]))


def test_basis_kats(kats):
    k = kats["basis_n8"]
    b = orc.Basis([17], 8)
    assert b.moduli == [17]
    assert b._b.tables[0].forward_roots[0] == 1
    with pytest.raises(orc.OracleError) as e:
        orc.Basis([19], 8)
    assert e.value.code == 3
    with pytest.raises(orc.OracleError) as e:
        orc.Basis([], 8)
    assert e.value.code == 2
    b = orc.Basis([17, 97, 113], 8)
    assert b.drop_last(1).moduli == [17, 97]
    with pytest.raises(orc.OracleError) as e:
        orc.Basis([17, 97], 8).drop_last(2)
    assert e.value.code == 4
    for case in ("reconstruct_centered_single_channel", "reconstruct_centered_two_channels"):
        c = k[case]
        bb = orc.Basis(c["moduli"], 8)
        for res, want in c["cases"]:
            assert bb.reconstruct_centered(res) == want


def test_poly_kats(kats):
    k = kats["poly_n8"]
    B2 = orc.Basis([17, 97], 8)
    B3 = orc.Basis([17, 97, 113], 8)

    c = k["from_coeffs_reduces_correctly"]
    p = orc.from_coeffs(B2, c["coeffs"])
    for ch, i, v in c["expect"]:
        assert p[ch, i] == v
    c = k["from_channels_rejects_unreduced_coefficient"]
    ch = np.array(c["channels"], dtype=np.uint64)
    assert orc.lib().or_from_channels_check(B2.ref, orc._p(ch), 2) == 6
    c = k["from_channels_rejects_wrong_channel_count"]
    ch = np.array(c["channels"], dtype=np.uint64)
    assert orc.lib().or_from_channels_check(B2.ref, orc._p(ch), 1) == 5

    c = k["ntt_roundtrip_preserves_coefficients"]
    p = orc.from_coeffs(B2, c["coeffs"])
    assert np.array_equal(orc.to_coeff(B2, orc.to_ntt(B2, p)), p)

    c = k["add_assign_computes_correct_sum"]
    s = orc.add(B2, orc.from_coeffs(B2, c["a"]), orc.from_coeffs(B2, c["b"]))
    assert (s == c["expect_all"]).all()
    c = k["add_assign_wraps_at_modulus"]
    s = orc.add(B2, orc.from_coeffs(B2, c["a"]), orc.from_coeffs(B2, c["b"]))
    assert s[0, 0] == 1
    c = k["neg_negates_coefficients"]
    s = orc.neg(B2, orc.from_coeffs(B2, c["a"]))
    assert s[0, 0] == 14 and s[0, 1] == 0
    for name in ("mul_assign_schoolbook_small", "mul_assign_wraps_around_quotient"):
        c = k[name]
        s = orc.mul(B2, orc.from_coeffs(B2, c["a"]), orc.from_coeffs(B2, c["b"]))
        assert list(orc.to_coeffs(B2, s)) == c["expect_coeffs"]
    c = k["to_coeffs_roundtrips_from_coeffs"]
    assert list(orc.to_coeffs(B2, orc.from_coeffs(B2, c["coeffs"]))) == c["coeffs"]
    c = k["to_coeffs_works_from_ntt_domain"]
    assert list(orc.to_coeffs(B2, orc.to_ntt(B2, orc.from_coeffs(B2, c["coeffs"])), True)) == c["coeffs"]
    c = k["mul_assign_ntt_domain_matches_coeff_domain"]
    a, b = orc.from_coeffs(B2, c["a"]), orc.from_coeffs(B2, c["b"])
    coeff = orc.mul(B2, a, b)
    ntt = orc.mul(B2, orc.to_ntt(B2, a), orc.to_ntt(B2, b), ntt=True)
    assert np.array_equal(orc.to_coeff(B2, ntt), coeff)
    c = k["automorphism_identity_preserves_coefficients"]
    p = orc.from_coeffs(B2, c["coeffs"])
    for g in c["exponents"]:
        assert list(orc.to_coeffs(B2, orc.automorphism(B2, p, g)[0])) == c["coeffs"]
    c = k["automorphism_applies_sign_change_correctly"]
    out, _ = orc.automorphism(B2, orc.from_coeffs(B2, c["coeffs"]), c["exponent"])
    assert list(orc.to_coeffs(B2, out)) == c["expect_coeffs"]
    c = k["automorphism_preserves_ntt_domain_flag"]
    _, f = orc.automorphism(B2, orc.to_ntt(B2, orc.from_coeffs(B2, c["coeffs"])), c["exponent"], in_ntt=True)
    assert f == c["expect_ntt"]
    c = k["mul_assign_matches_naive"]
    a, b = orc.from_coeffs(B2, c["a"]), orc.from_coeffs(B2, c["b"])
    assert np.array_equal(orc.mul(B2, a, b), orc.mul_naive(B2, a, b))
    c = k["rescale_is_exact_division_by_last_prime"]
    r = orc.rescale(B3, orc.from_coeffs(B3, c["coeffs"]))
    assert list(orc.to_coeffs(B3.drop_last(1), r)) == c["expect_coeffs"]
    c = k["rescale_from_ntt_domain_matches_coeff_domain"]
    p = orc.from_coeffs(B3, c["coeffs"])
    assert np.array_equal(orc.rescale(B3, p), orc.rescale(B3, orc.to_ntt(B3, p), in_ntt=True))
    B1 = orc.Basis([17], 8)
    with pytest.raises(orc.OracleError) as e:
        orc.rescale(B1, orc.from_coeffs(B1, k["rescale_on_single_channel_errors"]["coeffs"]))
    assert e.value.code == 4
    # mixed domains: the reference only debug_asserts (poly.rs:292-295)
    x = orc.from_coeffs(B2, [1] * 8)
    assert orc.lib().or_mul_assign(B2.ref, orc._p(x), 0, orc._p(x.copy()), 1) == 7


def test_oracle_matches_bigint_vectors(vectors, manifest):
    """Every ring vector of the independent Python restatement."""
    for name, m in manifest.items():
        if f"{name}/a" not in vectors:
            continue
        mod = [int(x) for x in vectors[f"{name}/moduli"]]
        B = orc.Basis(mod, m["n"])
        a, b = vectors[f"{name}/a"], vectors[f"{name}/b"]
        assert [B.psi(i) for i in range(B.L)] == [int(x) for x in vectors[f"{name}/psi"]]
        assert np.array_equal(orc.mul(B, a, b), vectors[f"{name}/mul"]), name
        assert np.array_equal(orc.to_ntt(B, a), vectors[f"{name}/ntt_a"]), name
        assert np.array_equal(orc.add(B, a, b), vectors[f"{name}/add"]), name
        if f"{name}/rescale_a" in vectors:
            assert np.array_equal(orc.rescale(B, a), vectors[f"{name}/rescale_a"]), name
        for key in vectors.files:
            if key.startswith(f"{name}/auto_"):
                g = int(key.split("_")[-1])
                assert np.array_equal(orc.automorphism(B, a, g)[0], vectors[key]), key
        if m["n"] <= 256:
            assert np.array_equal(orc.mul_naive(B, a, b), vectors[f"{name}/mul"])


def test_oracle_keyswitch_vectors(vectors, manifest):
    for name, m in manifest.items():
        if not name.startswith("ks_"):
            continue
        mod = [int(x) for x in vectors[f"{name}/moduli"]]
        B = orc.Basis(mod, m["n"])
        g = lambda k: vectors[f"{name}/{k}"]  # noqa: E731
        o0, o1 = orc.mul_ciphertexts_gadget(B, g("c0"), g("c1"), g("c0p"), g("c1p"), g("key_a"), g("key_b"))
        assert np.array_equal(o0, g("relin_out0")) and np.array_equal(o1, g("relin_out1"))
        for k in (1, -1, 3):
            r0, r1 = orc.rotate_ciphertext(B, g("c0"), g("c1"), k, g("key_a"), g("key_b"))
            assert np.array_equal(r0, g(f"rot{k}_out0")) and np.array_equal(r1, g(f"rot{k}_out1"))


def test_config_prime_chains(vectors, manifest):
    """BASELINE configs' primes and psi from the oracle."""
    for name, m in manifest.items():
        if not name.startswith("cfg"):
            continue
        mod = orc.generate_primes(m["bits"], m["L"], m["n"])
        assert mod == [int(x) for x in vectors[f"{name}/moduli"]]
        for q, psi in zip(mod, vectors[f"{name}/psi"]):
            assert orc.lib().or_find_primitive_root(q, 2 * m["n"]) == int(psi)


def test_channel_parallel_keyswitch_matches_serial():
    """or_*_mt (test infrastructure for the config-4/5 checks) give the
    serial restatement's results exactly."""
    n = 64
    mod = orc.generate_primes(31, 4, n)
    b = orc.Basis(mod, n)
    rng = np.random.default_rng(8)
    c = [orc.uniform_poly(mod, n, rng) for _ in range(4)]
    ka, kb = orc.uniform_poly(mod, n, rng, batch=4), orc.uniform_poly(mod, n, rng, batch=4)
    for x, y in zip(orc.mul_ciphertexts_gadget(b, *c, ka, kb), orc.mul_ciphertexts_gadget(b, *c, ka, kb, threads=3)):
        assert np.array_equal(x, y)
    for k in (1, -3, 0):
        for x, y in zip(orc.rotate_ciphertext(b, c[0], c[1], k, ka, kb),
                        orc.rotate_ciphertext(b, c[0], c[1], k, ka, kb, threads=3)):
            assert np.array_equal(x, y)
    for x, y in zip(orc.keyswitch(b, c[2], ka, kb), orc.keyswitch(b, c[2], ka, kb, threads=2)):
        assert np.array_equal(x, y)
