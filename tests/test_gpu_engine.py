"""Device-resident CKKS engine sequences on the GPU.

The host samplers are not the reference's RNG streams, so parity is
relational: key relations hold with small errors, and decryptions of
encrypt / multiply+relin / rescale / rotate match the exact plaintext
arithmetic within noise bounds.  This mirrors the reference's tolerance
tests (tests/integration_mul.rs).  The last two tests run the reference's
examples/encrypt_mul.rs and examples/rotation_demo.rs end to end through
the device encoder, with the examples' own parameters and error bounds.
"""
from __future__ import annotations

import numpy as np
import pytest


def _engine(rn, log_n=12, L=4, seed=3):
    from rns_ntt.engine import CkksEngine

    n = 1 << log_n
    eng = CkksEngine(rn.generate_primes(31, L, n), n, error_std=3.2, hamming_weight=64)
    return eng, np.random.default_rng(seed)


def _negacyclic(a, b):
    n = len(a)
    full = np.zeros(2 * n, dtype=object)
    for i, x in enumerate(a):
        if x:
            full[i:i + n] += int(x) * b.astype(object)
    return full[:n] - full[n:]


def _maxdiff(x, y):
    return max(abs(int(u) - int(v)) for u, v in zip(x, y))


@pytest.mark.gpu
def test_key_relations(gpu):
    rn = gpu
    eng, rng = _engine(rn)
    sk = eng.generate_secret_key(rng)
    pk = eng.generate_public_key(sk, rng)
    e = (pk.b + pk.a * sk).to_coeffs()  # b + a s = e
    assert np.abs(e).max() <= 8 * eng.error_std
    rlk = eng.generate_gadget_relin_key(sk, rng)
    s2 = (sk * sk).channels()
    L = eng.basis.channel_count()
    for i in range(L):  # b_i + a_i s - E_i(s^2) = e_i
        # prepared keys are NTT-resident: their channels are NTT-domain values
        ai = rn.RnsPoly.from_channels(rlk.a.channels()[i], eng.basis, in_ntt_domain=True)
        bi = rn.RnsPoly.from_channels(rlk.b.channels()[i], eng.basis, in_ntt_domain=True)
        plain = np.zeros_like(s2)
        plain[i] = s2[i]
        ai.to_coeff_domain()
        bi.to_coeff_domain()
        ei = (bi + ai * sk - rn.RnsPoly.from_channels(plain, eng.basis)).to_coeffs()
        assert np.abs(ei).max() <= 8 * eng.error_std, i


@pytest.mark.gpu
def test_encrypt_mul_relin_rescale_decrypt(gpu):
    rn = gpu
    from rns_ntt.engine import CkksEngine

    eng, rng = _engine(rn)
    n = eng.degree
    sk = eng.generate_secret_key(rng)
    pk = eng.generate_public_key(sk, rng)
    rlk = eng.generate_gadget_relin_key(sk, rng)
    delta = 1 << 20
    m1 = np.rint(rng.uniform(-1, 1, n) * delta).astype(np.int64)
    m2 = np.rint(rng.uniform(-1, 1, n) * delta).astype(np.int64)
    ct1 = eng.encrypt(rn.RnsPoly.from_coeffs(m1, eng.basis), pk, rng)
    ct2 = eng.encrypt(rn.RnsPoly.from_coeffs(m2, eng.basis), pk, rng)
    # encrypt / decrypt and add
    assert _maxdiff(CkksEngine.decrypt(ct1, sk).to_coeffs(), m1) < 1 << 12
    s = CkksEngine.decrypt(CkksEngine.add_ciphertexts(ct1, ct2), sk).to_coeffs()
    assert _maxdiff(s, m1 + m2) < 1 << 13
    # multiply + gadget relinearisation
    prod = _negacyclic(m1, m2)
    ct = CkksEngine.mul_ciphertexts_gadget(ct1, ct2, rlk)
    dec = CkksEngine.decrypt(ct, sk).to_coeffs_exact()
    assert _maxdiff(dec, prod) < 1 << 46, "relinearised product outside the noise bound"
    # rescale: floor-divide by q_L (R4), decrypt on the dropped basis
    r = CkksEngine.rescale_ciphertext(ct)
    q_last = eng.basis.moduli()[-1]
    dec2 = CkksEngine.decrypt(r, CkksEngine.secret_on(sk, r.c0.basis)).to_coeffs_exact()
    assert _maxdiff(dec2, [v // q_last for v in prod]) < 1 << 16
    assert r.logq == ct.logq - q_last.bit_length()


@pytest.mark.gpu
def test_rotation_key_switch(gpu):
    rn = gpu
    from rns_ntt.engine import CkksEngine

    eng, rng = _engine(rn, log_n=11, L=3)
    n = eng.degree
    sk = eng.generate_secret_key(rng)
    pk = eng.generate_public_key(sk, rng)
    m = rng.integers(-(1 << 24), 1 << 24, size=n, dtype=np.int64)
    ct = eng.encrypt(rn.RnsPoly.from_coeffs(m, eng.basis), pk, rng)
    for k in (1, 3, -2):
        rotk = eng.generate_gadget_rotation_key(sk, k, rng)
        out = CkksEngine.rotate_ciphertext(ct, rotk)
        want = rn.RnsPoly.from_coeffs(m, eng.basis).rotate_slots(k).to_coeffs()
        got = CkksEngine.decrypt(out, sk).to_coeffs_exact()
        assert _maxdiff(got, want) < 1 << 45, k


@pytest.mark.gpu
def test_encrypt_mul_example_slots(gpu):
    """examples/encrypt_mul.rs: N=16, 4 x 31-bit primes, scale 2^30; encode ->
    encrypt -> gadget mul -> rescale -> decrypt -> decode within 1e-4."""
    rn = gpu
    from rns_ntt.engine import CkksEngine

    n = 16
    eng = CkksEngine(rn.generate_primes(31, 4, n), n, error_std=3.2, hamming_weight=n // 2)
    rng = np.random.default_rng(42)
    sk = eng.generate_secret_key(rng)
    pk = eng.generate_public_key(sk, rng)
    rlk = eng.generate_gadget_relin_key(sk, rng)
    a, b = [1.0, 2.0, 3.0, 4.0], [0.5, 1.0, 1.5, 2.0]
    enc = rn.CkksEncoder(n, 30)
    logq = eng.basis.total_bits()
    ct_a = eng.encrypt(enc.encode(a, eng.basis), pk, rng, logq=logq)
    ct_b = eng.encrypt(enc.encode(b, eng.basis), pk, rng, logq=logq)
    assert ct_a.logp == 30
    prod = CkksEngine.rescale_ciphertext(CkksEngine.mul_ciphertexts_gadget(ct_a, ct_b, rlk))
    assert prod.logp == 60 - eng.basis.moduli()[-1].bit_length()
    pt = CkksEngine.decrypt_plaintext(prod, CkksEngine.secret_on(sk, prod.c0.basis))
    got = enc.decode(pt)[:4]
    assert np.max(np.abs(got - np.multiply(a, b))) <= 1e-4


@pytest.mark.gpu
def test_rotation_demo_example_slots(gpu):
    """examples/rotation_demo.rs: N=32, 3 x 30-bit primes, scale 2^58;
    rotate(+1), add the original, rotate(+2); every slot within 1e-4."""
    rn = gpu
    from rns_ntt.engine import CkksEngine

    n, slots = 32, 16
    eng = CkksEngine(rn.generate_primes(30, 3, n), n, error_std=3.2, hamming_weight=n // 2)
    rng = np.random.default_rng(7)
    sk = eng.generate_secret_key(rng)
    pk = eng.generate_public_key(sk, rng)
    rk1 = eng.generate_gadget_rotation_key(sk, 1, rng)
    rk2 = eng.generate_gadget_rotation_key(sk, 2, rng)
    enc = rn.CkksEncoder(n, 58)
    v = np.arange(1, slots + 1, dtype=np.float64)
    ct = eng.encrypt(enc.encode(v, eng.basis), pk, rng)
    r1 = CkksEngine.rotate_ciphertext(ct, rk1)
    out = CkksEngine.rotate_ciphertext(CkksEngine.add_ciphertexts(ct, r1), rk2)
    got = enc.decode(CkksEngine.decrypt_plaintext(out, sk))
    want = np.roll(v + np.roll(v, -1), -2)  # rotate_vec: slot i <- slot i + k
    assert np.max(np.abs(got - want)) <= 1e-4
