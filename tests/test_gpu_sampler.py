"""Device samplers (rnt_sample_*, rnt_sample.hip), SURVEY §8f row 2.

Bit-exact against the CPU restatement of the same Philox4x32-10
construction (oracle/sampler.py); the Gaussian allows a rounding-tie
difference where device and numpy log/cos differ in the last ulp.  Then the
reference's statistical sampler tests on the device output, the error
paths, and key generation / encryption driven entirely by the device RNG.
"""
from __future__ import annotations

import numpy as np
import pytest

import sampler as smp

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("log_n,mods", [(3, [17, 97]), (10, None), (12, "wide")])
def test_uniform_matches_oracle(gpu, log_n, mods):
    rn = gpu
    n = 1 << log_n
    if mods is None:
        mods = rn.generate_primes(31, 3, n)
    elif mods == "wide":
        mods = rn.generate_primes(61, 2, n)
    basis = rn.RnsBasis(mods, n)
    rng = rn.DeviceRng(0x1234_5678_9ABC_DEF0)
    rng.stream = 7
    got = rn.RnsPoly.sample_uniform(basis, rng, n_polys=3).channels()
    want = smp.uniform(mods, n, 3, 0x1234_5678_9ABC_DEF0, 7)
    assert np.array_equal(got, want)
    assert rng.stream == 8


def test_uniform_beyond_one_dispatch_grid(gpu):
    """1100 polys x 16 limbs at N = 2^16 (1.15e9 words, past the 2^30
    work-items of the capped grid, so the kernel's grid-stride loop covers
    the rest; 4096 polys -- 2^32 words -- used to fail the launch): the
    first and the last poly bit-exact against the oracle."""
    rn = gpu
    n, L, B = 1 << 16, 16, 1100
    mods = rn.generate_primes(31, L, n)
    basis = rn.RnsBasis(mods, n)
    rng = rn.DeviceRng(0xC0FFEE)
    rng.stream = 3
    x = rn.RnsPoly.sample_uniform(basis, rng, n_polys=B)
    for p in (0, B - 1):
        assert np.array_equal(x.channels_of(p)[0], smp.uniform_poly(mods, n, p, 0xC0FFEE, 3)), p
    del x


def test_gaussian_matches_oracle(gpu):
    rn = gpu
    n = 4096
    mods = rn.generate_primes(31, 3, n)
    basis = rn.RnsBasis(mods, n)
    rng = rn.DeviceRng(42)
    p = rn.RnsPoly.sample_gaussian(3.2, basis, rng, n_polys=2)
    got = np.asarray(p.to_coeffs())
    want = smp.gaussian_ints(n, 2, 3.2, 42, 0)
    assert np.abs(got - want).max() <= 1 and np.count_nonzero(got - want) <= 2
    assert np.array_equal(p.channels()[:, 1], smp.residues(got, mods)[:, 1])
    e = got.astype(np.float64)
    assert abs(e.mean()) < 0.1 and abs(e.var() - 3.2 ** 2 - 1 / 12) < 0.6  # sampling.rs:172-205
    noise = rn.RnsPoly.sample_noise(3.2 ** 2, basis, rng)  # poly.rs:471-477
    assert abs(np.asarray(noise.to_coeffs()).astype(np.float64).std() - 3.2) < 0.3


@pytest.mark.parametrize("log_n,h", [(3, 3), (6, 0), (6, 64), (12, 2048), (16, 32768), (17, 64)])
def test_ternary_matches_oracle(gpu, log_n, h):
    """Exact Hamming weight (poly.rs:978-987) and bit-exact selection."""
    rn = gpu
    n = 1 << log_n
    mods = [17, 97] if n == 8 else rn.generate_primes(31, 2, n)
    basis = rn.RnsBasis(mods, n)
    rng = rn.DeviceRng(99)
    rng.stream = 3
    p = rn.RnsPoly.sample_tribits(h, basis, rng, n_polys=2)
    got = np.asarray(p.to_coeffs()).reshape(2, n)
    assert all(int(np.count_nonzero(r)) == h for r in got)
    assert np.all(np.isin(got, [-1, 0, 1]))
    assert np.array_equal(got, smp.ternary_ints(n, 2, h, 99, 3))


def test_sampler_errors(gpu):
    rn = gpu
    basis = rn.RnsBasis([17, 97], 8)
    rng = rn.DeviceRng(1)
    with pytest.raises(rn.RnsNttError, match="BadArgument"):
        rn.RnsPoly.sample_tribits(9, basis, rng)  # sampling.rs:240-245
    for bad in (0.0, -1.0, float("inf"), float("nan")):
        with pytest.raises(rn.RnsNttError, match="BadArgument"):
            rn.RnsPoly.sample_gaussian(bad, basis, rng)  # sampling.rs:150-170


def test_keygen_and_encryption_on_device_rng(gpu):
    """engine.rs:288-399 with every sample drawn on the device: key
    relations within 8 sigma and an encrypt / mul / relin / rescale /
    decrypt / decode round trip within the encrypt_mul example's bound."""
    rn = gpu
    from rns_ntt.engine import CkksEngine

    n = 1 << 12
    eng = CkksEngine(rn.generate_primes(31, 4, n), n, error_std=3.2, hamming_weight=64)
    rng = rn.DeviceRng(2026)
    sk = eng.generate_secret_key(rng)
    assert int(np.count_nonzero(sk.to_coeffs())) == 64
    pk = eng.generate_public_key(sk, rng)
    assert np.abs((pk.b + pk.a * sk).to_coeffs()).max() <= 8 * 3.2
    rlk = eng.generate_gadget_relin_key(sk, rng)
    enc = rn.CkksEncoder(n, 30)
    x = np.linspace(-1, 1, n // 2)
    y = np.cos(np.arange(n // 2))
    logq = eng.basis.total_bits()
    ct = CkksEngine.mul_ciphertexts_gadget(eng.encrypt(enc.encode(x, eng.basis), pk, rng, logq=logq),
                                           eng.encrypt(enc.encode(y, eng.basis), pk, rng, logq=logq), rlk)
    r = CkksEngine.rescale_ciphertext(ct)
    got = enc.decode(CkksEngine.decrypt_plaintext(r, CkksEngine.secret_on(sk, r.c0.basis)))
    # the engine tracks logp -= bitlen(q_L) (engine.rs:263-282) while the true
    # scale is 2^60 / q_L: a known relative offset of 2^31 / q_L - 1 (~1e-4 here)
    q_last = eng.basis.moduli()[-1]
    err = np.abs(got - x * y * 2.0 ** (60 - r.logp) / q_last)
    # The reference's gadget digits are the [0, q_i) residues (engine.rs:505-528,
    # SURVEY R5), not centred: their mean q_i/2 times the all-ones polynomial
    # evaluates to ~2N/pi at zeta^(5^0) = exp(i pi/N), so slot 0 carries
    # ~N/8 times the relinearisation noise of the other slots (~2^-9 here).
    assert np.median(err) < 1e-4 and np.max(err[1:]) < 1e-3 and err[0] < 5e-3
