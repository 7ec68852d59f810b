"""GPU CKKS encoder/decoder (rnt_encode / rnt_decode, rnt_encode.hip) vs the
oracle (oracle/encoder.py), SURVEY §8f row 4.

Floating point, so parity is tolerance-based (as in ckks_encoder.rs:173-227):
* encode: integer coefficients equal the oracle's rounding of the same
  real values exactly, except where the f64 value sits within ~1e-6 of a
  rounding tie (at most a handful of coefficients, off by one);
* decode: slots within 1e-9 of the largest slot magnitude;
* full size (N=2^16, L=16 and N=2^17, L=32): decode(encode(v)) within the
  rounding bound N / 2^scale_bits of v.
"""
from __future__ import annotations

import numpy as np
import pytest

import encoder as enc

pytestmark = pytest.mark.gpu


def _coeffs(rn, poly):
    return np.asarray(poly.to_coeffs())


def _assert_coeffs_match(got, want_real, max_ties=4):
    want = enc.round_half_away(want_real)
    diff = np.abs(got.astype(np.int64) - want)
    bad = np.nonzero(diff)[0]
    assert diff.max() <= 1, f"coefficient off by {diff.max()}"
    assert len(bad) <= max_ties, f"{len(bad)} coefficients differ"
    if len(bad):  # only at rounding ties
        frac = np.abs(np.abs(want_real - np.trunc(want_real)) - 0.5)
        assert np.all(frac[bad] < 1e-6)


def test_encoder_reference_cases(gpu):
    """ckks_encoder.rs:173-214 through the device: N = 8, basis {97, 113},
    scale_bits 5; coefficients equal the restated encoder exactly."""
    rn = gpu
    basis = rn.RnsBasis([97, 113], 8)
    e = rn.CkksEncoder(8, 5)
    for values in ([1.0, -1.0, 0.5, -0.5], [3.0], [1.0, 2.0, 3.0]):
        pt = e.encode(values, basis)
        assert pt.slots == len(values)
        assert np.array_equal(_coeffs(rn, pt.poly), enc.encode_ref(values, 8, 5))
        out = e.decode(pt)
        assert out.shape == (len(values),)
        assert np.allclose(out, values, atol=0.1, rtol=0)
    cv = [1.0 + 0.5j, -0.5 + 0.25j]
    pt = e.encode_complex(cv, basis)
    assert np.allclose(e.decode_complex(pt), cv, atol=0.1, rtol=0)
    assert e.max_slots() == 4


def test_encoder_errors(gpu):
    rn = gpu
    basis = rn.RnsBasis([97, 113], 8)
    e = rn.CkksEncoder(8, 5)
    with pytest.raises(ValueError, match="exceed max slots"):
        e.encode([0.0] * 5, basis)
    with pytest.raises(ValueError):
        rn.CkksEncoder(8, 0)
    import ctypes

    x = np.zeros(10, dtype=np.complex128)
    p = rn.RnsPoly(basis, 1)
    with pytest.raises(rn.RnsNttError, match="BadArgument"):
        rn._lib.check(rn.load().rnt_encode(p.handle, x.ctypes.data_as(ctypes.c_void_p), 5, 5))
    with pytest.raises(rn.RnsNttError, match="BadArgument"):
        rn._lib.check(rn.load().rnt_encode(p.handle, x.ctypes.data_as(ctypes.c_void_p), 2, 0))


@pytest.mark.parametrize("log_n,L,bits", [(4, 2, 31), (10, 3, 31), (12, 4, 31), (13, 7, 61)])
def test_encode_matches_oracle(gpu, log_n, L, bits):
    """Batched encode of random complex slots (some rows partially filled)
    vs the oracle's FFT evaluation of the reference's special_idft."""
    rn = gpu
    n = 1 << log_n
    mods = rn.generate_primes(bits, L, n)
    basis = rn.RnsBasis(mods, n)
    rng = np.random.default_rng(log_n)
    scale = 30
    B, nv = 3, max(1, n // 2 - 3)
    v = rng.uniform(-4, 4, (B, nv)) + 1j * rng.uniform(-4, 4, (B, nv))
    pt = rn.CkksEncoder(n, scale).encode_complex(v, basis)
    got = np.asarray(pt.poly.to_coeffs())
    for p in range(B):
        _assert_coeffs_match(got[p], enc.encode_fft_real(v[p], n, scale))
    # residues are from_coeffs of those integers (poly.rs:55-61)
    ch = pt.poly.channels()
    want = np.stack([np.asarray(got[0], dtype=object) % q for q in mods]).astype(np.uint64)
    assert np.array_equal(ch[0], want)


@pytest.mark.parametrize("log_n,L", [(4, 2), (11, 3), (12, 4)])
def test_decode_matches_oracle(gpu, log_n, L):
    rn = gpu
    n = 1 << log_n
    mods = rn.generate_primes(31, L, n)
    basis = rn.RnsBasis(mods, n)
    rng = np.random.default_rng(100 + log_n)
    B = 2
    a = rng.integers(-(2 ** 40), 2 ** 40, (B, n))
    poly = rn.RnsPoly.from_coeffs(a, basis)
    scale = 25
    for slots in (n // 2, 3):
        z = rn.CkksEncoder(n, scale).decode_complex(rn.Plaintext(poly, scale, slots))
        for p in range(B):
            want = enc.decode_fft(a[p], n, scale, slots)
            assert np.allclose(z[p], want, atol=1e-9 * np.max(np.abs(want)), rtol=0)
    # NTT-domain input decodes through a coefficient-domain clone
    t = poly.clone()
    t.to_ntt_domain()
    zt = rn.CkksEncoder(n, scale).decode_complex(rn.Plaintext(t, scale, n // 2))
    z0 = rn.CkksEncoder(n, scale).decode_complex(rn.Plaintext(poly, scale, n // 2))
    assert np.array_equal(zt, z0)
    assert t.is_ntt_domain()


@pytest.mark.parametrize("log_n,L", [(16, 16), (17, 32)])
def test_full_size_roundtrip(gpu, log_n, L):
    """BASELINE configs 4/5 rings: decode(encode(v)) == v within the
    rounding bound, and the decode of a full-size encode matches the oracle."""
    rn = gpu
    n = 1 << log_n
    mods = rn.generate_primes(31, L, n)
    basis = rn.RnsBasis(mods, n)
    rng = np.random.default_rng(log_n)
    scale = 40
    v = rng.uniform(-1, 1, (2, n // 2)) + 1j * rng.uniform(-1, 1, (2, n // 2))
    e = rn.CkksEncoder(n, scale)
    pt = e.encode_complex(v, basis)
    back = e.decode_complex(pt)
    assert np.max(np.abs(back - v)) < n / 2.0 ** scale
    got = np.asarray(pt.poly.to_coeffs())
    _assert_coeffs_match(got[1], enc.encode_fft_real(v[1], n, scale), max_ties=16)
