"""CKKS encoder/decoder oracle (oracle/encoder.py) pinned on CPU.

The reference's encoder is floating point, so its own tests are tolerance
checks; the same cases are run here against the restatement
(special_fft.rs:250-339, ckks_encoder.rs:173-227), and the FFT-based
formulation the GPU tests use at full sizes is pinned against the
loop-for-loop restatement of the reference's O(N^2) Vandermonde sums.
"""
from __future__ import annotations

import numpy as np
import pytest

import encoder as enc
import pyoracle as orc


def _roundtrip(values, n, mods, scale_bits):
    """encode -> from_coeffs -> to_coeffs -> decode, through the oracle's
    RNS path (poly.rs:49-67, 404-427)."""
    ob = orc.Basis(mods, n)
    coeffs = enc.encode_ref(values, n, scale_bits)
    poly = orc.from_coeffs(ob, coeffs)
    back = orc.to_coeffs(ob, poly)
    assert np.array_equal(np.asarray(back, dtype=np.int64), coeffs)
    return enc.decode_ref(back, n, scale_bits, len(values))


def test_conjugate_slots_build_symmetry():
    """special_fft.rs:250-268."""
    inp = np.array([1 + 0.5j, -0.25 + 0.75j, -1j])
    s = enc.build_conjugate_slots(inp, 8)
    assert np.array_equal(s[:3], inp)
    assert np.array_equal(s[[7, 6, 5]], np.conj(inp))


def test_conjugate_slots_rejects_overflow():
    """special_fft.rs:284-291."""
    with pytest.raises(ValueError, match="exceeds slot capacity"):
        enc.build_conjugate_slots(np.zeros(5), 8)


def test_vandermonde_roundtrip():
    """special_fft.rs:325-339: dft then idft within 1e-9."""
    n = 8
    coeffs = np.array([k / 7.0 - 1j * k / 11.0 for k in range(n)])
    back = enc.special_idft_ref(enc.special_dft_ref(coeffs, n), n)
    assert np.allclose(back, coeffs, atol=1e-9, rtol=0)


def test_slot_roots_are_conjugate_pairs():
    """special_fft.rs:293-323 (table consistency)."""
    r = enc.slot_roots(8)
    assert np.allclose(np.abs(r), 1.0, atol=1e-12)
    assert np.allclose(r[::-1], np.conj(r), atol=1e-12)  # J-ordering pairs k <-> N-1-k


@pytest.mark.parametrize("values", [[1.0, -1.0, 0.5, -0.5], [3.0], [1.0, 2.0, 3.0]])
def test_encoder_reference_cases_real(values):
    """ckks_encoder.rs:173-214: N = 8, basis {97, 113}, scale_bits 5, eps 0.1."""
    got = _roundtrip(values, 8, [97, 113], 5)
    assert len(got) == len(values)
    assert np.allclose(got.real, values, atol=0.1, rtol=0)


def test_encoder_reference_case_complex():
    """ckks_encoder.rs:186-198."""
    values = [1.0 + 0.5j, -0.5 + 0.25j]
    got = _roundtrip(values, 8, [97, 113], 5)
    assert np.allclose(got, values, atol=0.1, rtol=0)


@pytest.mark.parametrize("n", [8, 64, 512])
def test_fft_formulation_matches_vandermonde(n):
    """The numpy-FFT evaluation (used by the GPU tests at full size) equals
    the restated O(N^2) sums."""
    rng = np.random.default_rng(n)
    v = rng.standard_normal(n // 2) + 1j * rng.standard_normal(n // 2)
    want = enc.special_idft_ref(enc.build_conjugate_slots(v * 2.0 ** 20, n), n)
    assert np.max(np.abs(want.imag)) < 1e-6  # real coefficients (Hermitian slots)
    got = enc.encode_fft_real(v, n, 20)
    assert np.allclose(got, want.real, atol=1e-6, rtol=0)
    assert np.array_equal(enc.encode_fft(v, n, 20), enc.encode_ref(v, n, 20))
    a = rng.integers(-(2 ** 40), 2 ** 40, n)
    z_ref = enc.decode_ref(a, n, 30, n // 2)
    z_fft = enc.decode_fft(a, n, 30, n // 2)
    assert np.allclose(z_fft, z_ref, atol=1e-9 * np.max(np.abs(z_ref)), rtol=0)


def test_round_half_away_matches_rust_round():
    x = np.array([0.5, -0.5, 1.5, -1.5, 2.4999999999999996, -2.5000000000000004, 0.0, -0.0])
    assert list(enc.round_half_away(x)) == [1, -1, 2, -2, 2, -3, 0, 0]
