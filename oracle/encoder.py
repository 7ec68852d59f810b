"""CPU restatement of the reference's CKKS encoder/decoder (TEST
INFRASTRUCTURE ONLY: imported by tests/ as the checker, never by the
product path).

Two independent formulations:

* ``special_idft_ref`` / ``special_dft_ref`` / ``encode_ref`` / ``decode_ref``
  restate the reference loop for loop: the J-function slot-root table
  (special_fft.rs:21-29, :88-137), the conjugate-symmetric slot vector
  (special_fft.rs:158-178), the O(N^2) Vandermonde evaluations
  (special_fft.rs:194-242) and the encoder's scale / round / from_coeffs and
  to_coeffs / lift / unscale sequences (ckks_encoder.rs:65-156).  Vectorised
  with numpy but the same sums; for N up to a few thousand.
* ``encode_fft`` / ``decode_fft`` evaluate the same maps through numpy's
  FFT of length 2N (the embedding is a(zeta^{5^k}), zeta = exp(i pi / N)),
  for full sizes.  Tests pin them against the restatement at small N and
  against the reference's own test cases (ckks_encoder.rs:173-227,
  special_fft.rs:250-339).

Parity for this floating-point path is tolerance-based, as in the
reference's tests; the tolerances live in the tests.
"""
from __future__ import annotations

import numpy as np


def j_exponents(n: int) -> np.ndarray:
    """special_fft.rs:101-107: 5^h mod 2N for h < N/2, then 2N - 5^h for h
    descending."""
    m2 = 2 * n
    plus = [pow(5, h, m2) for h in range(n // 2)]
    minus = [(m2 - pow(5, h, m2)) % m2 for h in reversed(range(n // 2))]
    return np.array(plus + minus, dtype=np.int64)


def slot_roots(n: int) -> np.ndarray:
    """special_fft.rs:109-113: psi^e with psi = exp(i pi / N)."""
    return np.exp(1j * np.pi * j_exponents(n) / n)


def build_conjugate_slots(values, n: int) -> np.ndarray:
    """special_fft.rs:158-178."""
    v = np.asarray(values, dtype=np.complex128)
    if v.size > n // 2:
        raise ValueError("input exceeds slot capacity")
    s = np.zeros(n, dtype=np.complex128)
    s[: v.size] = v
    s[n - 1 - np.arange(n // 2)] = np.conj(s[: n // 2])
    return s


def special_idft_ref(values: np.ndarray, n: int) -> np.ndarray:
    """special_fft.rs:194-220: permuted = reverse(values); coeff[j] =
    (1/N) sum_i permuted[i] root_i^j."""
    perm = np.asarray(values, dtype=np.complex128)[::-1]
    roots = slot_roots(n)
    j = np.arange(n)
    out = np.zeros(n, dtype=np.complex128)
    for i in range(n):  # one Vandermonde row per slot, as the reference loops
        out += perm[i] * roots[i] ** j
    return out * (1.0 / n)


def special_dft_ref(coeffs: np.ndarray, n: int) -> np.ndarray:
    """special_fft.rs:224-242: slot[i] = sum_j c_j conj(root_i)^j, reversed."""
    c = np.asarray(coeffs, dtype=np.complex128)
    inv = np.conj(slot_roots(n))
    j = np.arange(n)
    slots = np.array([np.sum(c * inv[i] ** j) for i in range(n)])
    return slots[::-1]


def round_half_away(x: np.ndarray) -> np.ndarray:
    """Rust f64::round (ties away from zero), then `as i64` (saturating)."""
    r = np.trunc(x)
    r = r + np.where(np.abs(x - r) >= 0.5, np.sign(x), 0.0)
    return np.clip(r, -(2.0 ** 63), 2.0 ** 63 - 1024).astype(np.int64)


def encode_ref(values, n: int, scale_bits: int) -> np.ndarray:
    """ckks_encoder.rs:85-122 (encode_complex): integer coefficients."""
    v = np.asarray(values, dtype=np.complex128) * (2.0 ** scale_bits)
    coeffs = special_idft_ref(build_conjugate_slots(v, n), n)
    return round_half_away(coeffs.real)


def decode_ref(int_coeffs, n: int, scale_bits: int, slots: int) -> np.ndarray:
    """ckks_encoder.rs:134-156 (decode_complex) from centred integer coeffs."""
    c = np.asarray(int_coeffs, dtype=np.int64).astype(np.float64)
    return special_dft_ref(c, n)[:slots] / (2.0 ** scale_bits)


def rot_group(n: int) -> np.ndarray:
    return np.array([pow(5, k, 2 * n) for k in range(n // 2)], dtype=np.int64)


def decode_fft(int_coeffs, n: int, scale_bits: int, slots: int) -> np.ndarray:
    """a(zeta^{5^k}) for k < slots via a length-2N FFT (zeta = exp(i pi/N))."""
    a = np.zeros(2 * n, dtype=np.complex128)
    a[:n] = np.asarray(int_coeffs, dtype=np.int64).astype(np.float64)
    ev = np.fft.ifft(a) * (2 * n)  # ev[e] = sum_j a_j exp(+2 pi i e j / 2N)
    return ev[rot_group(n)[:slots]] / (2.0 ** scale_bits)


def encode_fft_real(values, n: int, scale_bits: int) -> np.ndarray:
    """Unrounded coefficients of encode_complex: w_j = (1/(N/2)) sum_k v_k
    zeta^{-5^k j}; coefficient j = Re w_j, j + N/2 = Im w_j."""
    v = np.asarray(values, dtype=np.complex128) * (2.0 ** scale_bits)
    big = np.zeros(2 * n, dtype=np.complex128)
    big[rot_group(n)[: v.size]] = v
    w = np.fft.fft(big)[: n // 2] / (n // 2)  # sum_e V_e exp(-2 pi i e j / 2N)
    return np.concatenate([w.real, w.imag])


def encode_fft(values, n: int, scale_bits: int) -> np.ndarray:
    return round_half_away(encode_fft_real(values, n, scale_bits))
