"""ctypes binding of oracle/liboracle.so -- the CPU restatement of the
reference RNS-NTT path (see oracle.h).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker / CPU baseline.  The product
package (toy-heaan-ckks_amd/) never imports this module.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_double, c_int, c_int32, c_int64, c_size_t, c_uint32, c_uint64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# ORACLE_LIB: an alternative build of the same source (tools/sanitize.sh's
# ASan/UBSan variant)
LIB_PATH = os.environ.get("ORACLE_LIB") or os.path.join(HERE, "liboracle.so")

_U64P = POINTER(c_uint64)
_I64P = POINTER(c_int64)


class OrTable(ctypes.Structure):
    _fields_ = [
        ("modulus", c_uint64),
        ("n_inv", c_uint64),
        ("psi", c_uint64),
        ("forward_roots", _U64P),
        ("inverse_roots", _U64P),
        ("twist_factors", _U64P),
        ("untwist_factors", _U64P),
    ]


class OrBasis(ctypes.Structure):
    _fields_ = [
        ("n", c_size_t),
        ("channels", c_size_t),
        ("moduli", _U64P),
        ("tables", POINTER(OrTable)),
        ("owns_tables", c_int),
    ]


_B = POINTER(OrBasis)
_SIGS = {
    "or_mul_mod": (c_uint64, [c_uint64, c_uint64, c_uint64]),
    "or_add_mod": (c_uint64, [c_uint64, c_uint64, c_uint64]),
    "or_sub_mod": (c_uint64, [c_uint64, c_uint64, c_uint64]),
    "or_mod_pow": (c_uint64, [c_uint64, c_uint64, c_uint64]),
    "or_mod_inverse": (c_uint64, [c_uint64, c_uint64]),
    "or_is_prime": (c_int, [c_uint64]),
    "or_is_prime_reference": (c_int, [c_uint64]),
    "or_is_ntt_friendly_prime": (c_int, [c_uint64, c_uint64]),
    "or_get_first_prime_up": (c_uint64, [c_uint32, c_uint64]),
    "or_get_first_prime_down": (c_uint64, [c_uint64, c_uint64]),
    "or_generate_primes": (c_size_t, [c_uint32, c_size_t, c_uint64, _U64P]),
    "or_find_primitive_root": (c_uint64, [c_uint64, c_uint64]),
    "or_basis_new": (c_int, [_B, c_size_t, _U64P, c_size_t]),
    "or_basis_free": (None, [_B]),
    "or_basis_drop_last": (c_int, [_B, c_size_t, _B]),
    "or_basis_total_bits": (c_uint32, [_B]),
    "or_reconstruct_centered": (c_int64, [_B, _U64P]),
    "or_from_coeffs": (None, [_B, _I64P, _U64P]),
    "or_from_channels_check": (c_int, [_B, _U64P, c_size_t]),
    "or_to_coeffs": (None, [_B, _U64P, c_int, _I64P]),
    "or_to_ntt_domain": (None, [_B, _U64P]),
    "or_to_coeff_domain": (None, [_B, _U64P]),
    "or_mul_assign": (c_int, [_B, _U64P, c_int, _U64P, c_int]),
    "or_mul_assign_naive": (None, [_B, _U64P, _U64P]),
    "or_add_assign": (c_int, [_B, _U64P, c_int, _U64P, c_int]),
    "or_neg": (None, [_B, _U64P]),
    "or_rescale": (c_int, [_B, _U64P, c_int, _U64P]),
    "or_automorphism": (None, [_B, _U64P, c_int, c_uint64, _U64P, POINTER(c_int)]),
    "or_rotate_slots": (None, [_B, _U64P, c_int, c_int32, _U64P, POINTER(c_int)]),
    "or_gadget_keyswitch": (None, [_B, _U64P, _U64P, _U64P, _U64P, _U64P]),
    "or_mul_ciphertexts_gadget": (None, [_B, _U64P, _U64P, _U64P, _U64P, _U64P, _U64P, _U64P, _U64P]),
    "or_rotate_ciphertext": (None, [_B, _U64P, _U64P, c_int32, _U64P, _U64P, _U64P, _U64P]),
    "or_gadget_keyswitch_mt": (None, [_B, _U64P, _U64P, _U64P, _U64P, _U64P, c_int]),
    "or_mul_ciphertexts_gadget_mt": (None, [_B, _U64P, _U64P, _U64P, _U64P, _U64P, _U64P, _U64P, _U64P,
                                            c_int]),
    "or_rotate_ciphertext_mt": (None, [_B, _U64P, _U64P, c_int32, _U64P, _U64P, _U64P, _U64P, c_int]),
    "or_polymul_batch_mt": (c_double, [_B, _U64P, _U64P, c_size_t, c_int]),
}

_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"oracle not built: {LIB_PATH} (run make)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _p(a: np.ndarray):
    assert a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_U64P)


class OracleError(Exception):
    def __init__(self, code):
        self.code = code
        super().__init__(f"oracle error {code}")


class Basis:
    """RnsBasis<N> restated (basis.rs:90-180)."""

    def __init__(self, moduli, n, _drop_from=None):
        self._b = OrBasis()
        if _drop_from is not None:
            parent, k = _drop_from
            rc = lib().or_basis_drop_last(ctypes.byref(parent._b), k, ctypes.byref(self._b))
            self._parent = parent
        else:
            arr = np.ascontiguousarray(np.array(list(moduli) or [0], dtype=np.uint64))
            rc = lib().or_basis_new(ctypes.byref(self._b), n, _p(arr), len(moduli))
            self._parent = None
        if rc != 0:
            raise OracleError(rc)
        self.n = n
        self.L = int(self._b.channels)

    @property
    def ref(self):
        return ctypes.byref(self._b)

    @property
    def moduli(self):
        return [int(self._b.moduli[i]) for i in range(self.L)]

    def psi(self, i):
        return int(self._b.tables[i].psi)

    def drop_last(self, k):
        return Basis(None, self.n, _drop_from=(self, k))

    def total_bits(self):
        return int(lib().or_basis_total_bits(self.ref))

    def reconstruct_centered(self, residues):
        r = np.ascontiguousarray(np.array(residues, dtype=np.uint64))
        return int(lib().or_reconstruct_centered(self.ref, _p(r)))

    def __del__(self):
        if getattr(self, "_b", None) is not None and self._b.moduli:
            lib().or_basis_free(ctypes.byref(self._b))


def _poly(a):
    return np.ascontiguousarray(np.array(a, dtype=np.uint64))


def from_coeffs(b: Basis, coeffs):
    c = np.ascontiguousarray(np.array(coeffs, dtype=np.int64)[: b.n])
    out = np.zeros((b.L, b.n), dtype=np.uint64)
    lib().or_from_coeffs(b.ref, c.ctypes.data_as(_I64P), _p(out))
    return out


def to_coeffs(b: Basis, poly, in_ntt=False):
    p = _poly(poly)
    out = np.zeros(b.n, dtype=np.int64)
    lib().or_to_coeffs(b.ref, _p(p), int(in_ntt), out.ctypes.data_as(_I64P))
    return out


def to_ntt(b: Basis, poly):
    p = _poly(poly).copy()
    lib().or_to_ntt_domain(b.ref, _p(p))
    return p


def to_coeff(b: Basis, poly):
    p = _poly(poly).copy()
    lib().or_to_coeff_domain(b.ref, _p(p))
    return p


def mul(b: Basis, a, rhs, ntt=False):
    x = _poly(a).copy()
    y = _poly(rhs)
    rc = lib().or_mul_assign(b.ref, _p(x), int(ntt), _p(y), int(ntt))
    if rc:
        raise OracleError(rc)
    return x


def mul_naive(b: Basis, a, rhs):
    x = _poly(a).copy()
    lib().or_mul_assign_naive(b.ref, _p(x), _p(_poly(rhs)))
    return x


def add(b: Basis, a, rhs, ntt=False):
    x = _poly(a).copy()
    rc = lib().or_add_assign(b.ref, _p(x), int(ntt), _p(_poly(rhs)), int(ntt))
    if rc:
        raise OracleError(rc)
    return x


def neg(b: Basis, a):
    x = _poly(a).copy()
    lib().or_neg(b.ref, _p(x))
    return x


def rescale(b: Basis, a, in_ntt=False):
    x = _poly(a)
    out = np.zeros((max(b.L - 1, 1), b.n), dtype=np.uint64)
    rc = lib().or_rescale(b.ref, _p(x), int(in_ntt), _p(out))
    if rc:
        raise OracleError(rc)
    return out


def automorphism(b: Basis, a, g, in_ntt=False):
    x = _poly(a)
    out = np.zeros((b.L, b.n), dtype=np.uint64)
    f = c_int(0)
    lib().or_automorphism(b.ref, _p(x), int(in_ntt), g, _p(out), ctypes.byref(f))
    return out, bool(f.value)


def rotate_slots(b: Basis, a, k, in_ntt=False):
    x = _poly(a)
    out = np.zeros((b.L, b.n), dtype=np.uint64)
    f = c_int(0)
    lib().or_rotate_slots(b.ref, _p(x), int(in_ntt), k, _p(out), ctypes.byref(f))
    return out, bool(f.value)


def keyswitch(b: Basis, d, key_a, key_b, threads: int = 1):
    """key_a/key_b: [L][L][N] coefficient domain.  threads > 1 runs the
    channel-parallel form (same arithmetic per target channel)."""
    acc0 = np.zeros((b.L, b.n), dtype=np.uint64)
    acc1 = np.zeros((b.L, b.n), dtype=np.uint64)
    args = (b.ref, _p(_poly(d)), _p(_poly(key_a)), _p(_poly(key_b)), _p(acc0), _p(acc1))
    if threads > 1:
        lib().or_gadget_keyswitch_mt(*args, threads)
    else:
        lib().or_gadget_keyswitch(*args)
    return acc0, acc1


def mul_ciphertexts_gadget(b: Basis, c0, c1, c0p, c1p, key_a, key_b, threads: int = 1):
    o0 = np.zeros((b.L, b.n), dtype=np.uint64)
    o1 = np.zeros((b.L, b.n), dtype=np.uint64)
    args = (b.ref, _p(_poly(c0)), _p(_poly(c1)), _p(_poly(c0p)), _p(_poly(c1p)),
            _p(_poly(key_a)), _p(_poly(key_b)), _p(o0), _p(o1))
    if threads > 1:
        lib().or_mul_ciphertexts_gadget_mt(*args, threads)
    else:
        lib().or_mul_ciphertexts_gadget(*args)
    return o0, o1


def rotate_ciphertext(b: Basis, c0, c1, k, key_a, key_b, threads: int = 1):
    o0 = np.zeros((b.L, b.n), dtype=np.uint64)
    o1 = np.zeros((b.L, b.n), dtype=np.uint64)
    args = (b.ref, _p(_poly(c0)), _p(_poly(c1)), k, _p(_poly(key_a)), _p(_poly(key_b)), _p(o0), _p(o1))
    if threads > 1:
        lib().or_rotate_ciphertext_mt(*args, threads)
    else:
        lib().or_rotate_ciphertext(*args)
    return o0, o1


def host_threads(cap: int = 16) -> int:
    """Worker threads for the oracle on this host (the GPU box's CPU share is
    16; os.cpu_count() reports the whole machine)."""
    import os

    return max(1, min(cap, os.cpu_count() or 1))


def polymul_batch_mt(b: Basis, a, rhs, threads):
    """In-place a[i] *= rhs[i] for a [count][L][N] batch; returns seconds."""
    assert a.flags["C_CONTIGUOUS"] and a.dtype == np.uint64
    return float(lib().or_polymul_batch_mt(b.ref, _p(a), _p(_poly(rhs)), a.shape[0], threads))


def generate_primes(bits, count, degree):
    out = np.zeros(max(count, 1), dtype=np.uint64)
    k = lib().or_generate_primes(bits, count, degree, _p(out))
    if k != count:
        raise OracleError(11)
    return [int(x) for x in out[:count]]


def uniform_poly(moduli, n, rng, batch=None):
    """Seeded uniform residues in [0, q_i) (our own numpy PRNG, not Rust's)."""
    shape = (len(moduli), n) if batch is None else (batch, len(moduli), n)
    out = np.empty(shape, dtype=np.uint64)
    for i, q in enumerate(moduli):
        if batch is None:
            out[i] = rng.integers(0, q, size=n, dtype=np.uint64)
        else:
            out[:, i] = rng.integers(0, q, size=(batch, n), dtype=np.uint64)
    return out
