"""Device-resident CKKS engine sequences.

Mirrors the RNS half of `CkksEngine` (src/crypto/engine.rs): key
generation (:288-399), encrypt / decrypt / add (:84-151), and the gadget
multiply, rotate and rescale already in `rns_ntt`.  Every polynomial stays
in device memory and every ring operation runs through librnsntt; only the
random samples are drawn on the host.

The samplers run on the device when ``rng`` is an ``rns_ntt.DeviceRng``
(Philox4x32-10 streams, rnt_sample_*: ternary secret with a fixed Hamming
weight, rounded Gaussian errors, uniform residues), or on the host with a
numpy Generator; neither reproduces the reference's ChaCha20 + rand_distr
streams bit-exactly.  Parity for
these paths is therefore relational: key relations and decryption error
bounds (tests/test_gpu_engine.py), as SURVEY §8f prescribes.  Plaintexts
are either scaled integer coefficients (an RnsPoly) or slot-encoded
``Plaintext``s from ``CkksEncoder`` (the device special FFT, §8f row 4).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import (Ciphertext, DeviceRng, Plaintext, RnsBasis, RnsGadgetKey, RnsPoly, mul_ciphertexts_gadget,
               rescale_ciphertext, rotate_ciphertext)


@dataclass
class PublicKey:
    """public_key.rs: b = -a*s + e."""

    b: RnsPoly
    a: RnsPoly


class CkksEngine:
    """The RNS-backend engine over one basis.

    ``error_std`` is the Gaussian width of every error sample.  The
    reference passes sqrt(error_variance) in key generation (engine.rs:316)
    but error_variance itself in encrypt (engine.rs:92).  Both call sites
    here take ``error_std``, and the caller chooses its value.
    """

    def __init__(self, moduli, degree: int, error_std: float = 3.2,
                 hamming_weight: Optional[int] = None, device: int = 0):
        # an existing RnsBasis is shared, as CkksEngine::new(basis.clone(), ..)
        # shares the Arc (engine.rs:36-41): a level-l engine built on a
        # rescaled ciphertext's basis encrypts onto that same basis
        if isinstance(moduli, RnsBasis):
            if moduli.degree != degree:
                raise ValueError(f"basis degree {moduli.degree} != engine degree {degree}")
            self.basis = moduli
        else:
            self.basis = RnsBasis(list(moduli), degree, device=device)
        self.degree = degree
        self.error_std = error_std
        self.hamming_weight = hamming_weight if hamming_weight is not None else degree // 2

    # -- samplers (traits.rs PolySampler): device for a DeviceRng, else host -
    # count=None draws the reference's single polynomial, count=k a batch of k
    def _tern_poly(self, rng, count=None) -> RnsPoly:
        if isinstance(rng, DeviceRng):
            return RnsPoly.sample_tribits(self.hamming_weight, self.basis, rng, count)
        c = self._ternary(rng, count or 1)
        return RnsPoly.from_coeffs(c if count else c[0], self.basis)

    def _gauss_poly(self, rng, count=None) -> RnsPoly:
        if isinstance(rng, DeviceRng):
            return RnsPoly.sample_gaussian(self.error_std, self.basis, rng, count)
        c = self._gaussian(rng, count or 1)
        return RnsPoly.from_coeffs(c if count else c[0], self.basis)

    def _ternary(self, rng, count=1):
        n = self.degree
        out = np.zeros((count, n), dtype=np.int64)
        for c in range(count):
            idx = rng.choice(n, size=self.hamming_weight, replace=False)
            out[c, idx] = rng.choice(np.array([-1, 1], dtype=np.int64), size=self.hamming_weight)
        return out

    def _gaussian(self, rng, count=1):
        return np.rint(rng.normal(0.0, self.error_std, size=(count, self.degree))).astype(np.int64)

    def _uniform(self, rng, count=None, basis: Optional[RnsBasis] = None):
        b = basis or self.basis
        if isinstance(rng, DeviceRng):
            return RnsPoly.sample_uniform(b, rng, count)
        q = np.array(b.moduli(), dtype=np.uint64)[None, :, None]
        ch = rng.integers(0, 1 << 62, size=(count or 1, len(b.moduli()), self.degree), dtype=np.uint64) % q
        return RnsPoly.from_channels(ch if count else ch[0], b)

    # -- keys (engine.rs:288-399, keys/*.rs) ---------------------------------
    def generate_secret_key(self, rng) -> RnsPoly:
        return self._tern_poly(rng)

    def generate_public_key(self, sk: RnsPoly, rng) -> PublicKey:
        a = self._uniform(rng)
        b = -(a * sk) + self._gauss_poly(rng)
        return PublicKey(b, a)

    def _gadget_key(self, sk: RnsPoly, target: RnsPoly, rng, rotation=None) -> RnsGadgetKey:
        """b_i = -(a_i s) + e_i + e_i-plaintext(target) for every channel i,
        as one batch of L polys on the device."""
        L, n = self.basis.channel_count(), self.degree
        t = target.channels()  # [L][N], coefficient domain
        plain = np.zeros((L, L, n), dtype=np.uint64)
        for i in range(L):
            plain[i, i] = t[i]
        s_rep = RnsPoly.from_channels(np.broadcast_to(sk.channels(), (L, L, n)).copy(), self.basis)
        a = self._uniform(rng, count=L)
        e = self._gauss_poly(rng, count=L)
        b = -(a * s_rep) + e + RnsPoly.from_channels(plain, self.basis)
        return RnsGadgetKey(a, b, rotation)

    def generate_gadget_relin_key(self, sk: RnsPoly, rng) -> RnsGadgetKey:
        return self._gadget_key(sk, sk * sk, rng)

    def generate_gadget_rotation_key(self, sk: RnsPoly, rotation: int, rng) -> RnsGadgetKey:
        return self._gadget_key(sk, sk.rotate_slots(rotation), rng, rotation)

    # -- encryption (engine.rs:84-127) -----------------------------------------
    def encrypt(self, plaintext, pk: PublicKey, rng, logp: int = 0,
                logq: Optional[int] = None) -> Ciphertext:
        """``plaintext`` is an RnsPoly (with ``logp``) or a Plaintext, whose
        scale_bits become the ciphertext's logp (engine.rs:84-112)."""
        if isinstance(plaintext, Plaintext):
            logp, plaintext = plaintext.scale_bits, plaintext.poly
        u = self._tern_poly(rng)
        e0 = self._gauss_poly(rng)
        e1 = self._gauss_poly(rng)
        c0 = pk.b * u + e0 + plaintext
        c1 = pk.a * u + e1
        return Ciphertext(c0, c1, logp, self.basis.total_bits() if logq is None else logq)

    @staticmethod
    def decrypt(ct: Ciphertext, sk: RnsPoly) -> RnsPoly:
        """m = c0 + c1 * s (engine.rs:114-127); sk must share ct's basis."""
        return ct.c1 * sk + ct.c0

    @staticmethod
    def decrypt_plaintext(ct: Ciphertext, sk: RnsPoly) -> Plaintext:
        """engine.rs:114-128: the decryption as a Plaintext with
        scale_bits = logp and all N/2 slots, ready for CkksEncoder.decode."""
        return Plaintext(CkksEngine.decrypt(ct, sk), ct.logp, ct.c0.basis.degree // 2)

    @staticmethod
    def add_ciphertexts(ct1: Ciphertext, ct2: Ciphertext) -> Ciphertext:
        assert ct1.logp == ct2.logp, "logp mismatch in addition"
        assert ct1.logq == ct2.logq, "logq mismatch in addition"
        return Ciphertext(ct1.c0 + ct2.c0, ct1.c1 + ct2.c1, ct1.logp, ct1.logq)

    # the gadget multiply / rotate / rescale are the library calls
    mul_ciphertexts_gadget = staticmethod(mul_ciphertexts_gadget)
    rotate_ciphertext = staticmethod(rotate_ciphertext)
    rescale_ciphertext = staticmethod(rescale_ciphertext)

    @staticmethod
    def secret_on(sk: RnsPoly, basis: RnsBasis) -> RnsPoly:
        """The secret key restricted to a prefix basis (after rescale), built
        on that basis object (same basis = same context, as Arc::ptr_eq)."""
        ch = sk.channels()
        return RnsPoly.from_channels(ch[: basis.channel_count()], basis)
