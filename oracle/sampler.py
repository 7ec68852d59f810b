"""CPU restatement of the device samplers (rnt_sample.hip) -- TEST
INFRASTRUCTURE ONLY (imported by tests/ as the checker).

The device draws from Philox4x32-10 (Salmon, Moraes, Dror, Shaw, "Parallel
random numbers: as easy as 1, 2, 3", SC'11; the Random123 library's
philox4x32_10) instead of the reference's ChaCha20 + rand_distr streams,
which cannot be reproduced here.  This module restates
that construction -- the Philox rounds, the counter layout and the three
samplers -- so the device output can be checked bit-exactly; ``philox``
itself is pinned by the Random123 known-answer vectors in the tests.  The
samplers' distributions follow the reference's (poly.rs:438-477,
sampling.rs:9-90), checked statistically with the reference's own tests.
"""
from __future__ import annotations

import numpy as np

M32 = np.uint64(0xFFFFFFFF)
KIND_UNIFORM, KIND_GAUSS, KIND_TERN_KEY, KIND_TERN_SIGN = 1, 2, 3, 4


def philox(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 over numpy arrays of 32-bit words (as uint64)."""
    c = [np.asarray(x, dtype=np.uint64) & M32 for x in (c0, c1, c2, c3)]
    k0 = np.uint64(k0) & M32
    k1 = np.uint64(k1) & M32
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c[0]
        p1 = np.uint64(0xCD9E8D57) * c[2]
        c = [(p1 >> np.uint64(32)) ^ c[1] ^ k0, p1 & M32, (p0 >> np.uint64(32)) ^ c[3] ^ k1, p0 & M32]
        k0 = (k0 + np.uint64(0x9E3779B9)) & M32
        k1 = (k1 + np.uint64(0xBB67AE85)) & M32
    return c


def _key(seed: int, stream: int):
    return seed & 0xFFFFFFFF, ((seed >> 32) ^ (stream >> 32)) & 0xFFFFFFFF


def draw(seed, stream, index, attempt, poly, limb, kind):
    """rnt_sample.hip draw(): counter (index | attempt << 20, poly,
    limb | kind << 16, stream_lo), key (seed_lo, seed_hi ^ stream_hi)."""
    k0, k1 = _key(seed, stream)
    idx = np.asarray(index, dtype=np.uint64) | np.uint64(attempt << 20)
    shape = np.shape(idx)
    return philox(idx, np.full(shape, poly, np.uint64), np.full(shape, limb | (kind << 16), np.uint64),
                  np.full(shape, stream & 0xFFFFFFFF, np.uint64), k0, k1)


def _lo(v):
    return v[0] | (v[1] << np.uint64(32))


def _hi(v):
    return v[2] | (v[3] << np.uint64(32))


def uniform(moduli, n, n_polys, seed, stream):
    """[B][L][N] residues (sample_uniform)."""
    out = np.zeros((n_polys, len(moduli), n), dtype=np.uint64)
    idx = np.arange(n, dtype=np.uint64)
    for li, q in enumerate(moduli):
        rem = (1 << 64) % q
        lim = (1 << 64) - rem
        for p in range(n_polys):
            val = np.zeros(n, dtype=object)
            todo = np.ones(n, dtype=bool)
            for att in range(16):
                v = draw(seed, stream, idx, att, p, li, KIND_UNIFORM)
                for x in (_lo(v), _hi(v)):
                    ok = todo & ((rem == 0) | (x.astype(object) < lim))
                    val[ok] = x[ok].astype(object) % q
                    todo &= ~ok
                if not todo.any():
                    break
            out[p, li] = val.astype(np.uint64)
    return out


def uniform_poly(moduli, n, p, seed, stream):
    """[L][N] residues of poly p alone (the draws depend only on the poly,
    limb and index, so one poly of a large batch is checkable by itself)."""
    out = np.zeros((len(moduli), n), dtype=np.uint64)
    idx = np.arange(n, dtype=np.uint64)
    for li, q in enumerate(moduli):
        rem = (1 << 64) % q
        lim = (1 << 64) - rem
        val = np.zeros(n, dtype=object)
        todo = np.ones(n, dtype=bool)
        for att in range(16):
            v = draw(seed, stream, idx, att, p, li, KIND_UNIFORM)
            for x in (_lo(v), _hi(v)):
                ok = todo & ((rem == 0) | (x.astype(object) < lim))
                val[ok] = x[ok].astype(object) % q
                todo &= ~ok
            if not todo.any():
                break
        out[li] = val.astype(np.uint64)
    return out


def round_away(z):
    r = np.trunc(z)
    return (r + np.where(np.abs(z - r) >= 0.5, np.sign(z), 0.0)).astype(np.int64)


def gaussian_ints(n, n_polys, sigma, seed, stream):
    """[B][N] rounded N(0, sigma) integers (sample_gaussian before from_coeffs)."""
    idx = np.arange(n, dtype=np.uint64)
    out = np.zeros((n_polys, n), dtype=np.int64)
    for p in range(n_polys):
        v = draw(seed, stream, idx, 0, p, 0, KIND_GAUSS)
        u1 = ((_lo(v) >> np.uint64(11)) + np.uint64(1)).astype(np.float64) * 2.0 ** -53
        u2 = (_hi(v) >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
        z = np.sqrt(-2.0 * np.log(u1)) * np.cos(6.283185307179586 * u2) * sigma
        out[p] = round_away(z)
    return out


def ternary_ints(n, n_polys, h, seed, stream):
    """[B][N] coefficients in {-1, 0, 1} with exactly h nonzeros: the h
    smallest keys (philox << 17 | i) are selected, signs from a second draw."""
    idx = np.arange(n, dtype=np.uint64)
    out = np.zeros((n_polys, n), dtype=np.int64)
    for p in range(n_polys):
        key = (draw(seed, stream, idx, 0, p, 0, KIND_TERN_KEY)[0] << np.uint64(17)) | idx
        sel = np.argsort(key, kind="stable")[:h]
        sign = draw(seed, stream, idx, 0, p, 0, KIND_TERN_SIGN)[0] & np.uint64(1)
        out[p, sel] = np.where(sign[sel] == 1, 1, -1)
    return out


def residues(ints, moduli):
    """from_coeffs (poly.rs:55-61) of [B][N] integers -> [B][L][N]."""
    x = np.asarray(ints, dtype=object)
    return np.stack([np.asarray(x % q, dtype=np.uint64) for q in moduli], axis=1)
