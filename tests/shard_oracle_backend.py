"""CPU oracle backend for rns_ntt.sharded.LimbShardedPipeline (TEST ONLY).

Implements the backend interface with the oracle (oracle/pyoracle.py, the C
restatement of the reference) so the limb-sharded data flow -- which limbs
are gathered, broadcast and dropped where -- is checked on CPU ranks (gloo)
against the unsharded reference computation.  A "poly" here is an int64
torch tensor [L_r][B][N] of residues (coefficient domain).
"""
from __future__ import annotations

import numpy as np
import pyoracle as orc
import torch


class _Basis:
    def __init__(self, moduli, n):
        self.mods = [int(q) for q in moduli]
        self.n = n
        self.ob = orc.Basis(self.mods, n)

    def channel_count(self):
        return len(self.mods)


def _to_bln(poly: torch.Tensor) -> np.ndarray:
    return np.ascontiguousarray(poly.numpy().astype(np.uint64).transpose(1, 0, 2))


def _from_bln(a: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a.astype(np.int64).transpose(1, 0, 2)))


class OracleBackend:
    def make_basis(self, moduli, degree):
        return _Basis(moduli, degree)

    def drop_last(self, basis):
        return _Basis(basis.mods[:-1], basis.n)

    def batch(self, poly):
        return poly.shape[1]

    def upload(self, basis, channels):
        return _from_bln(np.asarray(channels, dtype=np.uint64))

    def download(self, poly):
        return _to_bln(poly)

    def key(self, basis, a_channels, b_channels):
        return np.asarray(a_channels, dtype=np.uint64), np.asarray(b_channels, dtype=np.uint64)

    def tensor(self, basis, c0, c1, c0p, c1p):
        a0, a1, b0, b1 = (_to_bln(x) for x in (c0, c1, c0p, c1p))
        ob = basis.ob
        d0 = np.stack([orc.mul(ob, a0[p], b0[p]) for p in range(a0.shape[0])])
        d1 = np.stack([orc.add(ob, orc.mul(ob, a0[p], b1[p]), orc.mul(ob, a1[p], b0[p]))
                       for p in range(a0.shape[0])])
        d2 = np.stack([orc.mul(ob, a1[p], b1[p]) for p in range(a0.shape[0])])
        return _from_bln(d0), _from_bln(d1), _from_bln(d2)

    def keyswitch(self, basis, src_full, key, d0, d1):
        """engine.rs:505-531 for this rank's target limbs: alpha_i = limb i of
        d2 (all global limbs) reduced mod each local q_j."""
        ka, kb = key
        src = src_full.numpy().astype(np.uint64)  # [L][B][N]
        ob = basis.ob
        B = src.shape[1]
        zero = np.zeros((B, len(basis.mods), basis.n), dtype=np.uint64)
        o0 = _to_bln(d0) if d0 is not None else zero.copy()
        o1 = _to_bln(d1) if d1 is not None else zero.copy()
        for p in range(B):
            for i in range(src.shape[0]):
                alpha = np.stack([src[i, p] % np.uint64(q) for q in basis.mods])
                o0[p] = orc.add(ob, o0[p], orc.mul(ob, alpha, kb[i]))
                o1[p] = orc.add(ob, o1[p], orc.mul(ob, alpha, ka[i]))
        return _from_bln(o0), _from_bln(o1)

    def rotate(self, basis, poly, k):
        """poly.rs:546-569 per poly on this rank's limbs."""
        x = _to_bln(poly)
        return _from_bln(np.stack([orc.rotate_slots(basis.ob, x[p], k)[0] for p in range(x.shape[0])]))

    rotate_planes = rotate

    def add(self, basis, a, b):
        x, y = _to_bln(a), _to_bln(b)
        return _from_bln(np.stack([orc.add(basis.ob, x[p], y[p]) for p in range(x.shape[0])]))

    def last_limb(self, poly):
        return poly[-1]

    def new_planes(self, basis, count, B):
        return torch.zeros((count, B, basis.n), dtype=torch.int64)

    def rescale(self, basis, out_basis, poly, last_plane, q_last):
        """poly.rs:211-224 restated: (c_i - (c_last mod q_i)) * (q_last mod q_i)^-1."""
        x = poly.numpy()
        last = last_plane.numpy()
        out = np.zeros((out_basis.channel_count(),) + x.shape[1:], dtype=np.int64)
        for li, q in enumerate(out_basis.mods):
            inv = pow(q_last % q, -1, q)
            for p in range(x.shape[1]):
                ci = [int(v) for v in x[li, p]]
                cl = [int(v) % q for v in last[p]]
                out[li, p] = [((a - b) % q) * inv % q for a, b in zip(ci, cl)]
        return torch.from_numpy(out)
