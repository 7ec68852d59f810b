"""Host model of the MFMA plane transform (dev tool; the design of
csrc/rnt_mfma.hip).

Checks, for a 31-bit prime at N = 2^16:
  1. the merged negacyclic CT network's radix-16 passes are block matrices
     M_U (U = the index bits above the pass) with M_U[j][k] = z_{U,j}^k;
  2. the twist factorisation M_U = F . diag(beta_U^k) with one F for all U
     and all passes (beta_U = z_{U,0});
  3. the four passes (exact modular matrices) reproduce the oracle's
     to_ntt_domain in the device's bit-reversed order;
  4. the digit arithmetic of one pass (balanced byte digits of the centred
     matrix and data, int32 digit sums as the i8 MFMA forms them, the
     shift-add recombination and the signed Montgomery reduction) is exact
     and stays within the stated ranges.

Run: python tools/mfma_model.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import pyoracle as orc  # noqa: E402

LOGN = 16
N = 1 << LOGN
R = 1 << 32


def brv(x, bits):
    return int(format(x, f"0{bits}b")[::-1], 2)


def tables(q, psi):
    tw = [1] * N
    for g in range(1, N):
        tw[g] = pow(psi, brv(g, LOGN), q)
    return tw


def pass_matrix(q, tw, p, U):
    """16x16 matrix of pass p (bits 15-4p .. 12-4p) for upper bits U."""
    b_lo = 12 - 4 * p
    M = [[0] * 16 for _ in range(16)]
    for k in range(16):
        v = [0] * 16
        v[k] = 1
        for sb in (3, 2, 1, 0):  # stage at index bit b_lo + sb
            b = b_lo + sb
            for kk in range(16):
                if kk & (1 << sb):
                    continue
                i = (U << (b_lo + 4)) | (kk << b_lo)
                w = tw[(N + i) >> (b + 1)]
                x, y = v[kk], v[kk | (1 << sb)]
                t = w * y % q
                v[kk], v[kk | (1 << sb)] = (x + t) % q, (x - t) % q
        for j in range(16):
            M[j][k] = v[j]
    return M


def centred(v, q):
    v %= q
    return v - q if v > q // 2 else v


def digits(v):
    """Balanced signed byte digits of |v| < 2^30 (v = sum d_a 256^a)."""
    u = (v + 0x80808080) & 0xFFFFFFFF
    return [((u >> (8 * a)) & 0xFF) - 128 for a in range(4)]


def main():
    mod = orc.generate_primes(31, 2, N)
    q = mod[0]
    Bo = orc.Basis([q], N)
    psi = Bo.psi(0)
    tw = tables(q, psi)
    # 1, 2: Vandermonde structure and the shared F
    F = None
    for p in range(4):
        for U in range(0, 1 << (4 * p), max(1, (1 << (4 * p)) // 37)):
            M = pass_matrix(q, tw, p, U)
            z = [M[j][1] for j in range(16)]
            for j in range(16):
                for k in range(16):
                    assert M[j][k] == pow(z[j], k, q), (p, U, j, k)
            beta = z[0]
            Fu = [[M[j][k] * pow(beta, (q - 1 - 1) * k % (q - 1), q) % q for k in range(16)] for j in range(16)]
            if F is None:
                F = Fu
            assert Fu == F, ("F differs", p, U)
    print("1, 2: M_U[j][k] = z_{U,j}^k and M_U = F diag(beta_U^k), one F for every pass and U: OK")
    # 3: the four passes reproduce to_ntt in device (bit-reversed) order
    rng = np.random.default_rng(5)
    a = rng.integers(0, q, size=N, dtype=np.uint64)
    x = [int(v) for v in a]
    for p in range(4):
        b_lo = 12 - 4 * p
        cache = {}
        y = [0] * N
        for i in range(N):
            if (i >> b_lo) & 15:
                continue
            U = i >> (b_lo + 4)
            M = cache.get(U)
            if M is None:
                M = cache[U] = pass_matrix(q, tw, p, U)
            grp = [x[i | (k << b_lo)] for k in range(16)]
            for j in range(16):
                y[i | (j << b_lo)] = sum(M[j][k] * grp[k] for k in range(16)) % q
        x = y
    want = orc.to_ntt(Bo, a[None, :])[0]
    dev = [int(want[brv(i, LOGN)]) for i in range(N)]
    assert x == dev
    print("3: four radix-16 passes == to_ntt_domain (device order): OK")
    # 4: digit arithmetic of one pass (p = 2 with the twist in VALU form)
    qinv_neg = (-pow(q, -1, R)) % R
    Ws = [[centred(F[j][k] * (1 << (8 * b)) * R, q) for b in range(4) for k in range(16)] for j in range(16)]
    worst_C, worst_T, worst_r = 0, 0, 0
    for trial in range(200):
        xs = [centred(int(v), q) for v in rng.integers(0, q, size=16)]
        if trial == 0:
            xs = [-(q // 2)] * 16
        if trial == 1:
            xs = [q // 2] * 16
        xd = [digits(v) for v in xs]
        for j in range(16):
            C = [0] * 4
            for kb, w in enumerate(Ws[j]):
                b, k = divmod(kb, 16)
                wd = digits(w)
                for aa in range(4):
                    C[aa] += wd[aa] * xd[k][b]
            worst_C = max(worst_C, *(abs(c) for c in C))
            lo = C[0] + (C[1] << 8)
            hi = C[2] + (C[3] << 8)
            T = lo + hi * 65536
            worst_T = max(worst_T, abs(T))
            m = ((T & (R - 1)) * qinv_neg) % R
            m = m - R if m >= R // 2 else m
            V = T + m * q
            assert V % R == 0
            r = V >> 32
            worst_r = max(worst_r, abs(r))
            assert (r - sum(F[j][k] * xs[k] for k in range(16))) % q == 0
    print(f"4: digit arithmetic exact; max |C_a| = {worst_C} (< 2^20 = {1 << 20}), max |T| = 2^{np.log2(worst_T):.2f},"
          f" max |r| = {worst_r} (q/2 + 2^14 = {q // 2 + (1 << 14)})")


if __name__ == "__main__":
    main()
