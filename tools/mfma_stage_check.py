"""GPU check of the MFMA transform kernels stage by stage (dev tool).

RNT_PLANE=5 (the MFMA path) at N = 2^16, L = 2: the forward transform's
prefixes (passes 0-1 and 0-2, words written canonical at their in-place
index by rnt_debug_mf_stage) against tools/mfma_model.py's exact passes,
then the whole forward / inverse transforms and the product against the
oracle.  Prints one line per check; exit status 1 on the first mismatch.

Run on the GPU box: python tools/mfma_stage_check.py
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "toy-heaan-ckks_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tools")):
    sys.path.insert(0, p)
os.environ["RNT_PLANE"] = "5"
import mfma_model as mm  # noqa: E402
import pyoracle as orc  # noqa: E402
import rns_ntt as rn  # noqa: E402

N = 1 << 16


def model_passes(q, psi, a, npass):
    """In-place words after the first npass radix-16 passes (numpy, exact)."""
    tw = mm.tables(q, psi)
    x = a.astype(object)
    for p in range(npass):
        b_lo = 12 - 4 * p
        y = np.zeros(N, dtype=object)
        idx = np.arange(N)
        grp_base = idx[((idx >> b_lo) & 15) == 0]
        U = grp_base >> (b_lo + 4)
        mats = {}
        for u in np.unique(U):
            mats[int(u)] = np.array(mm.pass_matrix(q, tw, p, int(u)), dtype=object)
        for base, u in zip(grp_base, U):
            M = mats[int(u)]
            g = x[base + (np.arange(16) << b_lo)]
            y[base + (np.arange(16) << b_lo)] = M.dot(g) % q
        x = y
    return np.array([int(v) for v in x], dtype=np.uint64)


def main():
    lib = rn.load()
    lib.rnt_debug_mf_stage.restype = ctypes.c_int
    lib.rnt_debug_mf_stage.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L = 2
    mod = rn.generate_primes(31, L, N)
    Bd, Bo = rn.RnsBasis(mod, N), orc.Basis(mod, N)
    rng = np.random.default_rng(11)
    a_h = orc.uniform_poly(mod, N, rng, batch=2)
    b_h = orc.uniform_poly(mod, N, rng, batch=2)
    ok = True
    for stop in (2, 3):
        t = rn.RnsPoly.from_channels(a_h, Bd)
        rn.check(lib.rnt_debug_mf_stage(t.handle, stop))
        got = t.channels()
        for i in range(2):
            for l in range(L):
                want = model_passes(mod[l], Bo.psi(l), a_h[i][l], stop)
                bad = int(np.count_nonzero(got[i][l] != want))
                print(f"stage {stop} poly {i} limb {l}: {'OK' if bad == 0 else f'{bad} mismatches'}", flush=True)
                if bad:
                    ok = False
                    idx = np.nonzero(got[i][l] != want)[0][:8]
                    print("   first bad idx", idx.tolist(), got[i][l][idx].tolist(), want[idx].tolist())
    t = rn.RnsPoly.from_channels(a_h, Bd)
    t.to_ntt_domain()
    nt = t.channels()
    for i in range(2):
        good = np.array_equal(nt[i], orc.to_ntt(Bo, a_h[i]))
        print(f"forward poly {i}: {'OK' if good else 'MISMATCH'}", flush=True)
        ok &= good
    x_h = orc.uniform_poly(mod, N, rng, batch=2)
    u = rn.RnsPoly.from_channels(x_h, Bd, in_ntt_domain=True)
    u.to_coeff_domain()
    ct = u.channels()
    for i in range(2):
        good = np.array_equal(ct[i], orc.to_coeff(Bo, x_h[i]))
        print(f"inverse poly {i}: {'OK' if good else 'MISMATCH'}", flush=True)
        ok &= good
    c = (rn.RnsPoly.from_channels(a_h, Bd) * rn.RnsPoly.from_channels(b_h, Bd)).channels()
    for i in range(2):
        good = np.array_equal(c[i], orc.mul(Bo, a_h[i], b_h[i]))
        print(f"product poly {i}: {'OK' if good else 'MISMATCH'}", flush=True)
        ok &= good
    print("ALL OK" if ok else "FAILED")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
