#!/usr/bin/env python3
"""debug_rot_small.py: rotation key-switch at N=2^17, L=32 for batches 1, 2
and 8 against the oracle, with host-uploaded and device-sampled keys; prints
which polys / limbs differ (diagnosis of the bench's B=1 spot check)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "toy-heaan-ckks_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import rns_ntt as rn  # noqa: E402
import pyoracle as orc  # noqa: E402

log_n, L = int(os.environ.get("LOGN", "17")), int(os.environ.get("LIMBS", "32"))
n = 1 << log_n
mod = rn.generate_primes(31, L, n)
Bs, ob = rn.RnsBasis(mod, n), orc.Basis(mod, n)
lib = rn.load()


def uniform(rng, count):
    q = np.array(mod, dtype=np.uint64)[None, :, None]
    return rng.integers(0, 1 << 62, size=(count, L, n), dtype=np.uint64) % q


for B in (1, 2, 8):
    for key_src in ("host", "device"):
        rng = np.random.default_rng(5)
        c0_h, c1_h = uniform(rng, B), uniform(rng, B)
        c0, c1 = rn.RnsPoly.from_channels(c0_h, Bs), rn.RnsPoly.from_channels(c1_h, Bs)
        if key_src == "host":
            ka_h, kb_h = uniform(rng, L), uniform(rng, L)
            key = rn.RnsGadgetKey.from_channels(ka_h, kb_h, Bs)
        else:
            drng = rn.DeviceRng(99)
            ka, kb = rn.RnsPoly.sample_uniform(Bs, drng, L), rn.RnsPoly.sample_uniform(Bs, drng, L)
            ka_h, kb_h = ka.channels(), kb.channels()
            key = rn.RnsGadgetKey(ka, kb)
        k = 1 << (log_n - 2)
        out0, out1 = rn.RnsPoly(Bs, B), rn.RnsPoly(Bs, B)
        rn.check(lib.rnt_ct_rotate(out0.handle, out1.handle, c0.handle, c1.handle, k, key.a.handle, key.b.handle))
        g0, g1 = out0.channels_of(0), out1.channels_of(0)
        w0, w1 = orc.rotate_ciphertext(ob, c0_h[0], c1_h[0], k, ka_h, kb_h, threads=16)
        bad0 = [l for l in range(L) if not np.array_equal(g0[0][l], w0[l])]
        bad1 = [l for l in range(L) if not np.array_equal(g1[0][l], w1[l])]
        print(f"B={B} key={key_src}: c0 bad limbs {bad0[:8]} ({len(bad0)}), c1 bad limbs {bad1[:8]} ({len(bad1)})",
              flush=True)
