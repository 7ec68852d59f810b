"""Repeated tensor products at the slot-scratch batch (N = 2^16, L = 16, 128
ciphertexts = 2048 (poly, limb) pairs): each round draws fresh ciphertexts,
runs rnt_ct_tensor on the default path (k_mf_tensor) and the four-step path
(RNT_PLANE=0), and checks sampled ciphertexts' d0^, d1^, d2 against the
oracle.  Prints the mismatches per path and round."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "toy-heaan-ckks_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
import pyoracle as orc  # noqa: E402
import rns_ntt as rn  # noqa: E402

N, L, Bc = 1 << 16, 16, 128
mod = rn.generate_primes(31, L, N)
Bo = orc.Basis(mod, N)
q = np.array(mod, dtype=object)[:, None]
rinv = np.array([pow(2, -32, int(x)) for x in mod], dtype=object)[:, None]


def want(c0, c1, c0p, c1p):
    sc = lambda x: ((x.astype(object) * rinv) % q).astype(np.uint64)  # noqa: E731
    return (sc(orc.to_ntt(Bo, orc.mul(Bo, c0, c0p))),
            sc(orc.to_ntt(Bo, orc.add(Bo, orc.mul(Bo, c0, c1p), orc.mul(Bo, c1, c0p)))),
            orc.mul(Bo, c1, c1p))


rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
bad_total = 0
for r in range(rounds):
    for plane in ("1", "0"):
        os.environ["RNT_PLANE"] = plane
        Bd = rn.RnsBasis(mod, N)
        drng = rn.DeviceRng(1000 + r)
        c = [rn.RnsPoly.sample_uniform(Bd, drng, Bc) for _ in range(4)]
        d = rn.ct_tensor(*c)
        bad = []
        for p in (0, 31, 64, 100, 127):
            w = want(*[x.channels_of(p)[0] for x in c])
            for i in range(3):
                g = d[i].channels_of(p)[0]
                if not np.array_equal(g, w[i]):
                    bad.append((p, i, int((g != w[i]).sum())))
        print(f"round {r} RNT_PLANE={plane}: {'ok' if not bad else bad}", flush=True)
        bad_total += len(bad)
sys.exit(1 if bad_total else 0)
