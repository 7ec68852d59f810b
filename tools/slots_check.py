"""k_plane_fused_slots (RNT_PLANE_SLOTS=1: a^ scratch indexed by CU) against
the per-plane scratch kernel on the metric batch (N = 2^16, L = 16, 1024
pairs): every word of every plane compared, in chunks of 16 polys."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "toy-heaan-ckks_amd"))
import rns_ntt as rn  # noqa: E402

n, L, B = 1 << 16, 16, 1024
mod = rn.generate_primes(31, L, n)
Bd = rn.RnsBasis(mod, n)
drng = rn.DeviceRng(77)
a = rn.RnsPoly.sample_uniform(Bd, drng, B)
b = rn.RnsPoly.sample_uniform(Bd, drng, B)
os.environ.pop("RNT_PLANE_SLOTS", None)
c1 = a * b
os.environ["RNT_PLANE_SLOTS"] = "1"
c2 = a * b
a *= b  # in place, out aliases a
Bd.sync()
bad = 0
for p0 in range(0, B, 16):
    x, y, z = c1.channels_of(p0, 16), c2.channels_of(p0, 16), a.channels_of(p0, 16)
    bad += int((x != y).sum()) + int((x != z).sum())
print("slots vs per-plane: mismatched words", bad)
sys.exit(1 if bad else 0)
