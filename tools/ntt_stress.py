"""Full-output check of the matrix-core transforms (k_mf_ntt) at N = 2^16,
L = 16: per round, argv[2] device-drawn polys (default 128) through
rnt_ntt_fwd on the default path and on the four-step kernels (RNT_PLANE=0),
every word compared, then the default inverse of the default forward
against the input.  argv[1] rounds.  RNSNTT_LIB picks the library."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "toy-heaan-ckks_amd"))
import rns_ntt as rn  # noqa: E402

N, L = 1 << 16, 16
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
B = int(sys.argv[2]) if len(sys.argv) > 2 else 128
mod = rn.generate_primes(31, L, N)
total = 0
for r in range(rounds):
    got = {}
    for plane in ("1", "0"):
        os.environ["RNT_PLANE"] = plane
        Bd = rn.RnsBasis(mod, N)
        x = rn.RnsPoly.sample_uniform(Bd, rn.DeviceRng(900 + r), B)
        x0 = x.channels() if plane == "1" else None
        x.to_ntt_domain()
        got[plane] = x.channels()
        if plane == "1":
            x.to_coeff_domain()
            back = x.channels()
            nb = int((back != x0).sum())
            total += nb
            print(f"round {r}: inverse(forward) vs input: {nb} words differ", flush=True)
            del x0, back
        del x, Bd
    bad = np.argwhere(got["1"] != got["0"])
    total += len(bad)
    print(f"round {r}: forward vs four-step: {len(bad)} words differ"
          + (f" in planes {sorted({(int(p), int(l)) for p, l, _ in bad[:2000]})[:6]}" if len(bad) else ""), flush=True)
    del got
sys.exit(1 if total else 0)
