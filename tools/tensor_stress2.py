"""Full-output comparison of the matrix-core tensor (default path) against
the four-step tensor (RNT_PLANE=0) on the same device-drawn ciphertexts:
N = 2^16, L = 16, Bc ciphertexts (argv[2], default 64 = 1024 pairs, the
per-pair scratch), argv[1] rounds.  Prints, per round and output, the
mismatched words and where they fall (poly, limb, device-order position
bits), to locate a hazard."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "toy-heaan-ckks_amd"))
import rns_ntt as rn  # noqa: E402

N, L = 1 << 16, 16
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
Bc = int(sys.argv[2]) if len(sys.argv) > 2 else 64
mod = rn.generate_primes(31, L, N)
total = 0
for r in range(rounds):
    outs = {}
    for plane in ("1", "0"):
        os.environ["RNT_PLANE"] = plane
        Bd = rn.RnsBasis(mod, N)
        drng = rn.DeviceRng(500 + r)
        c = [rn.RnsPoly.sample_uniform(Bd, drng, Bc) for _ in range(4)]
        d = rn.ct_tensor(*c)
        outs[plane] = [x.channels() for x in d]
        del c, d, Bd
    for i in range(3):
        a, b = outs["1"][i], outs["0"][i]
        bad = np.argwhere(a != b)
        total += len(bad)
        if len(bad):
            pl = sorted({(int(p), int(l)) for p, l, _ in bad[:20000]})
            pos = bad[:, 2]
            print(f"round {r} d{i}: {len(bad)} words differ in {len(pl)} (poly, limb) planes, first {pl[:8]}; "
                  f"positions min {pos.min()} max {pos.max()}, bits set counts "
                  f"{[int(((pos >> k) & 1).sum()) for k in range(16)]}", flush=True)
        else:
            print(f"round {r} d{i}: equal", flush=True)
    del outs
sys.exit(1 if total else 0)
