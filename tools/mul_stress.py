"""Full-output stress of the default N = 2^16 poly-mul (k_mf_mul) against
the four-step kernels (RNT_PLANE=0) on the same device-drawn operands:
every word of B pairs x 16 limbs (argv[2], default 1024: the metric's
batch and the CU-slot scratch path), argv[1] rounds, plus the VALU
whole-plane product (RNT_MF_MUL=0) on the first round.  Prints, per round,
the number of differing words and where they fall."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "toy-heaan-ckks_amd"))
import rns_ntt as rn  # noqa: E402

N, L = 1 << 16, 16
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
mod = rn.generate_primes(31, L, N)
total = 0
for r in range(rounds):
    outs = {}
    modes = [("mf_mul", {}), ("four_step", {"RNT_PLANE": "0"})]
    if r == 0:
        modes.append(("plane_fused", {"RNT_MF_MUL": "0"}))
    for name, env in modes:
        for k in ("RNT_PLANE", "RNT_MF_MUL"):
            os.environ.pop(k, None)
        os.environ.update(env)
        Bd = rn.RnsBasis(mod, N)
        drng = rn.DeviceRng(7000 + r)
        a = rn.RnsPoly.sample_uniform(Bd, drng, B)
        b = rn.RnsPoly.sample_uniform(Bd, drng, B)
        outs[name] = (a * b).channels_batch()
        del a, b, Bd
    for name in outs:
        if name == "four_step":
            continue
        bad = np.argwhere(outs[name] != outs["four_step"])
        total += len(bad)
        where = sorted({(int(p), int(l)) for p, l, _ in bad[:2000]})[:8]
        print(f"round {r} {name}: {len(bad)} words differ" + (f", planes {where}" if len(bad) else ""), flush=True)
sys.exit(1 if total else 0)
