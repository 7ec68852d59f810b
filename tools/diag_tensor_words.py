"""Locate wrong words of the matrix-core tensor (default path) against the
four-step tensor (RNT_PLANE=0) and infer which operand went wrong.

With a0 = c0^, a1 = c1^, b3 = c0'^, b4 = c1'^ (device-order forward
transforms), the tensor computes d0 = a0 b3 R^-1, d1 = (a1 b3 + a0 b4) R^-1
and d2 = INTT(a1 b4) (R = 2^32).  A wrong a1 shows as
  da1 = (d1_bad - d1) R / b3 = (NTT(d2_bad) - NTT(d2)) / b4   (mod q);
the script prints both quotients at each wrong d1 word, the implied bad a1
value and whether that value occurs anywhere among the batch's c0^..c1'^
words of the same limb (misrouted data) or among the last 2^20 words of any
operand.  Diagnostic only (the r05 split-load / persistent-forward
experiments, profiles/r05/ab_mf_ntt_split_load.txt)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "toy-heaan-ckks_amd"))
import rns_ntt as rn  # noqa: E402

N, L = 1 << 16, 16
Bc = int(sys.argv[2]) if len(sys.argv) > 2 else 16
mod = rn.generate_primes(31, L, N)
R = 1 << 32


def ntt_dev(Bd, ch):
    t = rn.RnsPoly.from_channels(ch, Bd)
    t.to_ntt_domain()
    return t.channels()


for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2):
    outs, fw = {}, {}
    for plane in ("1", "0"):
        os.environ["RNT_PLANE"] = plane
        Bd = rn.RnsBasis(mod, N)
        drng = rn.DeviceRng(900 + r)
        c = [rn.RnsPoly.sample_uniform(Bd, drng, Bc) for _ in range(4)]
        if plane == "0":
            for k in range(4):
                fw[k] = ntt_dev(Bd, c[k].channels())
        d = rn.ct_tensor(*c)
        outs[plane] = [x.channels() for x in d]
        if plane == "0":
            xx = {"1": ntt_dev(Bd, outs["1"][2]), "0": ntt_dev(Bd, outs["0"][2])}
        del c, d
    bad = np.argwhere(outs["1"][1] != outs["0"][1])
    bad2 = {(int(p), int(l)) for p, l in np.argwhere((outs["1"][2] != outs["0"][2]).any(axis=2))}
    bad1 = {(int(p), int(l)) for p, l, _ in bad}
    print(f"round {r}: d1 {len(bad)} wrong words in {len(bad1)} planes; d0 "
          f"{int((outs['1'][0] != outs['0'][0]).sum())} wrong; d2 wrong in {len(bad2)} planes, "
          f"same planes as d1: {bad1 == bad2}", flush=True)
    for p, l, x in bad[:40]:
        q = int(mod[l])
        d1b, d1g = int(outs["1"][1][p, l, x]), int(outs["0"][1][p, l, x])
        b3, b4 = int(fw[2][p, l, x]), int(fw[3][p, l, x])
        e1 = (d1b - d1g) * R * pow(b3, -1, q) % q
        e2 = (int(xx["1"][p, l, x]) - int(xx["0"][p, l, x])) * pow(b4, -1, q) % q
        a1 = int(fw[1][p, l, x])
        a1b = (a1 + e1) % q
        where = []
        for k in range(4):
            hit = np.argwhere(fw[k][:, l, :] == a1b)
            where += [f"c{k}^[p{int(a)}][{int(b)}]" for a, b in hit[:3]]
        print(f"  p{p} l{l} pos {x:5d} = {x:#06x}: da1 via d1 {e1} via d2 {e2} equal {e1 == e2}; "
              f"bad a1 {a1b} (a1 {a1}) found at {where}", flush=True)
