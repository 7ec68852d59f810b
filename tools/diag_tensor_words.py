"""Locate wrong words of the matrix-core tensor (default path) against the
four-step tensor (RNT_PLANE=0) and test what they equal: for each wrong d1
word, is it the forward transform of c0 or c1 (the values the tensor's
first two epilogues stored at that address), or the four-step value?
Diagnostic only (r05 split-load experiment)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "toy-heaan-ckks_amd"))
import rns_ntt as rn  # noqa: E402

N, L = 1 << 16, 16
Bc = int(sys.argv[2]) if len(sys.argv) > 2 else 16
mod = rn.generate_primes(31, L, N)
for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2):
    outs, fw = {}, {}
    for plane in ("1", "0"):
        os.environ["RNT_PLANE"] = plane
        Bd = rn.RnsBasis(mod, N)
        drng = rn.DeviceRng(900 + r)
        c = [rn.RnsPoly.sample_uniform(Bd, drng, Bc) for _ in range(4)]
        if plane == "0":
            for k in range(4):
                t = rn.RnsPoly.from_channels(c[k].channels(), Bd)
                t.to_ntt_domain()
                fw[k] = t.channels()
        d = rn.ct_tensor(*c)
        outs[plane] = [x.channels() for x in d]
        del c, d, Bd
    a, b = outs["1"][1], outs["0"][1]
    bad = np.argwhere(a != b)
    print(f"round {r}: d1 {len(bad)} wrong words, d0 {int((outs['1'][0] != outs['0'][0]).sum())}, "
          f"d2 {int((outs['1'][2] != outs['0'][2]).sum())}", flush=True)
    for p, l, x in bad[:24]:
        got = int(a[p, l, x])
        tags = [f"c{k}^" for k in range(4) if int(fw[k][p, l, x]) == got]
        # which other position of the same plane holds the wrong value
        same = np.flatnonzero(b[p, l] == got)[:3].tolist()
        print(f"  p{p} l{l} pos {x:5d} = {x:#06x}: got {got} want {int(b[p, l, x])} equals {tags} "
              f"four-step d1 at {same}", flush=True)
