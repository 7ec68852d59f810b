"""Phase timeline of the matrix-core forward transform k_mf_ntt<false>
(measurement build).

  MF_ONLY=1 bash tools/build_variant.sh mftrace -DRNT_MF_TRACE
  RNSNTT_LIB=toy-heaan-ckks_amd/lib/variants/librnsntt_mftrace.so \\
      python tools/mf_trace.py [batch]

Runs rnt_ntt_fwd on a batch of N = 2^16, L = 16 polys a few times and prints
the mean time per phase (first and last wave of a workgroup to reach each
boundary, 100 MHz real-time stamps), the mean workgroup lifetime, the span,
and how many workgroups are in their load phase at once.  Stamps wait only
for their own scalar read: loads and stores stay asynchronous, so a phase
includes the memory waits its first use of the data has.
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "toy-heaan-ckks_amd"))
import rns_ntt as rn  # noqa: E402

WG, WV, ST = 4096, 16, 16
PH = ["load_issue", "p1a(+load wait)", "x1w+p1b", "sync1", "x1r0+sync", "x1w1+p2a", "sync2", "x1r1+p2b",
      "swap+p3", "p4+stores", "store_drain"]


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    n, L = 1 << 16, 16
    mod = rn.generate_primes(31, L, n)
    basis = rn.RnsBasis(mod, n)
    x = rn.RnsPoly.sample_uniform(basis, rn.DeviceRng(3), B)
    lib = rn.load()
    lib.rnt_debug_mf_trace.argtypes = [ctypes.c_void_p]
    lib.rnt_debug_mf_trace.restype = ctypes.c_int
    for _ in range(3):
        x.to_ntt_domain()
        x.to_coeff_domain()
    x.to_ntt_domain()  # the traced launch is the last forward
    basis.sync()
    buf = np.zeros(WG * WV * ST, dtype=np.uint64)
    assert lib.rnt_debug_mf_trace(buf.ctypes.data) == 0
    tr = buf.reshape(WG, WV, ST).astype(np.int64)[:, :, : len(PH) + 1]
    nwg = min(B * L, WG)
    # the persistent forward (one workgroup per CU) stamps only its first
    # gridDim.x slots, each with the workgroup's last plane
    stamped = (tr[:nwg] != 0).all(axis=(1, 2))
    nwg = int(stamped.sum()) if not stamped.all() else nwg
    w = tr[:nwg]
    first, last = w.min(axis=1), w.max(axis=1)
    t0 = first[:, :1]
    out = {"batch": B, "workgroups": nwg,
           "boundaries": ["start"] + PH,
           "first_wave_us": [round(float(v), 2) for v in ((first - t0).mean(0) / 100)],
           "last_wave_us": [round(float(v), 2) for v in ((last - t0).mean(0) / 100)]}
    d = np.diff(last, axis=1) / 100.0
    out["phase_us_last_wave"] = {p: round(float(d[:, i].mean()), 3) for i, p in enumerate(PH)}
    life = (last[:, -1] - first[:, 0]) / 100.0
    out["wg_life_us_mean"] = round(float(life.mean()), 2)
    out["span_us"] = round(float((last[:, -1].max() - first[:, 0].min()) / 100.0), 1)
    # how many workgroups are waiting on their plane load / draining stores at once
    out["zero_stamps"] = int((w == 0).sum())
    g0 = first[:, 0].min()
    grid = np.arange(g0, last[:, -1].max(), 100)
    if len(grid):
        in_p1 = ((first[:, 0][None, :] <= grid[:, None]) & (last[:, 2][None, :] > grid[:, None])).sum(1)
        out["wg_in_load+p1a_mean"] = round(float(in_p1.mean()), 1)
        out["wg_in_load+p1a_max"] = int(in_p1.max())
    # per wave index: mean boundary time (us from the workgroup's first stamp)
    out["per_wave_boundary_us"] = [[round(float(v), 2) for v in ((w[:, k] - t0).mean(0) / 100)]
                                   for k in range(WV)]
    np.save(os.environ.get("MF_TRACE_NPY", "/tmp/mf_trace.npy"), w)
    # the first round (one workgroup per CU) against the later ones
    for name, sl in (("round0", slice(0, 256)), ("later", slice(256, nwg))):
        dd = d[sl]
        out["phase_us_last_wave_" + name] = {p: round(float(dd[:, i].mean()), 3) for i, p in enumerate(PH)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
