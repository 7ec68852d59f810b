"""Phase timeline of the whole-plane kernels (measurement build).

  bash tools/build_variant.sh trace -DRNT_PLANE_TRACE
  RNSNTT_LIB=toy-heaan-ckks_amd/lib/variants/librnsntt_trace.so \
      python tools/plane_trace.py [batch]

Runs the metric's poly-mul (N = 2^16, L = 16, 31-bit) a few times and prints,
for each kernel, the mean time wave 0 of a workgroup spends in each phase
(100 MHz real-time stamps, 10 ns resolution), the mean workgroup lifetime,
and the kernel's span from the first stamp to the last.  The stamps wait
for the wave's own memory operations, so "load" is the time to the last
load's return as wave 0 sees it.
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
PHASES = {
    "plane_fwd": ["load", "passA", "x1", "passB", "x2", "passC", "store"],
    "plane_mul": ["load", "passA", "x1", "passB", "x2", "passC", "product", "gsC", "ix2",
                  "gsB", "ix1", "gsA", "store"],
}


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    n, L = 1 << 16, 16
    mod = rn.generate_primes(31, L, n)
    basis = rn.RnsBasis(mod, n)
    drng = rn.DeviceRng(7)
    a = rn.RnsPoly.sample_uniform(basis, drng, B)
    b = rn.RnsPoly.sample_uniform(basis, drng, B)
    lib = rn.load()
    lib.rnt_debug_plane_trace.argtypes = [ctypes.c_void_p]
    lib.rnt_debug_plane_trace.restype = ctypes.c_int
    for _ in range(3):
        c = a * b
    basis.sync()
    buf = np.zeros(2 * WG * WV * ST, dtype=np.uint64)
    rc = lib.rnt_debug_plane_trace(buf.ctypes.data)
    assert rc == 0, rc
    tr = buf.reshape(2, WG, WV, ST).astype(np.int64)
    nwg = min(B * L, WG)
    out = {"batch": B, "workgroups_traced": nwg}
    for k, name in enumerate(("plane_fwd", "plane_mul")):
        ph = PHASES[name]
        w = tr[k, :nwg, :, : len(ph) + 1]
        # per phase boundary: the first and the last wave of the workgroup to reach it
        first, last = w.min(axis=1), w.max(axis=1)
        out[name + "_by_wave"] = {
            "boundary": ["start"] + ph,
            "first_wave_us": [round(float(v), 2) for v in ((first - first[:, :1]).mean(0) / 100)],
            "last_wave_us": [round(float(v), 2) for v in ((last - first[:, :1]).mean(0) / 100)],
            "wave0_us": [round(float(v), 2) for v in ((w[:, 0] - first[:, :1]).mean(0) / 100)],
        }
        s = last
        d = np.diff(s, axis=1) * 10.0 / 1000.0  # us
        life = (s[:, -1] - s[:, 0]) * 10.0 / 1000.0
        span = (s[:, -1].max() - s[:, 0].min()) * 10.0 / 1000.0
        start = np.sort(s[:, 0])
        per = {p: round(float(d[:, i].mean()), 3) for i, p in enumerate(ph)}
        out[name] = {"phase_us_mean": per, "wg_life_us_mean": round(float(life.mean()), 2),
                     "wg_life_us_p10_p90": [round(float(np.percentile(life, 10)), 2),
                                            round(float(np.percentile(life, 90)), 2)],
                     "span_us": round(float(span), 1),
                     "start_gap_us_median": round(float(np.median(np.diff(start))) * 10 / 1000, 4)}
        # time-resolved concurrency: how many workgroups are in their load phase at once
        t0 = s[:, 0].min()
        grid = np.arange(t0, s[:, -1].max(), 100)  # 1 us bins
        in_load = ((s[:, 0][None, :] <= grid[:, None]) & (s[:, 1][None, :] > grid[:, None])).sum(1)
        in_store = ((s[:, -2][None, :] <= grid[:, None]) & (s[:, -1][None, :] > grid[:, None])).sum(1)
        out[name]["wg_in_load_mean"] = round(float(in_load.mean()), 1)
        out[name]["wg_in_store_mean"] = round(float(in_store.mean()), 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
