#!/usr/bin/env python3
"""tensor_traffic.py <dir>: k_mf_tensor's PMC bytes per launch for the
shipped build and each RNT_MF_TENSOR_MEAS build (tools/gpu_tensor_traffic.sh)
-> profiles/r06/tensor_traffic.json.  P = one 64-ct chunk's plane set
(64 cts x 16 limbs x 256 KiB); the algorithmic floor is 7P, the
one-plane-resident floor 15P; each build's saving is set
against the bytes its dropped temporary moves (write + reads)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import pmc_summary  # noqa: E402

P = 64 * 16 * 256 * 1024
DROPS = {"tmeas1": ("c1^ -> scratch slot, read at c0'^ and c1'^", 1, 2),
         "tmeas2": ("t = c1^ c0'^ -> d2's plane, read at c1'^", 1, 1),
         "tmeas3": ("c0^ -> d1's plane, read at c0'^ and c1'^", 1, 2)}


def per_launch(d, counter):
    m = pmc_summary.counters(d)
    return m.get("mf_tensor", {}).get(counter)


def main():
    d = sys.argv[1]
    res = {}
    for v in ("base", "tmeas1", "tmeas2", "tmeas3"):
        f = per_launch(os.path.join(d, f"{v}_FETCH_SIZE"), "FETCH_SIZE")
        w = per_launch(os.path.join(d, f"{v}_WRITE_SIZE"), "WRITE_SIZE")
        if f is None or w is None:
            continue
        f, w = f * 1024, w * 1024  # rocprofv3 reports KB
        res[v] = {"fetch_x2_bytes": 2 * f, "write_bytes": w, "bytes": 2 * f + w, "planes": (2 * f + w) / P,
                  "read_planes": 2 * f / P, "write_planes": w / P}
    base = res["base"]
    for v, (what, wr, rd) in DROPS.items():
        if v not in res:
            continue
        r = res[v]
        r["dropped"] = what
        r["alg_saving_planes"] = {"write": wr, "read": rd, "total": wr + rd}
        r["measured_saving_planes"] = {"write": base["write_planes"] - r["write_planes"],
                                       "read": base["read_planes"] - r["read_planes"],
                                       "total": base["planes"] - r["planes"]}
    out = {"P_bytes": P, "shape": "one 64-ct chunk at N=2^16, L=16 (bench.py --workload ctmul --ct-batch 64)",
           "algorithmic_planes": 7, "one_plane_resident_floor_planes": 15, "builds": res}
    os.makedirs(os.path.join(ROOT, "profiles", "r06"), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "profiles", "r06", "tensor_traffic.json"), "w"), indent=1)
    for v, r in res.items():
        print(v, round(r["planes"], 2), "P  (reads", round(r["read_planes"], 2), "writes", round(r["write_planes"], 2), ")",
              r.get("measured_saving_planes", ""))


if __name__ == "__main__":
    main()
