#!/usr/bin/env python3
"""energy_model.py: the poly-mul's power-cap model ("the
ceiling"), fitted to measured workloads.

  energy_model.py collect <gpu_energy.sh dir>... <out.json>
      per workload: the bench line's rate, step time, package power and
      sclk (rocm-smi power probe while the step keeps running) and, from
      the rocprofv3 --pmc passes of the same shape, the per-step VALU and
      LDS wave instructions (SQ_INSTS_VALU / SQ_INSTS_LDS) and HBM bytes
      (2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md § HBM) of the
      step's kernels (per-dispatch means x launches per step).
  energy_model.py fit <data.json> [--json out.json]
      least squares  P = P0 + e_v * VALU/s + e_m * HBM bytes/s  over every
      workload, leave-one-out checks of power and of the rate each
      workload would run at with the power it drew, and the poly-mul's
      rate at the 1400 W cap for lower-traffic variants:
      rate = (cap - P0) / (e_v * V + e_m * M) per product, bounded by the
      VALU-only build's rate (no plane data moved, full clock).
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import re

import numpy as np

KMAP = [(r"^k_colt_fwd|^k_col_fwd", "col_fwd"), (r"^k_colt_inv|^k_col_inv", "col_inv"),
        (r"^k_row<[^,]+, 0", "row_fwd"), (r"^k_row<[^,]+, 1", "row_inv"), (r"^k_row<[^,]+, 2", "row_mul"),
        (r"^k_elementwise", "elementwise"), (r"^k_copy16", "copy"), (r"^k_ks_rows", "ks_rows"),
        (r"^k_colt_decompose|^k_col_decompose", "ks_decompose"), (r"^k_tensor_rows", "tensor_rows"),
        (r"^k_automorph", "automorphism"), (r"^k_rescale", "rescale")]


def kid(name: str):
    # "void rnt::k_row<unsigned int, 2, 8, false>(...)" -> "k_row<unsigned int, 2, ..."
    name = re.sub(r"^void ", "", name.strip())
    name = re.sub(r"^(rnt::)?(\(anonymous namespace\)::)?", "", name)
    for pat, k in KMAP:
        if re.search(pat, name):
            return k
    return None


def pmc(d: str) -> dict:
    """{kernel id: {counter: mean per dispatch}} (instances summed per dispatch)."""
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kid(r["Kernel_Name"])
            if k:
                per[(k, r["Counter_Name"])][r.get("Dispatch_Id", "")] += float(r["Counter_Value"])
    out = collections.defaultdict(dict)
    for (k, c), disp in per.items():
        out[k][c] = sum(disp.values()) / len(disp)
    return out


def collect(dirs, out_path):
    rows = []
    for d in dirs:
        for j in sorted(glob.glob(os.path.join(d, "*.json"))):
            tag = os.path.basename(j)[:-5]
            lines = [x for x in open(j).read().splitlines() if x.startswith("{")]
            if not lines:
                continue
            b = json.loads(lines[-1])
            pw = b.get("power") or {}
            if not pw.get("package_w_median") or not pw.get("sclk_mhz_median"):
                continue
            kern = (b.get("roofline") or {}).get("kernels") or {}
            counts = {}
            for part in ("sq", "fetch", "write"):
                for k, cs in pmc(os.path.join(d, f"{tag}_{part}")).items():
                    counts.setdefault(k, {}).update(cs)
            per_step = collections.Counter()
            for k, kv in kern.items():
                lps = kv["launches"] / b["steps"]
                for c, v in counts.get(k, {}).items():
                    per_step[c] += v * lps
            t = b["ms_per_step"] * 1e-3
            rows.append({
                "tag": tag, "P_w": pw["package_w_median"], "sclk_ghz": pw["sclk_mhz_median"] / 1e3,
                "rate": b["value"], "unit": b["unit"], "ms_per_step": b["ms_per_step"],
                "units_per_step": b["value"] * t,
                # per step, the step's kernels only
                "valu_insts": per_step["SQ_INSTS_VALU"], "lds_insts": per_step["SQ_INSTS_LDS"],
                # rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB
                "hbm_bytes": (2 * per_step["FETCH_SIZE"] + per_step["WRITE_SIZE"]) * 1024,
                "kernels": {k: round(kv["launches"] / b["steps"], 3) for k, kv in kern.items()},
            })
    json.dump({"source": "tools/gpu_energy.sh + tools/energy_model.py collect", "workloads": rows},
              open(out_path, "w"), indent=1)
    print(f"{len(rows)} workloads -> {out_path}")


def _rates(r):
    t = r["ms_per_step"] * 1e-3
    return r["valu_insts"] / t / 1e9, r["hbm_bytes"] / t / 1e12  # G wave-instr/s, TB/s


def _lstsq(rows):
    X = np.array([[1.0, *_rates(r)] for r in rows])
    y = np.array([r["P_w"] for r in rows])
    c, *_ = np.linalg.lstsq(X, y, rcond=None)
    return c


def _joules(c, r):
    n = r["units_per_step"]
    return c[1] * r["valu_insts"] / n / 1e9 + c[2] * r["hbm_bytes"] / n / 1e12  # J per unit


def fit(path, out_json=None, cap=1400.0, holdout=("polymul_meas3", "polymul_meas4",
                                                   "polymul_b256_meas3", "polymul_b256_meas4")):
    allrows = json.load(open(path))["workloads"]
    # the traffic-emulation builds (RNT_MEAS=3/4: every butterfly kept, the
    # 5- or 7-plane traffic of a fused design) are held out of the fit: they
    # test its what-if predictions
    rows = [r for r in allrows if r["tag"] not in holdout]
    held = [r for r in allrows if r["tag"] in holdout]
    c = _lstsq(rows)
    P0, ev, em = (float(x) for x in c)
    print(f"P = {P0:.0f} W + {ev:.3f} nJ x VALU wave-instr/s + {em:.1f} pJ x HBM B/s   ({len(rows)} workloads)")
    res = {"model": "P = P0 + e_v * VALU wave-instructions/s + e_m * HBM bytes/s",
           "P0_w": P0, "e_valu_nj_per_wave_instr": ev, "e_hbm_pj_per_byte": em, "points": []}
    print(f"{'workload':20s} {'P':>6s} {'fit':>6s} {'loo':>6s} {'GHz':>5s} {'VALU G/s':>8s} {'TB/s':>5s}"
          f" {'rate':>10s} {'loo rate':>10s} {'err':>6s}")
    for i, r in enumerate(rows):
        ci = _lstsq(rows[:i] + rows[i + 1:])
        v, m = _rates(r)
        pf, pl = c @ [1, v, m], ci @ [1, v, m]
        rate_loo = (r["P_w"] - ci[0]) / _joules(ci, r)  # the rate the drawn power buys
        err = rate_loo / r["rate"] - 1
        print(f"{r['tag']:20s} {r['P_w']:6.0f} {pf:6.0f} {pl:6.0f} {r['sclk_ghz']:5.2f} {v:8.1f} {m:5.2f}"
              f" {r['rate']:10.4g} {rate_loo:10.4g} {err * 100:+5.1f}%")
        res["points"].append({"tag": r["tag"], "P_w": r["P_w"], "fit_w": float(pf), "loo_w": float(pl),
                              "rate": r["rate"], "unit": r["unit"], "loo_rate": float(rate_loo),
                              "loo_rate_err": float(err), "valu_G_per_s": v, "hbm_TB_per_s": m,
                              "sclk_ghz": r["sclk_ghz"]})
    if held:
        print("\nheld out (traffic emulation builds):")
        res["held_out"] = []
        for r in held:
            v, m = _rates(r)
            rate_pred = min((min(r["P_w"], cap) - c[0]) / _joules(c, r), float("inf"))
            err = rate_pred / r["rate"] - 1
            print(f"{r['tag']:20s} {r['P_w']:6.0f} {c @ [1, v, m]:6.0f} {r['sclk_ghz']:5.2f} {v:8.1f} {m:5.2f}"
                  f" {r['rate']:10.4g} {rate_pred:10.4g} {err * 100:+5.1f}%  ({r['hbm_bytes'] / r['units_per_step'] / 1e6:.1f} MB/unit)")
            res["held_out"].append({"tag": r["tag"], "P_w": r["P_w"], "rate": r["rate"], "pred_rate": rate_pred,
                                    "err": err, "hbm_MB_per_unit": r["hbm_bytes"] / r["units_per_step"] / 1e6})
    base = next((r for r in rows if r["tag"] == "polymul"), None)
    valu_only = next((r for r in rows if r["tag"] == "polymul_meas1"), None)
    if base:
        n = base["units_per_step"]
        V, M = base["valu_insts"] / n, base["hbm_bytes"] / n
        ceiling = valu_only["rate"] * 2.4 / valu_only["sclk_ghz"] if valu_only else float("inf")
        print(f"\npoly-mul (N=2^16, L=16): {V / 1e6:.2f} M VALU wave-instr and {M / 1e6:.1f} MB of HBM per product;"
              f" energy {(ev * V / 1e9 + em * M / 1e12) * 1e3:.2f} mJ + P0 x time; VALU-only ceiling"
              f" {ceiling / 1e3:.0f}k/s at 2.4 GHz")
        res["polymul_per_product"] = {"valu_wave_instr": V, "hbm_bytes": M, "valu_only_ceiling": ceiling}
        res["at_cap"] = {}
        for name, planes, vf in (("as built: 9 planes of HBM per (poly, limb)", 9, 1.0),
                                 ("7 planes (row pass + inverse column pass fused on one CU)", 7, 1.0),
                                 ("5 planes (whole-plane fwd(a), then fwd(b) x a^ -> inverse)", 5, 1.0),
                                 ("3 planes (read a, read b, write c only)", 3, 1.0),
                                 ("9 planes, 10% fewer VALU instructions", 9, 0.9)):
            e = ev * V * vf / 1e9 + em * M * planes / 9 / 1e12
            rate = min((cap - P0) / e, ceiling)
            res["at_cap"][name] = rate
            print(f"  {name:62s} -> {rate / 1e3:6.1f}k poly-muls/s")
    if out_json:
        json.dump(res, open(out_json, "w"), indent=1)


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    c = sub.add_parser("collect")
    c.add_argument("paths", nargs="+")
    f = sub.add_parser("fit")
    f.add_argument("data")
    f.add_argument("--json")
    f.add_argument("--cap", type=float, default=1400.0)
    a = ap.parse_args()
    if a.cmd == "collect":
        collect(a.paths[:-1], a.paths[-1])
    else:
        fit(a.data, a.json, a.cap)


if __name__ == "__main__":
    main()
