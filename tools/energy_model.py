#!/usr/bin/env python3
"""energy_model.py <dir> [--json out.json]: the poly-mul's power-cap model
("the ceiling").

Input: tools/gpu_energy.sh's output -- per workload a bench JSON line (its
step time, per-kernel launches and the rocm-smi power probe: package watts
and sclk while the step keeps running) and rocprofv3 --pmc passes of the
same shape (SQ_INSTS_VALU, SQ_INSTS_LDS, FETCH_SIZE, WRITE_SIZE).

Model (least squares over every workload):
    P = a + b * f + e_v * VALU/s + e_l * LDS/s + e_m * HBM bytes/s
f = sclk (GHz), VALU/LDS = wave instructions (SQ_INSTS_*), HBM bytes =
2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md § HBM's gfx950 correction).
a + b f is what the chip draws at clock f beyond the counted work (static,
clock tree, fabric, everything not proportional to these counts).

Prediction at the 1400 W cap for a variant of the poly-mul: with its
counts per product (V, Ls, M) and its products per clock k (the measured
rate / sclk, i.e. cycles per product held fixed), the clock solves
a + b f + (e_v V + e_l Ls + e_m M) k f = cap, and the rate is k f (or the
clock ceiling 2.4 GHz times k, whichever is lower).
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
    name = re.sub(r"^void ", "", name.strip())
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


def load(d: str) -> list:
    rows = []
    for j in sorted(glob.glob(os.path.join(d, "*.json"))):
        tag = os.path.basename(j)[:-5]
        try:
            line = [x for x in open(j).read().splitlines() if x.startswith("{")][-1]
        except IndexError:
            continue
        b = json.loads(line)
        pw = b.get("power") or {}
        if not pw.get("package_w_median") or not pw.get("sclk_mhz_median"):
            continue
        kern = (b.get("roofline") or {}).get("kernels") or {}
        counts = {}
        for part in ("sq", "fetch", "write"):
            for k, cs in pmc(os.path.join(d, f"{tag}_{part}")).items():
                for c, v in cs.items():
                    counts.setdefault(k, {})[c] = v
        steps = b["steps"]
        per_step = collections.Counter()
        for k, kv in kern.items():
            lps = kv["launches"] / steps
            for c, v in counts.get(k, {}).items():
                per_step[c] += v * lps
        hbm = 2 * per_step["FETCH_SIZE"] * 1024 + per_step["WRITE_SIZE"] * 1024  # rocprofv3 reports KiB
        t = b["ms_per_step"] * 1e-3
        rows.append({"tag": tag, "P": pw["package_w_median"], "f": pw["sclk_mhz_median"] / 1e3,
                     "valu": per_step["SQ_INSTS_VALU"] / t / 1e9, "lds": per_step["SQ_INSTS_LDS"] / t / 1e9,
                     "hbm": hbm / t / 1e12, "value": b["value"], "unit": b["unit"], "ms": b["ms_per_step"],
                     "per_unit": {"valu": per_step["SQ_INSTS_VALU"], "lds": per_step["SQ_INSTS_LDS"], "hbm": hbm},
                     "units_per_step": b["value"] * t})
    return rows


def fit(rows):
    X = np.array([[1.0, r["f"], r["valu"], r["lds"], r["hbm"]] for r in rows])
    y = np.array([r["P"] for r in rows])
    coef, *_ = np.linalg.lstsq(X, y, rcond=None)
    return coef, X @ coef


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json")
    ap.add_argument("--cap", type=float, default=1400.0)
    args = ap.parse_args()
    rows = load(args.dir)
    if len(rows) < 6:
        raise SystemExit(f"need >= 6 workloads with power and PMC data, got {len(rows)}")
    coef, pred = fit(rows)
    names = ["a_W", "b_W_per_GHz", "e_valu_nJ_per_Ginstr(W per Ginstr/s)", "e_lds_W_per_Ginstr_s",
             "e_hbm_W_per_TBs"]
    print("fit:", {n: round(float(c), 3) for n, c in zip(names, coef)})
    loo = []
    for i in range(len(rows)):
        c, _ = fit(rows[:i] + rows[i + 1:])
        x = np.array([1.0, rows[i]["f"], rows[i]["valu"], rows[i]["lds"], rows[i]["hbm"]])
        loo.append(float(x @ c))
    out = {"coef": dict(zip(["a", "b", "e_valu", "e_lds", "e_hbm"], map(float, coef))), "points": []}
    print(f"{'workload':16s} {'P':>7s} {'fit':>7s} {'loo':>7s} {'GHz':>5s} {'VALU G/s':>9s} {'LDS G/s':>8s} {'HBM TB/s':>8s}")
    for r, p, l in zip(rows, pred, loo):
        print(f"{r['tag']:16s} {r['P']:7.0f} {p:7.0f} {l:7.0f} {r['f']:5.2f} {r['valu']:9.1f} {r['lds']:8.1f} {r['hbm']:8.2f}")
        out["points"].append({**{k: r[k] for k in ("tag", "P", "f", "valu", "lds", "hbm", "value", "unit", "ms")},
                              "fit": float(p), "loo": float(l)})
    # the poly-mul at the cap, and what-ifs
    base = next((r for r in rows if r["tag"] == "polymul"), None)
    if base:
        a, b, ev, el, em = coef
        n = base["units_per_step"]
        V, Ls, M = (base["per_unit"][k] / n for k in ("valu", "lds", "hbm"))
        k = base["value"] / base["f"]  # products per (GHz * s)

        def rate(Vx, Lx, Mx, kx):
            # joules per product: V, Ls in wave instructions, M in bytes
            # (the coefficients are W per G instr/s and W per TB/s)
            e = ev * Vx / 1e9 + el * Lx / 1e9 + em * Mx / 1e12
            f = (args.cap - a) / (b + e * kx)
            f = min(f, 2.4)
            return kx * f, f

        # k (products per GHz-second) is held fixed: the same cycles per
        # product, only the energy changes -- an upper bound for a variant
        # that moves fewer bytes, since it also assumes no new stalls
        scen = {"as measured (9 planes of HBM per limb)": (V, Ls, M, k),
                "5 planes (whole-plane fwd(a) + fused product)": (V, Ls, M * 5 / 9, k),
                "3 planes (read a, b, write c only)": (V, Ls, M * 3 / 9, k),
                "VALU instructions -10%": (V * 0.9, Ls, M, k),
                "no HBM traffic at all": (V, Ls, 0.0, k)}
        out["polymul_per_product"] = {"valu": V, "lds": Ls, "hbm_bytes": M, "products_per_GHz_s": k}
        out["scenarios"] = {}
        print(f"\npoly-mul per product: VALU {V:.3g}, LDS {Ls:.3g} wave-instr, HBM {M / 1e6:.1f} MB;"
              f" measured {base['value']:.0f}/s at {base['P']:.0f} W, {base['f']:.2f} GHz")
        for name, (Vx, Lx, Mx, kx) in scen.items():
            r, f = rate(Vx, Lx, Mx, kx)
            out["scenarios"][name] = {"rate": r, "GHz": f}
            print(f"  {name:48s} -> {r / 1e3:7.1f}k/s at {f:.2f} GHz")
    if args.json:
        json.dump(out, open(args.json, "w"), indent=1)


if __name__ == "__main__":
    main()
