#!/usr/bin/env python3
"""pmc_summary.py <prof_dir> <tag>: per-kernel averages from a
tools/profile_run.sh run -> profiles/<tag>_rocprof_kernel_stats.csv (copied),
profiles/<tag>_pmc.json and profiles/pmc_traffic.json (what bench.py reads
for roofline.traffic).  HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE per launch
(MI355X_MICROARCH.md § HBM: gfx950 FETCH_SIZE tallies 128-B requests at 64 B;
checked here against this kernel's own algorithmic reads)."""
import collections
import csv
import glob
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# u32 kernels -> bench.py's kernel ids (k_row's second template argument is
# its mode: 0 forward rows, 1 inverse rows, 2 poly-mul rows)
FN = {"k_colt_fwd": "col_fwd", "k_colt_inv": "col_inv", "k_ks_rows": "ks_rows",
      "k_colt_decompose": "ks_decompose", "k_tensor_rows": "tensor_rows",
      "k_automorph_odd": "automorphism", "k_rescale": "rescale"}
ROW_MODES = {"0": "row_fwd", "1": "row_inv", "2": "row_mul"}


def short(kname):
    m = re.search(r"\bk_mf_ntt<(true|false)>", kname)
    if m:
        return "mf_ntt_inv" if m.group(1) == "true" else "mf_ntt_fwd"
    if re.search(r"\bk_plane_fused(_slots)?\(", kname):
        return "plane_fused"
    if re.search(r"\bk_mf_tensor\(", kname):
        return "mf_tensor"
    if re.search(r"\bk_mf_mul\(", kname):
        return "mf_mul"
    if re.search(r"\bk_ks_whole<unsigned int", kname):
        return "ks_whole"
    if re.search(r"\bk_tensor_rows<unsigned (int|long), \d+, true>", kname):
        return "tensor_whole"
    m = re.search(r"\bk_row<unsigned (int|long), (\d), \d+, (true|false), true>", kname)
    if m:
        return ("whole_fwd", "whole_inv", "whole_mul")[int(m.group(2))]
    m = re.search(r"(k_\w+)<([^>]*)>", kname)
    if not m or not m.group(2).startswith(("unsigned int", "unsigned long")):
        return None
    fn, targs = m.group(1), [t.strip() for t in m.group(2).split(",")]
    sfx = "_u64" if targs[0] == "unsigned long" else ""  # the wide-prime (u64) kernels apart
    if fn == "k_row":
        r = ROW_MODES.get(targs[1])
    else:
        r = FN.get(fn)
    return r + sfx if r else None


def counters(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k:
                agg[k][(r["Counter_Name"], r.get("Dispatch_Id", ""))].append(float(r["Counter_Value"]))
    out = {}
    for k, d2 in agg.items():
        per = collections.defaultdict(list)
        for (c, _), vals in d2.items():
            per[c].append(sum(vals))  # sum over XCD/SE instances within one dispatch
        out[k] = {c: sum(v) / len(v) for c, v in per.items()}
    return out


def main():
    # pmc_summary.py <prof_dir> <tag> [workload batch log_n L]
    prof, tag = sys.argv[1], sys.argv[2]
    workload, batch, log_n, L = (sys.argv[3:7] + ["polymul", "256", "16", "16"][len(sys.argv[3:7]):])
    res = collections.defaultdict(dict)
    for sub in ("fetch", "write", "sq", "grbm"):
        for k, d in counters(os.path.join(prof, sub)).items():
            res[k].update(d)
    stats = glob.glob(os.path.join(prof, "trace", "**", "*kernel_stats.csv"), recursive=True)
    trace = {}
    if stats:
        shutil.copy(stats[0], os.path.join(ROOT, "profiles", f"{tag}_rocprof_kernel_stats.csv"))
        for r in csv.DictReader(open(stats[0])):
            k = short(r["Name"])
            if k:
                trace[k] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}
    kernels = {}
    for k, d in res.items():
        fetch = d.get("FETCH_SIZE", 0.0) * 1024  # rocprofv3 reports KB
        write = d.get("WRITE_SIZE", 0.0) * 1024
        e = {"fetch_size_bytes": fetch, "write_size_bytes": write,
             "bytes_per_launch": 2 * fetch + write, **{c: v for c, v in d.items() if c.startswith(("SQ_", "GRBM"))}}
        if k in trace:
            e.update(trace[k])
            if "GRBM_GUI_ACTIVE" in d:
                e["effective_clock_ghz"] = d["GRBM_GUI_ACTIVE"] / 8 / trace[k]["avg_ns"]
        if "SQ_WAVE_CYCLES" in d and d["SQ_WAVE_CYCLES"]:
            w = d["SQ_WAVE_CYCLES"]
            e["frac_active"] = d.get("SQ_ACTIVE_INST_ANY", 0) / w
            e["frac_issue_stall"] = d.get("SQ_WAIT_INST_ANY", 0) / w
            e["frac_waitcnt_barrier"] = d.get("SQ_WAIT_ANY", 0) / w
        kernels[k] = e
    meta = {"workload": workload, "batch": int(batch), "log_n": int(log_n), "L": int(L),
            "source": f"tools/profile_run.sh {tag}", "kernels": kernels}
    with open(os.path.join(ROOT, "profiles", f"{tag}_pmc.json"), "w") as f:
        json.dump(meta, f, indent=1)
    # profiles/pmc_traffic.json: one entry per workload shape (bench.py
    # roofline.traffic); a new pass of the same shape replaces the old one
    tpath = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    entries = []
    if os.path.exists(tpath):
        old = json.load(open(tpath))
        entries = old.get("entries", [dict(old, workload="polymul")] if "kernels" in old else [])
    key = (workload, int(batch), int(log_n), int(L))
    entries = [e for e in entries if (e.get("workload"), e.get("batch"), e.get("log_n"), e.get("L")) != key]
    entries.append(meta)
    with open(tpath, "w") as f:
        json.dump({"entries": entries}, f, indent=1)
    for k, e in kernels.items():
        print(k, {x: (round(y, 3) if isinstance(y, float) else y) for x, y in e.items()})


if __name__ == "__main__":
    main()
