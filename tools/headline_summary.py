#!/usr/bin/env python3
"""headline_summary.py <dir> <tag>: one-lease headline evidence
(tools/gpu_headline.sh) -> profiles/<tag>_headline.json and
profiles/<tag>_rocprof_kernel_stats.csv.  Reconciles the rocprof kernel
time with the bench line's ms_per_step (both from the same box, with the
sclk each run's power probe saw) and carries the line's live PMC traffic."""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import pmc_summary  # noqa: E402


def main():
    d, tag = sys.argv[1], sys.argv[2]
    line = json.loads(open(os.path.join(d, "bench.json")).read().strip().splitlines()[-1])
    tline = json.loads(open(os.path.join(d, "trace.json")).read().strip().splitlines()[-1])
    stats = glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True)[0]
    shutil.copy(stats, os.path.join(ROOT, "profiles", f"{tag}_rocprof_kernel_stats.csv"))
    kern = {}
    for r in csv.DictReader(open(stats)):
        k = pmc_summary.short(r["Name"])
        if k:
            kern[k] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                       "min_ms": float(r["MinNs"]) / 1e6, "max_ms": float(r["MaxNs"]) / 1e6}
    sq = pmc_summary.counters(os.path.join(d, "sq"))
    roof = line["roofline"]
    dom = next(iter(roof["kernels"]))
    out = {
        "what": "one lease: bench line (live PMC traffic), rocprofv3 kernel-trace of the same command, SQ pass",
        "bench": {"value": line["value"], "ms_per_step": line["ms_per_step"], "kernel_avg_ms_hip_events":
                  roof["kernels"][dom]["avg_ms"], "power": line.get("power"), "traffic": roof.get("traffic"),
                  "traffic_source": roof.get("traffic_source"), "traffic_live": roof.get("traffic_live"),
                  "traffic_ratio": roof.get("traffic_ratio"), "frac": roof["frac"],
                  "frac_u64_equiv": roof.get("frac_u64_equiv"), "parity_spot_check":
                  line["config"].get("parity_spot_check")},
        "trace_run": {"value": tline["value"], "ms_per_step": tline["ms_per_step"], "power": tline.get("power"),
                      "kernels_rocprof": kern},
        "sq": sq.get(dom),
    }
    rk = kern.get(dom)
    if rk:
        # the dominant kernel's dispatches in the trace run's timed region:
        # after its `warmup` launches, the next `steps` (the power probe's
        # launches follow them and enter rocprof's all-dispatch average)
        trows = []
        for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if pmc_summary.short(r["Kernel_Name"]) == dom:
                    trows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        trows.sort()
        w, st = tline["warmup"], tline["steps"]
        timed = trows[w:w + st]
        timed_ms = sum(e - b for b, e in timed) / len(timed) / 1e6 if timed else None
        out["reconcile"] = {
            "rocprof_avg_ms_all_dispatches": rk["avg_ms"], "rocprof_dispatches": rk["calls"],
            "rocprof_timed_avg_ms": timed_ms, "rocprof_timed_dispatches": len(timed),
            "trace_run_ms_per_step": tline["ms_per_step"],
            "rocprof_timed_over_trace_step": timed_ms / tline["ms_per_step"] if timed_ms else None,
            "bench_ms_per_step": line["ms_per_step"],
            "bench_kernel_avg_ms_hip_events": roof["kernels"][dom]["avg_ms"],
            "rocprof_timed_over_bench_step": timed_ms / line["ms_per_step"] if timed_ms else None,
            "sclk_bench_mhz": (line.get("power") or {}).get("sclk_mhz_median"),
            "sclk_trace_mhz": (tline.get("power") or {}).get("sclk_mhz_median"),
        }
    if out["sq"] and out["sq"].get("SQ_WAVE_CYCLES"):
        w = out["sq"]["SQ_WAVE_CYCLES"]
        out["sq_fracs"] = {"active": out["sq"].get("SQ_ACTIVE_INST_ANY", 0) / w,
                           "issue_stall": out["sq"].get("SQ_WAIT_INST_ANY", 0) / w,
                           "waitcnt_barrier": out["sq"].get("SQ_WAIT_ANY", 0) / w}
    path = os.path.join(ROOT, "profiles", f"{tag}_headline.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out.get("reconcile"), indent=1))
    print("traffic", out["bench"]["traffic"], out["bench"]["traffic_ratio"], out["bench"]["traffic_source"])


if __name__ == "__main__":
    main()
