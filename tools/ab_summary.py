#!/usr/bin/env python3
"""Median value and per-kernel average launch times over repeated bench runs."""
import json
import statistics
import sys

runs = [json.loads(open(f).read().strip().splitlines()[-1]) for f in sys.argv[1:]]
print("value  median %.1f  (%s)" % (statistics.median(r["value"] for r in runs),
                                   ", ".join("%.1f" % r["value"] for r in runs)))
pw = [r["power"] for r in runs if r.get("power")]
if pw:
    print("power  %s" % ", ".join("%sW %sMHz" % (p.get("package_w_median"), p.get("sclk_mhz_median")) for p in pw))
print("parity %s" % [r["config"].get("parity_spot_check") for r in runs])
for k in runs[0]["roofline"].get("kernels", {}):
    v = [r["roofline"]["kernels"][k]["avg_ms"] for r in runs]
    if any(x is None for x in v):
        continue
    print("%-8s median %.4f ms  (%s)" % (k, statistics.median(v), ", ".join("%.4f" % x for x in v)))
