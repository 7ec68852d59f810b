#!/usr/bin/env python3
"""pmc_table.py <prof_dir> [name-substr...]: per-kernel averages from a
tools/profile_any.sh run (HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE)."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
keys = sys.argv[2:]


def short(n):
    n = n.replace("void rnt::", "").replace("(anonymous namespace)::", "").split("(")[0]
    return n


vals = collections.defaultdict(lambda: collections.defaultdict(list))
for sub in ("fetch", "write", "sq", "grbm", "ic"):
    for f in glob.glob(os.path.join(d, sub, "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
trace = {}
for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        trace[short(r["Name"])] = (int(r["Calls"]), float(r["AverageNs"]))
for k, c in sorted(vals.items(), key=lambda kv: -trace.get(kv[0], (0, 0))[1] * trace.get(kv[0], (0, 0))[0]):
    if keys and not any(x in k for x in keys):
        continue
    if k not in trace:
        continue
    avg = {n: sum(v) / len(v) for n, v in c.items()}
    calls, ns = trace[k]
    hbm = 2 * avg.get("FETCH_SIZE", 0) * 1024 + avg.get("WRITE_SIZE", 0) * 1024
    w = avg.get("SQ_WAVE_CYCLES", 0) or 1
    clk = avg.get("GRBM_GUI_ACTIVE", 0) / 8 / ns if ns else 0
    print(f"{k[:48]:48s} calls {calls:4d} avg {ns/1e3:9.1f} us  HBM {hbm/1e6:9.1f} MB ({hbm/ns:6.2f} TB/s)  "
          f"clk {clk:4.2f}  active {avg.get('SQ_ACTIVE_INST_ANY',0)/w:4.2f} issue-stall {avg.get('SQ_WAIT_INST_ANY',0)/w:4.2f} "
          f"wait {avg.get('SQ_WAIT_ANY',0)/w:4.2f}  VALU/wave {avg.get('SQ_INSTS_VALU',0)/max(avg.get('SQ_WAVES',1),1):7.0f}")
    if "SQC_ICACHE_MISSES" in avg:
        print(f"{'':48s} icache misses {avg['SQC_ICACHE_MISSES']:.0f} hits {avg.get('SQC_ICACHE_HITS',0):.0f} "
              f"lds-issue-stall {avg.get('SQ_WAIT_INST_LDS',0)/w:4.2f} smem {avg.get('SQ_INSTS_SMEM',0)/max(avg.get('SQ_WAVES',1),1):.0f}/wave")
