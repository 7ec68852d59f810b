#!/usr/bin/env python3
"""stream_split_probe.py: poly-mul throughput of one batch on one stream
against the same pairs split over S contexts (each its own HIP stream),
issued round-robin with no cross-stream dependency.  N=2^16, L=16."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "toy-heaan-ckks_amd"))
import rns_ntt as rn  # noqa: E402

n, L, total = 1 << 16, 16, int(os.environ.get("PAIRS", "1024"))
mod = rn.generate_primes(31, L, n)
lib = rn.load()


def run(S, steps=30, warm=3):
    ctx = [rn.RnsBasis(mod, n) for _ in range(S)]
    per = total // S
    rng = rn.DeviceRng(7)
    ops = [(rn.RnsPoly(c, per), rn.RnsPoly.sample_uniform(c, rng, per), rn.RnsPoly.sample_uniform(c, rng, per))
           for c in ctx]
    for _ in range(warm):
        for o, a, b in ops:
            rn.check(lib.rnt_mul(o.handle, a.handle, b.handle))
    for c in ctx:
        c.sync()
    t = time.perf_counter()
    for _ in range(steps):
        for o, a, b in ops:
            rn.check(lib.rnt_mul(o.handle, a.handle, b.handle))
    for c in ctx:
        c.sync()
    return total * steps / (time.perf_counter() - t)


for rep in range(2):
    for S in (1, 2, 4):
        print(f"streams={S} pairs={total}: {run(S):.1f} poly-muls/s", flush=True)
