#!/usr/bin/env python3
"""RNS-NTT poly-mul throughput on MI355X (BASELINE.json metric).

Workload (BASELINE configs[3] ring, the metric's quoted shape): N = 2^16,
16 RNS primes from the reference's generate_primes(31, 16, N) rule.  One
step = one batched coefficient-domain poly-mul c = a * b (poly.rs:307-329,
the `a *= &b` of every CkksEngine call site) over `--batch` pairs per GPU,
inputs resident in HBM.  Multi-GPU: one process per GPU (torchrun); the
batch is sharded across ranks with no data-path collective (each rank owns
its own pairs), so scaling is weak; only the timing barrier / max-reduce
crosses ranks (gloo control plane).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "toy-heaan-ckks_amd")
sys.path.insert(0, PKG)

METRIC = "RNS-NTT poly-muls/sec (N=2^16, 16 primes) at 1/2/4/8 GPUs; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md chip table); 6.29 TB/s measured copy


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--batch", type=int, default=256, help="poly-mul pairs per GPU per step")
    p.add_argument("--log-n", type=int, default=16)
    p.add_argument("--limbs", type=int, default=16)
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget")
    p.add_argument("--no-cpu-baseline", action="store_true")
    return p.parse_args()


def relaunch_with_torchrun(args) -> int:
    """--gpus N > 1 without torchrun: start torchrun as a CHILD process (this
    process has not touched the GPU) and return its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", os.environ.get("MASTER_PORT", "29517"),
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def cpu_baseline(mod, n, budget_s):
    """The oracle (reference-faithful C restatement, u128 `%`) on this host's
    cores: a bounded sample of the same workload, timed in this run."""
    import numpy as np

    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle as orc

    threads = max(1, min(16, os.cpu_count() or 1))
    Bo = orc.Basis(mod, n)
    rng = np.random.default_rng(11)
    count = threads  # one pair per worker per pass; each pair = L (poly, limb) items
    a = orc.uniform_poly(mod, n, rng, batch=count)
    b = orc.uniform_poly(mod, n, rng, batch=count)
    done, elapsed = 0, 0.0
    while elapsed < budget_s:
        elapsed += orc.polymul_batch_mt(Bo, a, b, threads)
        done += count
    return {
        "value": done / elapsed,
        "unit": "poly-muls/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{done} coefficient-domain poly-muls (N={n}, L={len(mod)}), {count} per pass over "
                  f"{threads} threads, {elapsed:.1f} s wall; oracle/oracle.c restating poly.rs:307-329",
    }


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch_with_torchrun(args))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import numpy as np

    import rns_ntt as rn  # loads librnsntt.so (HIP runtime) before torch
    from rns_ntt.dist import Comm, weak_throughput

    comm = Comm.from_env()
    barrier, max_over_ranks = comm.barrier, comm.max

    n = 1 << args.log_n
    L = args.limbs
    mod = rn.generate_primes(31, L, n)
    B = rn.RnsBasis(mod, n, device=local_rank)
    batch = args.batch
    wb = 4 if max(mod) < (1 << 31) else 8

    # synthetic inputs: 16 seeded unique pairs tiled to the batch (rank-seeded)
    rng = np.random.default_rng(1234 + rank)
    uniq = min(16, batch)
    qa = np.array(mod, dtype=np.uint64)[None, :, None]
    a_u = (rng.integers(0, 1 << 62, size=(uniq, L, n), dtype=np.uint64) % qa)
    b_u = (rng.integers(0, 1 << 62, size=(uniq, L, n), dtype=np.uint64) % qa)
    reps = (batch + uniq - 1) // uniq
    a = rn.RnsPoly.from_channels(np.tile(a_u, (reps, 1, 1))[:batch], B)
    b = rn.RnsPoly.from_channels(np.tile(b_u, (reps, 1, 1))[:batch], B)
    del a_u, b_u
    out = rn.RnsPoly(B, batch)
    lib = rn.load()

    for _ in range(args.warmup):
        rn.check(lib.rnt_mul(out.handle, a.handle, b.handle))
    B.sync()
    barrier()
    B.profile_enable(True)
    B.sync()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        rn.check(lib.rnt_mul(out.handle, a.handle, b.handle))
    B.sync()
    t1 = time.perf_counter()
    barrier()
    elapsed = max_over_ranks(t1 - t0)
    kernels = {}
    for k in ("col_fwd", "row_mul", "col_inv"):
        cnt, ms = B.profile_read(k)
        kernels[k] = {"launches": cnt, "avg_ms": ms / cnt if cnt else None, "total_ms": ms}
    B.profile_enable(False)

    ms_per_step = elapsed / args.steps * 1e3
    value = weak_throughput(batch, world, elapsed, args.steps)

    # spot parity of the timed output against the first unique pair
    if rank == 0:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import pyoracle as orc

        ch = out.channels()
        Bo = orc.Basis(mod, n)
        rng2 = np.random.default_rng(1234 + rank)
        a_u = (rng2.integers(0, 1 << 62, size=(uniq, L, n), dtype=np.uint64) % qa)
        b_u = (rng2.integers(0, 1 << 62, size=(uniq, L, n), dtype=np.uint64) % qa)
        parity_ok = bool(np.array_equal(ch[0], orc.mul(Bo, a_u[0], b_u[0])))
        del ch
    else:
        parity_ok = True

    # roofline of the dominant kernel: algorithmic bytes per launch / average
    # launch time (a step may issue several launches when the batch is
    # chunked; bytes per launch = bytes per step * steps / launches)
    elem = L * batch * n
    step_bytes = {"col_fwd": 4 * elem * wb, "row_mul": 3 * elem * wb, "col_inv": 2 * elem * wb}
    dom = max(kernels, key=lambda k: kernels[k]["total_ms"])
    dom_ms = kernels[dom]["avg_ms"]
    alg_bytes = {k: step_bytes[k] * args.steps / max(kernels[k]["launches"], 1) for k in kernels}
    achieved = alg_bytes[dom] / (dom_ms * 1e-3) / 1e9
    traffic = None
    tpath = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if os.path.exists(tpath):
        try:
            with open(tpath) as f:
                t = json.load(f)
            kt = t.get("kernels", {}).get(dom)
            if kt and t.get("batch") == batch and t.get("log_n") == args.log_n and t.get("L") == L:
                traffic = kt.get("bytes_per_launch")
        except Exception:
            traffic = None
    op_bytes = 3 * L * n * wb  # read a, read b, write c per poly-mul at the device word width
    roofline = {
        "bound": "hbm",
        "kernel": dom,
        "achieved": achieved,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS,
        "traffic": traffic,
        "alg_bytes_per_launch": alg_bytes[dom],
        "whole_op_GBs": value / world * op_bytes / 1e9,
        "whole_op_frac": value / world * op_bytes / 1e9 / HBM_PEAK_GBS,
        "whole_op_frac_u64_equiv": value / world * 3 * L * n * 8 / 1e9 / HBM_PEAK_GBS,
        "kernels": kernels,
    }

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(mod, n, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "poly-muls/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32" if wb == 4 else "u64",
            "data": "synthetic (seeded uniform residues)",
            "config": {
                "workload": f"coefficient-domain RNS-NTT poly-mul c=a*b, N=2^{args.log_n}, L={L} x 31-bit primes",
                "N": n,
                "L": L,
                "batch_per_gpu": batch,
                "global_batch": batch * world,
                "parallelism": f"batch-sharded x{world}, no collective",
                "parity_spot_check": parity_ok,
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    comm.close()


if __name__ == "__main__":
    main()
