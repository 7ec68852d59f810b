#!/usr/bin/env python3
"""RNS-NTT poly-mul throughput on MI355X (BASELINE.json metric).

Default workload (the metric's shape, BASELINE configs[3] ring): N = 2^16,
16 RNS primes from the reference's generate_primes(31, 16, N) rule.  One
step = one batched coefficient-domain poly-mul c = a * b (poly.rs:307-329,
the `a *= &b` of every CkksEngine call site) over `--batch` pairs' worth of
work per GPU, inputs resident in HBM.

Multi-GPU: one process per GPU (torchrun).  `--shard limb`
(default) gives rank r a contiguous run of the 16 limbs of a global batch of
batch * N_gpus pairs -- the north star's limb sharding; `--shard batch`
gives each rank its own `--batch` pairs over all limbs.  Both keep the work
per GPU fixed (weak scaling) and need no data-path collective for poly-mul;
only the timing barrier / max-reduce crosses ranks (gloo control plane).

`--workload ctmul` times BASELINE config 4's pipeline instead: ct x ct ->
gadget relinearisation -> rescale.  Its default layout at N > 1 is config
4's own, `--shard limb`: the RCCL all-gather of d2 and the broadcast of the
last limb (rns_ntt.sharded).  `--shard batch` is SURVEY §8e's zero-collective
comparison (each rank its own ciphertexts over all limbs, a full key
replica); the line's config.parallelism names the layout that ran.

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
CT_METRIC = "ct x ct -> relin -> rescale ciphertexts/sec (N=2^{log_n}, {L} primes)"
ROT_METRIC = "rotation key-switches/sec (N=2^17, 32 primes, power-of-two Galois offsets)"
ENC_METRIC = "CKKS encode+decode round trips/sec (N=2^16, 16 primes, N/2 complex slots)"
NTT_METRIC = "RNS-NTT forward+inverse transform pairs/sec (N=2^16, 16 primes)"
PW_METRIC = "NTT-domain pointwise poly-muls/sec (N=2^16, 16 primes)"
HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md chip table); ~6.3 TB/s achievable
# VALU peak in radix-2 butterflies/s: all 1024 SIMDs (256 CUs
# x 4) issue the canonical 31-bit CT butterfly -- 3 half-rate + 8 full-rate
# wave64 instructions -- for 64 lanes at a time, at the per-instruction costs
# measured on this chip (tools/oprate.hip: 4.1 and 2.2 SIMD cycles) and the
# 2.4 GHz maximum clock: 1024 * 64 * 2.4e9 / 29.9 = 5.26e12 butterflies/s.
VALU_BFLY_CYCLES = 3 * 4.1 + 8 * 2.2
VALU_PEAK_BFLY = 1024 * 64 * 2.4e9 / VALU_BFLY_CYCLES
MFMA_PEAK_I8 = 5.0e15  # dense i8 MFMA ops/s (MI355X_MICROARCH.md: 2x BF16's ~2.5e15 per clock)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--workload", choices=("polymul", "ctmul", "rotate", "encode", "ntt", "pointwise", "copy"),
                   default="polymul")
    p.add_argument("--shard", choices=("limb", "batch"), default="limb",
                   help="multi-GPU layout: limb (default, the north star's and config 4's layout; "
                        "ctmul/rotate join over RCCL) or batch (SURVEY 8e's zero-collective comparison)")
    p.add_argument("--batch", type=int, default=1024, help="poly-mul pairs per GPU per step")
    p.add_argument("--inputs", choices=("device", "host"), default="device",
                   help="poly-mul operands: seeded uniform residues drawn on the device (Philox, "
                        "rnt_sample_uniform) or 16 seeded host pairs tiled to the batch and uploaded")
    p.add_argument("--ct-batch", type=int, default=128, help="ciphertext pairs per GPU per step (ctmul)")
    p.add_argument("--chunk", type=int, default=None,
                   help="ctmul: ciphertexts per pipeline chunk (default 64, the library's key-switch "
                        "chunk at N=2^16 under the default 4 GiB RNT_KS_WS_MB)")
    p.add_argument("--rot-batch", type=int, default=8, help="ciphertexts per rotation (rotate)")
    p.add_argument("--enc-batch", type=int, default=64, help="plaintexts per step (encode)")
    p.add_argument("--log-n", type=int, default=16)
    p.add_argument("--limbs", type=int, default=16)
    p.add_argument("--prime-bits", type=int, default=31,
                   help="poly-mul primes from generate_primes(bits, L, N); 30 takes the lazy path")
    p.add_argument("--cpu-seconds", type=float, default=16.0, help="CPU baseline sample budget")
    p.add_argument("--rot-keys", choices=("per-offset", "shared"), default="per-offset",
                   help="rotate: a distinct gadget key per offset (SURVEY 8d sweep 1) or one resident key")
    p.add_argument("--rot-offsets", choices=("pow2", "all"), default="pow2",
                   help="rotate: the log2(N/2) power-of-two offsets, or every offset 1..N/2-1 with "
                        "one resident key (SURVEY 8d sweep 2)")
    p.add_argument("--graph", action="store_true",
                   help="ctmul / rotate: the reference engine's call shape -- fused per-call C-ABI ops "
                        "(rnt_ct_mul_relin + rnt_ct_rescale, rnt_ct_rotate) on each GPU's own ciphertexts, "
                        "the step recorded once as a HIP graph and replayed (rnt_capture_begin / "
                        "rnt_graph_launch); reports device-busy = kernel time / step time")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-power", action="store_true", help="skip the rocm-smi power/clock samples")
    p.add_argument("--no-live-pmc", action="store_true",
                   help="poly-mul at N=1: skip the two rocprofv3 --pmc child passes that measure "
                        "roofline.traffic in this run (then it comes from the committed pass)")
    p.add_argument("--strong", action="store_true",
                   help="poly-mul: --batch is the fixed global batch split over the ranks (strong "
                        "scaling) instead of the per-GPU batch (weak, the default)")
    return p.parse_args()


def relaunch_with_torchrun(args) -> int:
    """--gpus N > 1 without torchrun: start torchrun as a CHILD process (this
    process has not touched the GPU) and return its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", os.environ.get("MASTER_PORT", "29517"),
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def data_backend() -> str:
    """The limb-sharded joins' process-group backend: "nccl" (RCCL over
    xGMI, one GPU per rank).  BENCH_ONE_DEVICE=1 rehearsals put every rank
    on device 0, where RCCL refuses to run, so they join over gloo (host
    copies of the same tensors) to exercise the rest of the N-rank path."""
    return "gloo" if os.environ.get("BENCH_ONE_DEVICE") == "1" else "nccl"


def oracle():
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle as orc

    return orc


def host_info():
    """What the CPU baseline ran on: lscpu model and sockets, the machine's
    CPU count and the CPUs this process may use (the GPU box gives each job a
    share of 16 of the machine's many CPUs; os.cpu_count() reports them all)."""
    info = {"cpu_count": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["affinity"] = os.cpu_count()
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "Model name":
                info["model"] = v
            elif k == "Socket(s)":
                info["sockets"] = int(v) if v.isdigit() else v
            elif k == "Core(s) per socket":
                info["cores_per_socket"] = int(v) if v.isdigit() else v
            elif k == "Thread(s) per core":
                info["threads_per_core"] = int(v) if v.isdigit() else v
    except (OSError, subprocess.SubprocessError):
        pass
    return info


def usable_threads() -> int:
    """The CPU threads this job may use for the CPU baseline: the job's CPU
    share as the GPU box sets it (OMP_NUM_THREADS, 16 per GPU on the
    MI355X boxes, whose rules cap a job's worker pools at that share), else
    every CPU in this process' affinity mask.  The host itself is reported
    beside it (host_info: 2 x 64-core EPYC 9575F, 256 CPUs shared by the
    host's 8 GPUs' jobs)."""
    aff = host_info()["affinity"] or 1
    try:
        share = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        share = 0
    return max(1, min(aff, share) if share > 0 else aff)


def cpu_baseline(mod, n, budget_s):
    """The oracle (reference-faithful C restatement of poly.rs:307-329, u128
    `%`) on this host: single-threaded, as the reference runs, and over every
    usable core (std::thread-style workers over (poly, limb) items), each on a
    bounded sample of the same workload timed in this run."""
    import numpy as np

    orc = oracle()
    Bo = orc.Basis(mod, n)
    rng = np.random.default_rng(11)

    def timed(threads, budget):
        count = threads  # one pair per worker per pass; each pair = L (poly, limb) items
        a = orc.uniform_poly(mod, n, rng, batch=count)
        b = orc.uniform_poly(mod, n, rng, batch=count)
        done, elapsed = 0, 0.0
        while elapsed < budget:
            elapsed += orc.polymul_batch_mt(Bo, a, b, threads)
            done += count
        return done, elapsed

    threads = usable_threads()
    d1, e1 = timed(1, budget_s / 2)
    dn, en = timed(threads, budget_s / 2)
    host = host_info()
    return {
        "value": dn / en,
        "unit": "poly-muls/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{dn} coefficient-domain poly-muls (N={n}, L={len(mod)}), {threads} per pass over "
                  f"{threads} threads, {en:.1f} s wall; oracle/oracle.c restating poly.rs:307-329",
        "cores_basis": (f"the job's CPU share (OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS')}, "
                        f"affinity {host.get('affinity')} of {host.get('cpu_count')} CPUs)"
                        if os.environ.get("OMP_NUM_THREADS") else
                        f"every CPU of the affinity mask ({host.get('affinity')})"),
        "single_thread": {"value": d1 / e1, "cores": 1,
                          "sample": f"{d1} poly-muls on one thread, {e1:.1f} s wall"},
        "host": host,
    }


def power_probe(step, sync, device, seconds=3.0):
    """Package power and graphics clock while `step` keeps the GPU busy for
    `seconds` after the timed region: rocm-smi (read-only) sampled from a
    thread, the first sample dropped as ramp-up.  Evidence for the power-cap
    ceiling of DESIGN.md §4; None when rocm-smi is unavailable."""
    import re
    import statistics
    import threading

    def smi(*flags):
        try:
            return subprocess.run(["rocm-smi", "-d", str(device), *flags], capture_output=True,
                                  text=True, timeout=15).stdout
        except (OSError, subprocess.SubprocessError):
            return ""

    cap = re.search(r"Max Graphics Package Power \(W\):\s*([\d.]+)", smi("--showmaxpower"))
    samples, stop = [], threading.Event()

    def sampler():
        while not stop.is_set():
            out = smi("--showpower", "--showclocks")
            w = re.search(r"Package Power \(W\):\s*([\d.]+)", out)
            c = re.search(r"sclk clock level:[^(]*\((\d+)Mhz\)", out)
            if not w:
                return
            samples.append((float(w.group(1)), int(c.group(1)) if c else None))

    th = threading.Thread(target=sampler, daemon=True)
    t_end = time.perf_counter() + seconds
    th.start()
    while time.perf_counter() < t_end:
        for _ in range(8):
            step()
        sync()
    stop.set()
    th.join(timeout=20)
    samples = samples[1:]
    if not samples:
        return None
    clocks = [c for _, c in samples if c]
    return {"package_w_median": statistics.median(w for w, _ in samples),
            "sclk_mhz_median": statistics.median(clocks) if clocks else None,
            "cap_w": float(cap.group(1)) if cap else None, "samples": len(samples),
            "how": f"rocm-smi --showpower --showclocks on device {device} while the same step ran "
                   f"{seconds:.0f} s more after the timed region"}


def uniform(rng, mods, count, n):
    import numpy as np

    q = np.array(mods, dtype=np.uint64)[None, :, None]
    return rng.integers(0, 1 << 62, size=(count, len(mods), n), dtype=np.uint64) % q


def pmc_field(kernel, workload, batch, log_n, L, field):
    """Another per-launch field (e.g. SQ_INSTS_VALU) of the same committed
    pass as traffic_for; None when none of this shape is committed."""
    tpath = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(tpath) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    for e in t.get("entries", []):
        if (e.get("workload"), e.get("batch"), e.get("log_n"), e.get("L")) == (workload, batch, log_n, L):
            return e.get("kernels", {}).get(kernel, {}).get(field)
    return None


def traffic_for(kernel, workload, batch, log_n, L):
    """HBM bytes per launch of `kernel` (2 x FETCH_SIZE + WRITE_SIZE, the
    gfx950 correction of MI355X_MICROARCH.md § HBM) from the committed
    rocprofv3 --pmc passes of this exact workload shape
    (profiles/pmc_traffic.json, tools/profile_run.sh + tools/pmc_summary.py);
    None when no pass of this shape is committed."""
    tpath = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(tpath) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    for e in t.get("entries", []):
        if (e.get("workload"), e.get("batch"), e.get("log_n"), e.get("L")) == (workload, batch, log_n, L):
            kt = e.get("kernels", {}).get(kernel)
            return kt.get("bytes_per_launch") if kt else None
    return None


def _pmc_csv_means(d, kernel_re):
    """Per-dispatch counter values of the kernels matching kernel_re in a
    rocprofv3 --pmc output dir (summed over the XCD/SE instances of one
    dispatch), averaged over dispatches: {counter: mean per launch}."""
    import collections
    import csv
    import glob
    import re

    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if re.search(kernel_re, r["Kernel_Name"]):
                per[r["Counter_Name"]][r.get("Dispatch_Id", "")] += float(r["Counter_Value"])
    return {c: sum(v.values()) / len(v) for c, v in per.items() if v}


def live_pmc(args, kernel_re):
    """roofline.traffic measured in THIS run: two rocprofv3 --pmc passes of the
    same workload shape (FETCH_SIZE; WRITE_SIZE + GRBM_GUI_ACTIVE: the
    per-block counter limits allow no single pass), each a child process
    (python3 bench.py after `--`, as the profiler requires) under its own
    time limit, on this box right after the timed region.  HBM bytes per
    launch = 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md § HBM: gfx950
    FETCH_SIZE tallies 128-B requests at 64 B; rocprofv3 reports KB).
    None (and the reason) when the profiler is missing or a pass fails."""
    import shutil
    import tempfile

    prof = shutil.which("rocprofv3")
    if not prof:
        return None, "rocprofv3 not found"
    child = [sys.executable, os.path.abspath(__file__), "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
             "--no-power", "--no-live-pmc", "--batch", str(args.batch), "--log-n", str(args.log_n),
             "--limbs", str(args.limbs), "--prime-bits", str(args.prime_bits), "--inputs", args.inputs]
    res = {}
    tmp = tempfile.mkdtemp(prefix="bench_pmc_")
    env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    try:
        for name, ctrs in (("fetch", ["FETCH_SIZE"]), ("write", ["WRITE_SIZE", "GRBM_GUI_ACTIVE"])):
            out = os.path.join(tmp, name)
            cmd = ["timeout", "-s", "KILL", "120", prof, "--pmc", *ctrs, "--output-format", "csv", "-d", out,
                   "-o", "run", "--", *child]
            t0 = time.perf_counter()
            r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
            if r.returncode != 0:
                return None, f"rocprofv3 --pmc {' '.join(ctrs)} exited {r.returncode}: {r.stderr[-300:]}"
            m = _pmc_csv_means(out, kernel_re)
            if not all(c in m for c in ctrs):
                return None, f"no {kernel_re} dispatches with {ctrs} in the pass"
            res.update(m)
            res[f"{name}_pass_s"] = time.perf_counter() - t0
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    fetch, write = res["FETCH_SIZE"] * 1024, res["WRITE_SIZE"] * 1024
    return {"bytes_per_launch": 2 * fetch + write, "fetch_size_bytes": fetch, "write_size_bytes": write,
            "grbm_gui_active": res["GRBM_GUI_ACTIVE"],
            "pass_seconds": [round(res["fetch_pass_s"], 1), round(res["write_pass_s"], 1)]}, None


def run_polymul(args, comm, world, rank, local_rank):
    import numpy as np

    import rns_ntt as rn
    from rns_ntt.dist import limb_shard, shard

    n = 1 << args.log_n
    L = args.limbs
    mod = rn.generate_primes(args.prime_bits, L, n)
    global_batch = args.batch if args.strong else args.batch * world
    if args.shard == "limb":
        limbs = limb_shard(L, world, rank)
        batch = global_batch  # every rank holds its limbs of the whole global batch
    else:
        limbs = range(L)
        batch = shard(global_batch, world, rank)[1]  # its own pairs over all limbs
    lmod = mod[limbs.start:limbs.stop]
    Lr = len(lmod)
    B = rn.RnsBasis(lmod, n, device=local_rank)
    wb = 4 if max(lmod) < (1 << 31) else 8

    if args.inputs == "device":
        # seeded uniform residues drawn on the device: no host copy of the
        # gigabytes of operands (a rank's draws depend on its local limbs)
        drng = rn.DeviceRng(1234 + rank)
        a = rn.RnsPoly.sample_uniform(B, drng, batch)
        b = rn.RnsPoly.sample_uniform(B, drng, batch)
    else:
        # 16 seeded unique pairs tiled to the batch
        rng = np.random.default_rng(1234 + (rank if args.shard == "batch" else 0))
        uniq = min(16, batch)
        a_u = uniform(rng, mod, uniq, n)[:, limbs.start:limbs.stop]
        b_u = uniform(rng, mod, uniq, n)[:, limbs.start:limbs.stop]
        reps = (batch + uniq - 1) // uniq
        a = rn.RnsPoly.from_channels(np.tile(a_u, (reps, 1, 1))[:batch], B)
        b = rn.RnsPoly.from_channels(np.tile(b_u, (reps, 1, 1))[:batch], B)
    out = rn.RnsPoly(B, batch)
    lib = rn.load()

    for _ in range(args.warmup):
        rn.check(lib.rnt_mul(out.handle, a.handle, b.handle))
    B.sync()
    comm.barrier()
    B.profile_enable(True)
    B.sync()
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        rn.check(lib.rnt_mul(out.handle, a.handle, b.handle))
    B.sync()
    t1 = time.perf_counter()
    comm.barrier()
    elapsed = comm.max(t1 - t0)
    kernels = {}
    for k in ("col_fwd", "row_mul", "col_inv", "plane_fused", "mf_mul", "whole_mul"):
        cnt, ms = B.profile_read(k)
        if cnt:
            kernels[k] = {"launches": cnt, "avg_ms": ms / cnt, "total_ms": ms}
    B.profile_enable(False)
    power = None
    if rank == 0 and not args.no_power:
        power = power_probe(lambda: rn.check(lib.rnt_mul(out.handle, a.handle, b.handle)), B.sync,
                            local_rank)
    # the measured stream-copy bandwidth (report against it too):
    # a device-to-device copy of one operand batch, read + write
    # (rnt_copy: a plain 16-byte-per-lane copy kernel, k_copy16, timed by its
    # HIP events)
    copy_gbs = None
    if rank == 0:
        dst = rn.RnsPoly(B, batch)
        rn.check(lib.rnt_copy(dst.handle, a.handle))
        B.sync()
        B.profile_enable(True)
        for _ in range(5):
            rn.check(lib.rnt_copy(dst.handle, a.handle))
        cnt, cms = B.profile_read("copy")
        B.profile_enable(False)
        if cnt:
            copy_gbs = cnt * 2 * Lr * batch * n * wb / (cms * 1e-3) / 1e9
        del dst

    ms_per_step = elapsed / args.steps * 1e3
    value = global_batch * args.steps / elapsed  # whole-job poly-muls / s (slowest rank's time)

    # spot parity of the timed output (this rank's limbs of the first and the
    # last pair) vs the oracle
    parity_ok = True
    if rank == 0:
        orc = oracle()
        ob = orc.Basis(lmod, n)
        for pi in sorted({0, batch - 1}):
            got = out.channels_of(pi)[0]
            want = orc.mul(ob, a.channels_of(pi)[0], b.channels_of(pi)[0])
            parity_ok &= bool(np.array_equal(got, want))

    # roofline.  Headline (`frac`): the whole rnt_mul -- the metric's unit --
    # as one launch of the path: its algorithmic bytes (read a, read b, write
    # c at the device word width) over the summed average launch
    # times of its kernels, each measured with HIP events on the library's
    # stream (the same kernels rocprofv3 lists; their sum is within a few us
    # of ms_per_step, so frac = whole-op bytes / ms_per_step / 8 TB/s).
    # Per-kernel figures follow in `kernels_roofline`, each with the bound
    # that really holds it (the row kernel is VALU-bound).
    elem = Lr * batch * n
    launches = max(kernels[k]["launches"] for k in kernels)
    op_ms = sum(kernels[k]["total_ms"] for k in kernels) / args.steps  # per rnt_mul
    op_bytes = 3 * elem * wb
    achieved = op_bytes / (op_ms * 1e-3) / 1e9
    step_bytes = {"col_fwd": 4 * elem * wb, "row_mul": 3 * elem * wb, "col_inv": 2 * elem * wb,
                  "plane_fused": 3 * elem * wb, "mf_mul": 3 * elem * wb, "whole_mul": 3 * elem * wb}
    per_gpu = value / world
    pmc = {k: traffic_for(k, "polymul", batch, args.log_n, Lr) if args.prime_bits == 31 else None
           for k in kernels}
    kroof = {}
    for k, kv in kernels.items():
        kb = step_bytes.get(k)
        ent = {"avg_ms": kv["avg_ms"], "launches": kv["launches"], "alg_bytes_per_launch": kb,
               "bound": ("power (mfma + valu)" if k == "mf_mul" else
                         "valu" if k in ("row_mul", "plane_fused", "whole_mul") else "hbm"),
               "pmc_bytes_per_launch": pmc.get(k)}
        if kb:
            ent["hbm_GBs"] = kb / (kv["avg_ms"] * 1e-3) / 1e9
            ent["hbm_frac"] = ent["hbm_GBs"] / HBM_PEAK_GBS
        kroof[k] = ent
    traffic = sum(v for v in pmc.values() if v) if all(pmc.values()) else None
    traffic_source = "profiles/pmc_traffic.json (committed rocprofv3 --pmc passes, not this run)"
    traffic_committed = traffic
    live = None
    if rank == 0 and world == 1 and not args.no_live_pmc and len(kernels) == 1:
        (kname,) = kernels
        kre = {"mf_mul": r"\bk_mf_mul\(", "plane_fused": r"\bk_plane_fused(_slots)?\(",
               "whole_mul": r"\bk_row<unsigned (int|long), 2, \d+, (true|false), true>"}.get(kname)
        if kre:
            live, why = live_pmc(args, kre)
            if live:
                traffic = live["bytes_per_launch"]
                traffic_source = ("live: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE child passes of this "
                                  "workload in this run, 2 x FETCH_SIZE + WRITE_SIZE per launch")
                # the kernel's clock under the counter pass: GRBM_GUI_ACTIVE
                # (summed over the 8 XCDs) over this run's HIP-event launch time
                live["clock_ghz_est"] = live["grbm_gui_active"] / 8 / (kernels[kname]["avg_ms"] * 1e6)
            else:
                live = {"error": why}
    roofline = {
        "bound": "hbm",
        "kernel": "rnt_mul (" + " + ".join(kernels) + ")",
        "achieved": achieved,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS,
        # HBM bytes per rnt_mul from the committed PMC passes of this shape
        # (profiles/pmc_traffic.json: 2 x FETCH_SIZE + WRITE_SIZE per kernel)
        "traffic": traffic,
        "traffic_source": traffic_source,
        "traffic_committed": traffic_committed,
        "traffic_live": live,
        "traffic_ratio": traffic / op_bytes if traffic else None,
        "alg_bytes_per_launch": op_bytes,
        "launch_ms": op_ms,
        "launches": launches,
        # SURVEY §8d's u64 accounting (3*L*N*8 B per poly-mul) of the same rate
        "frac_u64_equiv": per_gpu * 3 * L * n * 8 / 1e9 / HBM_PEAK_GBS,
        "whole_op_GBs_wall": per_gpu * 3 * L * n * wb / 1e9,
        "stream_copy_GBs": copy_gbs,
        "frac_of_copy": achieved / copy_gbs if copy_gbs else None,
        "kernels_roofline": kroof,
        "kernels": kernels,
    }
    if "row_mul" in kernels:
        # the row kernel is VALU-bound: the butterflies it
        # executes (both forward row transforms and the inverse one) per
        # second of its time.  With the truncated transform (u32 canonical
        # bases, rows of 2^(4k) words) each row transform runs
        # two stages fewer and the degree-3 block products are not counted.
        log_r = max(args.log_n // 2, 4) if args.log_n >= 8 else max(args.log_n - 4, 0)
        log_c = args.log_n - log_r
        lazy = max(lmod) < (1 << 30) and log_r >= 5
        trunc = wb == 4 and not lazy and log_c >= 4 and log_c % 4 == 0
        stages = log_c - 2 if trunc else log_c
        rb = 3 * elem * stages // 2 * args.steps / kernels["row_mul"]["launches"]
        ra = rb / (kernels["row_mul"]["avg_ms"] * 1e-3)
        kroof["row_mul"].update(valu_unit="butterflies/s", bfly_per_launch=rb,
                                row_stages_per_transform=stages, truncated_transform=trunc,
                                valu_achieved=ra, valu_peak=VALU_PEAK_BFLY, valu_frac=ra / VALU_PEAK_BFLY)
    if "plane_fused" in kernels:
        # the whole-plane kernel is bound by VALU issue: its
        # butterflies per second (three truncated 14-stage transforms per
        # (poly, limb); block products not counted) against VALU_PEAK_BFLY,
        # and its VALU wave-instructions (committed PMC pass of this shape)
        # per second against one wave64 instruction per 4 cycles per SIMD at
        # 2.4 GHz -- the issue cost tools/bflyrate.hip measures for these
        # 32-bit integer ops.
        pb = 21 * elem * args.steps / kernels["plane_fused"]["launches"]
        pa = pb / (kernels["plane_fused"]["avg_ms"] * 1e-3)
        kroof["plane_fused"].update(valu_unit="butterflies/s", bfly_per_launch=pb, valu_achieved=pa,
                                    valu_peak=VALU_PEAK_BFLY, valu_frac=pa / VALU_PEAK_BFLY)
        vi = pmc_field("plane_fused", "polymul", batch, args.log_n, Lr, "SQ_INSTS_VALU") \
            if args.prime_bits == 31 else None
        if vi:
            ipeak = 1024 * 2.4e9 / 4
            ia = vi / (kernels["plane_fused"]["avg_ms"] * 1e-3)
            kroof["plane_fused"].update(valu_instr_per_launch_pmc=vi, valu_issue_per_s=ia,
                                        valu_issue_peak=ipeak, valu_issue_frac=ia / ipeak)
    if "mf_mul" in kernels:
        # the matrix-core product (k_mf_mul): three transforms
        # of four radix-16 passes per (poly, limb), each pass 16 tiles x 4
        # v_mfma_i32_16x16x64_i8 (16 x 16 x 64 MACs) per wave, 16 waves; its
        # MFMA ops per second against the dense i8 peak (2x the BF16 rate
        # per clock, MI355X_MICROARCH.md: ~5e15 ops/s).  The kernel runs at
        # the package power limit, not at either peak.
        mops = 3 * 4 * 16 * 4 * 16 * (16 * 16 * 64) * 2 * (Lr * batch) * args.steps \
            / kernels["mf_mul"]["launches"]
        ma = mops / (kernels["mf_mul"]["avg_ms"] * 1e-3)
        kroof["mf_mul"].update(mfma_unit="i8 ops/s", mfma_ops_per_launch=mops, mfma_achieved=ma,
                               mfma_peak=MFMA_PEAK_I8, mfma_frac=ma / MFMA_PEAK_I8)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(mod, n, args.cpu_seconds)
    par = (f"limb-sharded x{world} ({Lr} of {L} limbs per GPU), no collective" if args.shard == "limb"
           else f"batch-sharded x{world}, no collective")
    return {
        "metric": METRIC,
        "value": value,
        "unit": "poly-muls/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None,
        "dtype": "u32" if wb == 4 else "u64",
        "data": ("synthetic (seeded uniform residues drawn on the device)" if args.inputs == "device"
                 else "synthetic (seeded uniform residues, 16 host pairs tiled)"),
        "config": {
            "workload": f"coefficient-domain RNS-NTT poly-mul c=a*b, N=2^{args.log_n}, L={L} x "
                        f"{args.prime_bits}-bit primes",
            "N": n,
            "L": L,
            "pairs_per_gpu_per_step": global_batch / world,
            "global_batch": global_batch,
            "parallelism": par,
            "parity_spot_check": parity_ok,
        },
        "roofline": roofline,
        "cpu_baseline": cpu,
        "power": power,
    }


def _graph_step_timing(basis, step, steps, warmup, comm, kernel_names):
    """Warm `step` eagerly, time one eager step's kernels with HIP events
    (kernel ms per step), record the step as a HIP graph and time `steps`
    replays (barrier + sync on both sides).  Returns (graph, elapsed_max_s,
    kernel_ms_per_step, kernels)."""
    for _ in range(max(warmup, 1)):
        step()
    basis.sync()
    basis.profile_enable(True)
    step()
    basis.sync()
    kernels, kms = {}, 0.0
    for k in kernel_names:
        cnt, ms = basis.profile_read(k)
        if cnt:
            kernels[k] = {"launches": cnt, "avg_ms": ms / cnt, "total_ms": ms}
            kms += ms
    basis.profile_enable(False)
    with basis.capture() as g:
        step()
    for _ in range(max(warmup, 1)):
        g.replay()
    basis.sync()
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        g.replay()
    basis.sync()
    t1 = time.perf_counter()
    comm.barrier()
    return g, comm.max(t1 - t0), kms, kernels


def run_ctmul_graph(args, comm, world, rank, local_rank):
    """The reference engine's own call shape for config 4's arithmetic:
    mul_ciphertexts_gadget then rescale_ciphertext on `--ct-batch`
    ciphertexts per call (1 = one ciphertext, as engine.rs:473-539 and
    263-282 are called), through the fused C-ABI ops, the step replayed
    from a recorded HIP graph; every GPU its own ciphertexts (replicas)."""
    import numpy as np

    import rns_ntt as rn

    n = 1 << args.log_n
    L = args.limbs
    mod = rn.generate_primes(args.prime_bits, L, n)
    wb = 4 if max(mod) < (1 << 31) else 8
    Bs = rn.RnsBasis(mod, n, device=local_rank)
    Bs1 = Bs.drop_last(1)
    B = args.ct_batch
    rng = np.random.default_rng(77 + rank)
    cts = [uniform(rng, mod, B, n) for _ in range(4)]
    key_a, key_b = uniform(rng, mod, L, n), uniform(rng, mod, L, n)
    c = [rn.RnsPoly.from_channels(x, Bs) for x in cts]
    key = rn.RnsGadgetKey.from_channels(key_a, key_b, Bs)
    o0, o1, r0, r1 = rn.RnsPoly(Bs, B), rn.RnsPoly(Bs, B), rn.RnsPoly(Bs1, B), rn.RnsPoly(Bs1, B)
    lib = rn.load()

    def step():
        rn.check(lib.rnt_ct_mul_relin(o0.handle, o1.handle, c[0].handle, c[1].handle, c[2].handle,
                                      c[3].handle, key.a.handle, key.b.handle))
        rn.check(lib.rnt_ct_rescale(r0.handle, r1.handle, o0.handle, o1.handle))

    g, elapsed, kms, kernels = _graph_step_timing(
        Bs, step, args.steps, args.warmup, comm,
        ("col_fwd", "tensor_rows", "col_inv", "ks_decompose", "ks_rows", "rescale", "elementwise", "tensor_whole",
         "ks_whole", "mf_tensor"))
    ms_per_step = elapsed / args.steps * 1e3
    value = B * args.steps * world / elapsed
    parity_ok = None
    if rank == 0:
        orc = oracle()
        ob = orc.Basis(mod, n)
        parity_ok = True
        for pi in sorted({0, B - 1}):
            w0, w1 = orc.mul_ciphertexts_gadget(ob, cts[0][pi], cts[1][pi], cts[2][pi], cts[3][pi], key_a, key_b,
                                                threads=usable_threads())
            parity_ok &= bool(np.array_equal(r0.channels_of(pi)[0], orc.rescale(ob, w0))
                              and np.array_equal(r1.channels_of(pi)[0], orc.rescale(ob, w1)))
    log_c = args.log_n - max(args.log_n // 2, 4)
    roof = {"bound": "valu", "kernel": "ks_rows", "unit": "butterflies/s", "peak": VALU_PEAK_BFLY,
            "achieved": None, "frac": None, "traffic": None, "kernels": kernels}
    if "ks_rows" in kernels:
        bfly = B * (L * L + 2 * L) * (n // 2) * log_c
        ach = bfly / (kernels["ks_rows"]["total_ms"] * 1e-3)
        roof.update(achieved=ach, frac=ach / VALU_PEAK_BFLY, bfly_per_launch=bfly / kernels["ks_rows"]["launches"])
    elif "ks_whole" in kernels:
        # k_ks_whole: whole forward transforms of every (source, target) pair
        # and whole inverses of both accumulators
        bfly = B * args.steps * (L * L + 2 * L) * (n // 2) * args.log_n
        ach = bfly / (kernels["ks_whole"]["total_ms"] * 1e-3)
        roof.update(kernel="ks_whole", achieved=ach, frac=ach / VALU_PEAK_BFLY,
                    bfly_per_launch=bfly / kernels["ks_whole"]["launches"])
    return {
        "metric": CT_METRIC.format(log_n=args.log_n, L=args.limbs),
        "value": value,
        "unit": "ct-muls/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32" if wb == 4 else "u64",
        "data": "synthetic (seeded uniform residues and key)",
        "config": {
            "workload": f"engine call shape: mul_ciphertexts_gadget + rescale_ciphertext of {B} ciphertext(s) per "
                        f"call, N=2^{args.log_n}, L={L} x {args.prime_bits}-bit primes, replayed HIP graph",
            "ct_pairs_per_gpu_per_step": B,
            "parallelism": f"replicas x{world} (each GPU its own ciphertexts)",
            "parity_spot_check": parity_ok,
            "kernel_ms_per_step": kms,
            "device_busy": kms / ms_per_step,
        },
        "roofline": roof,
        "cpu_baseline": None,
    }


def run_ctmul(args, comm, world, rank, local_rank):
    """BASELINE config 4: ct x ct + gadget relin + rescale, limb-sharded."""
    if args.graph:
        return run_ctmul_graph(args, comm, world, rank, local_rank)
    import numpy as np
    import torch

    import rns_ntt as rn
    from rns_ntt.sharded import GpuBackend, LimbShardedPipeline, SingleComm, TorchDistComm

    n = 1 << args.log_n
    L = args.limbs
    mod = rn.generate_primes(args.prime_bits, L, n)
    wb = 4 if max(mod) < (1 << 31) else 8
    torch.cuda.set_device(local_rank)
    # --shard limb (default): the north star's limb shard with RCCL joins;
    # --shard batch: every rank runs the whole pipeline on its own
    # ciphertexts over all limbs with a full key replica (SURVEY §8e's
    # zero-collective fallback)
    batch_shard = world > 1 and args.shard == "batch"
    if world > 1 and not batch_shard:
        import torch.distributed as dist

        data_comm = TorchDistComm(dist.new_group(backend=data_backend()))  # RCCL over xGMI
    else:
        data_comm = SingleComm()
    B_global = args.ct_batch * world  # weak scaling
    B = args.ct_batch if batch_shard else B_global  # ciphertexts this rank's pipeline holds
    pipe = LimbShardedPipeline(mod, n, data_comm, GpuBackend(local_rank), chunk=args.chunk)
    rng = np.random.default_rng(77)
    uniq = min(4, B)
    reps = (B + uniq - 1) // uniq
    cts = [np.tile(uniform(rng, mod, uniq, n), (reps, 1, 1))[:B] for _ in range(4)]
    key_a, key_b = uniform(rng, mod, L, n), uniform(rng, mod, L, n)
    c = [pipe.upload(x) for x in cts]
    key = pipe.upload_key(key_a, key_b)
    state0 = (pipe.basis, pipe.moduli, list(pipe.counts), pipe.limbs, pipe.owner_last)
    # shared stream (the default at every N): torch's ops and the RCCL joins
    # are queued against the library's own HIP stream, so the pipeline runs
    # without host syncs and each chunk's all-gather overlaps the compute of
    # its neighbours (LimbShardedPipeline); RNT_SHARED_STREAM=0 restores
    # torch's stream and the per-op host syncs (A/B)
    shared = os.environ.get("RNT_SHARED_STREAM", "1") != "0"
    lib_stream = pipe.backend.shared_stream(pipe.basis) if shared else torch.cuda.current_stream()

    def step():
        # every step starts from the same level (rescale drops a limb)
        pipe.basis, pipe.moduli, counts, pipe.limbs, pipe.owner_last = state0
        pipe.counts = list(counts)
        with torch.cuda.stream(lib_stream):  # torch ops share the library's stream
            # (a world of one: the fused rnt_ct_mul_relin_rescale per chunk;
            # limb-sharded: mul_relin, then rescale, with their RCCL joins)
            return pipe.mul_relin_rescale(c[0], c[1], c[2], c[3], key)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    comm.barrier()
    prof_basis = state0[0]  # drop_last views share its tables and profiler
    prof_basis.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r = step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    comm.barrier()
    elapsed = comm.max(t1 - t0)
    value = B_global * args.steps / elapsed
    kernels = {}
    for k in ("col_fwd", "tensor_rows", "col_inv", "ks_decompose", "ks_rows", "rescale", "elementwise",
              "tensor_whole", "ks_whole", "mf_tensor"):
        cnt, ms = prof_basis.profile_read(k)
        if cnt:
            kernels[k] = {"launches": cnt, "avg_ms": ms / cnt, "total_ms": ms}
    prof_basis.profile_enable(False)
    power = None
    if rank == 0 and world == 1 and not args.no_power:
        power = power_probe(step, torch.cuda.synchronize, local_rank)

    parity_ok = None
    cpu = None
    Lr = state0[2][0 if batch_shard else rank]  # this rank's target limbs
    # sampled parity of the timed output: the first pair, the first pair of
    # the second pipeline chunk and the batch's last pair.  Limb-sharded:
    # every rank sends its limbs of those pairs (after the rescale) to rank
    # 0 over the gloo control plane, which assembles the full ciphertexts.
    # the first pair, the first of the second pipeline chunk (or, one chunk,
    # of the library's second key-switch chunk at N = 2^16: 256), the last
    check_pairs = sorted({0, min(pipe.chunk, 256, B - 1), B - 1})
    mine = {pi: pipe.download(r[0], first=pi, count=1)[0] for pi in check_pairs}
    if world > 1 and not batch_shard:
        parts = comm.gather((rank, pipe.limbs.start, mine))
    else:
        parts = [(0, 0, mine)]
    if rank == 0:
        orc = oracle()
        ob = orc.Basis(mod, n)
        threads = usable_threads()
        parts = sorted(parts, key=lambda t: t[1])  # by first limb
        parity_ok = True
        for pi in check_pairs:
            got = np.concatenate([pr[2][pi] for pr in parts], axis=0)  # [L-1][N]
            u = pi % uniq
            o0, _ = orc.mul_ciphertexts_gadget(ob, cts[0][u], cts[1][u], cts[2][u], cts[3][u], key_a, key_b,
                                               threads=threads)
            parity_ok &= bool(np.array_equal(got, orc.rescale(ob, o0)))
        if not args.no_cpu_baseline and world == 1:
            def t_pair(th):
                t = time.perf_counter()
                o0, o1 = orc.mul_ciphertexts_gadget(ob, cts[0][0], cts[1][0], cts[2][0], cts[3][0], key_a, key_b,
                                                    threads=th)
                orc.rescale(ob, o0), orc.rescale(ob, o1)
                return time.perf_counter() - t
            s1 = t_pair(1)
            sn = t_pair(threads)
            cpu = {"value": 1.0 / sn, "unit": "ct-muls/s", "cores": threads, "kind": "port",
                   "sample": f"1 ciphertext pair (N={n}, L={L}) through oracle mul_ciphertexts_gadget + rescale "
                             f"of c0 and c1, channel-parallel over {threads} threads, {sn:.1f} s",
                   "single_thread": {"value": 1.0 / s1, "cores": 1, "sample": f"the same pair on one thread, {s1:.1f} s"},
                   "host": host_info()}
    # bytes per ciphertext: (4L + 2(L-1)) * N * 8
    ct_bytes = (4 * L + 2 * (L - 1)) * n * 8
    log_c = args.log_n - max(args.log_n // 2, 4)
    roof = {"bound": "valu", "kernel": "ks_rows", "unit": "butterflies/s", "peak": VALU_PEAK_BFLY,
            "achieved": None, "frac": None, "traffic": None, "kernels": kernels,
            "whole_pipeline_hbm": {"unit": "GB/s", "achieved": value / world * ct_bytes / 1e9,
                                   "peak": HBM_PEAK_GBS,
                                   "frac": value / world * ct_bytes / 1e9 / HBM_PEAK_GBS}}
    if "ks_rows" in kernels:
        # k_ks_rows per ciphertext on this rank: the forward row stages of
        # alpha_i mod q_j for every (source i, own target j) and the inverse
        # row stages of both accumulators (L_r target limbs)
        bfly = B * args.steps * (L * Lr + 2 * Lr) * (n // 2) * log_c
        ach = bfly / (kernels["ks_rows"]["total_ms"] * 1e-3)
        roof.update(achieved=ach, frac=ach / VALU_PEAK_BFLY,
                    bfly_per_launch=bfly / kernels["ks_rows"]["launches"],
                    traffic=traffic_for("ks_rows", "ctmul", args.ct_batch, args.log_n, L))
    elif "ks_whole" in kernels:
        bfly = B * args.steps * (L * Lr + 2 * Lr) * (n // 2) * args.log_n
        ach = bfly / (kernels["ks_whole"]["total_ms"] * 1e-3)
        roof.update(kernel="ks_whole", achieved=ach, frac=ach / VALU_PEAK_BFLY,
                    bfly_per_launch=bfly / kernels["ks_whole"]["launches"])
    return {
        "metric": CT_METRIC.format(log_n=args.log_n, L=args.limbs),
        "value": value,
        "unit": "ct-muls/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32" if wb == 4 else "u64",
        "data": "synthetic (seeded uniform residues and key)",
        "config": {
            "workload": f"ct x ct + gadget relin + rescale, N=2^{args.log_n}, L={L} x {args.prime_bits}-bit primes",
            "ct_pairs_per_gpu_per_step": args.ct_batch,
            "global_batch": B_global,
            "parallelism": (f"batch-sharded x{world}: no collective, full key per GPU, fused "
                            f"rnt_ct_mul_relin_rescale per chunk" if batch_shard else
                            "single GPU: fused rnt_ct_mul_relin_rescale per chunk (no join)" if world == 1 else
                            f"limb-sharded x{world}: RCCL all-gather of d2, broadcast of q_L limb"),
            "parity_spot_check": parity_ok,
            "parity_pairs": check_pairs,
            "pipeline_chunk": pipe.chunk,
            "shared_stream": shared,
        },
        "roofline": roof,
        "cpu_baseline": cpu,
        "power": power,
    }


def rotation_offsets(args, log_n):
    n = 1 << log_n
    if args.rot_offsets == "all":
        return list(range(1, n // 2))  # every slot offset (one resident key, SURVEY §8d sweep 2)
    return [1 << e for e in range(log_n - 1)]  # 1 .. N/4: all power-of-two slot offsets


def run_rotate(args, comm, world, rank, local_rank):
    """BASELINE config 5: rotate_ciphertext (engine.rs:412-463)
    over the log2(N/2) power-of-two slot offsets, each with its own gadget
    rotation key (generate_gadget_rotation_key, engine.rs:348-399: 2 GiB of
    u64 key per offset in the reference, 1 GiB resident here at u32), or with
    --rot-offsets all every offset 1..N/2-1 reusing one resident key (the
    arithmetic per offset is identical).  Defaults to N = 2^17, L = 32 when
    --log-n/--limbs are the poly-mul defaults."""
    import numpy as np

    import rns_ntt as rn

    log_n = 17 if args.log_n == 16 else args.log_n
    L = 32 if args.limbs == 16 else args.limbs
    n = 1 << log_n
    mod = rn.generate_primes(args.prime_bits, L, n)
    wb = 4 if max(mod) < (1 << 31) else 8
    if world > 1 and args.shard == "limb":
        return run_rotate_sharded(args, comm, world, rank, local_rank, log_n, L, mod)
    Bs = rn.RnsBasis(mod, n, device=local_rank)
    B = args.rot_batch
    rng = np.random.default_rng(5 + rank)
    c0_h, c1_h = uniform(rng, mod, B, n), uniform(rng, mod, B, n)
    c0 = rn.RnsPoly.from_channels(c0_h, Bs)
    c1 = rn.RnsPoly.from_channels(c1_h, Bs)
    offsets = rotation_offsets(args, log_n)
    per_offset = args.rot_keys == "per-offset" and args.rot_offsets == "pow2"
    # keys: uniform a_i, b_i drawn on the device (the key relation does not
    # change the arithmetic); key 0 also comes back to the host for the check
    drng = rn.DeviceRng(99 + rank)
    nkeys = len(offsets) if per_offset else 1
    keys, check_key = [], None
    for i in range(nkeys):
        ka, kb = rn.RnsPoly.sample_uniform(Bs, drng, L), rn.RnsPoly.sample_uniform(Bs, drng, L)
        if i == nkeys - 1:  # the key of the checked offset, coefficient domain (before prepare)
            check_key = (ka.channels(), kb.channels())
        keys.append(rn.RnsGadgetKey(ka, kb))
    out0, out1 = rn.RnsPoly(Bs, B), rn.RnsPoly(Bs, B)  # reused: the workspace stays allocated
    lib = rn.load()

    def step():
        for i, k in enumerate(offsets):
            key = keys[i if per_offset else 0]
            rn.check(lib.rnt_ct_rotate(out0.handle, out1.handle, c0.handle, c1.handle, k,
                                       key.a.handle, key.b.handle))

    rot_kernels = ("ks_decompose", "ks_rows", "col_inv", "automorphism", "col_fwd", "row_fwd", "ks_whole")
    graph_info = None
    if args.graph:
        # the reference's call shape replayed: the whole sweep step recorded
        # once as a HIP graph (rnt_capture_begin), kernels timed eagerly
        g, elapsed, kms, kernels = _graph_step_timing(Bs, step, args.steps, args.warmup, comm, rot_kernels)
        graph_info = {"kernel_ms_per_step": kms, "device_busy": kms / (elapsed / args.steps * 1e3)}
        for kv in kernels.values():  # one eager step profiled: scale to the timed steps
            kv["launches"] *= args.steps
            kv["total_ms"] *= args.steps
    else:
        for _ in range(args.warmup):
            step()
        Bs.sync()
        comm.barrier()
        Bs.profile_enable(True)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        Bs.sync()
        t1 = time.perf_counter()
        comm.barrier()
        elapsed = comm.max(t1 - t0)
        kernels = {}
        for k in rot_kernels:
            cnt, ms = Bs.profile_read(k)
            if cnt:
                kernels[k] = {"launches": cnt, "avg_ms": ms / cnt, "total_ms": ms}
        Bs.profile_enable(False)
        kms = sum(kv["total_ms"] for kv in kernels.values()) / args.steps
        graph_info = {"kernel_ms_per_step": kms, "device_busy": kms / (elapsed / args.steps * 1e3)}
    power = None
    if rank == 0 and not args.no_power:
        power = power_probe(step, Bs.sync, local_rank)
    rots = B * len(offsets) * args.steps * world
    value = rots / elapsed
    log_c = log_n - max(log_n // 2, 4)
    # k_ks_rows per rotation: forward row stages of alpha_i mod q_j for all
    # (i, j) and the inverse row stages of both accumulators
    bfly_rows = B * len(offsets) * args.steps * (L * L + 2 * L) * (n // 2) * log_c
    roof = {"bound": "valu", "kernel": "ks_rows", "unit": "butterflies/s", "peak": VALU_PEAK_BFLY,
            "achieved": None, "frac": None, "traffic": None, "kernels": kernels,
            "whole_op_bfly_per_s": value / world * (L * L + 2 * L) * (n // 2) * log_n}
    if "ks_rows" in kernels:
        ach = bfly_rows / (kernels["ks_rows"]["total_ms"] * 1e-3)
        roof.update(achieved=ach, frac=ach / VALU_PEAK_BFLY,
                    bfly_per_launch=bfly_rows / kernels["ks_rows"]["launches"],
                    traffic=traffic_for("ks_rows", "rotate", B, log_n, L))
    elif "ks_whole" in kernels:
        bfly = B * len(offsets) * args.steps * (L * L + 2 * L) * (n // 2) * log_n
        ach = bfly / (kernels["ks_whole"]["total_ms"] * 1e-3)
        roof.update(kernel="ks_whole", achieved=ach, frac=ach / VALU_PEAK_BFLY,
                    bfly_per_launch=bfly / kernels["ks_whole"]["launches"])

    parity_ok = None
    cpu = None
    if rank == 0:
        # the last offset of the sweep, ciphertext 0 and the batch's last one,
        # against the oracle's rotate_ciphertext (channel-parallel)
        orc = oracle()
        ob = orc.Basis(mod, n)
        threads = usable_threads()
        ki = len(offsets) - 1
        key = keys[-1]
        ka, kb = check_key
        rn.check(lib.rnt_ct_rotate(out0.handle, out1.handle, c0.handle, c1.handle, offsets[ki],
                                   key.a.handle, key.b.handle))
        parity_ok = True
        t = time.perf_counter()
        for pi in sorted({0, B - 1}):
            # channels_of: [1][L][N] whatever the batch (channels() drops the
            # batch axis of a one-poly buffer)
            g0, g1 = out0.channels_of(pi)[0], out1.channels_of(pi)[0]
            w0, w1 = orc.rotate_ciphertext(ob, c0_h[pi], c1_h[pi], offsets[ki], ka, kb, threads=threads)
            parity_ok &= bool(np.array_equal(g0, w0) and np.array_equal(g1, w1))
        sn = (time.perf_counter() - t) / len({0, B - 1})
        if world == 1 and not args.no_cpu_baseline:
            cpu = {"value": 1.0 / sn, "unit": "rotations/s", "cores": threads, "kind": "port",
                   "sample": f"1 rotation (N={n}, L={L}) through oracle rotate_ciphertext (automorphism + "
                             f"gadget key-switch, engine.rs:412-463), channel-parallel over {threads} threads, "
                             f"{sn:.1f} s; single thread not run: one rotation is 6L^2 limb NTTs (~{16 * sn:.0f} s)",
                   "host": host_info()}
    return {
        "metric": ROT_METRIC,
        "value": value,
        "unit": "rotations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32" if wb == 4 else "u64",
        "data": ("synthetic (seeded uniform residues; a distinct device-sampled gadget key per offset)"
                 if per_offset else "synthetic (seeded uniform residues; one device-sampled key reused for every offset)"),
        "config": {
            "workload": f"rotate_ciphertext sweep over {len(offsets)} "
                        f"{'power-of-two' if args.rot_offsets == 'pow2' else 'slot'} offsets, "
                        f"N=2^{log_n}, L={L} x {args.prime_bits}-bit primes, {B} ciphertexts",
            "keys": len(keys),
            "parallelism": f"replicas x{world} (each GPU its own ciphertexts)",
            "parity_spot_check": parity_ok,
            "replayed_graph": bool(args.graph),
            **graph_info,
        },
        "roofline": roof,
        "cpu_baseline": cpu,
        "power": power,
    }


def run_encode(args, comm, world, rank, local_rank):
    """CkksEncoder.encode_complex + decode_complex
    (ckks_encoder.rs:85-156) of a batch of full-slot plaintexts through the
    device special FFT (rnt_encode / rnt_decode).  Slot values start and end
    on the host, so the wall rate includes their PCIe copies; the special-FFT
    kernels are timed with HIP events for the roofline."""
    import numpy as np

    import rns_ntt as rn

    n = 1 << args.log_n
    L = args.limbs
    mod = rn.generate_primes(31, L, n)
    Bs = rn.RnsBasis(mod, n, device=local_rank)
    B = args.enc_batch
    rng = np.random.default_rng(3 + rank)
    v = rng.uniform(-1, 1, (B, n // 2)) + 1j * rng.uniform(-1, 1, (B, n // 2))
    scale = 40
    enc = rn.CkksEncoder(n, scale)

    def step():
        return enc.decode_complex(enc.encode_complex(v, Bs))

    for _ in range(args.warmup):
        step()
    Bs.sync()
    comm.barrier()
    Bs.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    Bs.sync()
    t1 = time.perf_counter()
    comm.barrier()
    elapsed = comm.max(t1 - t0)
    kernels = {}
    for k in ("sfft", "crt", "import"):
        cnt, ms = Bs.profile_read(k)
        if cnt:
            kernels[k] = {"launches": cnt, "avg_ms": ms / cnt, "total_ms": ms}
    Bs.profile_enable(False)
    err = float(np.max(np.abs(out - v)))
    # algorithmic bytes of one special-FFT launch (encode or decode of the
    # batch): the N/2 complex slots (16 B) and the N i64 coefficients (8 B)
    alg = B * (n // 2 * 16 + n * 8)
    sf = kernels.get("sfft", {"avg_ms": float("nan")})
    achieved = alg / (sf["avg_ms"] * 1e-3) / 1e9
    return {
        "metric": ENC_METRIC,
        "value": B * args.steps * world / elapsed,
        "unit": "round-trips/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded uniform complex slots in [-1, 1]^2)",
        "config": {
            "workload": f"encode_complex + decode_complex, N=2^{args.log_n}, L={L} x 31-bit primes, "
                        f"{n // 2} slots, scale 2^{scale}, {B} plaintexts per step",
            "parallelism": f"replicas x{world}",
            "roundtrip_max_err": err,
            "parity_spot_check": err < n / 2.0 ** scale,
        },
        "roofline": {"bound": "hbm", "kernel": "sfft", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "alg_bytes_per_launch": alg, "kernels": kernels},
        "cpu_baseline": None,
    }


def run_ntt(args, comm, world, rank, local_rank):
    """SURVEY §8a rows a4/a5 on their own: to_ntt_domain then to_coeff_domain
    (poly.rs:136-166) of a batch of `--batch` polys over all limbs, in place.
    One step = one forward and one inverse transform of the batch (column +
    row launches each way); replicas at N > 1 (no collective)."""
    import numpy as np

    import rns_ntt as rn

    n = 1 << args.log_n
    L = args.limbs
    mod = rn.generate_primes(args.prime_bits, L, n)
    B = rn.RnsBasis(mod, n, device=local_rank)
    wb = 4 if max(mod) < (1 << 31) else 8
    batch = args.batch
    x = rn.RnsPoly.sample_uniform(B, rn.DeviceRng(4321 + rank), batch)
    first, last = x.channels_of(0)[0], x.channels_of(batch - 1)[0]

    def step():
        x.to_ntt_domain()
        x.to_coeff_domain()

    for _ in range(args.warmup):
        step()
    B.sync()
    comm.barrier()
    B.profile_enable(True)
    B.sync()
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    B.sync()
    t1 = time.perf_counter()
    comm.barrier()
    elapsed = comm.max(t1 - t0)
    kernels = {}
    for k in ("col_fwd", "row_fwd", "row_inv", "col_inv", "mf_ntt_fwd", "mf_ntt_inv", "whole_fwd", "whole_inv"):
        cnt, ms = B.profile_read(k)
        if cnt:
            kernels[k] = {"launches": cnt, "avg_ms": ms / cnt, "total_ms": ms}
    B.profile_enable(False)
    power = None
    if rank == 0 and not args.no_power:
        power = power_probe(step, B.sync, local_rank)
    # parity: the round trips returned the operands (bit-exact identity), and
    # one more forward transform matches the oracle's natural-order NTT
    parity_ok = bool(np.array_equal(x.channels_of(0)[0], first)
                     and np.array_equal(x.channels_of(batch - 1)[0], last))
    cpu = None
    if rank == 0:
        orc = oracle()
        ob = orc.Basis(mod, n)
        x.to_ntt_domain()
        parity_ok &= bool(np.array_equal(x.channels_of(batch - 1)[0], orc.to_ntt(ob, last)))
        if world == 1 and not args.no_cpu_baseline:
            # the oracle's transforms (poly.rs:574-625) on one thread, as the
            # reference runs them, on a bounded sample
            done, el = 0, 0.0
            while el < args.cpu_seconds / 2:
                t = time.perf_counter()
                orc.to_coeff(ob, orc.to_ntt(ob, first))
                el += time.perf_counter() - t
                done += 1
            cpu = {"value": done / el, "unit": "transform pairs/s", "cores": 1, "kind": "port",
                   "sample": f"{done} forward+inverse transforms of one poly (N={n}, L={L}) on one "
                             f"thread, {el:.1f} s; oracle/oracle.c restating poly.rs:574-625",
                   "host": host_info()}
    # every launch moves its batch once in and once out: 2 L B N w bytes
    alg = 2 * L * batch * n * wb
    dom = max(kernels, key=lambda k: kernels[k]["total_ms"])
    achieved = alg / (kernels[dom]["avg_ms"] * 1e-3) / 1e9
    value = batch * args.steps * world / elapsed
    return {
        "metric": NTT_METRIC,
        "value": value,
        "unit": "transform pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32" if wb == 4 else "u64",
        "data": "synthetic (seeded uniform residues drawn on the device)",
        "config": {
            "workload": f"to_ntt_domain + to_coeff_domain in place, N=2^{args.log_n}, L={L} x "
                        f"{args.prime_bits}-bit primes, {batch} polys per step",
            "parallelism": f"replicas x{world}",
            "parity_spot_check": parity_ok,
        },
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic_for(dom, "ntt", batch, args.log_n, L),
                     "alg_bytes_per_launch": alg,
                     # bytes the device moves per pair: each launch moves the batch once in
                     # and once out (four launches per pair on the four-step kernels, two
                     # on the whole-plane ones)
                     "whole_op_GBs": value / world * (sum(v["launches"] for v in kernels.values())
                                                      / args.steps) * alg / batch / 1e9,
                     "kernels": kernels},
        "cpu_baseline": cpu,
        "power": power,
    }


def run_pointwise(args, comm, world, rank, local_rank):
    """SURVEY §8d's secondary figure: MulAssign with both operands in the NTT
    domain (poly.rs:297-306, a Montgomery pointwise product per residue),
    `--batch` pairs per step, in place of the first operand's copy."""
    import numpy as np

    import rns_ntt as rn

    n = 1 << args.log_n
    L = args.limbs
    mod = rn.generate_primes(args.prime_bits, L, n)
    B = rn.RnsBasis(mod, n, device=local_rank)
    wb = 4 if max(mod) < (1 << 31) else 8
    batch = args.batch
    drng = rn.DeviceRng(777 + rank)
    a = rn.RnsPoly.sample_uniform(B, drng, batch)
    b = rn.RnsPoly.sample_uniform(B, drng, batch)
    a.to_ntt_domain()
    b.to_ntt_domain()
    out = rn.RnsPoly(B, batch)
    lib = rn.load()
    for _ in range(args.warmup):
        rn.check(lib.rnt_mul(out.handle, a.handle, b.handle))
    B.sync()
    comm.barrier()
    B.profile_enable(True)
    B.sync()
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        rn.check(lib.rnt_mul(out.handle, a.handle, b.handle))
    B.sync()
    t1 = time.perf_counter()
    comm.barrier()
    elapsed = comm.max(t1 - t0)
    cnt, ms = B.profile_read("elementwise")
    B.profile_enable(False)
    power = None
    if rank == 0 and not args.no_power:
        power = power_probe(lambda: rn.check(lib.rnt_mul(out.handle, a.handle, b.handle)), B.sync, local_rank)
    parity_ok = True
    if rank == 0:
        orc = oracle()
        ob = orc.Basis(mod, n)
        for pi in sorted({0, batch - 1}):
            want = orc.mul(ob, a.channels_of(pi)[0], b.channels_of(pi)[0], ntt=True)
            parity_ok &= bool(np.array_equal(out.channels_of(pi)[0], want))
    alg = 3 * L * batch * n * wb  # read a, read b, write out
    achieved = alg / (ms / cnt * 1e-3) / 1e9 if cnt else None
    value = batch * args.steps * world / elapsed
    return {
        "metric": PW_METRIC,
        "value": value,
        "unit": "poly-muls/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32" if wb == 4 else "u64",
        "data": "synthetic (seeded uniform residues drawn on the device, transformed)",
        "config": {
            "workload": f"NTT-domain MulAssign, N=2^{args.log_n}, L={L} x {args.prime_bits}-bit primes, "
                        f"{batch} pairs per step",
            "parallelism": f"replicas x{world}",
            "parity_spot_check": parity_ok,
        },
        "roofline": {"bound": "hbm", "kernel": "elementwise", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS if achieved else None,
                     "traffic": None, "alg_bytes_per_launch": alg,
                     "kernels": {"elementwise": {"launches": cnt, "avg_ms": ms / cnt if cnt else None,
                                                 "total_ms": ms}}},
        "cpu_baseline": None,
        "power": power,
    }


def run_copy(args, comm, world, rank, local_rank):
    """A plain device copy of `--batch` polys (rnt_copy = k_copy16, 16 bytes
    per lane): the measured streaming bandwidth the roofline fractions are
    compared against, and a pure-HBM point of the energy model
    (tools/energy_model.py)."""
    import rns_ntt as rn

    n = 1 << args.log_n
    L = args.limbs
    mod = rn.generate_primes(args.prime_bits, L, n)
    B = rn.RnsBasis(mod, n, device=local_rank)
    wb = 4 if max(mod) < (1 << 31) else 8
    a = rn.RnsPoly.sample_uniform(B, rn.DeviceRng(55 + rank), args.batch)
    dst = rn.RnsPoly(B, args.batch)
    lib = rn.load()

    def step():
        rn.check(lib.rnt_copy(dst.handle, a.handle))

    for _ in range(args.warmup):
        step()
    B.sync()
    comm.barrier()
    B.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    B.sync()
    t1 = time.perf_counter()
    comm.barrier()
    elapsed = comm.max(t1 - t0)
    cnt, ms = B.profile_read("copy")
    B.profile_enable(False)
    power = power_probe(step, B.sync, local_rank) if rank == 0 and not args.no_power else None
    alg = 2 * L * args.batch * n * wb
    achieved = alg / (ms / cnt * 1e-3) / 1e9
    return {
        "metric": "device copy GB/s (read + write)",
        "value": alg * args.steps * world / elapsed / 1e9,
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32" if wb == 4 else "u64",
        "data": "synthetic (seeded uniform residues drawn on the device)",
        "config": {"workload": f"rnt_copy of {args.batch} polys, N=2^{args.log_n}, L={L}",
                   "parallelism": f"replicas x{world}"},
        "roofline": {"bound": "hbm", "kernel": "copy", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None, "alg_bytes_per_launch": alg,
                     "kernels": {"copy": {"launches": cnt, "avg_ms": ms / cnt, "total_ms": ms}}},
        "cpu_baseline": None,
        "power": power,
    }


def run_rotate_sharded(args, comm, world, rank, local_rank, log_n, L, mod):
    """Config 5 limb-sharded: each rank owns L/world limbs of a
    global batch of rot_batch * world ciphertexts and a [L][L_r][N] slice of
    the rotation key; per offset: limb-local slot rotation, RCCL all-gather
    of sigma(c1) per pipeline chunk, key-switch of the local target limbs,
    all queued on the library's stream (shared stream; RNT_SHARED_STREAM=0:
    torch's stream with per-op host syncs)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from rns_ntt.sharded import GpuBackend, LimbShardedPipeline, TorchDistComm

    n = 1 << log_n
    torch.cuda.set_device(local_rank)
    pipe = LimbShardedPipeline(mod, n, TorchDistComm(dist.new_group(backend=data_backend())), GpuBackend(local_rank))
    B = args.rot_batch * world
    rng = np.random.default_rng(5)
    uniq = min(2, B)
    reps = (B + uniq - 1) // uniq
    c0_u, c1_u = uniform(rng, mod, uniq, n), uniform(rng, mod, uniq, n)
    c0 = pipe.upload(np.tile(c0_u, (reps, 1, 1))[:B])
    c1 = pipe.upload(np.tile(c1_u, (reps, 1, 1))[:B])
    ka, kb = uniform(rng, mod, L, n), uniform(rng, mod, L, n)
    key = pipe.upload_key(ka, kb)
    offsets = [1 << e for e in range(log_n - 1)]
    shared = os.environ.get("RNT_SHARED_STREAM", "1") != "0"
    lib_stream = pipe.backend.shared_stream(pipe.basis) if shared else torch.cuda.current_stream()

    def step():
        with torch.cuda.stream(lib_stream):
            for k in offsets:
                out = pipe.rotate(c0, c1, k, key)
        return out

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    comm.barrier()
    elapsed = comm.max(t1 - t0)
    value = B * len(offsets) * args.steps / elapsed
    bfly = (L * L + 2 * L) * (n // 2) * log_n
    # sampled parity of the last offset's output: ciphertext 0 and the last
    # one, every rank's limbs gathered to rank 0 over the gloo control plane
    check = sorted({0, B - 1})
    mine = {p: (pipe.download(out[0], first=p, count=1)[0], pipe.download(out[1], first=p, count=1)[0])
            for p in check}
    parts = comm.gather((pipe.limbs.start, mine))
    parity_ok = None
    if rank == 0:
        orc = oracle()
        ob = orc.Basis(mod, n)
        parts = sorted(parts, key=lambda t: t[0])
        parity_ok = True
        for p in check:
            g0 = np.concatenate([pr[1][p][0] for pr in parts], axis=0)
            g1 = np.concatenate([pr[1][p][1] for pr in parts], axis=0)
            w0, w1 = orc.rotate_ciphertext(ob, c0_u[p % uniq], c1_u[p % uniq], offsets[-1], ka, kb,
                                           threads=usable_threads())
            parity_ok &= bool(np.array_equal(g0, w0) and np.array_equal(g1, w1))
    return {
        "metric": ROT_METRIC,
        "value": value,
        "unit": "rotations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32" if max(mod) < (1 << 31) else "u64",
        "data": "synthetic (seeded uniform residues and key; one key reused for every offset)",
        "config": {
            "workload": f"rotate_ciphertext sweep over {len(offsets)} power-of-two offsets, "
                        f"N=2^{log_n}, L={L} x 31-bit primes, {B} ciphertexts (global)",
            "parallelism": f"limb-sharded x{world}: RCCL all-gather of sigma(c1) per offset and chunk",
            "parity_spot_check": parity_ok,
            "parity_ciphertexts": check,
            "shared_stream": shared,
        },
        # whole key-switch butterflies per GPU (no per-kernel events on this path)
        "roofline": {"bound": "valu", "kernel": "whole key-switch", "unit": "butterflies/s",
                     "achieved": value / world * bfly, "peak": VALU_PEAK_BFLY,
                     "frac": value / world * bfly / VALU_PEAK_BFLY, "traffic": None},
        "cpu_baseline": None,
    }


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch_with_torchrun(args))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("BENCH_ONE_DEVICE") == "1":
        # rehearsal of the N-rank control plane on a one-GPU box: every rank
        # on device 0 (poly-mul / ntt / encode only; RCCL refuses two ranks
        # on one device)
        local_rank = 0

    # the JSON line is the only thing on stdout: everything else written to
    # fd 1 (gloo's and RCCL's connection messages, library prints) goes to
    # stderr, and the line goes to a private copy of the original stdout
    sys.stdout.flush()
    result_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    import rns_ntt  # noqa: F401
    from rns_ntt.dist import Comm

    comm = Comm.from_env()
    run = {"polymul": run_polymul, "ctmul": run_ctmul, "rotate": run_rotate,
           "encode": run_encode, "ntt": run_ntt,
           "pointwise": run_pointwise, "copy": run_copy}[args.workload]
    line = run(args, comm, world, rank, local_rank)
    if rank == 0:
        result_out.write(json.dumps(line) + "\n")
        result_out.flush()
    comm.close()


if __name__ == "__main__":
    main()
