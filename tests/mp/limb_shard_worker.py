"""One rank of the multi-process limb-sharded pipeline test
(tests/test_gpu_multiproc.py): launched by torch.distributed.run with
world_size 2 on ONE GPU, gloo process group (or world_size 1 over RCCL,
--backend nccl).  Each rank runs
LimbShardedPipeline with GpuBackend on device 0 -- its limbs in its own
library context, the joins (all-gather of d2 / sigma(c1), broadcast of the
last limb) as torch collectives between the processes over buffers the
library reads and writes in place (rnt_buf_wrap) -- and saves its limbs of
the results for the parent to compare against the oracle."""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "toy-heaan-ckks_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--inputs", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--shared", action="store_true",
                    help="queue torch's ops and the joins on the library's stream (GpuBackend.shared_stream)")
    ap.add_argument("--chunk", type=int, default=None)
    ap.add_argument("--backend", default="gloo", choices=["gloo", "nccl", "gloo+nccl"],
                    help="the process group of the joins (nccl = RCCL: one GPU per rank); gloo+nccl: "
                         "bench.py's layout, a gloo default group and an nccl group for the joins")
    args = ap.parse_args()

    import rns_ntt  # noqa: F401  (loads librnsntt before torch initialises HIP)
    import torch
    import torch.distributed as dist

    from rns_ntt.sharded import GpuBackend, LimbShardedPipeline, TorchDistComm

    torch.cuda.set_device(0)
    dist.init_process_group(args.backend.split("+")[0])
    rank = dist.get_rank()
    data_group = dist.new_group(backend="nccl") if args.backend == "gloo+nccl" else None
    z = np.load(args.inputs)
    mod = [int(q) for q in z["moduli"]]
    n = int(z["n"])
    import contextlib

    be = GpuBackend(0)
    pipe = LimbShardedPipeline(mod, n, TorchDistComm(data_group), be, chunk=args.chunk)
    scope = torch.cuda.stream(be.shared_stream(pipe.basis)) if args.shared else contextlib.nullcontext()
    scope.__enter__()
    c = [pipe.upload(z[k]) for k in ("c0", "c1", "c0p", "c1p")]
    rlk = pipe.upload_key(z["ka"], z["kb"])
    rotk = pipe.upload_key(z["ra"], z["rb"])
    lo, hi = pipe.limbs.start, pipe.limbs.stop
    res = {"limbs": np.array([lo, hi])}
    # rotation join first (the pipeline's level is unchanged by it)
    r0, r1 = pipe.rotate(c[0], c[1], int(z["k"]), rotk)
    res["rot0"], res["rot1"] = pipe.download(r0), pipe.download(r1)
    m0, m1 = pipe.mul_relin(c[0], c[1], c[2], c[3], rlk)
    res["mul0"], res["mul1"] = pipe.download(m0), pipe.download(m1)
    s0, s1 = pipe.rescale(m0, m1)
    res["res0"], res["res1"] = pipe.download(s0), pipe.download(s1)
    res["res_limbs"] = np.array([pipe.limbs.start, pipe.limbs.stop])
    scope.__exit__(None, None, None)
    torch.cuda.synchronize()
    np.savez(f"{args.out}.rank{rank}.npz", **res)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
