#!/usr/bin/env python3
"""Per-step time and free device memory of the single-GPU ct-mul pipeline
(bench.py --workload ctmul) over many steps: finds allocation growth."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "toy-heaan-ckks_amd"))
import numpy as np
import torch

import rns_ntt as rn
from rns_ntt.sharded import GpuBackend, LimbShardedPipeline, SingleComm

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
n, L = 1 << 16, 16
mod = rn.generate_primes(31, L, n)
torch.cuda.set_device(0)
pipe = LimbShardedPipeline(mod, n, SingleComm(), GpuBackend(0))
rng = np.random.default_rng(1)
cts = [rng.integers(0, 2**30, (B, L, n), dtype=np.uint64) for _ in range(4)]
c = [pipe.upload(x) for x in cts]
key = pipe.upload_key(rng.integers(0, 2**30, (L, L, n), dtype=np.uint64),
                      rng.integers(0, 2**30, (L, L, n), dtype=np.uint64))
state0 = (pipe.basis, pipe.moduli, list(pipe.counts), pipe.limbs, pipe.owner_last)
for s in range(steps):
    t = time.perf_counter()
    pipe.basis, pipe.moduli, counts, pipe.limbs, pipe.owner_last = state0
    pipe.counts = list(counts)
    m0, m1 = pipe.mul_relin(c[0], c[1], c[2], c[3], key)
    r = pipe.rescale(m0, m1)
    del m0, m1
    torch.cuda.synchronize()
    free, total = torch.cuda.mem_get_info()
    print(f"step {s:3d} {1e3 * (time.perf_counter() - t):8.2f} ms  free {free / 2**30:7.1f} GiB"
          f"  torch reserved {torch.cuda.memory_reserved() / 2**30:6.1f} GiB", flush=True)
