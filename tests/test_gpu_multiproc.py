"""The limb-sharded pipeline across PROCESSES on one MI355X (VERDICT r01
"do this" #7): world_size 2 under torch.distributed.run with a gloo process
group, each rank a separate process with its own library context on device
0, running LimbShardedPipeline + GpuBackend (tests/mp/limb_shard_worker.py).
This covers what the thread-rank test cannot: TorchDistComm.all_gather_limbs
and .broadcast between processes over torch CUDA tensors that the library
reads and writes in place (rnt_buf_wrap).  Uneven shards: L = 5 gives the
ranks 3 and 2 limbs.  Results are bit-exact against the unsharded oracle:
rotate_ciphertext (engine.rs:412-463), mul_ciphertexts_gadget
(engine.rs:473-539) and rescale_ciphertext (engine.rs:263-282).  RCCL itself
needs one GPU per rank: on a one-GPU box it runs at world_size 1
(test_single_rank_rccl_limb_pipeline: every join an RCCL collective on the
library's buffers), across GPUs only in the driver's multi-GPU bench."""
from __future__ import annotations

import os
import subprocess
import sys

import numpy as np
import pytest

import pyoracle as orc

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("shared", [False, True], ids=["torch-stream", "shared-stream"])
def test_two_process_limb_sharded_pipeline(gpu, tmp_path, shared):
    """shared: each rank queues torch's ops and the (async, per-chunk) joins
    on its library context's stream -- the bench's default at every N -- with
    B = 3 in pipeline chunks of 2."""
    rn = gpu
    n, L, B, k = 1 << 12, 5, 3, -3
    mod = rn.generate_primes(31, L, n)
    rng = np.random.default_rng(2024)
    u = lambda b=None: orc.uniform_poly(mod, n, rng, batch=b)  # noqa: E731
    z = {"moduli": np.array(mod, dtype=np.uint64), "n": n, "k": k,
         "c0": u(B), "c1": u(B), "c0p": u(B), "c1p": u(B), "ka": u(L), "kb": u(L), "ra": u(L), "rb": u(L)}
    inp = str(tmp_path / "inputs.npz")
    np.savez(inp, **z)
    out = str(tmp_path / "res")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(29611 + int(shared)),
           os.path.join(REPO, "tests", "mp", "limb_shard_worker.py"), "--inputs", inp, "--out", out,
           "--chunk", "2"] + (["--shared"] if shared else [])
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    ranks = [np.load(f"{out}.rank{r}.npz") for r in range(2)]
    assert [tuple(r["limbs"]) for r in ranks] == [(0, 3), (3, 5)]

    def gather(key, limbs_key="limbs"):
        parts = sorted(((int(r[limbs_key][0]), r[key]) for r in ranks), key=lambda t: t[0])
        return np.concatenate([p for _, p in parts], axis=1)

    Bo = orc.Basis(mod, n)
    rot0, rot1 = gather("rot0"), gather("rot1")
    mul0, mul1 = gather("mul0"), gather("mul1")
    res0, res1 = gather("res0", "res_limbs"), gather("res1", "res_limbs")
    for p in range(B):
        w0, w1 = orc.rotate_ciphertext(Bo, z["c0"][p], z["c1"][p], k, z["ra"], z["rb"])
        assert np.array_equal(rot0[p], w0) and np.array_equal(rot1[p], w1), p
        m0, m1 = orc.mul_ciphertexts_gadget(Bo, z["c0"][p], z["c1"][p], z["c0p"][p], z["c1p"][p], z["ka"], z["kb"])
        assert np.array_equal(mul0[p], m0) and np.array_equal(mul1[p], m1), p
        assert np.array_equal(res0[p], orc.rescale(Bo, m0)) and np.array_equal(res1[p], orc.rescale(Bo, m1)), p


@pytest.mark.parametrize("backend", ["nccl", "gloo+nccl"])
def test_single_rank_rccl_limb_pipeline(gpu, tmp_path, backend):
    """The joins over RCCL itself (backend nccl, the driver's multi-GPU
    layout), at the one rank a one-GPU box allows: rotate_ciphertext's
    all-gather of sigma(c1), mul_ciphertexts_gadget's all-gather of d2 (both
    all_gather_into_tensor: equal limb counts) and rescale_ciphertext's
    broadcast of the last limb run as RCCL collectives on the library's
    buffers (rnt_buf_wrap), bit-exact against the oracle.  gloo+nccl is
    bench.py's layout: a gloo default group (control plane) and the joins on
    dist.new_group(backend="nccl")."""
    rn = gpu
    n, L, B, k = 1 << 12, 4, 3, 5
    mod = rn.generate_primes(31, L, n)
    rng = np.random.default_rng(4242)
    u = lambda b=None: orc.uniform_poly(mod, n, rng, batch=b)  # noqa: E731
    z = {"moduli": np.array(mod, dtype=np.uint64), "n": n, "k": k,
         "c0": u(B), "c1": u(B), "c0p": u(B), "c1p": u(B), "ka": u(L), "kb": u(L), "ra": u(L), "rb": u(L)}
    inp = str(tmp_path / "inputs.npz")
    np.savez(inp, **z)
    out = str(tmp_path / "res")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0", NCCL_SOCKET_IFNAME="lo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", str(29631 + (backend != "nccl")),
           os.path.join(REPO, "tests", "mp", "limb_shard_worker.py"), "--inputs", inp, "--out", out,
           "--backend", backend]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    r = np.load(f"{out}.rank0.npz")
    assert tuple(r["limbs"]) == (0, L)
    Bo = orc.Basis(mod, n)
    for q in range(B):
        w0, w1 = orc.rotate_ciphertext(Bo, z["c0"][q], z["c1"][q], k, z["ra"], z["rb"])
        assert np.array_equal(r["rot0"][q], w0) and np.array_equal(r["rot1"][q], w1), q
        m0, m1 = orc.mul_ciphertexts_gadget(Bo, z["c0"][q], z["c1"][q], z["c0p"][q], z["c1p"][q], z["ka"], z["kb"])
        assert np.array_equal(r["mul0"][q], m0) and np.array_equal(r["mul1"][q], m1), q
        assert np.array_equal(r["res0"][q], orc.rescale(Bo, m0)) and np.array_equal(r["res1"][q], orc.rescale(Bo, m1)), q
