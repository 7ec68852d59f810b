"""BASELINE configs 4 and 5 limb-sharded at their real sizes (VERDICT r02
"next round" #1): LimbShardedPipeline with 8 simulated ranks (ThreadComm,
one thread per rank, every rank its own library context on device 0 --
the 8-GPU layout of SURVEY §8e, each rank owning L/8 limbs).

* config 4: N = 2^16, L = 16 (2 limbs per rank), 66 ciphertext pairs in
  pipeline chunks of 64 (two chunks, the second ragged), ct x ct -> gadget
  relin (all-gather of d2 per chunk) -> rescale (broadcast of the last
  limb per chunk);
* config 5: N = 2^17, L = 32 (4 limbs per rank), rotate_ciphertext at
  k in {1, -3, 2^15} (all-gather of sigma(c1)), 3 ciphertexts in chunks of 2.

Sampled ciphertexts (the first, the first of the second chunk, the last)
are compared bit-exactly with the oracle's mul_ciphertexts_gadget + rescale
(engine.rs:473-539, 263-282) and rotate_ciphertext (engine.rs:412-463).
Both stream modes of GpuBackend run config 4: torch's stream with host
syncs, and the library's stream shared with torch (the bench default).
"""
from __future__ import annotations

import contextlib
import threading

import numpy as np
import pytest

import pyoracle as orc

pytestmark = pytest.mark.gpu

T = 16  # oracle worker threads


def _run_ranks(comm, body):
    """body(rank) on comm.world threads; a failing rank aborts the others'
    barriers, and the first failure fails the test."""
    world = comm.world
    errors, results = [], [None] * world

    def main(r):
        try:
            results[r] = body(r)
        except BaseException as e:  # surface thread failures in the test
            errors.append(e)
            comm.abort()

    ths = [threading.Thread(target=main, args=(r,)) for r in range(world)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=900)
    assert not errors, errors
    assert all(r is not None for r in results)
    return results


@pytest.mark.parametrize("shared", [True, False], ids=["shared-stream", "torch-stream"])
def test_config4_limb_sharded_8_ranks(gpu, shared):
    import torch

    rn = gpu
    from rns_ntt.sharded import GpuBackend, LimbShardedPipeline, ThreadComm

    n, L, B, world, chunk = 1 << 16, 16, 66, 8, 64
    mods = rn.generate_primes(31, L, n)
    rng = np.random.default_rng(4016)
    cts = [orc.uniform_poly(mods, n, rng, batch=B) for _ in range(4)]
    ka, kb = orc.uniform_poly(mods, n, rng, batch=L), orc.uniform_poly(mods, n, rng, batch=L)
    check = (0, chunk, B - 1)
    comm = ThreadComm(world)

    def rank(r):
        be = GpuBackend(0)
        pipe = LimbShardedPipeline(mods, n, comm.rank_view(r), be, chunk=chunk)
        assert len(pipe.limbs) == 2
        ctx = torch.cuda.stream(be.shared_stream(pipe.basis)) if shared else contextlib.nullcontext()
        with ctx:
            c = [pipe.upload(x) for x in cts]
            assert [be.batch(x) for x in c[0]] == [64, 2]
            key = pipe.upload_key(ka, kb)
            m0, m1 = pipe.mul_relin(c[0], c[1], c[2], c[3], key)
            relin = {p: (pipe.download(m0, p, 1)[0], pipe.download(m1, p, 1)[0]) for p in check}
            s0, s1 = pipe.rescale(m0, m1)
            resc = {p: (pipe.download(s0, p, 1)[0], pipe.download(s1, p, 1)[0]) for p in check}
        torch.cuda.synchronize()
        return pipe.limbs.start, relin, resc

    res = sorted(_run_ranks(comm, rank), key=lambda t: t[0])
    ob = orc.Basis(mods, n)
    for p in check:
        w0, w1 = orc.mul_ciphertexts_gadget(ob, cts[0][p], cts[1][p], cts[2][p], cts[3][p], ka, kb, threads=T)
        g0 = np.concatenate([x[1][p][0] for x in res], axis=0)
        g1 = np.concatenate([x[1][p][1] for x in res], axis=0)
        assert np.array_equal(g0, w0) and np.array_equal(g1, w1), ("relin", p)
        r0 = np.concatenate([x[2][p][0] for x in res], axis=0)
        r1 = np.concatenate([x[2][p][1] for x in res], axis=0)
        assert r0.shape == (L - 1, n)
        assert np.array_equal(r0, orc.rescale(ob, w0)) and np.array_equal(r1, orc.rescale(ob, w1)), ("rescale", p)


@pytest.mark.parametrize("k", [1, -3, 1 << 15])
def test_config5_limb_sharded_rotation_8_ranks(gpu, k):
    import torch

    rn = gpu
    from rns_ntt.sharded import GpuBackend, LimbShardedPipeline, ThreadComm

    n, L, B, world, chunk = 1 << 17, 32, 3, 8, 2
    mods = rn.generate_primes(31, L, n)
    rng = np.random.default_rng(5017 + k)
    c0 = orc.uniform_poly(mods, n, rng, batch=B)
    c1 = orc.uniform_poly(mods, n, rng, batch=B)
    ka, kb = orc.uniform_poly(mods, n, rng, batch=L), orc.uniform_poly(mods, n, rng, batch=L)
    check = (0, B - 1)
    comm = ThreadComm(world)

    def rank(r):
        be = GpuBackend(0)
        pipe = LimbShardedPipeline(mods, n, comm.rank_view(r), be, chunk=chunk)
        assert len(pipe.limbs) == 4
        with torch.cuda.stream(be.shared_stream(pipe.basis)):
            x0, x1 = pipe.upload(c0), pipe.upload(c1)
            key = pipe.upload_key(ka, kb)
            o0, o1 = pipe.rotate(x0, x1, k, key)
            out = {p: (pipe.download(o0, p, 1)[0], pipe.download(o1, p, 1)[0]) for p in check}
        torch.cuda.synchronize()
        return pipe.limbs.start, out

    res = sorted(_run_ranks(comm, rank), key=lambda t: t[0])
    ob = orc.Basis(mods, n)
    for p in check:
        w0, w1 = orc.rotate_ciphertext(ob, c0[p], c1[p], k, ka, kb, threads=T)
        g0 = np.concatenate([x[1][p][0] for x in res], axis=0)
        g1 = np.concatenate([x[1][p][1] for x in res], axis=0)
        assert np.array_equal(g0, w0) and np.array_equal(g1, w1), (k, p)
