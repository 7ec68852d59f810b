"""Limb-sharded ct x ct -> relin -> rescale and
limb-sharded rotation key-switch.

CPU: world_size 2/3 gloo ranks run rns_ntt.sharded.LimbShardedPipeline with
the oracle backend (tests/shard_oracle_backend.py); the assembled per-rank
limbs must equal the unsharded oracle pipeline (oracle/oracle.c restating
engine.rs:473-539 and poly.rs:187-228) bit-exactly.

GPU: the same pipeline on one MI355X with the ranks simulated as threads
(ThreadComm), through librnsntt's rnt_ct_tensor / rnt_keyswitch_ext /
rnt_rescale_ext, against the unsharded library path and the oracle.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import pyoracle as orc


def _inputs(mods, n, B, seed):
    rng = np.random.default_rng(seed)
    L = len(mods)
    cts = [orc.uniform_poly(mods, n, rng, batch=B) for _ in range(4)]  # c0 c1 c0' c1'
    key_a = orc.uniform_poly(mods, n, rng, batch=L)
    key_b = orc.uniform_poly(mods, n, rng, batch=L)
    return cts, key_a, key_b


def _oracle_reference(mods, n, cts, key_a, key_b):
    ob = orc.Basis(mods, n)
    r0, r1, s0, s1 = [], [], [], []
    for p in range(cts[0].shape[0]):
        o0, o1 = orc.mul_ciphertexts_gadget(ob, cts[0][p], cts[1][p], cts[2][p], cts[3][p], key_a, key_b)
        r0.append(o0)
        r1.append(o1)
        s0.append(orc.rescale(ob, o0))
        s1.append(orc.rescale(ob, o1))
    return np.stack(r0), np.stack(r1), np.stack(s0), np.stack(s1)


def _run_rank(pipe, cts, key_a, key_b):
    c = [pipe.upload(x) for x in cts]
    key = pipe.upload_key(key_a, key_b)
    m0, m1 = pipe.mul_relin(c[0], c[1], c[2], c[3], key)
    relin = (pipe.download(m0), pipe.download(m1))
    r0, r1 = pipe.rescale(m0, m1)
    return relin, (pipe.download(r0), pipe.download(r1))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gloo_worker(rank, world, port, mods, n, B, seed, q, chunk=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from rns_ntt.sharded import LimbShardedPipeline, TorchDistComm
    from shard_oracle_backend import OracleBackend

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cts, key_a, key_b = _inputs(mods, n, B, seed)
        pipe = LimbShardedPipeline(mods, n, TorchDistComm(), OracleBackend(), chunk=chunk)
        limbs = (pipe.limbs.start, pipe.limbs.stop)
        relin, resc = _run_rank(pipe, cts, key_a, key_b)
        q.put((rank, limbs, relin, resc))
    finally:
        dist.destroy_process_group()


def _collect(q, procs, count, timeout=300.0):
    """Results from the workers; fail fast if one of them dies."""
    import queue
    import time

    out, t0 = [], time.time()
    while len(out) < count:
        try:
            out.append(q.get(timeout=2))
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead, f"worker exited with {dead}"
            assert time.time() - t0 < timeout, "workers timed out"
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def _assemble(results):
    results = sorted(results, key=lambda r: r[0])
    relin0 = np.concatenate([r[2][0] for r in results], axis=1)
    relin1 = np.concatenate([r[2][1] for r in results], axis=1)
    resc0 = np.concatenate([r[3][0] for r in results], axis=1)
    resc1 = np.concatenate([r[3][1] for r in results], axis=1)
    return relin0, relin1, resc0, resc1


@pytest.mark.parametrize("world,L,B,chunk", [(2, 4, 2, None), (3, 7, 3, 2), (2, 5, 3, 1)])
def test_limb_sharded_gloo_matches_unsharded(world, L, B, chunk):
    """chunk: ciphertexts per pipeline chunk (each chunk's joins start as
    soon as its tensor product exists); 2 and 1 split B = 3 into uneven
    chunks."""
    n, seed = 32, 5
    mods = orc.generate_primes(31, L, n)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_worker, args=(r, world, port, mods, n, B, seed, q, chunk))
             for r in range(world)]
    for p in procs:
        p.start()
    results = _collect(q, procs, world)
    # contiguous limb runs in rank order covering the basis
    spans = [r[1] for r in sorted(results, key=lambda r: r[0])]
    assert spans[0][0] == 0 and spans[-1][1] == L
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    cts, key_a, key_b = _inputs(mods, n, B, seed)
    want = _oracle_reference(mods, n, cts, key_a, key_b)
    got = _assemble(results)
    for g, w in zip(got, want):
        assert np.array_equal(g.astype(np.uint64), w)


@pytest.mark.parametrize("world,L,B,chunk", [(2, 4, 3, 1), (3, 7, 5, 2)])
def test_limb_sharded_thread_ranks_async_joins(world, L, B, chunk):
    """ThreadComm's joins run on helper threads and wait() blocks until the
    join is done.  The joins are held at a gate until every rank has issued
    the relin all-gather of EVERY chunk (which it can only do if starting a
    join does not wait for it: the chunks' tensor products run while the
    earlier chunks' joins are in flight); then the pipeline finishes and the
    assembled limbs must equal the unsharded oracle pipeline."""
    import threading
    import time

    from rns_ntt.sharded import LimbShardedPipeline, ThreadComm
    from shard_oracle_backend import OracleBackend

    n, seed = 32, 9
    mods = orc.generate_primes(31, L, n)
    cts, key_a, key_b = _inputs(mods, n, B, seed)
    comm = ThreadComm(world)
    gate, lock, calls = threading.Event(), threading.Lock(), []
    real_join = comm._join

    class Gated:
        def __init__(self, bar):
            self._b = bar

        def wait(self):
            gate.wait()
            return self._b.wait()

        def abort(self):
            self._b.abort()

    def recording_join(seq):
        j = real_join(seq)
        with lock:
            calls.append(seq)
            if not isinstance(j.bar, Gated):
                j.bar = Gated(j.bar)
        return j

    comm._join = recording_join
    results, errors = [None] * world, []

    def rank_main(r):
        try:
            pipe = LimbShardedPipeline(mods, n, comm.rank_view(r), OracleBackend(), chunk=chunk)
            relin, resc = _run_rank(pipe, cts, key_a, key_b)
            results[r] = (r, (pipe.limbs.start, pipe.limbs.stop), relin, resc)
        except BaseException as e:  # surface thread failures in the test
            errors.append(e)
            comm.abort()

    threads = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in threads:
        t.start()
    chunks = -(-B // chunk)
    t0 = time.time()
    while len(calls) < world * chunks and time.time() - t0 < 60:
        time.sleep(0.01)
    issued = len(calls)
    gate.set()
    for t in threads:
        t.join(timeout=120)
    assert issued == world * chunks, (issued, world * chunks)
    assert not errors, errors
    got = _assemble(results)
    want = _oracle_reference(mods, n, cts, key_a, key_b)
    for g, w in zip(got, want):
        assert np.array_equal(g.astype(np.uint64), w)


ROT_K = (1, -3, 0)  # slot offsets; negative = rotate_slots(k < 0), 0 = identity


def _rot_inputs(mods, n, B, seed):
    rng = np.random.default_rng(seed)
    L = len(mods)
    c0 = orc.uniform_poly(mods, n, rng, batch=B)
    c1 = orc.uniform_poly(mods, n, rng, batch=B)
    key_a = orc.uniform_poly(mods, n, rng, batch=L)
    key_b = orc.uniform_poly(mods, n, rng, batch=L)
    return c0, c1, key_a, key_b


def _rot_oracle(mods, n, c0, c1, key_a, key_b, k):
    """engine.rs:412-463 restated (oracle/oracle.c or_rotate_ciphertext)."""
    ob = orc.Basis(mods, n)
    r = [orc.rotate_ciphertext(ob, c0[p], c1[p], k, key_a, key_b) for p in range(c0.shape[0])]
    return np.stack([x[0] for x in r]), np.stack([x[1] for x in r])


def _run_rank_rotate(pipe, c0, c1, key_a, key_b):
    x0, x1 = pipe.upload(c0), pipe.upload(c1)
    key = pipe.upload_key(key_a, key_b)
    outs = []
    for k in ROT_K:
        o0, o1 = pipe.rotate(x0, x1, k, key)
        outs.append((pipe.download(o0), pipe.download(o1)))
    return outs


def _gloo_rot_worker(rank, world, port, mods, n, B, seed, q, chunk=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from rns_ntt.sharded import LimbShardedPipeline, TorchDistComm
    from shard_oracle_backend import OracleBackend

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c0, c1, key_a, key_b = _rot_inputs(mods, n, B, seed)
        pipe = LimbShardedPipeline(mods, n, TorchDistComm(), OracleBackend(), chunk=chunk)
        q.put((rank, _run_rank_rotate(pipe, c0, c1, key_a, key_b)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,L,B,chunk", [(2, 4, 2, None), (3, 5, 3, 2)])
def test_limb_sharded_rotation_gloo_matches_unsharded(world, L, B, chunk):
    n, seed = 32, 21
    mods = orc.generate_primes(31, L, n)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_rot_worker, args=(r, world, port, mods, n, B, seed, q, chunk))
             for r in range(world)]
    for p in procs:
        p.start()
    results = sorted(_collect(q, procs, world), key=lambda r: r[0])
    c0, c1, key_a, key_b = _rot_inputs(mods, n, B, seed)
    for ki, k in enumerate(ROT_K):
        want0, want1 = _rot_oracle(mods, n, c0, c1, key_a, key_b, k)
        got0 = np.concatenate([r[1][ki][0] for r in results], axis=1)
        got1 = np.concatenate([r[1][ki][1] for r in results], axis=1)
        assert np.array_equal(got0.astype(np.uint64), want0), k
        assert np.array_equal(got1.astype(np.uint64), want1), k


def test_sharded_layout_bookkeeping():
    """Rescale drops the last limb only on its owner; later joins follow."""
    from rns_ntt.sharded import LimbShardedPipeline

    class _Comm:
        def __init__(self, rank, world):
            self.rank, self.world = rank, world

    class _NullBackend:
        def make_basis(self, moduli, degree):
            return list(moduli)

    pipes = [LimbShardedPipeline(list(range(101, 117)), 8, _Comm(r, 3), _NullBackend()) for r in range(3)]
    assert [(p.limbs.start, p.limbs.stop) for p in pipes] == [(0, 6), (6, 11), (11, 16)]
    assert all(p.owner_last == 2 for p in pipes)


# ---------------------------------------------------------------------------
# GPU: simulated ranks (threads) on one MI355X through librnsntt
# ---------------------------------------------------------------------------


@pytest.mark.gpu
@pytest.mark.parametrize("shared", [False, True], ids=["torch-stream", "shared-stream"])
@pytest.mark.parametrize("world", [2, 4])
def test_limb_sharded_gpu_threads_match_unsharded(gpu, world, shared):
    import contextlib
    import threading

    import torch

    import rns_ntt as rn
    from rns_ntt.sharded import GpuBackend, LimbShardedPipeline, ThreadComm

    n, L, B, seed = 4096, 8, 2, 11
    mods = rn.generate_primes(31, L, n)
    cts, key_a, key_b = _inputs(mods, n, B, seed)
    comm = ThreadComm(world)
    results, errors = [None] * world, []

    def rank_main(r):
        try:
            be = GpuBackend(0)
            pipe = LimbShardedPipeline(mods, n, comm.rank_view(r), be)
            # shared: torch runs on the library's stream and the host syncs drop out
            ctx = torch.cuda.stream(be.shared_stream(pipe.basis)) if shared else contextlib.nullcontext()
            with ctx:
                relin, resc = _run_rank(pipe, cts, key_a, key_b)
            results[r] = (r, (pipe.limbs.start, pipe.limbs.stop), relin, resc)
        except BaseException as e:  # surface thread failures in the test
            errors.append(e)
            comm.abort()

    threads = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=600)
    assert not errors, errors
    got = _assemble(results)

    # unsharded library path (oracle-checked elsewhere) ...
    Bf = rn.RnsBasis(mods, n)
    c = [rn.RnsPoly.from_channels(x, Bf) for x in cts]
    key = rn.RnsGadgetKey.from_channels(key_a, key_b, Bf)
    m = rn.mul_ciphertexts_gadget(rn.Ciphertext(c[0], c[1]), rn.Ciphertext(c[2], c[3]), key)
    r = rn.rescale_ciphertext(m)
    for g, w in zip(got, (m.c0.channels(), m.c1.channels(), r.c0.channels(), r.c1.channels())):
        assert np.array_equal(g, w)
    # ... and the oracle on one ciphertext
    want = _oracle_reference(mods, n, [x[:1] for x in cts], key_a, key_b)
    for g, w in zip(got, want):
        assert np.array_equal(g[:1], w)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_limb_sharded_rotation_gpu_threads_match_unsharded(gpu, world):
    """Config 5's limb-sharded rotation on simulated ranks (threads) vs the
    fused unsharded rnt_ct_rotate and the oracle."""
    import threading

    import rns_ntt as rn
    from rns_ntt.sharded import GpuBackend, LimbShardedPipeline, ThreadComm

    n, L, B, seed = 2048, 6, 2, 31
    mods = rn.generate_primes(31, L, n)
    c0, c1, key_a, key_b = _rot_inputs(mods, n, B, seed)
    comm = ThreadComm(world)
    results, errors = [None] * world, []

    def rank_main(r):
        try:
            pipe = LimbShardedPipeline(mods, n, comm.rank_view(r), GpuBackend(0))
            results[r] = _run_rank_rotate(pipe, c0, c1, key_a, key_b)
        except BaseException as e:  # surface thread failures in the test
            errors.append(e)
            comm.abort()

    threads = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=600)
    assert not errors, errors
    Bf = rn.RnsBasis(mods, n)
    x0, x1 = rn.RnsPoly.from_channels(c0, Bf), rn.RnsPoly.from_channels(c1, Bf)
    for ki, k in enumerate(ROT_K):
        got0 = np.concatenate([results[r][ki][0] for r in range(world)], axis=1)
        got1 = np.concatenate([results[r][ki][1] for r in range(world)], axis=1)
        key = rn.RnsGadgetKey.from_channels(key_a, key_b, Bf, rotation=k)
        ref = rn.rotate_ciphertext(rn.Ciphertext(x0, x1), key)
        assert np.array_equal(got0, ref.c0.channels()), k
        assert np.array_equal(got1, ref.c1.channels()), k
        want0, want1 = _rot_oracle(mods, n, c0[:1], c1[:1], key_a, key_b, k)
        assert np.array_equal(got0[:1], want0) and np.array_equal(got1[:1], want1), k


@pytest.mark.gpu
def test_keyswitch_ext_and_rescale_ext_match_fused(gpu):
    """rnt_ct_tensor + rnt_keyswitch_ext (source = the local d2) equals the
    fused rnt_ct_mul_relin; rnt_rescale_ext by the own last limb equals
    rnt_rescale; by a foreign modulus it keeps every limb."""
    import rns_ntt as rn

    n, L, B = 1024, 4, 3
    mods = rn.generate_primes(31, L + 1, n)
    base, extra = mods[:L], mods[L]
    cts, key_a, key_b = _inputs(base, n, B, 3)
    Bf = rn.RnsBasis(base, n)
    c = [rn.RnsPoly.from_channels(x, Bf) for x in cts]
    key = rn.RnsGadgetKey.from_channels(key_a, key_b, Bf)
    d0, d1, d2 = rn.ct_tensor(*c)
    ptr, wb = d2.device_ptr()
    assert wb == 4 and ptr != 0
    o0, o1 = rn.keyswitch_ext(ptr, L, key, Bf, B, d0, d1)
    m = rn.mul_ciphertexts_gadget(rn.Ciphertext(c[0], c[1]), rn.Ciphertext(c[2], c[3]), key)
    assert np.array_equal(o0.channels(), m.c0.channels())
    assert np.array_equal(o1.channels(), m.c1.channels())
    # own last limb -> same as rescale
    last_ptr = ptr + (L - 1) * B * n * wb
    rs = rn.rescale_ext(d2, last_ptr, base[-1], Bf.drop_last(1))
    assert np.array_equal(rs.channels(), d2.rescale().channels())
    # a foreign modulus: every limb kept, matches the oracle formula
    Bx = rn.RnsBasis(base + [extra], n)
    xl = orc.uniform_poly([extra], n, np.random.default_rng(9), batch=B)[:, 0]  # [B][N] mod extra
    full = np.concatenate([d2.channels(), xl[:, None, :]], axis=1)
    want = rn.RnsPoly.from_channels(full, Bx).rescale().channels()
    xdev = rn.RnsPoly.from_channels(xl[:, None, :], rn.RnsBasis([extra], n))
    xptr, _ = xdev.device_ptr()
    got = rn.rescale_ext(d2, xptr, extra, Bf)
    assert np.array_equal(got.channels(), want)
