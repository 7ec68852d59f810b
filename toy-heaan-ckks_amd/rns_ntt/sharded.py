"""Limb-sharded ciphertext pipeline (BASELINE configs 4 and 5).

One process (rank) per GPU owns a contiguous run of the global RNS basis'
limbs and holds every ciphertext of the batch restricted to them.  Every
ring op is limb-local; the two joins of ct x ct -> relin -> rescale are:

* relinearisation (engine.rs:498-531): every target limb j needs every
  source limb i of d2 = c1 c1' to form alpha_i mod q_j, so d2
  (coefficient domain, [L_r][B][N] per rank) is ALL-GATHERED into
  [L][B][N] on every rank, then each rank runs the gadget sum for its own
  target limbs (rnt_keyswitch_ext) with its slice of the key;
* rescale (poly.rs:187-228, engine.rs:263-282): every limb needs the last
  limb of c0 and c1, so its owner BROADCASTS those two [B][N] planes and
  every rank rescales its limbs by them (rnt_rescale_ext); the owner also
  drops the limb.
* rotation (engine.rs:412-463): the slot rotation X -> X^g permutes the
  coefficients of each limb, so it is limb-local; the gadget sum over
  sigma(c1) needs every source limb, so sigma(c1) is ALL-GATHERED (the
  rotation join) and each rank forms its own target limbs of
  c0' = sigma(c0) + acc0, c1' = acc1 with its slice of the rotation key.

The collectives run on torch tensors: over RCCL (backend "nccl") between
GPUs on xGMI, over gloo between CPU processes (tests), or between threads
of one process (ThreadComm: simulated ranks sharing one GPU).  The compute
goes through a backend: GpuBackend (this library) in production; the tests
pass a CPU oracle backend to check the data flow itself.
"""
from __future__ import annotations

import threading
from typing import Any, Optional, Sequence

import numpy as np

from .dist import shard


# ---------------------------------------------------------------------------
# communicators
# ---------------------------------------------------------------------------


class _Done:
    """A join that has already completed (synchronous communicators)."""

    def __init__(self, value):
        self._v = value

    def wait(self):
        return self._v


class _Pending:
    """An in-flight torch.distributed collective; wait() returns its result.
    On RCCL, wait() makes the CURRENT stream wait for the collective's stream
    (no host wait), so the library work queued after it on that stream is
    ordered behind the join while the host moves on."""

    def __init__(self, work, finish):
        self._work, self._finish = work, finish

    def wait(self):
        self._work.wait()
        return self._finish()


class TorchDistComm:
    """torch.distributed process group (nccl = RCCL on ROCm, or gloo)."""

    def __init__(self, group=None):
        import torch.distributed as dist

        self._dist = dist
        self._group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self._gloo = dist.get_backend(group) == "gloo"

    def all_gather_limbs(self, local, counts: Sequence[int]):
        return self.all_gather_limbs_async(local, counts).wait()

    def all_gather_limbs_async(self, local, counts: Sequence[int]):
        """Start the limb all-gather of a [L_r][B][N] tensor into [L][B][N];
        returns a handle whose wait() gives the gathered tensor."""
        import torch

        B, N = local.shape[1], local.shape[2]
        if not self._gloo and len(set(counts)) == 1:
            out = torch.empty((sum(counts), B, N), dtype=local.dtype, device=local.device)
            w = self._dist.all_gather_into_tensor(out, local.contiguous(), group=self._group, async_op=True)
            return _Pending(w, lambda: out)
        # uneven limb counts (or gloo): pad every shard to the largest, gather, trim
        m = max(counts)
        pad = torch.zeros((m, B, N), dtype=local.dtype, device=local.device)
        pad[: local.shape[0]].copy_(local)
        parts = [torch.empty((m, B, N), dtype=local.dtype, device=local.device) for _ in counts]
        w = self._dist.all_gather(parts, pad, group=self._group, async_op=True)
        return _Pending(w, lambda: torch.cat([p[:c] for p, c in zip(parts, counts)], 0))

    def broadcast(self, t, src: int):
        return self.broadcast_async(t, src).wait()

    def broadcast_async(self, t, src: int):
        w = self._dist.broadcast(t, src, group=self._group, async_op=True)
        return _Pending(w, lambda: t)


class SingleComm:
    """World of one: the joins are local."""

    rank = 0
    world = 1

    def all_gather_limbs(self, local, counts: Sequence[int]):
        return local

    def all_gather_limbs_async(self, local, counts: Sequence[int]):
        return _Done(local)

    def broadcast(self, t, src: int):
        return t

    def broadcast_async(self, t, src: int):
        return _Done(t)


class ThreadComm:
    """`world` simulated ranks as threads of one process (one GPU).

    The async joins are real: each starts a helper thread that waits for the
    producing rank's stream, meets the other ranks' helpers of the same join
    (the k-th join of every rank: the ranks issue their joins in the same
    order) at that join's own barrier, and builds the result; wait() blocks
    until the helper is done.  So the pipeline's overlap and ordering -- the
    joins of chunk k in flight while chunk k+1's tensor product runs, each
    consumer waiting only for its own join -- are exercised as on RCCL."""

    def __init__(self, world: int):
        self.world = world
        self._bar = threading.Barrier(world)
        self._lock = threading.Lock()
        self._joins: dict[int, "_ThreadJoin"] = {}
        self._aborted = False

    def rank_view(self, rank: int) -> "_ThreadRank":
        return _ThreadRank(self, rank)

    def _join(self, seq: int) -> "_ThreadJoin":
        with self._lock:
            j = self._joins.get(seq)
            if j is None:
                j = self._joins[seq] = _ThreadJoin(self.world)
                if self._aborted:
                    j.bar.abort()
            return j

    def _done(self, seq: int, j: "_ThreadJoin"):
        with self._lock:
            j.finished += 1
            if j.finished == self.world:
                self._joins.pop(seq, None)

    def abort(self):
        """Break every barrier (a failing rank must not leave the others
        waiting in a join)."""
        self._bar.abort()
        with self._lock:
            for j in self._joins.values():
                j.bar.abort()
            self._aborted = True


class _ThreadJoin:
    def __init__(self, world: int):
        self.bar = threading.Barrier(world)
        self.slots: list[Any] = [None] * world
        self.finished = 0


class _ThreadPending:
    """A join running on a helper thread; wait() blocks until it is done and
    returns its result (re-raising the helper's exception).  On a GPU the
    result is also marked as used by the waiter's current stream, so the
    caching allocator keeps it until that stream's queued work is done."""

    def __init__(self, fn):
        self._res: list[Any] = []
        self._err: list[BaseException] = []

        def run():
            try:
                self._res.append(fn())
            except BaseException as e:  # surfaced by wait()
                self._err.append(e)

        self._t = threading.Thread(target=run, daemon=True)
        self._t.start()

    def wait(self):
        self._t.join()
        if self._err:
            raise self._err[0]
        out = self._res[0]
        if getattr(out, "is_cuda", False):
            import torch

            out.record_stream(torch.cuda.current_stream(out.device))
        return out


class _ThreadRank:
    def __init__(self, comm: ThreadComm, rank: int):
        self._c = comm
        self.rank = rank
        self.world = comm.world
        self._seq = 0

    def _next(self) -> tuple[int, "_ThreadJoin"]:
        seq = self._seq
        self._seq += 1
        return seq, self._c._join(seq)

    def all_gather_limbs(self, local, counts: Sequence[int]):
        return self.all_gather_limbs_async(local, counts).wait()

    def all_gather_limbs_async(self, local, counts: Sequence[int]):
        seq, j = self._next()
        producer = _current_stream(local)  # the rank's stream that wrote `local`

        def run():
            import torch

            _device_of(local)
            _stream_sync(producer)
            j.slots[self.rank] = local
            j.bar.wait()
            out = torch.cat(list(j.slots), 0)
            _stream_sync(_current_stream(out))
            j.bar.wait()  # every rank has its copy before the slots go
            self._c._done(seq, j)
            return out

        return _ThreadPending(run)

    def broadcast(self, t, src: int):
        return self.broadcast_async(t, src).wait()

    def broadcast_async(self, t, src: int):
        seq, j = self._next()
        producer = _current_stream(t)

        def run():
            _device_of(t)
            _stream_sync(producer)
            if self.rank == src:
                j.slots[src] = t
            j.bar.wait()
            if self.rank != src:
                t.copy_(j.slots[src])
                _stream_sync(_current_stream(t))
            j.bar.wait()
            self._c._done(seq, j)
            return t

        return _ThreadPending(run)


def _current_stream(t):
    """The calling thread's current stream on `t`'s device (None on the CPU)."""
    if getattr(t, "is_cuda", False):
        import torch

        return torch.cuda.current_stream(t.device)
    return None


def _stream_sync(stream):
    if stream is not None:
        stream.synchronize()


def _device_of(t):
    """Make `t`'s device current in a helper thread."""
    if getattr(t, "is_cuda", False):
        import torch

        torch.cuda.set_device(t.device)


# ---------------------------------------------------------------------------
# GPU backend (this library)
# ---------------------------------------------------------------------------


class GpuBackend:
    """Compute on this rank's GPU through librnsntt; exchange buffers are
    torch tensors wrapped as non-owning RnsPoly views (rnt_buf_wrap), so the
    collectives read and write library data in place."""

    def __init__(self, device: int = 0):
        import torch

        self.torch = torch
        self.device = device
        self.tdev = torch.device("cuda", device)

    def make_basis(self, moduli: Sequence[int], degree: int):
        from . import RnsBasis

        return RnsBasis(list(moduli), degree, device=self.device)

    def drop_last(self, basis):
        return basis.drop_last(1)

    def _dtype(self, basis):
        return self.torch.int32 if max(basis.moduli()) < (1 << 31) else self.torch.int64

    def shared_stream(self, basis):
        """One stream for torch and the library context.  Run the pipeline
        under ``with torch.cuda.stream(backend.shared_stream(basis))`` and
        torch's allocations, copies and collective joins are ordered with the
        library's kernels on one stream, so the host syncs below drop out.

        The stream is torch's (from its stream pool, alive until the process
        ends) and the context is moved onto it (rnt_ctx_set_stream), not the
        other way round: torch keeps stream handles beyond any tensor it
        hands out -- a block allocated under the stream, or marked with
        record_stream, has an event recorded on that stream when it is
        freed, whenever that is.  Wrapping the context's own stream
        (ExternalStream, r04) let those events land on a stream the
        context's teardown had destroyed; with 8 thread ranks dropping their
        contexts while gathered tensors were still alive, that took the
        process down inside torch's allocator (the r04 segfault in
        torch.empty)."""
        s = getattr(basis, "_torch_stream", None)
        if s is None or basis.stream() != s.cuda_stream:
            s = self.torch.cuda.Stream(device=self.tdev)
            basis.set_stream(s.cuda_stream)
            basis._torch_stream = s
        return s

    def _same_stream(self, basis) -> bool:
        return self.torch.cuda.current_stream(self.tdev).cuda_stream == basis.stream()

    def _sync_torch(self, basis=None):
        """Before a library op on torch memory: torch's stream must be done
        with it, unless torch is running on the library's own stream."""
        if basis is not None and self._same_stream(basis):
            return
        self.torch.cuda.synchronize(self.tdev)

    def _lib_done(self, basis):
        """After a library op whose output torch reads next."""
        if not self._same_stream(basis):
            basis.sync()

    def _empty(self, basis, shape):
        try:
            return self.torch.empty(shape, dtype=self._dtype(basis), device=self.tdev)
        except self.torch.cuda.OutOfMemoryError:
            # the library's device block cache may hold the memory torch needs
            from . import pool_trim

            if pool_trim(self.device) == 0:
                raise
            return self.torch.empty(shape, dtype=self._dtype(basis), device=self.tdev)

    def _wrap(self, basis, t, B, ntt=False):
        from . import RnsPoly

        return RnsPoly.wrap(basis, t.data_ptr(), B, ntt, owner=t)

    def batch(self, poly) -> int:
        return poly.n_polys

    def upload(self, basis, channels: np.ndarray):
        from . import RnsPoly

        return RnsPoly.from_channels(channels, basis)

    def download(self, poly) -> np.ndarray:
        return poly.channels_batch()

    def key(self, basis, a_channels: np.ndarray, b_channels: np.ndarray):
        from . import RnsGadgetKey

        return RnsGadgetKey.from_channels(a_channels, b_channels, basis)

    def tensor(self, basis, c0, c1, c0p, c1p):
        from . import ct_tensor

        B, N = c0.n_polys, basis.degree
        self._sync_torch(basis)  # torch may hand back memory its stream last used
        d2_t = self._empty(basis, (basis.channel_count(), B, N))
        d0, d1, _ = ct_tensor(c0, c1, c0p, c1p, d2_out=self._wrap(basis, d2_t, B))
        self._lib_done(basis)
        return d0, d1, d2_t

    def keyswitch(self, basis, src_full, key, d0, d1):
        """Gadget sum for this rank's limbs over the gathered source limbs
        ([L][B][N] torch tensor); d0/d1 are NTT-domain seeds or None."""
        from . import keyswitch_ext

        B, N, L = int(src_full.shape[1]), basis.degree, basis.channel_count()
        self._sync_torch(basis)
        out_t = self._empty(basis, (2, L, B, N))
        o0, o1 = self._wrap(basis, out_t[0], B), self._wrap(basis, out_t[1], B)
        keyswitch_ext(src_full.data_ptr(), src_full.shape[0], key, basis, B, d0, d1, o0, o1)
        self._lib_done(basis)
        return o0, o1

    def rotate(self, basis, poly, k: int):
        """rotate_slots (poly.rs:546-569) on this rank's limbs."""
        return poly.rotate_slots(k)

    def rotate_planes(self, basis, poly, k: int):
        """rotate_slots into a torch-owned [L_r][B][N] tensor (the source of
        the rotation join's all-gather)."""
        from . import check, load

        B = poly.n_polys
        self._sync_torch(basis)
        t = self._empty(basis, (basis.channel_count(), B, basis.degree))
        out = self._wrap(basis, t, B)
        check(load().rnt_rotate_slots(out.handle, poly.handle, int(k)))
        self._lib_done(basis)
        return t

    def add(self, basis, a, b):
        return a + b

    def last_limb(self, poly):
        """[B][N] torch view of the last local limb (poly must be torch-backed)."""
        return poly._owner[-1]

    def new_planes(self, basis, count: int, B: int):
        return self._empty(basis, (count, B, basis.degree))

    def mul_relin_rescale(self, basis, out_basis, x0, x1, y0, y1, key):
        """One rank holding every limb: ct-mul + relin + rescale of a chunk
        as the library's fused op (rnt_ct_mul_relin_rescale)."""
        from . import Ciphertext, mul_ciphertexts_gadget_rescale

        self._sync_torch(basis)
        r = mul_ciphertexts_gadget_rescale(Ciphertext(x0, x1), Ciphertext(y0, y1), key)
        self._lib_done(basis)
        return r.c0, r.c1

    def rescale(self, basis, out_basis, poly, last_plane, q_last: int):
        from . import rescale_ext

        B = poly.n_polys
        self._sync_torch(basis)
        out_t = self._empty(basis, (out_basis.channel_count(), B, basis.degree))
        out = rescale_ext(poly, last_plane.data_ptr(), q_last, out_basis, out=self._wrap(out_basis, out_t, B))
        self._lib_done(basis)
        return out


# ---------------------------------------------------------------------------
# the pipeline (per rank)
# ---------------------------------------------------------------------------


class Chunked:
    """A limb-sharded batch held as consecutive chunks of ciphertexts (each a
    backend poly over this rank's limbs), so every join can run per chunk
    and overlap the compute of the chunks around it."""

    def __init__(self, chunks: list):
        self.chunks = list(chunks)

    def __len__(self):
        return len(self.chunks)

    def __iter__(self):
        return iter(self.chunks)

    def __getitem__(self, i):
        return self.chunks[i]


class LimbShardedPipeline:
    """One rank's view of a limb-sharded batch of ciphertexts.

    ``moduli`` is the GLOBAL basis; this rank owns the contiguous limbs
    ``self.limbs``.  Inputs are given as full host channel arrays and sliced
    here (a real deployment would load only its slice).  A batch is held as
    chunks of ``chunk`` ciphertexts (:class:`Chunked`); every join is
    started per chunk as soon as that chunk's input exists and waited for
    only by the compute that consumes it, so on RCCL (with the library's
    stream as torch's current stream, GpuBackend.shared_stream) the
    all-gather of chunk k runs beside the tensor product of chunk k+1 and the
    key-switch of chunk k-1 (overlap the join with compute)."""

    def __init__(self, moduli: Sequence[int], degree: int, comm, backend, chunk: Optional[int] = None):
        self.comm = comm
        self.backend = backend
        self.degree = degree
        self.moduli = list(moduli)
        # default: 64 ciphertexts with limb-sharded joins (each chunk's join
        # overlaps its neighbours' compute); a rank holding every limb has no
        # join to overlap, so its batch is one chunk and the library chunks
        # it by its own key-switch cap (256 cts at N = 2^16, 16 limbs): config
        # 3 at 1024 cts 141.8k -> 148.1k ct-muls/s against 256-ct pipeline
        # chunks, config 4 flat (profiles/r06/ab_ks_chunk.txt)
        self.chunk = int(chunk) if chunk else (1 << 30 if comm.world == 1 else 64)
        if comm.world > len(self.moduli):
            raise ValueError(f"{comm.world} ranks for {len(self.moduli)} limbs")
        self._layout()
        self.basis = backend.make_basis(self.moduli[self.limbs.start:self.limbs.stop], degree)

    def _layout(self):
        L, W = len(self.moduli), self.comm.world
        self.counts = [shard(L, W, r)[1] for r in range(W)]
        start, count = shard(L, W, self.comm.rank)
        self.limbs = range(start, start + count)
        # owner of the last global limb: the last rank with any limbs
        self.owner_last = max(r for r in range(W) if self.counts[r] > 0)

    # -- data in / out ------------------------------------------------------
    def upload(self, channels_full: np.ndarray) -> Chunked:
        """[B][L][N] (global limbs) -> this rank's slice on its device, in
        chunks of ``self.chunk`` ciphertexts."""
        ch = np.asarray(channels_full)
        loc = ch[:, self.limbs.start:self.limbs.stop]
        return Chunked([self.backend.upload(self.basis, np.ascontiguousarray(loc[s:s + self.chunk]))
                        for s in range(0, ch.shape[0], self.chunk)])

    def upload_key(self, a_full: np.ndarray, b_full: np.ndarray):
        """Gadget key [L][L][N] (source poly i, global limb j) -> the
        [L][L_r][N] slice of this rank's target limbs."""
        s = slice(self.limbs.start, self.limbs.stop)
        return self.backend.key(self.basis, np.ascontiguousarray(a_full[:, s]),
                                np.ascontiguousarray(b_full[:, s]))

    def download(self, x: Chunked, first: int = 0, count: Optional[int] = None) -> np.ndarray:
        """This rank's limbs of ciphertexts [first, first + count) as
        [count][L_r][N] (all of them by default)."""
        out, pos = [], 0
        stop = None if count is None else first + count
        for c in x:
            b = self.backend.batch(c)
            if (stop is None or pos < stop) and pos + b > first:
                arr = self.backend.download(c)
                lo, hi = max(first - pos, 0), b if stop is None else min(stop - pos, b)
                out.append(arr[lo:hi])
            pos += b
        return np.concatenate(out, axis=0)

    # -- ct x ct + relin (engine.rs:473-539) ---------------------------------
    def mul_relin(self, c0: Chunked, c1: Chunked, c0p: Chunked, c1p: Chunked, key):
        """Tensor product per chunk, the relin join (all-gather of d2) started
        per chunk right behind it, then per chunk: wait for its join, gadget
        sum for the local target limbs seeded by d0/d1."""
        pend = []
        for x0, x1, y0, y1 in zip(c0, c1, c0p, c1p):
            d0, d1, d2 = self.backend.tensor(self.basis, x0, x1, y0, y1)
            pend.append((d0, d1, self.comm.all_gather_limbs_async(d2, self.counts)))  # the relin join
        o0, o1 = [], []
        for d0, d1, h in pend:
            a0, a1 = self.backend.keyswitch(self.basis, h.wait(), key, d0, d1)
            o0.append(a0)
            o1.append(a1)
        return Chunked(o0), Chunked(o1)

    def mul_relin_rescale(self, c0: Chunked, c1: Chunked, c0p: Chunked, c1p: Chunked, key):
        """ct x ct -> relin -> rescale (engine.rs:473-539 then :263-282).  A
        world of one with a backend that has the fused op runs it per chunk
        (the rescale inside the key-switch inverse, no join to wait for);
        otherwise mul_relin, then rescale with its joins."""
        if self.comm.world == 1 and hasattr(self.backend, "mul_relin_rescale"):
            out_basis = self.backend.drop_last(self.basis)
            r0, r1 = [], []
            for x0, x1, y0, y1 in zip(c0, c1, c0p, c1p):
                a0, a1 = self.backend.mul_relin_rescale(self.basis, out_basis, x0, x1, y0, y1, key)
                r0.append(a0)
                r1.append(a1)
            self.moduli = self.moduli[:-1]
            self.counts[self.owner_last] -= 1
            self.limbs = range(self.limbs.start, self.limbs.stop - 1)
            self.basis = out_basis
            return Chunked(r0), Chunked(r1)
        m0, m1 = self.mul_relin(c0, c1, c0p, c1p, key)
        return self.rescale(m0, m1)

    # -- rotation (engine.rs:412-463) ---------------------------------------
    def rotate(self, c0: Chunked, c1: Chunked, k: int, key):
        """rotate_ciphertext with slot offset k and this rank's slice of the
        rotation key (upload_key): sigma is limb-local, sigma(c1) is
        all-gathered per chunk, the gadget sum runs on the local target limbs."""
        pend = []
        for x0, x1 in zip(c0, c1):
            r0 = self.backend.rotate(self.basis, x0, k)
            r1 = self.backend.rotate_planes(self.basis, x1, k)
            pend.append((r0, self.comm.all_gather_limbs_async(r1, self.counts)))  # the rotation join
        o0, o1 = [], []
        for r0, h in pend:
            a0, a1 = self.backend.keyswitch(self.basis, h.wait(), key, None, None)
            o0.append(self.backend.add(self.basis, a0, r0))
            o1.append(a1)
        return Chunked(o0), Chunked(o1)

    # -- rescale (engine.rs:263-282) -----------------------------------------
    def rescale(self, c0: Chunked, c1: Chunked):
        q_last = self.moduli[-1]
        owner = self.rank == self.owner_last
        # every rank knows the owner's count: all raise together, before the
        # collective, instead of the others waiting in it
        if self.counts[self.owner_last] < 2:
            raise ValueError("rescale would leave the owner of the last limb with no limbs")
        pend = []
        for x0, x1 in zip(c0, c1):
            planes = self.backend.new_planes(self.basis, 2, self.backend.batch(x0))
            if owner:
                planes[0].copy_(self.backend.last_limb(x0))
                planes[1].copy_(self.backend.last_limb(x1))
            pend.append(self.comm.broadcast_async(planes, self.owner_last))  # the rescale join
        out_basis = self.backend.drop_last(self.basis) if owner else self.basis
        r0, r1 = [], []
        for x0, x1, h in zip(c0, c1, pend):
            planes = h.wait()
            r0.append(self.backend.rescale(self.basis, out_basis, x0, planes[0], q_last))
            r1.append(self.backend.rescale(self.basis, out_basis, x1, planes[1], q_last))
        # the global basis lost its last limb, which only its owner held
        self.moduli = self.moduli[:-1]
        self.counts[self.owner_last] -= 1
        if owner:
            self.limbs = range(self.limbs.start, self.limbs.stop - 1)
        self.owner_last = max(r for r in range(self.comm.world) if self.counts[r] > 0)
        self.basis = out_basis
        return Chunked(r0), Chunked(r1)

    @property
    def rank(self) -> int:
        return self.comm.rank
