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
        import torch

        B, N = local.shape[1], local.shape[2]
        if not self._gloo and len(set(counts)) == 1:
            out = torch.empty((sum(counts), B, N), dtype=local.dtype, device=local.device)
            self._dist.all_gather_into_tensor(out, local.contiguous(), group=self._group)
            return out
        # uneven limb counts: pad every shard to the largest, gather, trim
        m = max(counts)
        pad = torch.zeros((m, B, N), dtype=local.dtype, device=local.device)
        pad[: local.shape[0]].copy_(local)
        parts = [torch.empty((m, B, N), dtype=local.dtype, device=local.device) for _ in counts]
        self._dist.all_gather(parts, pad, group=self._group)
        return torch.cat([p[:c] for p, c in zip(parts, counts)], 0)

    def broadcast(self, t, src: int):
        self._dist.broadcast(t, src, group=self._group)
        return t


class SingleComm:
    """World of one: the joins are local."""

    rank = 0
    world = 1

    def all_gather_limbs(self, local, counts: Sequence[int]):
        return local

    def broadcast(self, t, src: int):
        return t


class ThreadComm:
    """`world` simulated ranks as threads of one process (one GPU)."""

    def __init__(self, world: int):
        self.world = world
        self._bar = threading.Barrier(world)
        self._slots: list[Any] = [None] * world

    def rank_view(self, rank: int) -> "_ThreadRank":
        return _ThreadRank(self, rank)


class _ThreadRank:
    def __init__(self, comm: ThreadComm, rank: int):
        self._c = comm
        self.rank = rank
        self.world = comm.world

    def all_gather_limbs(self, local, counts: Sequence[int]):
        import torch

        c = self._c
        c._slots[self.rank] = local
        _stream_done(local)  # ranks read each other's tensors from their own streams
        c._bar.wait()
        out = torch.cat([s for s in c._slots], 0)
        _stream_done(out)
        c._bar.wait()
        return out

    def broadcast(self, t, src: int):
        c = self._c
        if self.rank == src:
            c._slots[src] = t
            _stream_done(t)
        c._bar.wait()
        if self.rank != src:
            t.copy_(c._slots[src])
            _stream_done(t)
        c._bar.wait()
        return t


def _stream_done(t):
    """Wait for this thread's current stream when `t` lives on a GPU."""
    if getattr(t, "is_cuda", False):
        import torch

        torch.cuda.current_stream(t.device).synchronize()


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
        """The library context's HIP stream as a torch stream.  Run the
        pipeline under ``with torch.cuda.stream(backend.shared_stream(basis))``
        and torch's allocations, copies and collective joins are ordered with
        the library's kernels on one stream, so the host syncs below drop out."""
        return self.torch.cuda.ExternalStream(basis.stream(), device=self.tdev)

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


class LimbShardedPipeline:
    """One rank's view of a limb-sharded batch of ciphertexts.

    ``moduli`` is the GLOBAL basis; this rank owns the contiguous limbs
    ``self.limbs``.  Inputs are given as full host channel arrays and sliced
    here (a real deployment would load only its slice)."""

    def __init__(self, moduli: Sequence[int], degree: int, comm, backend):
        self.comm = comm
        self.backend = backend
        self.degree = degree
        self.moduli = list(moduli)
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
    def upload(self, channels_full: np.ndarray):
        """[B][L][N] (global limbs) -> this rank's slice on its device."""
        ch = np.asarray(channels_full)
        return self.backend.upload(self.basis, np.ascontiguousarray(ch[:, self.limbs.start:self.limbs.stop]))

    def upload_key(self, a_full: np.ndarray, b_full: np.ndarray):
        """Gadget key [L][L][N] (source poly i, global limb j) -> the
        [L][L_r][N] slice of this rank's target limbs."""
        s = slice(self.limbs.start, self.limbs.stop)
        return self.backend.key(self.basis, np.ascontiguousarray(a_full[:, s]),
                                np.ascontiguousarray(b_full[:, s]))

    def download(self, poly) -> np.ndarray:
        return self.backend.download(poly)

    # -- ct x ct + relin (engine.rs:473-539) ---------------------------------
    def mul_relin(self, c0, c1, c0p, c1p, key):
        d0, d1, d2 = self.backend.tensor(self.basis, c0, c1, c0p, c1p)
        d2_full = self.comm.all_gather_limbs(d2, self.counts)  # the relin join
        return self.backend.keyswitch(self.basis, d2_full, key, d0, d1)

    # -- rotation (engine.rs:412-463) ---------------------------------------
    def rotate(self, c0, c1, k: int, key):
        """rotate_ciphertext with slot offset k and this rank's slice of the
        rotation key (upload_key): sigma is limb-local, sigma(c1) is
        all-gathered, the gadget sum runs on the local target limbs."""
        r0 = self.backend.rotate(self.basis, c0, k)
        r1 = self.backend.rotate_planes(self.basis, c1, k)
        full = self.comm.all_gather_limbs(r1, self.counts)  # the rotation join
        a0, a1 = self.backend.keyswitch(self.basis, full, key, None, None)
        return self.backend.add(self.basis, a0, r0), a1

    # -- rescale (engine.rs:263-282) -----------------------------------------
    def rescale(self, c0, c1):
        q_last = self.moduli[-1]
        B = self.backend.batch(c0)
        owner = self.rank == self.owner_last
        # every rank knows the owner's count: all raise together, before the
        # collective, instead of the others waiting in it
        if self.counts[self.owner_last] < 2:
            raise ValueError("rescale would leave the owner of the last limb with no limbs")
        planes = self.backend.new_planes(self.basis, 2, B)
        if owner:
            planes[0].copy_(self.backend.last_limb(c0))
            planes[1].copy_(self.backend.last_limb(c1))
        self.comm.broadcast(planes, self.owner_last)  # the rescale join
        out_basis = self.backend.drop_last(self.basis) if owner else self.basis
        r0 = self.backend.rescale(self.basis, out_basis, c0, planes[0], q_last)
        r1 = self.backend.rescale(self.basis, out_basis, c1, planes[1], q_last)
        # the global basis lost its last limb, which only its owner held
        self.moduli = self.moduli[:-1]
        self.counts[self.owner_last] -= 1
        if owner:
            self.limbs = range(self.limbs.start, self.limbs.stop - 1)
        self.owner_last = max(r for r in range(self.comm.world) if self.counts[r] > 0)
        self.basis = out_basis
        return r0, r1

    @property
    def rank(self) -> int:
        return self.comm.rank
