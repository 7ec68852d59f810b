"""Multi-rank plumbing: one process per GPU, launched by torchrun.

The poly-mul path has no cross-limb or cross-poly dependency,
so ranks never exchange residues: each owns its own batch (weak scaling) or
its own slice of a fixed batch / of the RNS limbs (strong scaling).  Only the
control plane crosses ranks -- the timing barrier and the max-over-ranks
reduction -- over gloo, so it works identically on CPU-only hosts (tests)
and GPU nodes.
"""
from __future__ import annotations

import os
from dataclasses import dataclass


def shard(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [start, start + count) slice of `total` items owned by
    `rank`; the first `total % world` ranks take one extra item."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def limb_shard(L: int, world: int, rank: int) -> range:
    """RNS limbs owned by `rank` under limb sharding (§8e: GPU g owns limbs
    {g*L/G, ...}): a contiguous run, so its device slab is contiguous in the
    [L][B][N] layout."""
    start, count = shard(L, world, rank)
    return range(start, start + count)


def weak_throughput(units_per_rank: int, world: int, elapsed_max_s: float, steps: int) -> float:
    """Whole-job units/s when every rank processes `units_per_rank` per step
    and the slowest rank took `elapsed_max_s` for `steps` steps."""
    if elapsed_max_s <= 0 or steps <= 0:
        raise ValueError("elapsed and steps must be positive")
    return world * units_per_rank * steps / elapsed_max_s


@dataclass
class Comm:
    rank: int = 0
    world: int = 1
    _torch: object = None
    _dist: object = None

    @classmethod
    def from_env(cls) -> "Comm":
        """torchrun environment -> gloo process group (control plane only);
        a single process gets a no-op communicator."""
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        if world == 1:
            return cls(rank, world)
        import torch
        import torch.distributed as dist

        if not dist.is_initialized():
            dist.init_process_group("gloo", rank=rank, world_size=world)
        return cls(rank, world, torch, dist)

    def barrier(self) -> None:
        if self._dist is not None:
            self._dist.barrier()

    def max(self, x: float) -> float:
        return self._reduce(x, "MAX")

    def sum(self, x: float) -> float:
        return self._reduce(x, "SUM")

    def _reduce(self, x: float, op: str) -> float:
        if self._dist is None:
            return float(x)
        t = self._torch.tensor([float(x)], dtype=self._torch.float64)
        self._dist.all_reduce(t, op=getattr(self._dist.ReduceOp, op))
        return float(t.item())

    def gather(self, obj, dst: int = 0):
        """Every rank's picklable `obj` as a list on rank `dst` (None
        elsewhere); a single process gets [obj].  Control plane only (gloo):
        used for the sampled parity checks of sharded outputs."""
        if self._dist is None:
            return [obj]
        out = [None] * self.world if self.rank == dst else None
        self._dist.gather_object(obj, out, dst=dst)
        return out

    def close(self) -> None:
        if self._dist is not None and self._dist.is_initialized():
            self._dist.destroy_process_group()
