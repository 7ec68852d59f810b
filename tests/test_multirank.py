"""Multi-rank control plane on CPU (gloo, world_size 2): the same helpers
bench.py uses for its timing barrier, max-over-ranks and whole-job value
(poly-mul shards with no data-path collective)."""
from __future__ import annotations

import os
import socket

import pytest
import torch.multiprocessing as mp

from rns_ntt.dist import Comm, limb_shard, shard, weak_throughput


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank: int, world: int, port: int, q) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    comm = Comm.from_env()
    try:
        comm.barrier()
        # bench.py: each rank times its own batch; the job time is the slowest
        elapsed = 0.1 * (rank + 1)
        emax = comm.max(elapsed)
        total = comm.sum(rank + 1)
        value = weak_throughput(256, comm.world, emax, 20)
        # each rank's slice of a fixed batch / of the RNS limbs
        start, count = shard(1000, world, rank)
        limbs = list(limb_shard(16, world, rank))
        q.put((rank, emax, total, value, start, count, limbs))
    finally:
        comm.close()


def test_two_rank_control_plane():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, emax, total, value, start, count, limbs in results:
        assert emax == pytest.approx(0.2)          # max over ranks, seen by every rank
        assert total == pytest.approx(3.0)
        assert value == pytest.approx(2 * 256 * 20 / 0.2)  # whole-job units/s
    # slices tile the range exactly, in rank order
    assert [(r[4], r[5]) for r in results] == [(0, 500), (500, 500)]
    assert results[0][6] == list(range(0, 8)) and results[1][6] == list(range(8, 16))


@pytest.mark.parametrize("total,world", [(0, 3), (7, 3), (16, 8), (5, 8), (1024, 8)])
def test_shard_covers_range(total, world):
    seen = []
    for r in range(world):
        start, count = shard(total, world, r)
        seen.extend(range(start, start + count))
    assert seen == list(range(total))
    counts = [shard(total, world, r)[1] for r in range(world)]
    assert max(counts) - min(counts) <= 1


def test_single_process_comm_is_noop():
    c = Comm()
    c.barrier()
    assert c.max(1.5) == 1.5 and c.sum(2.0) == 2.0
    with pytest.raises(ValueError):
        shard(4, 2, 2)
    with pytest.raises(ValueError):
        weak_throughput(1, 1, 0.0, 1)
