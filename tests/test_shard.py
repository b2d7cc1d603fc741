"""Sharding helpers (cobrix_amd/shard.py) on CPU: ranges, and the count all-gather over gloo with
world_size 2 and 3 (the same code runs over RCCL on the GPUs)."""
from __future__ import annotations

import os
import socket

import pytest

torch = pytest.importorskip("torch")
import torch.multiprocessing as mp  # noqa: E402

from cobrix_amd.shard import byte_shard, global_bases, shard_range  # noqa: E402


def test_shard_ranges_cover_exactly():
    for n in (0, 1, 7, 64, 1000, 50_000_001):
        for w in (1, 2, 3, 8):
            rs = [shard_range(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1
    assert byte_shard(10 * 200 + 13, 200, 3, 2) == (6 * 200, 10 * 200)
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rows = 10 * (rank + 1)
    sizes = [torch.tensor([100 + rank], dtype=torch.int64), 7 * rank]
    rb, sb, tot = global_bases(rows, sizes)
    q.put((rank, int(rb), [int(x) for x in sb], [int(x) for x in tot]))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_global_bases_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rows = [10 * (r + 1) for r in range(world)]
    s0 = [100 + r for r in range(world)]
    s1 = [7 * r for r in range(world)]
    for rank, rb, sb, tot in res:
        assert rb == sum(rows[:rank])
        assert sb == [sum(s0[:rank]), sum(s1[:rank])]
        assert tot == [sum(rows), sum(s0), sum(s1)]
