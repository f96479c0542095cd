"""Multi-rank path on CPU (gloo, world_size 2): request sharding and the global
throughput reduction bench.py uses under torchrun."""
from __future__ import annotations

import os
import socket

import pytest

from lodestar_amd.shard import shard_by_request


def test_shard_partition_and_balance():
    weights = [1] * 1000 + [128] * 20 + [512] * 3
    for world in (1, 2, 4, 8):
        shards = shard_by_request(weights, world)
        flat = sorted(i for s in shards for i in s)
        assert flat == list(range(len(weights)))
        loads = [sum(weights[i] for i in s) for s in shards]
        assert max(loads) - min(loads) <= 512


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, q):
    import torch.distributed as dist

    from lodestar_amd.shard import global_throughput, shard_by_request

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    weights = [1] * 64 + [8] * 4
    mine = shard_by_request(weights, world)[rank]
    local_sets = sum(weights[i] for i in mine)
    elapsed = 0.5 + 0.25 * rank          # rank 1 is the slow one
    dist.barrier()
    rate, emax = global_throughput(local_sets, elapsed, dist)
    q.put((rank, local_sets, rate, emax))
    dist.destroy_process_group()


def test_gloo_world2_throughput():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    total = sum(r[1] for r in res)
    assert total == 64 + 32
    for _, _, rate, emax in res:
        assert emax == pytest.approx(0.75)
        assert rate == pytest.approx(total / 0.75)
