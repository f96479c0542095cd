"""Multi-GPU sharding of verify work: one process per GPU, calls
(requests) sharded by cumulative set weight, no data-path collective; the only
cross-rank traffic is the benchmark's barrier and the max-of-elapsed reduction.

Works with any torch.distributed backend: "nccl" (RCCL over xGMI) on the GPU box,
"gloo" in the CPU tests."""
from __future__ import annotations


def shard_by_request(weights: list[int], world: int) -> list[list[int]]:
    """Assign request indices to ranks: greedy by weight (an aggregate set of k keys
    weighs k, a single set 1), heaviest first, to the least-loaded rank; a request
    is never split (its fallback stays on one GPU)."""
    loads = [0] * world
    out: list[list[int]] = [[] for _ in range(world)]
    for r in sorted(range(len(weights)), key=lambda i: (-weights[i], i)):
        k = min(range(world), key=lambda j: (loads[j], j))
        out[k].append(r)
        loads[k] += weights[r]
    for lst in out:
        lst.sort()
    return out


def global_throughput(local_sets: int, local_elapsed_s: float, dist=None, device=None) -> tuple[float, float]:
    """(sets/s over all ranks, max elapsed): all ranks' sets / the slowest rank's time."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return local_sets / local_elapsed_s, local_elapsed_s
    import torch

    t = torch.tensor([float(local_sets), local_elapsed_s], dtype=torch.float64, device=device)
    s = t[:1].clone()
    e = t[1:].clone()
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    dist.all_reduce(e, op=dist.ReduceOp.MAX)
    return float(s.item()) / float(e.item()), float(e.item())
