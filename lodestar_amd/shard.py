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


# ---------------------------------------------------------------------------
# One call split across GPUs (the north_star's "each GPU reduces its shard to an
# Fp12 partial, the partials are combined over RCCL/xGMI, and one final
# exponentiation follows").  The exchange is a 580-byte all-gather per rank.
# ---------------------------------------------------------------------------
PARTIAL_BYTES = 576


def shard_bounds(n_sets: int, world: int) -> list[tuple[int, int]]:
    """Contiguous [beg, end) slices of a call's sets, sizes differing by at most 1, so
    set i of the call keeps its index (and its random scalar) whichever rank holds it."""
    q, r = divmod(n_sets, world)
    out, beg = [], 0
    for k in range(world):
        end = beg + q + (1 if k < r else 0)
        out.append((beg, end))
        beg = end
    return out


class GpuPartialBackend:
    """Adapter from a GpuContext (C-ABI bls_gpu_partial / bls_gpu_final_check)."""

    def __init__(self, gpu):
        self.gpu = gpu

    def partial(self, sets, set_index_base: int, seed: bytes):
        from .native import pack_requests

        part, status, _ = self.gpu.partial(pack_requests([(True, sets)], seed=seed), set_index_base)
        return part, status

    def final_check(self, partials: list[bytes]) -> bool:
        return self.gpu.final_check(partials)


def verify_call_sharded(sets, seed: bytes, backend, dist=None, device=None, localize: bool = True):
    """verifySignatureSets on ONE call whose sets are spread over the ranks.

    Semantics: an undecodable set rejects the call with its code (the
    first failing set in call order wins); otherwise the verdict is the random-scalar
    batch check of all sets (maybeBatch.ts:18-25), done as one final exponentiation
    over the product of the ranks' Miller-loop partials.  Every rank passes the whole
    call's `sets` (each uses only its contiguous shard) and the same 32-byte `seed`.

    Returns (verdict, info): verdict True / False, or a negative error code;
    info["bad_shards"] lists the ranks whose own partial fails its final
    exponentiation (only computed when the call fails and `localize`)."""
    import numpy as np

    world = dist.get_world_size() if dist is not None and dist.is_initialized() else 1
    rank = dist.get_rank() if world > 1 else 0
    n = len(sets)
    if n < 2:
        raise ValueError("a sharded call needs >= 2 sets (1-set calls take the non-batched path)")
    beg, end = shard_bounds(n, world)[rank]
    rec = np.zeros(4 + PARTIAL_BYTES, dtype=np.uint8)
    rec[:4] = np.frombuffer(np.int32(1).tobytes(), dtype=np.uint8)  # 1 = empty shard
    if end > beg:
        part, status = backend.partial(sets[beg:end], beg, seed)
        rec[:4] = np.frombuffer(np.int32(status).tobytes(), dtype=np.uint8)
        if part is not None:
            rec[4:] = np.frombuffer(part, dtype=np.uint8)
    recs = _all_gather_bytes(rec, dist, device) if world > 1 else [rec]
    statuses = [int(np.frombuffer(r[:4].tobytes(), dtype=np.int32)[0]) for r in recs]
    for st in statuses:                       # ranks hold the call in order
        if st < 0:
            return st, {"bad_shards": []}
    partials = [r[4:].tobytes() for r, st in zip(recs, statuses) if st == 0]
    # one final exponentiation for the whole call (rank 0), verdict broadcast
    ok = backend.final_check(partials) if rank == 0 else False
    if world > 1:
        ok = bool(_broadcast_int(int(ok), dist, device))
    info = {"bad_shards": []}
    if not ok and localize:
        mine = 1
        if statuses[rank] == 0:
            mine = int(backend.final_check([recs[rank][4:].tobytes()]))
        flags = _all_gather_bytes(np.array([mine], dtype=np.uint8), dist, device) if world > 1 else [[mine]]
        info["bad_shards"] = [k for k, f in enumerate(flags) if int(f[0]) == 0]
    return ok, info


def _all_gather_bytes(arr, dist, device):
    import numpy as np
    import torch

    t = torch.from_numpy(arr.copy()).to(device) if device else torch.from_numpy(arr.copy())
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [np.asarray(o.cpu().numpy(), dtype=np.uint8) for o in out]


def _broadcast_int(v: int, dist, device) -> int:
    import torch

    t = torch.tensor([v], dtype=torch.int32, device=device) if device else torch.tensor([v], dtype=torch.int32)
    dist.broadcast(t, src=0)
    return int(t.item())
