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


def _grouped(dist) -> bool:
    """A process group exists: the exchange goes through it whatever its size (a
    world-1 group on the GPU box still runs the RCCL collectives, tests/test_gpu_rccl.py)."""
    return dist is not None and dist.is_initialized()


def global_throughput(local_sets: int, local_elapsed_s: float, dist=None, device=None) -> tuple[float, float]:
    """(sets/s over all ranks, max elapsed): all ranks' sets / the slowest rank's time."""
    if not _grouped(dist):
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
# exponentiation follows").  The exchange is a 588-byte all-gather per rank.
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
        """(576-byte partial or None, status 0 / -code, (class, shard-local index) or None)"""
        from .native import pack_requests

        part, status, err, _ = self.gpu.partial(pack_requests([(True, sets)], seed=seed), set_index_base)
        return part, status, err

    def final_check(self, partials: list[bytes]) -> bool:
        return self.gpu.final_check(partials)


RECORD_BYTES = 12 + PARTIAL_BYTES   # int32 status, int32 error class, uint32 call index, Fp12 partial


def first_error(records) -> int:
    """The call's rejection code from the ranks' (status, class, call index) triples:
    the lowest error class first (0 a pubkey that does not decode / aggregate, 1 a
    signature that does not decode, 2 an infinity pubkey -- the order in which the
    reference's worker meets them, worker.ts:45 then maybeBatch.ts:19-24), then the
    lowest index in the call; 0 if no rank failed."""
    bad = [(cls, idx, st) for st, cls, idx in records if st < 0]
    return min(bad)[2] if bad else 0


def verify_call_sharded(sets, seed: bytes, backend, dist=None, device=None, localize: bool = True):
    """verifySignatureSets on ONE call whose sets are spread over the ranks.

    Semantics: an undecodable set rejects the call with its code (the
    first error in the reference's order, `first_error`); otherwise the verdict is the
    random-scalar batch check of all sets (maybeBatch.ts:18-25), done as one final
    exponentiation over the product of the ranks' Miller-loop partials.  Every shard is
    verified with the rules of a multi-set call, so a sharded call gives the verdict of
    the same call unsharded.  Every rank passes the whole call's `sets` (each uses only
    its contiguous shard) and the same 32-byte `seed`.

    Returns (verdict, info): verdict True / False, or a negative error code;
    info["bad_shards"] lists the ranks whose own partial fails its final
    exponentiation (only computed when the call fails and `localize`)."""
    import numpy as np

    grouped = _grouped(dist)
    world = dist.get_world_size() if grouped else 1
    rank = dist.get_rank() if grouped else 0
    n = len(sets)
    if n < 2:
        raise ValueError("a sharded call needs >= 2 sets (1-set calls take the non-batched path)")
    beg, end = shard_bounds(n, world)[rank]
    rec = np.zeros(RECORD_BYTES, dtype=np.uint8)
    head = np.array([1, 3, 0], dtype=np.int32)  # status 1 = empty shard
    if end > beg:
        part, status, err = backend.partial(sets[beg:end], beg, seed)
        head[0] = status
        if err is not None:
            head[1], head[2] = err[0], beg + err[1]
        if part is not None:
            rec[12:] = np.frombuffer(part, dtype=np.uint8)
    rec[:12] = head.view(np.uint8)
    recs = _all_gather_bytes(rec, dist, device) if grouped else [rec]
    heads = [np.frombuffer(r[:12].tobytes(), dtype=np.int32) for r in recs]
    code = first_error([(int(h[0]), int(h[1]), int(h[2])) for h in heads])
    if code < 0:
        return code, {"bad_shards": []}
    partials = [r[12:].tobytes() for r, h in zip(recs, heads) if int(h[0]) == 0]
    # one final exponentiation for the whole call (rank 0), verdict broadcast
    ok = backend.final_check(partials) if rank == 0 else False
    if grouped:
        ok = bool(_broadcast_int(int(ok), dist, device))
    info = {"bad_shards": []}
    if not ok and localize:
        mine = 1
        if int(heads[rank][0]) == 0:
            mine = int(backend.final_check([recs[rank][12:].tobytes()]))
        flags = _all_gather_bytes(np.array([mine], dtype=np.uint8), dist, device) if grouped else [[mine]]
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
