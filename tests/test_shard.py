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


# ---------------------------------------------------------------------------
# One call sharded over ranks: Fp12 partials + one final exponentiation
# (lodestar_amd.shard.verify_call_sharded).  The orchestration runs over gloo here
# with an oracle-backed partial backend (test infrastructure, never the product);
# tests/test_gpu_parity.py drives the same function with the GPU backend.
# ---------------------------------------------------------------------------
def test_shard_bounds_contiguous():
    from lodestar_amd.shard import shard_bounds

    for n in (2, 3, 7, 128, 1000):
        for world in (1, 2, 3, 8):
            b = shard_bounds(n, world)
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[k][1] == b[k + 1][0] for k in range(world - 1))
            sizes = [e - s for s, e in b]
            assert max(sizes) - min(sizes) <= 1


class OraclePartialBackend:
    """partial = prod_i ML(r_i pk_i, H(m_i)) * ML(-g1, r_i sig_i) in the oracle's Fp12,
    serialised as 12 big-endian 48-byte words; scalars from (seed, call index)."""

    def __init__(self):
        from oracle import bls_oracle as O

        self.O = O

    def _scalar(self, seed, i):
        import hashlib

        r = int.from_bytes(hashlib.sha256(seed + i.to_bytes(4, "little")).digest()[:8], "big")
        return r or 1

    def partial(self, sets, base, seed):
        O = self.O
        f = O.F12_ONE
        for k, (pk96, msg, sig) in enumerate(sets):
            try:
                s = O.signature_from_bytes(sig, validate=True)
            except O.BlsError as e:
                return None, -e.code
            _, pk = O.g1_deserialize(pk96)
            r = self._scalar(seed, base + k)
            f = O.f12_mul(f, O.miller_loop(O.E1.mul(pk, r), O.hash_to_g2(msg)))
            f = O.f12_mul(f, O.miller_loop(O.E1.neg(O.G1), O.E2.mul(s, r)))
        return b"".join(v.to_bytes(48, "big") for c in f for v in c), 0

    def final_check(self, partials):
        O = self.O
        f = O.F12_ONE
        for p in partials:
            w = [int.from_bytes(p[48 * k: 48 * k + 48], "big") for k in range(12)]
            f = O.f12_mul(f, [(w[2 * j], w[2 * j + 1]) for j in range(6)])
        return O.f12_is_one(O.final_exponentiation(f))


def _sharded_cases():
    import hashlib

    from oracle import bls_oracle as O

    sks = [O.interop_secret_key(i) for i in range(4)]
    msgs = [hashlib.sha256(b"shard%d" % i).digest() for i in range(4)]
    sigs = [O.g2_compress(O.sign(s, m)) for s, m in zip(sks, msgs)]
    pks = [O.g1_serialize(O.sk_to_pk(s)) for s in sks]
    good = list(zip(pks, msgs, sigs))
    wrong_msg = good[:3] + [(pks[3], msgs[0], sigs[3])]          # invalid set in rank 1's shard
    bad_enc = good[:1] + [(pks[1], msgs[1], b"\x00" * 96)] + good[2:]  # undecodable (no compression flag)
    return {"good": good, "wrong_msg": wrong_msg, "bad_enc": bad_enc}


def _sharded_rank(rank, world, port, q):
    import torch.distributed as dist

    from lodestar_amd.shard import verify_call_sharded

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    be = OraclePartialBackend()
    seed = bytes(range(32))
    out = {}
    for name, sets in _sharded_cases().items():
        out[name] = verify_call_sharded(sets, seed, be, dist)
    q.put((rank, out))
    dist.destroy_process_group()


def test_gloo_world2_sharded_call_partials():
    import torch.multiprocessing as mp

    from oracle import bls_oracle as O

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in (0, 1):
        out = res[rank]
        assert out["good"] == (True, {"bad_shards": []})
        assert out["wrong_msg"] == (False, {"bad_shards": [1]})
        assert out["bad_enc"][0] == -O.E_BAD_ENCODING
