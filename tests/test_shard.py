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
        """(partial, status, (class, local index)) with multi-set rules, first error of
        the lowest class: 0 pubkey decode, 1 signature decode, 2 infinity pubkey."""
        O = self.O
        decoded = []
        for k, (pk96, _, _) in enumerate(sets):
            code, pk = O.g1_deserialize(pk96)
            if code != O.E_OK:
                return None, -code, (0, k)
            decoded.append(pk)
        sigs = []
        for k, (_, _, sig) in enumerate(sets):
            try:
                sigs.append(O.signature_from_bytes(sig, validate=True))
            except O.BlsError as e:
                return None, -e.code, (1, k)
        for k, pk in enumerate(decoded):
            if pk is None:
                return None, -O.E_PK_IS_INFINITY, (2, k)
        f = O.F12_ONE
        for k, ((_, msg, _), pk, s) in enumerate(zip(sets, decoded, sigs)):
            r = self._scalar(seed, base + k)
            f = O.f12_mul(f, O.miller_loop(O.E1.mul(pk, r), O.hash_to_g2(msg)))
            if s is not None:
                f = O.f12_mul(f, O.miller_loop(O.E1.neg(O.G1), O.E2.mul(s, r)))
        return b"".join(v.to_bytes(48, "big") for c in f for v in c), 0, None

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
    # the unsharded call decides these, not the shards' own rules
    inf_sig = bytes([0xC0]) + bytes(95)
    two_inf = [good[0], (pks[1], msgs[1], inf_sig)]               # 1-set shards: false, not ZERO_SIGNATURE
    bad_pk = bytes([0x80]) + pks[3][1:]
    order = [(pks[0], msgs[0], sigs[0][:32])] + good[1:3] + [(bad_pk, msgs[3], sigs[3])]
    inf_pk = good[:2] + [(O.g1_serialize(None), msgs[2], sigs[2]), good[3]]
    return {"good": good, "wrong_msg": wrong_msg, "bad_enc": bad_enc, "two_inf": two_inf, "order": order,
            "inf_pk": inf_pk}


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
        # a 2-set call over 2 ranks with an infinity signature: the multi-set verdict
        # (false), as unsharded (oracle verify_multiple), not the 1-set ZERO_SIGNATURE
        assert out["two_inf"][0] is False
        # a signature error in rank 0's shard and a pubkey error in rank 1's: the pubkey
        # error wins (deserializeSet runs first, worker.ts:45)
        assert out["order"][0] == -O.E_BAD_ENCODING
        assert out["inf_pk"][0] == -O.E_PK_IS_INFINITY


def test_first_error_order():
    from lodestar_amd.shard import first_error

    assert first_error([(0, 3, 0), (0, 3, 0)]) == 0
    assert first_error([(-8, 1, 0), (-2, 0, 7)]) == -2         # pubkey class before signature class
    assert first_error([(-3, 1, 9), (-8, 1, 4)]) == -8         # same class: lower call index
    assert first_error([(-6, 2, 1), (-1, 1, 5)]) == -1


# ---------------------------------------------------------------------------
# bench.py --mode sharded, dry run: the bench's own timed loop (run_sharded) and
# max-over-ranks reduction over gloo with two ranks; only the per-rank partial backend
# is the oracle's (no GPU here).
# ---------------------------------------------------------------------------
def _bench_sharded_rank(rank, world, port, q):
    import hashlib

    import torch.distributed as dist

    import bench
    from lodestar_amd.shard import global_throughput

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sets = _sharded_cases()["good"]
    seed = hashlib.sha256(b"sharded-bench").digest()
    elapsed, total = bench.run_sharded(OraclePartialBackend(), sets, seed, 1, 0, dist, None)
    value, emax = global_throughput(total * 1 / world, elapsed, dist)
    q.put((rank, total, value, emax, elapsed))
    dist.destroy_process_group()


def test_bench_sharded_mode_gloo_world2():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_sharded_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    emax = max(r[4] for r in res)
    for _, total, value, e, _ in res:
        assert total == 4
        assert e == pytest.approx(emax)
        assert value == pytest.approx(4 / emax)
