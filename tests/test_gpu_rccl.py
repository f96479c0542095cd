"""The multi-GPU bench's runtime combination, run once on one GPU.

`bench.py --gpus N` (and torchrun) ranks call torch.cuda.set_device(local_rank) and
init_process_group("nccl") before opening their verifier contexts, so in a rank the
library binds to torch's bundled HIP runtime (same soname, libamdhip64.so.7) and the
sharded call's exchange runs over RCCL.  This test starts a fresh `spawn` child (never
a re-exec) that does exactly that with a world-1 RCCL group on cuda:0, then:

* verifies one 1024-set cfg2 call (1024 batchable single-set requests) and the same
  call with invalid sets, verdicts checked against validity by construction;
* runs shard.global_throughput (two all_reduce) and shard.verify_call_sharded (the
  588-byte all_gather, the verdict broadcast, the bad-shard all_gather) with
  device="cuda:0", so every collective of the multi-GPU path goes through RCCL.

Reference split mirrored: multithread/index.ts:153-166 (one message per worker).
"""
from __future__ import annotations

import hashlib
import socket

import pytest

pytestmark = pytest.mark.gpu


def _rccl_child(port, q):
    import os

    import torch
    import torch.distributed as dist

    out = {}
    try:
        torch.cuda.set_device(0)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("nccl", rank=0, world_size=1)
        out["backend"] = dist.get_backend()
        out["world"] = dist.get_world_size()

        from lodestar_amd import workloads as W
        from lodestar_amd.native import GpuContext, mapped_hip_runtime, pack_requests
        from lodestar_amd.shard import GpuPartialBackend, global_throughput, verify_call_sharded

        with GpuContext(0) as gpu:
            out["hip_runtime"] = mapped_hip_runtime()
            n = 1024
            W.load_table([gpu], 64)
            sks = W.interop_sks(64)
            msgs = [W.message(j, b"RCCL") for j in range(n)]
            sigs = W._sign_all(gpu, [sks[j % 64] for j in range(n)], msgs)
            sets = [([j % 64], msgs[j], sigs[j]) for j in range(n)]
            v, _ = gpu.verify_packed(pack_requests([(True, [s]) for s in sets]))
            out["cfg2_valid"] = [int(x) for x in v]
            bad = list(sets)
            for j in (3, 517, 1000):
                bad[j] = (bad[j][0], msgs[(j + 1) % n], bad[j][2])
            v, _ = gpu.verify_packed(pack_requests([(True, [s]) for s in bad]))
            out["cfg2_invalid"] = [int(x) for x in v]
            rate, el = global_throughput(2048, 0.5, dist, device="cuda:0")
            out["throughput"] = (rate, el)
            raw, _ = gpu.aggregate_pubkeys([[j % 64] for j in range(256)])
            rsets = [(bytes(raw[j]), msgs[j], sigs[j]) for j in range(256)]
            be = GpuPartialBackend(gpu)
            out["sharded_good"] = verify_call_sharded(rsets, bytes(32), be, dist, device="cuda:0")
            rbad = list(rsets)
            rbad[100] = (rbad[100][0], msgs[101], rbad[100][2])
            out["sharded_bad"] = verify_call_sharded(rbad, bytes(32), be, dist, device="cuda:0")
        dist.destroy_process_group()
    except Exception as e:  # reported to the parent, which fails the test with it
        out["error"] = f"{type(e).__name__}: {e}"
    q.put(out)


def test_rccl_world1_runtime_and_collectives():
    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_child, args=(port, q))
    p.start()
    out = q.get(timeout=110)
    p.join(timeout=30)
    assert "error" not in out, out["error"]
    assert p.exitcode == 0
    assert out["backend"] == "nccl" and out["world"] == 1
    assert any("torch" in h for h in out["hip_runtime"]), out["hip_runtime"]
    assert out["cfg2_valid"] == [1] * 1024
    assert out["cfg2_invalid"] == [0 if j in (3, 517, 1000) else 1 for j in range(1024)]
    assert out["throughput"] == (4096.0, 0.5)
    assert out["sharded_good"] == (True, {"bad_shards": []})
    assert out["sharded_bad"] == (False, {"bad_shards": [0]})


_GLOO_RANK = r"""
import json, os, sys
sys.path.insert(0, os.environ["REPO"])
from lodestar_amd._abi import load_library
load_library()                       # before torch: the runtime of the N = 1 line
import torch.distributed as dist
dist.init_process_group("gloo", rank=0, world_size=1)
from lodestar_amd import workloads as W
from lodestar_amd.native import GpuContext, library_hip_runtime, pack_requests
from lodestar_amd.shard import global_throughput
out = {"backend": dist.get_backend()}
with GpuContext(0) as gpu:
    n = 1024
    W.load_table([gpu], 64)
    sks = W.interop_sks(64)
    msgs = [W.message(j, b"GLOO") for j in range(n)]
    sigs = W._sign_all(gpu, [sks[j % 64] for j in range(n)], msgs)
    v, _ = gpu.verify_packed(pack_requests([(True, [([j % 64], msgs[j], sigs[j])]) for j in range(n)]))
    out["cfg2_valid"] = int((v == 1).sum())
    out["throughput"] = global_throughput(2048, 0.5, dist, device=None)
    out["library_hip_runtime"] = library_hip_runtime()
dist.destroy_process_group()
print(json.dumps(out))
"""


def test_gloo_rank_binds_library_to_opt_rocm():
    """The cfg2 / cfg4 / cfg5 rank modes of `bench.py --gpus N` (no data-path collective)
    load the library before torch and use gloo for the barrier and the max-over-ranks
    reduction, so a rank's HIP calls go to /opt/rocm's runtime as the N = 1 line's do
    (VERDICT r5 item 2).  A fresh child process does exactly that (world 1) and verifies a
    1024-set cfg2 call."""
    import json
    import os
    import subprocess
    import sys
    from pathlib import Path

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
               REPO=str(Path(__file__).resolve().parent.parent))
    r = subprocess.run([sys.executable, "-c", _GLOO_RANK], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["backend"] == "gloo" and out["cfg2_valid"] == 1024
    assert out["throughput"] == [4096.0, 0.5]
    assert out["library_hip_runtime"].startswith("/opt/rocm"), out["library_hip_runtime"]
