"""The N-API addon (integration/napi/lodestar_bls_napi.c) and the JS GpuBlsVerifier
(integration/js/gpuBlsVerifier.js): the reference's pool e2e test
(beacon-node/test/e2e/chain/bls/multithread.test.ts) run under Node against the GPU."""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
ADDON = ROOT / "lodestar_amd" / "_native" / "lodestar_bls.node"
NODE = shutil.which("node")

pytestmark = pytest.mark.skipif(NODE is None or not ADDON.exists(), reason="node or the N-API addon is absent")


def test_addon_exports():
    code = ("const a = require(process.argv[1]);"
            "console.log(JSON.stringify(['init','close','loadPubkeys','verify','verifySync','sszRoots','partial','finalCheck']"
            ".map(k => typeof a[k])))")
    out = subprocess.run([NODE, "-e", code, str(ADDON)], capture_output=True, text=True, timeout=60, check=True)
    assert json.loads(out.stdout) == ["function"] * 8


@pytest.mark.gpu
def test_js_pool_matches_reference_tests(gpu, golden, oracle, tmp_path):
    sks = [oracle.interop_secret_key(i).to_bytes(32, "big") for i in range(3)]
    msgs = [hashlib.sha256(b"napi%d" % i).digest() for i in range(3)]
    sigs = gpu.sign(b"".join(sks), b"".join(msgs))
    data = {"pubkeys48": "".join(golden["kat2_interop_pubkeys"]),
            "sets": [{"idx": i, "msg": msgs[i].hex(), "sig": sigs[i].tobytes().hex()} for i in range(3)]}
    f = tmp_path / "sets.json"
    f.write_text(json.dumps(data))
    out = subprocess.run([NODE, str(ROOT / "integration" / "js" / "poolTest.js"), str(f)], capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["chunkify"] == [[[0]], [[0, 1]], [[0, 1, 2]], [[0, 1, 2, 3]], [[0, 1, 2, 3, 4]],
                             [[0, 1, 2], [3, 4, 5]], [[0, 1, 2, 3], [4, 5, 6]], [[0, 1, 2, 3], [4, 5, 6, 7]]]
    for k in ("sync", "async", "batched", "mainThread", "firstInvalidOthers"):
        assert r[k] == [True] * 8, k
    assert "BLST_INVALID_SIZE" in r["firstInvalid"]
    assert r["wrongMessage"] is False
    assert r["empty"] == "Empty signature set"
    # state-transition verifySignatureSet through verifySync (signatureSets.ts:24-38)
    assert r["stfSync"] == [True, False, "BLST_ERROR: BLST_INVALID_SIZE"]
    assert r["stfEach"] == [True, False, True, False]
    assert r["stfEachInvalid"] == [False, "BLST_ERROR: BLST_INVALID_SIZE"]


def test_js_adapter_host_side():
    """The adapter's queueing with a stand-in addon (no GPU): per-set gossip calls are
    buffered (>32 sigs / 100 ms) and coalesced into calls of up to 1024 sets, verdicts
    map back to their calls, an error code rejects only its own call, close() waits for
    calls in flight and rejects queued jobs."""
    out = subprocess.run([NODE, str(ROOT / "integration" / "js" / "adapterTest.js")], capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["verdicts_ok"] and r["max_call_sets"] == 1024 and 4 <= r["calls"] <= 6
    assert r["rejected"] == "BLST_ERROR: BLST_INVALID_SIZE" and r["others_true"]
    assert r["closed"] == "QUEUE_ABORTED" and r["inflight_at_close"] == 0
    # batchRetries, batchSigsSuccess, latencyToWorker, latencyFromWorker move (calls with a
    # failing chunk), queueLength is sampled on collect (multithread/index.ts:130,357-366)
    assert all(x > 0 for x in r["series"]) and not r["series_bad"] and r["queue_length_metric"]
    assert r["stats_retries"] > 0
    # raw-key calls stay one worker message each (prepareWork: jobs until >= 128 sets)
    assert r["raw_max_call_sets"] == 128
    # verifyOnMainThread runs on the dedicated high-priority context
    assert r["main_handles"] == 1 and r["main_calls"] == [1] and r["pool_high"] == 2
    # the libuv pool warning reads the pool the process started with (a stand-in of 4)
    assert r["pool_warning"] and "4 threads < contexts + 2 = 5" in r["pool_warning"]
    # admission: a refused pool context is recorded and the pool runs on the others; with
    # none admitted, queued work rejects with the first error (multithread/index.ts:247-253)
    assert r["admitted_partial"] == {"ctxs": 1, "errors": 2, "verdict": True}
    assert r["admitted_none"] == "BLS_ERR_ADMISSION: stand-in refusal"


@pytest.mark.gpu
def test_js_signing_roots_kat1(gpu):
    """GpuBlsVerifier.computeSigningRoots through the addon: KAT-1's deposit signing root
    (genesisState.test.ts:65-69) and the computeDomain it needs (fork data on the GPU)."""
    g = json.loads((ROOT / "tests" / "golden" / "ssz_golden.json").read_text())["kat1_deposit"]
    code = f"""
const {{GpuBlsVerifier}} = require({json.dumps(str(ROOT / "integration" / "js" / "gpuBlsVerifier.js"))});
const v = new GpuBlsVerifier({{contexts: 1}});
const fd = v.computeSigningRoots("forkData", Buffer.from("{g['fork_version']}" + "00".repeat(32), "hex"), null);
const domain = Buffer.concat([Buffer.from("03000000", "hex"), Buffer.from(fd).subarray(0, 28)]);
const amount = Buffer.alloc(8); amount.writeUInt32LE({g['amount']} % 2 ** 32, 0); amount.writeUInt32LE(Math.floor({g['amount']} / 2 ** 32), 4);
const msg = Buffer.concat([Buffer.from("{g['pubkey']}", "hex"), Buffer.from("{g['withdrawal_credentials']}", "hex"), amount]);
const r = v.computeSigningRoots("depositMessage", msg, domain);
console.log(JSON.stringify({{domain: domain.toString("hex"), root: Buffer.from(r).toString("hex")}}));
v.close();
"""
    out = subprocess.run([NODE, "-e", code], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r == {"domain": g["domain"], "root": g["signing_root"]}


@pytest.mark.gpu
def test_js_main_thread_lane_not_behind_pool(gpu, tmp_path):
    """verifyOnMainThread (multithread/index.ts:138-151) while a 4096-set pool call is in
    flight: the adapter runs it on its own high-priority context, so it resolves before
    the pool call does, in a fraction of the pool call's time."""
    from lodestar_amd import workloads as W

    n, keys = 4096, 1024
    sks = W.interop_sks(keys)
    pks48 = gpu.sk_to_pk(b"".join(s.to_bytes(32, "big") for s in sks)).tobytes()
    msgs = [W.message(j, b"MAIN") for j in range(n)]
    sigs = gpu.sign(b"".join(sks[j % keys].to_bytes(32, "big") for j in range(n)), b"".join(msgs))
    f = tmp_path / "work.json"
    f.write_text(json.dumps({"pubkeys48": pks48.hex(), "sets": [
        {"idx": j % keys, "msg": msgs[j].hex(), "sig": sigs[j].tobytes().hex()} for j in range(n)]}))
    out = subprocess.run([NODE, str(ROOT / "integration" / "js" / "mainLaneTest.js"), str(f)], capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    r = json.loads(out.stdout.strip().splitlines()[-1])
    for run in r["runs"]:
        assert run["main_ok"] is True and run["pool_ok"] is True
        assert run["main_before_pool"], run
        assert run["main_ms"] < 0.7 * run["pool_ms"], run


def _multi_checks(r):
    assert r["slots"] == [2, 2]
    assert r["gossipOk"] is True
    assert sum(r["slotSets"]) == 512 and min(r["slotSets"]) > 0, r["slotSets"]
    assert r["splitValid"] is True and r["splitInvalid"] is False and r["badShards"] == [1]
    assert r["splitError"] == "BLST_ERROR: BLST_INVALID_SIZE"
    assert r["splitStats"]["calls"] == 2 and r["splitStats"]["rerouted"] == 1 and r["splitStats"]["failed"] == 1
    assert r["batchableValid"] is True and r["splitCallsAfterBatchable"] == 2


def test_js_multi_device_host_side():
    """The adapter over two device slots with a stand-in addon (no GPU): per-set gossip
    calls spread over both slots with their verdicts; a 512-set non-batchable call split
    in two shards of 256 with one shared seed (addon.partial), one finalCheck over both
    partials (then one per shard to localise a failing call); an undecodable signature
    re-runs the call as the reference's jobs and rejects with BLST_INVALID_SIZE."""
    out = subprocess.run([NODE, str(ROOT / "integration" / "js" / "multiDeviceTest.js"), "--stand-in"],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    r = json.loads(out.stdout.strip().splitlines()[-1])
    _multi_checks(r)
    assert r["partials"] == [[0, 256], [256, 256]] and r["sharedSeed"] is True
    assert r["finals"] == [2, 2, 1, 1]


@pytest.mark.gpu
def test_js_multi_device_on_one_gpu(gpu, oracle, tmp_path):
    """The same through the real addon with devices [0, 0] (two slots on the box's one
    GPU): real signatures, bls_gpu_partial / bls_gpu_final_check for the split call."""
    n = 512
    sks = [oracle.interop_secret_key(i % 100).to_bytes(32, "big") for i in range(n)]
    msgs = [hashlib.sha256(b"jsmulti%d" % i).digest() for i in range(n)]
    sigs = gpu.sign(b"".join(sks), b"".join(msgs))
    pks48 = gpu.sk_to_pk(b"".join(sks[:100])).tobytes()
    f = tmp_path / "work.json"
    f.write_text(json.dumps({"pubkeys48": pks48.hex(), "sets": [
        {"idx": i % 100, "msg": msgs[i].hex(), "sig": sigs[i].tobytes().hex()} for i in range(n)]}))
    out = subprocess.run([NODE, str(ROOT / "integration" / "js" / "multiDeviceTest.js"), str(f)], capture_output=True,
                         text=True, timeout=300, env=dict(os.environ, UV_THREADPOOL_SIZE="16"))
    assert out.returncode == 0, out.stderr
    _multi_checks(json.loads(out.stdout.strip().splitlines()[-1]))


@pytest.mark.gpu
def test_js_bench_exits_cleanly_with_16_contexts(gpu, tmp_path):
    """benchNapi.js at the bench's 16 contexts (plus the main lane) exits with status 0
    after closing every handle: before the handles were wrapped objects whose wrap
    close() removes, Node ran their finalizers during environment teardown and the
    16-context bench died at exit with SIGSEGV (profiles/r06_napi_exit_crash.txt)."""
    from lodestar_amd import workloads as W

    n, keys = 4096, 1024
    sks = W.interop_sks(keys)
    pks48 = gpu.sk_to_pk(b"".join(s.to_bytes(32, "big") for s in sks)).tobytes()
    msgs = [W.message(j, b"EXIT") for j in range(n)]
    sigs = gpu.sign(b"".join(sks[j % keys].to_bytes(32, "big") for j in range(n)), b"".join(msgs))
    f = tmp_path / "work.json"
    f.write_text(json.dumps({"pubkeys48": pks48.hex(), "sets": [
        {"idx": j % keys, "msg": msgs[j].hex(), "sig": sigs[j].tobytes().hex()} for j in range(n)]}))
    for per_call in ("1024", "1"):
        out = subprocess.run([NODE, str(ROOT / "integration" / "js" / "benchNapi.js"), str(f), "2", "16", str(n),
                              per_call, str(n), "0"], capture_output=True, text=True, timeout=300,
                             env=dict(os.environ, UV_THREADPOOL_SIZE="18"))
        assert out.returncode == 0, (per_call, out.returncode, out.stderr[-2000:])
        r = json.loads(out.stdout.strip().splitlines()[-1])
        assert r["contexts"] == 16 and r["sets_per_step"] == 16 * n
