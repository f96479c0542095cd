"""GpuBlsVerifier: the IBlsVerifier contract over the MI355X C-ABI.

Mirrors `BlsMultiThreadWorkerPool` (beacon-node/src/chain/bls/multithread/index.ts)
with GPU contexts in place of worker threads:

* `verify_signature_sets(sets, batchable, verify_on_main_thread)` (interface.ts:20-46,
  index.ts:134-174): the main-thread branch (`verify_on_main_thread` and not
  `verify_all_multi_thread`) runs the call at once as one non-batchable request
  (verifySignatureSetsMaybeBatch semantics, maybeBatch.ts:16-39) on a dedicated
  high-priority context that no pool call uses (the reference runs it on the main
  thread, outside the worker queue, index.ts:138-151); otherwise the sets
  are split by chunkifyMaximizeChunkSize(sets, 128) into jobs (index.ts:156) whose
  results are AND-ed.
* job queue (index.ts:238-285): batchable jobs are buffered until more than 32
  signatures are waiting or 100 ms passed since the first (MAX_BUFFERED_SIGS,
  MAX_BUFFER_WAIT_MS); other jobs go straight to the queue.
* dispatch (runJob / prepareWork, index.ts:290-400): an idle context takes queued
  jobs up to `max_sets_per_call` signature sets and runs one verifyManySignatureSets
  call (bls_gpu_verify, worker.ts:32-108); per job a verdict resolves the job's
  future, an error code rejects it with the blst-style message ("BLST_ERROR:
  BLST_INVALID_SIZE", "Empty signature set", ...).  The reference caps a worker
  message at 128 sets (MAX_SIGNATURE_SETS_PER_JOB, sized for one CPU core); a GPU call
  wants ~1024 (one call of 128 sets fills 43 of 1024 SIMDs), so the default
  coalesces queued jobs up to GPU_SETS_PER_CALL.  For table-index keys verdicts per
  job are unchanged: the worker chunks a message by request (worker.ts:56) and
  re-verifies a failing chunk's requests alone, so which jobs share a message changes
  only batchRetries.  Raw-key jobs are different: deserializeSet rejects a whole worker
  message when one key does not decode (worker.ts:43-46), so they go to the GPU as the
  reference's messages (prepareWork: jobs until >= 128 sets, index.ts:385-400), each
  its own message of one bls_gpu_verify_many submission.
* metrics: `metrics.bls.aggregatedPubkeys` and the `metrics.blsThreadPool.*` series
  under the reference's names (lodestar_amd/metrics.py, lodestar.ts:378-446).
* `close()` (index.ts:176-197) rejects pending jobs with QUEUE_ABORTED.

* several devices (`devices=[0, 1, ...]`, one verifier per node): the reference's pool
  spreads one call's 128-set jobs over every worker of the process (index.ts:153-166,
  199-233, poolSize.ts:3-11); here every device slot opens `n_contexts` contexts with
  its own replica of the pubkey table, and an idle context takes queued jobs only while
  its slot carries the least outstanding set weight among slots with an idle context
  (`set_weight`: an aggregate set of k keys weighs 1 + k / 1024, its share of a set's
  Fp products), so jobs go to the least-loaded device.  A non-batchable call of at
  least `split_call_min_sets` sets is split across the slots instead (the
  in-process form of lodestar_amd/shard.py): each slot computes the Fp12 Miller-loop
  partial of a contiguous shard (bls_gpu_partial, scalars from the call's shared seed
  at the set's call index, so the shards are one random-scalar batch), the partials
  are gathered on the host and ONE final exponentiation decides the call
  (bls_gpu_final_check); a failing call is localised to its shards for the record.
  The verdict equals the reference's AND over the call's jobs (each a batch of
  verifySignatureSetsMaybeBatch, maybeBatch.ts:16-39; non-batchable jobs move no
  worker counter, worker.ts:90-97); when any shard reports a set that does not
  decode, the call is re-run as the reference's jobs so the rejection is the one its
  Promise.all would give.  `devices=[0, 0]` gives two slots on one GPU (the 1-GPU
  test of the routing and the split).

Sets are `SignatureSet(pubkey, signing_root, signature)` where pubkey is an int
index into the context's device pubkey table (Index2PubkeyCache), a list of
indices (an aggregate set, getAggregatedPubkey, utils.ts:5-16), or 96 raw bytes
(uncompressed affine, the worker wire format of index.ts:126).
"""
from __future__ import annotations

import os
import threading
import time
from concurrent.futures import Future
from dataclasses import dataclass
from typing import Sequence, Union

from ._abi import ERROR_MESSAGES
from .metrics import BlsMetrics, get_aggregated_pubkeys_count
from .native import GpuContext, NativeError, pack_requests
from .shard import shard_bounds

MAX_SIGNATURE_SETS_PER_JOB = 128   # multithread/index.ts:39
GPU_SETS_PER_CALL = 1024           # sets per bls_gpu_verify call (cfg2 shape)
MAX_BUFFERED_SIGS = 32             # multithread/index.ts:48 (flush when >)
MAX_BUFFER_WAIT_MS = 100           # multithread/index.ts:57
SPLIT_CALL_MIN_SETS = 4096         # non-batchable calls this large are split across device slots
AGG_KEY_WEIGHT = 1024              # keys of an aggregate set per set of weight (set_weight)

PubkeyRef = Union[int, Sequence[int], bytes]


@dataclass
class SignatureSet:
    """ISignatureSet (state-transition/src/util/signatureSets.ts:5-22)."""

    pubkey: PubkeyRef
    signing_root: bytes
    signature: bytes


class BlsError(Exception):
    """A rejected verification (the worker's WorkResult error, types.ts:26-38)."""


class QueueAborted(Exception):
    """QueueError QUEUE_ABORTED (util/queue)."""


def chunkify_maximize_chunk_size(arr: list, min_per_chunk: int) -> list:
    """multithread/utils.ts:4-19."""
    chunk_count = len(arr) // min_per_chunk
    if chunk_count <= 1:
        return [arr]
    per = -(-len(arr) // chunk_count)
    return [arr[i: i + per] for i in range(0, len(arr), per)]


@dataclass
class _Job:
    sets: list
    batchable: bool
    future: Future
    added: float


def set_weight(pk) -> float:
    """Routing weight of one set: 1 for a single key, 1 + k / AGG_KEY_WEIGHT for an
    aggregate of k table keys (a G1 addition is ~11 of a set's ~12.7k Fp products, so
    a 512-key committee costs about 1.5 sets), 1 for raw keys."""
    if isinstance(pk, int) or isinstance(pk, (bytes, bytearray, memoryview)):
        return 1.0
    k = len(pk)
    return 1.0 + (k / AGG_KEY_WEIGHT if k > 1 else 0.0)


def _wire(s: SignatureSet):
    pk = s.pubkey
    if isinstance(pk, int):
        pk = [pk]
    elif not isinstance(pk, (bytes, bytearray, memoryview)):
        pk = list(pk)
    return (pk, bytes(s.signing_root), bytes(s.signature))


class _Pinned:
    """One shard of a split call, for one device slot (bls_gpu_partial)."""

    __slots__ = ("sets", "base", "seed", "done")

    def __init__(self, sets, base, seed, done):
        self.sets, self.base, self.seed, self.done = sets, base, seed, done


class GpuBlsVerifier:
    """IBlsVerifier on one or more GPUs: `n_contexts` contexts (HIP streams) per device
    slot, plus one high-priority main-thread context on the first slot's device."""

    def __init__(self, device: int = 0, n_contexts: int = 2, verify_all_multi_thread: bool = False,
                 max_sets_per_call: int = GPU_SETS_PER_CALL, pubkeys48: bytes | None = None,
                 metrics: BlsMetrics | None = None, devices: Sequence[int] | None = None,
                 split_call_min_sets: int = SPLIT_CALL_MIN_SETS, context_factory=None, record_calls: bool = False):
        self.verify_all_multi_thread = verify_all_multi_thread
        self.max_sets_per_call = max_sets_per_call
        self.devices = list(devices) if devices is not None else [device]
        if not self.devices:
            raise ValueError("devices: at least one device")
        self.split_call_min_sets = max(2, int(split_call_min_sets))
        make = context_factory or (lambda dev, high: GpuContext(dev, high_priority=high))
        # the main-thread lane first (its own high-priority context, never used by the
        # pool), then the pool's contexts: a context the library refuses (scratch
        # admission, BLS_ERR_ADMISSION) or that fails to start is recorded and the pool runs
        # on the others, as the reference's pool keeps the workers that started
        # (multithread/index.ts:221-229); with none at all, queued work raises the first
        # error (index.ts:247-253)
        self._main = make(self.devices[0], True)
        self._ctxs: list = []
        self._ctx_slot: list[int] = []
        self.init_errors: list[Exception] = []
        for slot, dev in enumerate(self.devices):
            for _ in range(n_contexts):
                try:
                    self._ctxs.append(make(dev, False))
                    self._ctx_slot.append(slot)
                except NativeError as e:
                    self.init_errors.append(e)
        self._main_lock = threading.Lock()
        if pubkeys48 is not None:
            self.load_pubkeys(pubkeys48)
        self._cv = threading.Condition()
        self._jobs: list[_Job] = []
        self._buffer: list[_Job] = []
        self._buffer_sigs = 0
        self._buffer_first = 0.0
        self._closed = False
        n_slots = len(self.devices)
        self._slot_ctxs = [sum(1 for s in self._ctx_slot if s == k) for k in range(n_slots)]
        self._idle = [0] * n_slots          # contexts of the slot waiting for work
        self._load = [0.0] * n_slots        # set weight the slot's contexts are running
        self._pinned: list[list[_Pinned]] = [[] for _ in range(n_slots)]
        # per slot: calls, sets and set weight run (the routing's record, tests / bench)
        self.slot_stats = [{"calls": 0, "sets": 0, "weight": 0.0} for _ in range(n_slots)]
        self.split_stats = {"calls": 0, "rerouted": 0, "failed": 0, "bad_shards": []}
        # record_calls: every pool GPU call as (slot, [(batchable, wire sets) per job]), so a
        # test can replay the calls through the oracle's worker semantics
        self.call_log: list | None = [] if record_calls else None
        self.metrics = metrics if metrics is not None else BlsMetrics()
        self._threads = [threading.Thread(target=self._worker, args=(c, self._ctx_slot[k], k), daemon=True)
                         for k, c in enumerate(self._ctxs)]
        self._timer = threading.Thread(target=self._buffer_timer, daemon=True)
        for t in self._threads:
            t.start()
        self._timer.start()

    # -- pubkey cache -----------------------------------------------------------
    def load_pubkeys(self, pubkeys48: bytes) -> None:
        """Append validator pubkeys (48 B compressed) to every context's device table on
        every device, all or nothing: bls_gpu_load_pubkeys appends no key of a batch that
        holds an undecodable one, so a failure on the first context leaves every table as
        it was and validator indices stay aligned across contexts and devices."""
        first = self._ctxs[0] if self._ctxs else self._main
        codes = first.load_pubkeys(pubkeys48, 48)
        if (codes != 0).any():
            bad = int((codes != 0).argmax())
            raise BlsError(f"invalid pubkey at batch index {bad} (code {int(codes[bad])}); no key appended")
        for c in [c for c in self._ctxs + [self._main] if c is not first]:
            codes = c.load_pubkeys(pubkeys48, 48)
            if (codes != 0).any():  # same bytes as context 0: cannot happen short of a device fault
                raise BlsError("pubkey tables diverged across contexts")

    # -- IBlsVerifier --------------------------------------------------------------
    def verify_signature_sets(self, sets: Sequence[SignatureSet], batchable: bool = False,
                              verify_on_main_thread: bool = False) -> bool:
        return self.verify_signature_sets_async(sets, batchable, verify_on_main_thread).result()

    def verify_signature_sets_async(self, sets: Sequence[SignatureSet], batchable: bool = False,
                                    verify_on_main_thread: bool = False) -> Future:
        # pubkeys are aggregated (on the device) whichever branch runs (index.ts:136)
        self.metrics.bls.aggregatedPubkeys.inc(get_aggregated_pubkeys_count(sets))
        if verify_on_main_thread and not self.verify_all_multi_thread:
            fut: Future = Future()
            stop = self.metrics.blsThreadPool.mainThreadDurationInThreadPool.start_timer()
            try:
                with self._main_lock:
                    fut.set_result(self._run_now(list(sets)))
            except Exception as e:  # noqa: BLE001 - the contract rejects with the error
                fut.set_exception(e)
            finally:
                stop()
            return fut
        sets = list(sets)
        if (not batchable and len(self.devices) > 1 and len(sets) >= self.split_call_min_sets
                and sum(self._slot_ctxs) > 0 and all(self._slot_ctxs)):
            return self._split_call(sets)
        return self._queue_call(sets, batchable)

    def _queue_call(self, sets: list, batchable: bool) -> Future:
        """The reference's path: chunkifyMaximizeChunkSize(sets, 128) jobs, AND-ed."""
        jobs = [self._queue(chunk, batchable) for chunk in chunkify_maximize_chunk_size(sets, MAX_SIGNATURE_SETS_PER_JOB)]
        out: Future = Future()
        pending = [len(jobs)]
        results = [None] * len(jobs)
        lock = threading.Lock()

        def done(k, f):
            with lock:
                if out.done():
                    return
                if f.exception() is not None:
                    out.set_exception(f.exception())
                    return
                results[k] = f.result()
                pending[0] -= 1
                if pending[0] == 0:
                    out.set_result(all(r is True for r in results))

        for k, j in enumerate(jobs):
            j.future.add_done_callback(lambda f, k=k: done(k, f))
        return out

    def _split_call(self, sets: list) -> Future:
        """One non-batchable call split over the device slots: a contiguous shard per slot
        -> bls_gpu_partial (Fp12 Miller-loop product, scalars from the shared seed at the
        set's call index) -> host gather -> one bls_gpu_final_check (see the module doc)."""
        out: Future = Future()
        wires = [_wire(s) for s in sets]
        seed = os.urandom(32)
        bounds = [(b, e) for b, e in shard_bounds(len(wires), len(self.devices))]
        results: list = [None] * len(bounds)
        pending = [len(bounds)]
        lock = threading.Lock()
        tp = self.metrics.blsThreadPool
        tp.totalJobsGroupsStarted.inc(len(bounds))
        tp.totalJobsStarted.inc(len(bounds))
        tp.totalSigSetsStarted.inc(len(wires))

        def finish(ctx):
            # every shard is in: runs on the worker thread of the last one, on its context
            if any(r is None or isinstance(r, Exception) for r in results):
                err = next((r for r in results if isinstance(r, Exception)), None)
                out.set_exception(err or NativeError("split call: a shard did not run"))
                tp.errorJobsSignatureSetsCount.inc(len(wires))
                return
            if any(st != 0 for _, st, _ in results):
                # a set that does not decode: the rejection must be the reference's, whose
                # jobs are the 128-set chunks -- run the call as those jobs
                self.split_stats["rerouted"] += 1
                inner = self._queue_call(sets, False)
                inner.add_done_callback(lambda f: out.set_exception(f.exception()) if f.exception() is not None
                                        else out.set_result(f.result()))
                return
            parts = [p for p, _, _ in results]
            try:
                ok = bool(ctx.final_check(parts))
                bad = []
                if not ok:
                    bad = [k for k, p in enumerate(parts) if not ctx.final_check([p])]
            except Exception as e:  # noqa: BLE001 - reject the call with the device error
                out.set_exception(e)
                tp.errorJobsSignatureSetsCount.inc(len(wires))
                return
            with self._cv:
                self.split_stats["calls"] += 1
                if not ok:
                    self.split_stats["failed"] += 1
                    self.split_stats["bad_shards"] = bad
            tp.successJobsSignatureSetsCount.inc(len(wires))
            out.set_result(ok)

        def shard_done(k, res, ctx):
            results[k] = res
            with lock:
                pending[0] -= 1
                last = pending[0] == 0
            if last:
                finish(ctx)

        with self._cv:
            if self._closed:
                out.set_exception(QueueAborted("QUEUE_ABORTED"))
                return out
            for k, (b, e) in enumerate(bounds):
                self._pinned[k].append(_Pinned(wires[b:e], b, seed, lambda res, ctx, k=k: shard_done(k, res, ctx)))
            self._cv.notify_all()
        return out

    def close(self) -> None:
        with self._cv:
            self._closed = True
            pending = self._jobs + self._buffer
            pinned = [p for lst in self._pinned for p in lst]
            self._jobs, self._buffer = [], []
            self._pinned = [[] for _ in self._pinned]
            self._cv.notify_all()
        for j in pending:
            if not j.future.done():
                j.future.set_exception(QueueAborted("QUEUE_ABORTED"))
        for p in pinned:
            p.done(QueueAborted("QUEUE_ABORTED"), None)
        for t in self._threads:
            t.join(timeout=30)
        for c in self._ctxs + [self._main]:
            c.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- internals ------------------------------------------------------------------
    def _run_now(self, sets: list) -> bool:
        v, _ = self._call(self._main, [(False, [_wire(s) for s in sets])])
        return self._verdict(int(v[0]))

    @staticmethod
    def _verdict(code: int) -> bool:
        if code < 0:
            raise BlsError(ERROR_MESSAGES.get(-code, f"BLST_ERROR: {-code}"))
        return code == 1

    def _call(self, ctx, reqs, worker_id: int = 0):
        """One GPU submission per pubkey form: table-index requests as one message
        (bls_gpu_verify), raw-key requests as the reference's worker messages (jobs until
        >= 128 sets each) through one bls_gpu_verify_many."""
        def is_raw(req):
            return any(isinstance(pk, (bytes, bytearray, memoryview)) for pk, _, _ in req[1])
        groups = {}
        for k, r in enumerate(reqs):
            groups.setdefault(is_raw(r), []).append(k)
        verdicts = [0] * len(reqs)
        stats = None
        tp = self.metrics.blsThreadPool
        for raw, idx in groups.items():
            t0 = time.perf_counter()
            if raw:
                msgs, cur, n = [], [], 0
                for k in idx:
                    cur.append(k)
                    n += len(reqs[k][1])
                    if n >= MAX_SIGNATURE_SETS_PER_JOB:
                        msgs.append(cur)
                        cur, n = [], 0
                if cur:
                    msgs.append(cur)
                pbs = [pack_requests([reqs[k] for k in m]) for m in msgs]
                t1 = time.perf_counter()
                vs, stats = ctx.verify_many(pbs)
                v = [x for part in vs for x in part]
                idx = [k for m in msgs for k in m]
            else:
                pb = pack_requests([reqs[k] for k in idx])
                t1 = time.perf_counter()
                v, stats = ctx.verify_packed(pb)
            t2 = time.perf_counter()
            for k, x in zip(idx, v):
                verdicts[k] = int(x)
            # the context is the "worker": its time is the call's device time; the
            # latencies to / from it are the host packing and the verdict hand-back
            tp.jobsWorkerTime.inc({"workerId": worker_id}, stats.device_ms / 1e3)
            tp.latencyToWorker.observe(t1 - t0)
            tp.latencyFromWorker.observe(max(0.0, (t2 - t1) - stats.device_ms / 1e3))
            tp.batchRetries.inc(stats.batch_retries)
            tp.batchSigsSuccess.inc(stats.batch_sigs_success)
        return verdicts, stats

    def _queue(self, sets: list, batchable: bool) -> _Job:
        if not self._ctxs and self.init_errors:
            raise self.init_errors[0]  # every pool context failed to start (index.ts:247-253)
        job = _Job([_wire(s) for s in sets], batchable, Future(), time.monotonic())
        with self._cv:
            if self._closed:
                job.future.set_exception(QueueAborted("QUEUE_ABORTED"))
                return job
            if batchable:
                if not self._buffer:
                    self._buffer_first = time.monotonic()
                self._buffer.append(job)
                self._buffer_sigs += len(sets)
                if self._buffer_sigs > MAX_BUFFERED_SIGS:
                    self._flush_locked()
            else:
                self._jobs.append(job)
            self._cv.notify_all()
        return job

    def _flush_locked(self):
        self._jobs.extend(self._buffer)
        self._buffer, self._buffer_sigs = [], 0

    def _buffer_timer(self):
        while True:
            with self._cv:
                if self._closed:
                    return
                if self._buffer and time.monotonic() - self._buffer_first >= MAX_BUFFER_WAIT_MS / 1e3:
                    self._flush_locked()
                    self._cv.notify_all()
                wait = MAX_BUFFER_WAIT_MS / 1e3
                if self._buffer:
                    wait = max(0.0, self._buffer_first + MAX_BUFFER_WAIT_MS / 1e3 - time.monotonic())
                self._cv.wait(timeout=wait if self._buffer else 0.05)

    def _prepare_work(self) -> list:
        """prepareWork (index.ts:385-400): take jobs up to max_sets_per_call sets."""
        jobs, total = [], 0
        while self._jobs and total < self.max_sets_per_call:
            j = self._jobs.pop(0)
            jobs.append(j)
            total += len(j.sets)
        return jobs

    def _my_turn(self, slot: int) -> bool:
        """Least-loaded routing: the slot takes queued jobs only while no other slot with
        an idle context carries less outstanding set weight (ties: the lower slot)."""
        mine = (self._load[slot], slot)
        return all(mine <= (self._load[k], k) for k in range(len(self._load)) if self._idle[k] > 0)

    def queue_length(self) -> int:
        """blsThreadPool.queueLength (index.ts:130, set on collect)."""
        with self._cv:
            n = len(self._jobs)
        self.metrics.blsThreadPool.queueLength.set(n)
        return n

    def _worker(self, ctx, slot: int, wid: int):
        tp = self.metrics.blsThreadPool
        while True:
            pin, jobs = None, None
            with self._cv:
                self._idle[slot] += 1
                while True:
                    if self._closed:
                        self._idle[slot] -= 1
                        return
                    if self._pinned[slot]:
                        pin = self._pinned[slot].pop(0)
                        break
                    if self._jobs and self._my_turn(slot):
                        jobs = self._prepare_work()
                        if jobs:
                            break
                    self._cv.wait(timeout=0.05)
                self._idle[slot] -= 1
                sets = pin.sets if pin is not None else [s for j in jobs for s in j.sets]
                weight = sum(set_weight(pk) for pk, _, _ in sets)
                self._load[slot] += weight
                st = self.slot_stats[slot]
                st["calls"] += 1
                st["sets"] += len(sets)
                st["weight"] += weight
            try:
                if pin is not None:
                    self._run_pinned(ctx, pin)
                else:
                    self._run_jobs(ctx, jobs, wid, tp)
            finally:
                with self._cv:
                    self._load[slot] -= weight
                    self._cv.notify_all()

    def _run_pinned(self, ctx, pin: _Pinned):
        try:
            part, status, err, _ = ctx.partial(pack_requests([(False, pin.sets)], seed=pin.seed), pin.base)
            res = (part, int(status), err)
        except Exception as e:  # noqa: BLE001 - the call rejects with it
            res = e
        pin.done(res, ctx)

    def _run_jobs(self, ctx, jobs, wid, tp):
        if self.call_log is not None:
            with self._cv:
                self.call_log.append((self._ctx_slot[wid], [(j.batchable, j.sets) for j in jobs]))
        now = time.monotonic()
        for j in jobs:
            tp.jobWaitTime.observe(now - j.added)
        tp.totalJobsGroupsStarted.inc(1)
        tp.totalJobsStarted.inc(len(jobs))
        tp.totalSigSetsStarted.inc(sum(len(j.sets) for j in jobs))
        try:
            verdicts, _ = self._call(ctx, [(j.batchable, j.sets) for j in jobs], wid)
        except Exception as e:  # noqa: BLE001 - reject every job of the call
            for j in jobs:
                j.future.set_exception(e)
            tp.errorJobsSignatureSetsCount.inc(sum(len(j.sets) for j in jobs))
            return
        for j, code in zip(jobs, verdicts):
            try:
                j.future.set_result(self._verdict(code))
                tp.successJobsSignatureSetsCount.inc(len(j.sets))
            except BlsError as e:
                j.future.set_exception(e)
                tp.errorJobsSignatureSetsCount.inc(len(j.sets))
