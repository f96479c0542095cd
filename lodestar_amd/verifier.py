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

Sets are `SignatureSet(pubkey, signing_root, signature)` where pubkey is an int
index into the context's device pubkey table (Index2PubkeyCache), a list of
indices (an aggregate set, getAggregatedPubkey, utils.ts:5-16), or 96 raw bytes
(uncompressed affine, the worker wire format of index.ts:126).
"""
from __future__ import annotations

import threading
import time
from concurrent.futures import Future
from dataclasses import dataclass
from typing import Sequence, Union

from ._abi import ERROR_MESSAGES
from .metrics import BlsMetrics, get_aggregated_pubkeys_count
from .native import GpuContext, NativeError, pack_requests

MAX_SIGNATURE_SETS_PER_JOB = 128   # multithread/index.ts:39
GPU_SETS_PER_CALL = 1024           # sets per bls_gpu_verify call (cfg2 shape)
MAX_BUFFERED_SIGS = 32             # multithread/index.ts:48 (flush when >)
MAX_BUFFER_WAIT_MS = 100           # multithread/index.ts:57

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


def _wire(s: SignatureSet):
    pk = s.pubkey
    if isinstance(pk, int):
        pk = [pk]
    elif not isinstance(pk, (bytes, bytearray, memoryview)):
        pk = list(pk)
    return (pk, bytes(s.signing_root), bytes(s.signature))


class GpuBlsVerifier:
    """IBlsVerifier on one GPU with `n_contexts` contexts (HIP streams) in flight."""

    def __init__(self, device: int = 0, n_contexts: int = 2, verify_all_multi_thread: bool = False,
                 max_sets_per_call: int = GPU_SETS_PER_CALL, pubkeys48: bytes | None = None,
                 metrics: BlsMetrics | None = None):
        self.verify_all_multi_thread = verify_all_multi_thread
        self.max_sets_per_call = max_sets_per_call
        # the main-thread lane first (its own high-priority context, never used by the
        # pool), then the pool's contexts: a context the library refuses (scratch
        # admission, BLS_ERR_ADMISSION) or that fails to start is recorded and the pool runs
        # on the others, as the reference's pool keeps the workers that started
        # (multithread/index.ts:221-229); with none at all, queued work raises the first
        # error (index.ts:247-253)
        self._main = GpuContext(device, high_priority=True)
        self._ctxs: list[GpuContext] = []
        self.init_errors: list[Exception] = []
        for _ in range(n_contexts):
            try:
                self._ctxs.append(GpuContext(device))
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
        self.metrics = metrics if metrics is not None else BlsMetrics()
        self._threads = [threading.Thread(target=self._worker, args=(c,), daemon=True) for c in self._ctxs]
        self._timer = threading.Thread(target=self._buffer_timer, daemon=True)
        for t in self._threads:
            t.start()
        self._timer.start()

    # -- pubkey cache -----------------------------------------------------------
    def load_pubkeys(self, pubkeys48: bytes) -> None:
        """Append validator pubkeys (48 B compressed) to every context's device table,
        all or nothing: bls_gpu_load_pubkeys appends no key of a batch that holds an
        undecodable one, so a failure on the first context leaves every table as it was
        and validator indices stay aligned across contexts."""
        codes = self._ctxs[0].load_pubkeys(pubkeys48, 48)
        if (codes != 0).any():
            bad = int((codes != 0).argmax())
            raise BlsError(f"invalid pubkey at batch index {bad} (code {int(codes[bad])}); no key appended")
        for c in self._ctxs[1:] + [self._main]:
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
        jobs = [self._queue(chunk, batchable)
                for chunk in chunkify_maximize_chunk_size(list(sets), MAX_SIGNATURE_SETS_PER_JOB)]
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

    def close(self) -> None:
        with self._cv:
            self._closed = True
            pending = self._jobs + self._buffer
            self._jobs, self._buffer = [], []
            self._cv.notify_all()
        for j in pending:
            if not j.future.done():
                j.future.set_exception(QueueAborted("QUEUE_ABORTED"))
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

    def _call(self, ctx: GpuContext, reqs, worker_id: int = 0):
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

    def queue_length(self) -> int:
        """blsThreadPool.queueLength (index.ts:130, set on collect)."""
        with self._cv:
            n = len(self._jobs)
        self.metrics.blsThreadPool.queueLength.set(n)
        return n

    def _worker(self, ctx: GpuContext):
        while True:
            with self._cv:
                while not self._jobs and not self._closed:
                    self._cv.wait(timeout=0.05)
                if self._closed:
                    return
                jobs = self._prepare_work()
            if not jobs:
                continue
            tp = self.metrics.blsThreadPool
            now = time.monotonic()
            for j in jobs:
                tp.jobWaitTime.observe(now - j.added)
            tp.totalJobsGroupsStarted.inc(1)
            tp.totalJobsStarted.inc(len(jobs))
            tp.totalSigSetsStarted.inc(sum(len(j.sets) for j in jobs))
            try:
                verdicts, _ = self._call(ctx, [(j.batchable, j.sets) for j in jobs], self._ctxs.index(ctx))
            except Exception as e:  # noqa: BLE001 - reject every job of the call
                for j in jobs:
                    j.future.set_exception(e)
                tp.errorJobsSignatureSetsCount.inc(sum(len(j.sets) for j in jobs))
                continue
            for j, code in zip(jobs, verdicts):
                try:
                    j.future.set_result(self._verdict(code))
                    tp.successJobsSignatureSetsCount.inc(len(j.sets))
                except BlsError as e:
                    j.future.set_exception(e)
                    tp.errorJobsSignatureSetsCount.inc(len(j.sets))
