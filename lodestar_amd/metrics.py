"""Verifier metrics under the reference's names (beacon-node/src/metrics/metrics/lodestar.ts:378-446).

`BlsMultiThreadWorkerPool` feeds `metrics.bls.aggregatedPubkeys` and the
`metrics.blsThreadPool.*` series (multithread/index.ts:130,136,139,317-366); the GPU
verifier feeds the same series so existing dashboards keep working.  A GPU context
plays the role of a worker: `workerId` is the context index, the "worker time" is
the device time of the call (HIP events), and the latencies to / from the worker are
the host staging before the call and the verdict hand-back after it.

Dependency-free: counters, gauges and histograms with the reference's metric names,
label sets and buckets, rendered in the Prometheus text format by `expose()`.
"""
from __future__ import annotations

import threading
import time
from collections import defaultdict


class _Metric:
    def __init__(self, name: str, help_: str, kind: str, label_names=(), buckets=None):
        self.name, self.help, self.kind = name, help_, kind
        self.label_names = tuple(label_names)
        self.buckets = tuple(buckets) if buckets else None
        self._lock = threading.Lock()
        self._values = defaultdict(float)
        self._hist = defaultdict(lambda: [[0] * (len(self.buckets) + 1), 0.0, 0])

    def _key(self, labels):
        labels = labels or {}
        return tuple(str(labels.get(k, "")) for k in self.label_names)

    # gauge / counter (the reference registers its counters as gauges and .inc()s them)
    def inc(self, labels=None, value: float = 1.0):
        if not isinstance(labels, dict) and labels is not None:
            labels, value = None, labels
        with self._lock:
            self._values[self._key(labels)] += value

    def set(self, value: float, labels=None):
        with self._lock:
            self._values[self._key(labels)] = value

    def get(self, labels=None) -> float:
        with self._lock:
            return self._values.get(self._key(labels), 0.0)

    # histogram
    def observe(self, value: float, labels=None):
        with self._lock:
            h = self._hist[self._key(labels)]
            for i, b in enumerate(self.buckets):
                if value <= b:
                    h[0][i] += 1
            h[0][-1] += 1
            h[1] += value
            h[2] += 1

    def count(self, labels=None) -> int:
        with self._lock:
            return self._hist[self._key(labels)][2] if self._key(labels) in self._hist else 0

    def start_timer(self, labels=None):
        t0 = time.perf_counter()
        return lambda: self.observe(time.perf_counter() - t0, labels)

    def expose(self) -> str:
        out = [f"# HELP {self.name} {self.help}", f"# TYPE {self.name} {self.kind}"]

        def lab(key, extra=""):
            parts = [f'{k}="{v}"' for k, v in zip(self.label_names, key) if v != ""]
            if extra:
                parts.append(extra)
            return "{" + ",".join(parts) + "}" if parts else ""

        with self._lock:
            if self.kind == "histogram":
                for key, (cnts, s, n) in self._hist.items():
                    for b, c in zip(self.buckets, cnts):
                        le = 'le="%s"' % b
                        out.append(f"{self.name}_bucket{lab(key, le)} {c}")
                    le = 'le="+Inf"'
                    out.append(f"{self.name}_bucket{lab(key, le)} {cnts[-1]}")
                    out.append(f"{self.name}_sum{lab(key)} {s}")
                    out.append(f"{self.name}_count{lab(key)} {n}")
            else:
                for key, v in self._values.items():
                    out.append(f"{self.name}{lab(key)} {v}")
        return "\n".join(out)


class _Group:
    def __init__(self, **metrics):
        self.__dict__.update(metrics)

    def all(self):
        return list(self.__dict__.values())


class BlsMetrics:
    """metrics.bls and metrics.blsThreadPool of lodestar.ts:378-446."""

    def __init__(self):
        g, h = "gauge", "histogram"
        self.bls = _Group(
            aggregatedPubkeys=_Metric("lodestar_bls_aggregated_pubkeys_total",
                                      "Total aggregated pubkeys for BLS validation", g),
        )
        self.blsThreadPool = _Group(
            jobsWorkerTime=_Metric("lodestar_bls_thread_pool_time_seconds_sum",
                                   "Total time spent verifying signature sets measured on the worker", g,
                                   ["workerId"]),
            successJobsSignatureSetsCount=_Metric("lodestar_bls_thread_pool_success_jobs_signature_sets_count",
                                                  "Count of total verified signature sets", g),
            errorJobsSignatureSetsCount=_Metric("lodestar_bls_thread_pool_error_jobs_signature_sets_count",
                                                "Count of total error-ed signature sets", g),
            jobWaitTime=_Metric("lodestar_bls_thread_pool_queue_job_wait_time_seconds",
                                "Time from job added to the queue to starting the job in seconds", h,
                                buckets=[0.1, 1, 10]),
            queueLength=_Metric("lodestar_bls_thread_pool_queue_length",
                                "Count of total block processor queue length", g),
            totalJobsGroupsStarted=_Metric("lodestar_bls_thread_pool_job_groups_started_total",
                                           "Count of total jobs groups started in bls thread pool, job groups "
                                           "include +1 jobs", g),
            totalJobsStarted=_Metric("lodestar_bls_thread_pool_jobs_started_total",
                                     "Count of total jobs started in bls thread pool, jobs include +1 signature "
                                     "sets", g),
            totalSigSetsStarted=_Metric("lodestar_bls_thread_pool_sig_sets_started_total",
                                        "Count of total signature sets started in bls thread pool, sig sets "
                                        "include 1 pk, msg, sig", g),
            batchRetries=_Metric("lodestar_bls_thread_pool_batch_retries_total",
                                 "Count of total batches that failed and had to be verified again.", g),
            batchSigsSuccess=_Metric("lodestar_bls_thread_pool_batch_sigs_success_total",
                                     "Count of total batches that failed and had to be verified again.", g),
            latencyToWorker=_Metric("lodestar_bls_thread_pool_latency_to_worker",
                                    "Time from sending the job to the worker and the worker receiving it", h,
                                    buckets=[0.1]),
            latencyFromWorker=_Metric("lodestar_bls_thread_pool_latency_from_worker",
                                      "Time from the worker sending the result and the main thread receiving it",
                                      h, buckets=[0.1]),
            mainThreadDurationInThreadPool=_Metric("lodestar_bls_thread_pool_main_thread_time_seconds",
                                                   "Time to verify signatures in main thread with thread pool mode",
                                                   h, buckets=[0.1, 1]),
        )

    def expose(self) -> str:
        return "\n".join(m.expose() for m in self.bls.all() + self.blsThreadPool.all()) + "\n"


def get_aggregated_pubkeys_count(sets) -> int:
    """getAggregatedPubkeysCount (chain/bls/utils.ts:18-26): the pubkeys of the
    aggregate-type sets (a set whose pubkey is a list of table indices)."""
    n = 0
    for s in sets:
        pk = s.pubkey
        if not isinstance(pk, (int, bytes, bytearray, memoryview)):
            n += len(pk)
    return n
