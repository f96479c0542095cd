"""Metric names and getAggregatedPubkeysCount (CPU): the GPU verifier feeds the
reference's bls / blsThreadPool series (beacon-node/src/metrics/metrics/lodestar.ts:378-446)."""
from __future__ import annotations

from lodestar_amd.metrics import BlsMetrics, get_aggregated_pubkeys_count
from lodestar_amd.verifier import SignatureSet

REFERENCE_NAMES = {
    "lodestar_bls_aggregated_pubkeys_total",
    "lodestar_bls_thread_pool_time_seconds_sum",
    "lodestar_bls_thread_pool_success_jobs_signature_sets_count",
    "lodestar_bls_thread_pool_error_jobs_signature_sets_count",
    "lodestar_bls_thread_pool_queue_job_wait_time_seconds",
    "lodestar_bls_thread_pool_queue_length",
    "lodestar_bls_thread_pool_job_groups_started_total",
    "lodestar_bls_thread_pool_jobs_started_total",
    "lodestar_bls_thread_pool_sig_sets_started_total",
    "lodestar_bls_thread_pool_batch_retries_total",
    "lodestar_bls_thread_pool_batch_sigs_success_total",
    "lodestar_bls_thread_pool_latency_to_worker",
    "lodestar_bls_thread_pool_latency_from_worker",
    "lodestar_bls_thread_pool_main_thread_time_seconds",
}


def test_metric_names_match_reference():
    m = BlsMetrics()
    names = {x.name for x in m.bls.all() + m.blsThreadPool.all()}
    assert names == REFERENCE_NAMES
    assert m.blsThreadPool.jobWaitTime.buckets == (0.1, 1, 10)
    assert m.blsThreadPool.mainThreadDurationInThreadPool.buckets == (0.1, 1)
    assert m.blsThreadPool.jobsWorkerTime.label_names == ("workerId",)


def test_metric_values_and_exposition():
    m = BlsMetrics()
    tp = m.blsThreadPool
    tp.jobsWorkerTime.inc({"workerId": 3}, 0.25)
    tp.jobsWorkerTime.inc({"workerId": 3}, 0.5)
    tp.batchRetries.inc(2)
    tp.jobWaitTime.observe(0.05)
    tp.jobWaitTime.observe(5.0)
    assert tp.jobsWorkerTime.get({"workerId": 3}) == 0.75
    assert tp.batchRetries.get() == 2
    text = m.expose()
    assert 'lodestar_bls_thread_pool_time_seconds_sum{workerId="3"} 0.75' in text
    assert 'lodestar_bls_thread_pool_queue_job_wait_time_seconds_bucket{le="0.1"} 1' in text
    assert 'lodestar_bls_thread_pool_queue_job_wait_time_seconds_bucket{le="10"} 2' in text
    assert 'lodestar_bls_thread_pool_queue_job_wait_time_seconds_count 2' in text


def test_get_aggregated_pubkeys_count():
    """chain/bls/utils.ts:18-26: only aggregate-type sets count, by their key count."""
    sets = [SignatureSet(5, b"\0" * 32, b""), SignatureSet([1, 2, 3], b"\0" * 32, b""),
            SignatureSet(b"\1" * 96, b"\0" * 32, b""), SignatureSet([7], b"\0" * 32, b""),
            SignatureSet([], b"\0" * 32, b"")]
    assert get_aggregated_pubkeys_count(sets) == 4
    assert get_aggregated_pubkeys_count([]) == 0
