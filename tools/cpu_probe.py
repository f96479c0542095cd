"""Host CPU the cfg2 timed region costs: process CPU seconds per wall second and the
cgroup's throttling counters over bench.timed_calls at the default shape, to tell whether
the threads waiting on the device (hipStreamSynchronize) compete for the job's CPU quota.
Measurement tool.

  python tools/cpu_probe.py [--inflight 16] [--calls-per-pass 22] [--steps 8]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def cpu_stat() -> dict:
    try:
        return {k: int(v) for k, v in (ln.split() for ln in open("/sys/fs/cgroup/cpu.stat"))}
    except OSError:
        return {}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--inflight", type=int, default=16)
    ap.add_argument("--calls-per-pass", type=int, default=22)
    ap.add_argument("--steps", type=int, default=8)
    a = ap.parse_args()
    from lodestar_amd.native import GpuContext, pack_requests

    ctxs = [GpuContext(0) for _ in range(a.inflight)]
    try:
        n = 1024 * a.calls_per_pass
        w = bench.make_workload(ctxs[0], n, 0, 0)
        sets = w[2]
        pks48 = ctxs[0].sk_to_pk(b"".join(bench.interop_sk(i) for i in range(len(sets)))).tobytes()
        for c in ctxs[1:]:
            c.load_pubkeys(pks48, 48)
        calls = [pack_requests([(True, [s]) for s in sets[k:k + 1024]]) for k in range(0, len(sets), 1024)]
        batches = [calls] * len(ctxs)
        bench.timed_calls(ctxs, batches, 2)
        t0, s0 = os.times(), cpu_stat()
        el, _, ok = bench.timed_calls(ctxs, batches, a.steps)
        t1, s1 = os.times(), cpu_stat()
        cpu = (t1.user + t1.system) - (t0.user + t0.system)
        print(json.dumps({"sets_per_s": round(a.steps * len(ctxs) * n / el, 1), "verdicts_ok": ok,
                          "cpu_s_per_wall_s": round(cpu / el, 3),
                          "user_s_per_wall_s": round((t1.user - t0.user) / el, 3),
                          "cgroup": {k: s1.get(k, 0) - s0.get(k, 0) for k in ("usage_usec", "nr_throttled",
                                                                               "throttled_usec")},
                          "env": {k: v for k, v in os.environ.items() if k.startswith(("BLS_", "HIP_", "ROC_", "HSA_"))
                                  and k != "HSA_ENABLE_IPC_MODE_LEGACY"}}))
    finally:
        for c in ctxs:
            c.close()


if __name__ == "__main__":
    main()
