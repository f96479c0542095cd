#!/bin/bash
# round 3, first GPU call: GPU tests, design probes, a short bench, a solo kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3a
mkdir -p $O
{ nproc; python3 -c "import os;print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo; } > $O/sys.txt 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
timeout -k 10 240 python -u tools/probe_ml.py > $O/probe.json 2> $O/probe.err || { echo "probe failed"; tail $O/probe.err; exit 1; }
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o solo -- python3 "$GRAFT_REPO_ROOT/bench.py" --sets 8192 --inflight 1 --calls-per-pass 1 --steps 3 --warmup 1 --no-cpu-baseline --latency-runs 3 > "$GRAFT_REPO_ROOT/$O/solo.json" 2> "$GRAFT_REPO_ROOT/$O/solo.err" || { echo "rocprof failed"; exit 1; }
echo done
