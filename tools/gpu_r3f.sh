#!/bin/bash
# round 3 (re-entry): GPU tests, default bench with sub-records + CPU baseline, Miller-loop variants, solo trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3f
mkdir -p $O
{ nproc; python3 -c "import os;print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo; } > $O/sys.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-sub-records"
run() { local name=$1; shift; local envs=$1; shift; env $envs timeout -k 10 300 $B "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail $O/$name.err; exit 1; }; }
run split_10x8 BLS_ML_SIMT=2
run coop_10x8 BLS_ML_SIMT=0
run split_14x8 BLS_ML_SIMT=2 --inflight 14
timeout -k 10 600 python -u bench.py > $O/default.json 2> $O/default.err || { echo "default failed"; tail $O/default.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o solo -- python3 "$GRAFT_REPO_ROOT/bench.py" --sets 8192 --inflight 1 --calls-per-pass 1 --steps 3 --warmup 1 --no-cpu-baseline --no-sub-records --latency-runs 3 > "$GRAFT_REPO_ROOT/$O/solo.json" 2> "$GRAFT_REPO_ROOT/$O/solo.err" || { echo "rocprof failed"; exit 1; }
echo done
